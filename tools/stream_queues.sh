# the streaming map with the markers throttle at several GPU_MAX_HW_QUEUES (the stall after markers scans)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q AOS_BENCH_STREAM_THROTTLE=1 timeout -k 10 300 python -u bench.py --stream --steps 12 --warmup 2 > gpurun_out/sq$q.log 2>&1 || { tail -20 gpurun_out/sq$q.log; exit 1; }
  grep '^{' gpurun_out/sq$q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stream']; print('queues $q', s['scan_latency_ms'], s['scan_markers'])"
done
