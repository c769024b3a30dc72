# cgroup CPU throttling during the stream (throttled markers) and the pipelined bench: cpu.stat deltas
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.stat
AOS_BENCH_STREAM_THROTTLE=1 timeout -k 10 300 python -u bench.py --stream --steps 12 --warmup 2 > gpurun_out/tp1.log 2>&1 || { tail -20 gpurun_out/tp1.log; exit 1; }
grep '^{' gpurun_out/tp1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stream']; print('stream', s['scan_latency_ms'])"
cat /sys/fs/cgroup/cpu.stat
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device-rate --steps 20 --warmup 5 > gpurun_out/tp2.log 2>&1 || { tail -20 gpurun_out/tp2.log; exit 1; }
grep '^{' gpurun_out/tp2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['frame_latency_ms'])"
cat /sys/fs/cgroup/cpu.stat
