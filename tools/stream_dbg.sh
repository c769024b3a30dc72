set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in "" "--markers-every-frame"; do
timeout -k 10 300 python -u bench.py --stream --steps 16 --warmup 2 $m > gpurun_out/sdbg.log 2>&1 || { tail -20 gpurun_out/sdbg.log; exit 1; }
grep '^{' gpurun_out/sdbg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stream']; print('$m'); print(s['scan_latency_ms']); print(s['scan_markers']); print(s['scan_delaunay_ms'])"
done
