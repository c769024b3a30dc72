# final round-2 check: GPU suite, smoke, the default bench line (CPU baseline included), depth 6 vs 8 at 20 steps
set -e
export TMPDIR=/tmp
TAG=r02s
mkdir -p gpurun_out
TAG=$TAG STEPS="test smoke" bash tools/gpu_r02.sh
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
grep '^{' gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default@20', d['value'], d['value_median'], d['ms_per_step'], d['frame_latency_ms'], d['roofline']['frac'], d['cpu_baseline']['value'], d['device_resident']['value'])"
for d in 6 8; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device-rate --steps 20 --warmup 5 --depth $d > gpurun_out/${TAG}_d$d.log 2>&1 || { tail -20 gpurun_out/${TAG}_d$d.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_d$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('depth $d', d['value'], d['value_median'], d['frame_latency_ms'])"
done
