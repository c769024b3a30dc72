# pipeline depth A/B with the cloud prefetch: depth 6 / 8 / 10, twice
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do for d in 8 10 12; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device-rate --steps 20 --warmup 5 --depth $d > gpurun_out/dd.log 2>&1 || { tail -20 gpurun_out/dd.log; exit 1; }
  grep '^{' gpurun_out/dd.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[depth $d]', d['value'], d['value_median'], d['ms_per_step'], d['frame_latency_ms'], d['stages_ms']['gvd_delaunay'])"
done; done
