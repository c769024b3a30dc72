# cloud prefetch: pipeline tests, full GPU suite, bench with / without prefetch at depth 6 and 8
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r02u_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r02u_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r02u_pytest_gpu.log
for args in "" "--no-prefetch" "--depth 8"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device-rate --steps 20 --warmup 5 $args > gpurun_out/r02u_bench.log 2>&1 || { tail -20 gpurun_out/r02u_bench.log; exit 1; }
  grep '^{' gpurun_out/r02u_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$args]', d['value'], d['value_median'], d['ms_per_step'], d['frame_latency_ms'])"
done
