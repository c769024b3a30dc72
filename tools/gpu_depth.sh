set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r02c_pytest_pipe.log 2>&1 || { tail -40 gpurun_out/r02c_pytest_pipe.log; exit 1; }
tail -2 gpurun_out/r02c_pytest_pipe.log
for d in 4 1 6 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --depth $d --steps 20 --warmup 5 > gpurun_out/r02c_bench_d$d.log 2> gpurun_out/r02c_bench_d$d.err || { tail -20 gpurun_out/r02c_bench_d$d.err; exit 1; }
  grep '^{' gpurun_out/r02c_bench_d$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('depth', $d, d['value'], d['value_median'], d['ms_per_step'], d['frame_latency_ms'], d['device_resident']['value'], d['stages_ms']['gvd_delaunay'], d['stages_ms']['gvd_cells'])"
done
