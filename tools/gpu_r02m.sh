#!/bin/bash
# new thinning predicate / shrinking rows: GPU suite, thinning A/B (default vs _h128), bench depth 4 vs 6
set -e
export TMPDIR=/tmp
TAG=${TAG:-r02m}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
AOS_GPU_LIB=$PWD/active-orchard-slam_amd/libaos_gpu_h128.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 -k "golden or c1 or blob" > gpurun_out/${TAG}_pytest_h128.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_h128.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_h128.log
VARIANTS="_h128" bash tools/ab_thin.sh
for d in 4 6; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device-rate --steps 20 --warmup 5 --depth $d > gpurun_out/${TAG}_bench_d$d.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_d$d.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_bench_d$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('depth', $d, 'value', d['value'], 'median', d['value_median'], 'ms', d['ms_per_step'], 'lat', d['frame_latency_ms'], 'thin', d['stages_ms']['seedgen_thin'], 'delaunay', d['stages_ms']['gvd_delaunay'])"
done
