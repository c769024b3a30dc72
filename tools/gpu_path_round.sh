#!/bin/bash
# GPU check of the path planner (aos_path_plan): its parity tests, then the C2 planning latency.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_path.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_path.log 2>&1 || { tail -60 gpurun_out/pytest_path.log; exit 1; }
tail -3 gpurun_out/pytest_path.log
timeout -k 10 600 python -u tools/bench_path.py --config ${CFG:-C2} > gpurun_out/bench_path.log 2>&1 || { tail -30 gpurun_out/bench_path.log; exit 1; }
grep '^{' gpurun_out/bench_path.log
