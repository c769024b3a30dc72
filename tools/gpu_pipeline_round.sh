#!/bin/bash
# GPU check of the pipelined GVD: the GPU suite (incl. test_gpu_pipeline.py), then the C2 bench
# sequential (default) and pipelined over 40 frames, and the C4 stream bench.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | cut -c1-200
timeout -k 10 400 python bench.py --no-cpu-baseline --pipeline --steps 40 --warmup 3 > gpurun_out/bench_pipe.log 2>&1 || { tail -20 gpurun_out/bench_pipe.log; exit 1; }
grep '^{' gpurun_out/bench_pipe.log | cut -c1-200
timeout -k 10 400 python bench.py --stream --steps 10 --warmup 2 > gpurun_out/bench_stream.log 2>&1 || { tail -20 gpurun_out/bench_stream.log; exit 1; }
grep '^{' gpurun_out/bench_stream.log | cut -c1-200
