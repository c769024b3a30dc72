#!/bin/bash
# round-3 validation: GPU tests, default bench, pipelined depth 4 and 6 (frame latency), stream
set -e
mkdir -p gpurun_out
STEPS="test bench stream" TAG=r03g bash tools/gpu_r03.sh
for d in 4 6; do
  timeout -k 10 300 python -u bench.py --pipelined --depth $d --steps 30 --warmup 4 --no-cpu-baseline --no-device-rate > gpurun_out/r03g_pipe_d$d.log 2> gpurun_out/r03g_pipe_d$d.err || { tail -20 gpurun_out/r03g_pipe_d$d.err; exit 1; }
  grep '^{' gpurun_out/r03g_pipe_d$d.log | cut -c1-400
done
