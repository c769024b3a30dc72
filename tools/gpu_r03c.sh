#!/bin/bash
# r03c: sequential bench (copy-stream overlap), C4 stream with the allocation / cells trace
set -e
mkdir -p gpurun_out
STEPS="bench" TAG=r03c BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_r03.sh
AOS_TRACE=1 STEPS="stream" TAG=r03c STREAM_ARGS="--trace --steps 16" bash tools/gpu_r03.sh
