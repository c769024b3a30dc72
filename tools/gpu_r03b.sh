#!/bin/bash
# r03b: ROR variants (rorbench), the GPU suite, the sequential bench, the C4 stream with host trace
set -e
mkdir -p gpurun_out
timeout -k 10 400 bash tools/rorbench/run_variants.sh
STEPS="test bench" TAG=r03b BENCH_ARGS="--trace" bash tools/gpu_r03.sh
AOS_TRACE=1 STEPS="stream" TAG=r03b STREAM_ARGS="--trace" bash tools/gpu_r03.sh
