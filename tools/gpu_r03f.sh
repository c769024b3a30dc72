#!/bin/bash
# r03f: the stream stall with numpy's hugepage madvise off; ROR default rebuilt
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
AOS_BENCH_NUMPY_HUGEPAGE=0 AOS_TRACE=1 timeout -k 10 300 python -u bench.py --stream --steps 12 --warmup 2 --trace > gpurun_out/r03f_stream_nohuge.log 2> gpurun_out/r03f_stream_nohuge.err
grep "dedup" gpurun_out/r03f_stream_nohuge.err | awk '{print $10,$11}' | tr '\n' ' '; echo
timeout -k 10 200 tools/rorbench/rorbench 4096 10000000 10 12 | tail -2
