#!/bin/bash
# r03e: the stream stall with glibc kept from returning freed memory to the OS (no munmap / heap trim),
# then the ROR count-pass / neighbour-scan variants
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
MALLOC_TRIM_THRESHOLD_=17179869184 MALLOC_MMAP_THRESHOLD_=17179869184 AOS_TRACE=1 timeout -k 10 300 python -u bench.py --stream --steps 12 --warmup 2 --trace > gpurun_out/r03e_stream_nomunmap.log 2> gpurun_out/r03e_stream_nomunmap.err
grep "dedup" gpurun_out/r03e_stream_nomunmap.err | awk '{print $10,$11}' | tr '\n' ' '; echo
timeout -k 10 600 bash tools/rorbench/run_variants.sh
