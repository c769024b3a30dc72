#!/bin/bash
# runs the rorbench_* binaries built by count_variants.sh (one GPU step each, own time limit)
set -e
mkdir -p gpurun_out
for b in tools/rorbench/rorbench_*; do
  [ -x "$b" ] || continue
  for fl in 0 512; do
    timeout -k 10 120 $b 4096 10000000 10 12 $fl > gpurun_out/cv_$(basename $b)_$fl.log 2>&1 || { tail -5 gpurun_out/cv_$(basename $b)_$fl.log; exit 1; }
    echo "$(basename $b) flush $fl: $(tail -2 gpurun_out/cv_$(basename $b)_$fl.log | head -1) $(tail -1 gpurun_out/cv_$(basename $b)_$fl.log | cut -c1-60)"
  done
done
