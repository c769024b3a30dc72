#!/bin/bash
# runs the rorbench_* binaries built by count_variants.sh (one GPU step each, own time limit) with the cache
# states in MODES (flush_mb argument: 0 warm, 512 = 512 MB memset between frames, -1 = the cloud re-uploaded
# from pinned host memory each frame, as in a product frame)
set -e
mkdir -p gpurun_out
for b in tools/rorbench/rorbench_*; do
  [ -x "$b" ] || continue
  for fl in ${MODES:-0 512 -1}; do
    log=gpurun_out/cv_$(basename $b)_$fl.log
    timeout -k 10 120 $b 4096 10000000 10 12 $fl > $log 2>&1 || { tail -5 $log; exit 1; }
    echo "$(basename $b) flush $fl: $(tail -2 $log | head -1 | cut -c1-60) $(tail -1 $log | cut -c1-75)"
  done
done
