#!/bin/bash
# runs every built tools/rorbench/rorbench_* variant on the C2 cloud (one GPU step each, own time limit)
set -e
mkdir -p gpurun_out
for b in tools/rorbench/rorbench tools/rorbench/rorbench_*; do
  [ -x "$b" ] || continue
  echo "== $(basename $b)"
  timeout -k 10 120 $b 4096 10000000 10 > gpurun_out/$(basename $b).log 2>&1 || { tail -5 gpurun_out/$(basename $b).log; exit 1; }
  tail -3 gpurun_out/$(basename $b).log
done
