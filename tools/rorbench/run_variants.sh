#!/bin/bash
# runs every built tools/rorbench/rorbench_* variant on the C2 cloud (one GPU step each, own time limit)
set -e
mkdir -p gpurun_out
for b in tools/rorbench/rorbench tools/rorbench/rorbench_*; do
  [ -x "$b" ] || continue
  echo "== $(basename $b)"
  for st in 16 12; do
    timeout -k 10 120 $b 4096 10000000 10 $st > gpurun_out/$(basename $b)_$st.log 2>&1 || { tail -5 gpurun_out/$(basename $b)_$st.log; exit 1; }
    echo "-- step $st"; tail -3 gpurun_out/$(basename $b)_$st.log
  done
done
