#!/bin/bash
# ROR A/B on the box: builds tools/rorbench (the product's flags) and the variants named in RB_VARIANTS
# ("tag:DEFS" pairs, DEFS comma-separated, e.g. "_g1024:-DAOS_RT_G=1024,-DAOS_RT_STB=1024") there, then runs
# them alternating, 3 rounds, on the C2 cloud (RB_STEP: 12 = the packed layout of the host upload, 16).
# RB_ENV: extra environment for every run (e.g. "RORBENCH_CS=1.6").
set -e
mkdir -p gpurun_out
timeout -k 10 300 bash tools/rorbench/build.sh > gpurun_out/rb_build.log 2>&1 || { tail -20 gpurun_out/rb_build.log; exit 1; }
for v in ${RB_VARIANTS:-}; do
  TAG=${v%%:*} DEFS="$(echo ${v#*:} | tr , " ")" timeout -k 10 300 bash tools/rorbench/build.sh >> gpurun_out/rb_build.log 2>&1 \
    || { tail -20 gpurun_out/rb_build.log; exit 1; }
done
for rep in 1 2 3; do
  for b in tools/rorbench/rorbench $(for v in ${RB_VARIANTS:-}; do echo tools/rorbench/rorbench${v%%:*}; done); do
    log=gpurun_out/rb_$(basename $b)_$rep.log
    env ${RB_ENV:-} timeout -k 10 120 $b 4096 10000000 10 ${RB_STEP:-12} > $log 2>&1 || { tail -5 $log; exit 1; }
    echo "$(basename $b) rep $rep: $(grep -o 'hash [0-9a-f]*' $log) | $(tail -1 $log | cut -c1-110)"
  done
done
