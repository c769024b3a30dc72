#!/bin/bash
# Kernel-trace A/B of environment settings on the C2 bench: for each entry of AB_SETS (space separated; an entry
# is VAR=value[,VAR=value...], "-" for none) one rocprofv3 --kernel-trace run, then the per-frame trace line and
# the kernels matching KERNELS (a grep -E pattern) from tools/kt_summary.py. Lines go to gpurun_out/${TAG}_abenv.txt.
# Usage: TAG=r05j AB_SETS="- AOS_CCL_TB=1024 AOS_CCL_CHUNK=1024" KERNELS="k_ccl" bash tools/ab_env.sh
set -e
TAG=${TAG:-r05x}
R=$PWD
out=gpurun_out/${TAG}_abenv.txt
mkdir -p gpurun_out
: > $out
k=0
for set in ${AB_SETS:--}; do
  k=$((k + 1))
  envs=()
  [ "$set" != "-" ] && IFS=',' read -ra envs <<< "$set"
  d=gpurun_out/${TAG}_ab$k
  rm -rf $d
  (cd /tmp && env "${envs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$d -o kt \
    -- python3 $R/bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 10 --warmup 2 > $R/$d.log 2>&1)
  python3 tools/kt_summary.py $d 12 > $d.txt
  {
    echo "== $set: $(grep -o '"p50": [0-9.]*' $d.log | head -1)"
    grep "trace frames" $d.txt || true
    grep -E "${KERNELS:-k_}" $d.txt | head -12 || true
  } | tee -a $out
done
