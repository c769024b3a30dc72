#!/bin/bash
# Bench-only A/B of environment settings on the C2 bench (no profiler): for each entry of AB_SETS (space separated;
# an entry is VAR=value[,VAR=value...], "-" for none) one bench process, ROUNDS times in alternation; prints the frame
# p50 and the stage medians named in STAGES. Lines go to gpurun_out/${TAG}_abbench.txt.
# Usage: TAG=r05m AB_SETS="AOS_UP_THREADS=8 AOS_UP_THREADS=16" ROUNDS=2 bash tools/ab_bench_env.sh
set -e
TAG=${TAG:-r05x}
out=gpurun_out/${TAG}_abbench.txt
mkdir -p gpurun_out
: > $out
for r in $(seq 1 ${ROUNDS:-2}); do
  k=0
  for set in ${AB_SETS:--}; do
    k=$((k + 1))
    envs=()
    [ "$set" != "-" ] && IFS=',' read -ra envs <<< "$set"
    log=gpurun_out/${TAG}_abb_${r}_$k.log
    env "${envs[@]}" timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate \
      --steps ${STEPS_N:-20} --warmup 5 > $log 2> $log.err
    python3 - "$set" "$log" "${STAGES:-seedgen_total}" <<'EOF' | tee -a $out
import json, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][-1]
s = d["stages_ms_p50"]
print(sys.argv[1], "frame p50", d["frame_ms"]["p50"], " ".join(f"{k} {s.get(k)}" for k in sys.argv[3].split(",")))
EOF
  done
done
