#!/bin/bash
# Upload A/B on the box: for each entry of AB_SETS (VAR=value[,VAR=value...]) one C2 bench process with AOS_TRACE=1,
# ROUNDS times alternating; prints the frame p50 and the medians of the upload's gather end and DMA end (AOS_TRACE
# "upload" lines, ms after the upload started).
set -e
mkdir -p gpurun_out
out=gpurun_out/${TAG:-r05x}_abupload.txt
: > $out
for r in $(seq 1 ${ROUNDS:-2}); do
  for set in ${AB_SETS:--}; do
    envs=()
    [ "$set" != "-" ] && IFS=',' read -ra envs <<< "$set"
    log=gpurun_out/${TAG:-r05x}_abu.log
    env "${envs[@]}" AOS_TRACE=1 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate \
      --steps 12 --warmup 3 > $log 2> $log.err
    python3 - "$set" "$log" <<'PY' | tee -a $out
import json, re, statistics, sys
d = [json.loads(l) for l in open(sys.argv[2]) if l.startswith("{")][-1]
g, m = [], []
for l in open(sys.argv[2] + ".err"):
    x = re.search(r"trace upload\] at [0-9.]+: gathered ([0-9.]+) dma_done ([0-9.]+)", l)
    if x: g.append(float(x.group(1))); m.append(float(x.group(2)))
print(sys.argv[1], "frame p50", d["frame_ms"]["p50"], "gathered", round(statistics.median(g), 3), "dma_done",
      round(statistics.median(m), 3), "gvd_total", d["stages_ms_p50"]["gvd_total"])
PY
  done
done
