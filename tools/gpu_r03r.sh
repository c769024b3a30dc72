#!/bin/bash
# placement of the grids' D2H (AOS_GRID_COPY 0: beside the cluster stage, 1: after it), A/B/A/B
set -e
mkdir -p gpurun_out
for k in 1 2; do
  for m in 0 1; do
    AOS_GRID_COPY=$m timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-device-rate --no-pipelined-rate > gpurun_out/r03r_copy${m}_$k.log 2> gpurun_out/r03r_copy${m}_$k.err || { tail -20 gpurun_out/r03r_copy${m}_$k.err; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/r03r_copy${m}_$k.log'):
    if l.startswith('{'):
        d=json.loads(l); s=d['stages_ms']; print('copy=$m run $k', d['value'], d['frame_ms']['p50'], 'seedgen', s['seedgen_total'], 'cluster', s['seedgen_cluster'], 'seeds', s['seedgen_seeds'], 'thin', s['seedgen_thin'], 'delaunay', s['gvd_delaunay'])
"
  done
done
