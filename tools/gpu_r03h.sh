#!/bin/bash
# distributed cluster stage on the GPU (tiled tests) + numpy hugepage A/B of the sequential bench
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiled.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03h_pytest_tiled.log 2>&1 || { tail -60 gpurun_out/r03h_pytest_tiled.log; exit 1; }
tail -3 gpurun_out/r03h_pytest_tiled.log
for k in 1 2; do
  for hp in 0 1; do
    AOS_NUMPY_HUGEPAGE=$hp timeout -k 10 200 python -u bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-device-rate --no-pipelined-rate > gpurun_out/r03h_bench_hp${hp}_$k.log 2> gpurun_out/r03h_bench_hp${hp}_$k.err || { tail -20 gpurun_out/r03h_bench_hp${hp}_$k.err; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/r03h_bench_hp${hp}_$k.log'):
    if l.startswith('{'):
        d=json.loads(l); print('hp=$hp run $k', d['value'], d['frame_ms'], d['stages_ms']['gvd_delaunay'], d['stages_ms'].get('gvd_cells'))
"
  done
done
