#!/bin/bash
# A/B of ROR kernel variants: default build vs libaos_gpu_a.so (see the DEFS it was built with). Parity tests run against each build first.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "" _a; do
  L=$PWD/active-orchard-slam_amd/libaos_gpu$v.so
  AOS_GPU_LIB=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 -k "c0 or c1 or overflow or golden" > gpurun_out/ab_pytest$v.log 2>&1 || { tail -30 gpurun_out/ab_pytest$v.log; exit 1; }
  tail -1 gpurun_out/ab_pytest$v.log
  AOS_GPU_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/ab$v.log 2>&1 || { tail -20 gpurun_out/ab$v.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab$v.log') if l.startswith('{')][0]); s=d['stages_ms']; print('variant[$v]', d['ms_per_step'], 'bin', s['seedgen_ror_bin'], 'scatter', s['seedgen_ror_scatter'], 'count', s['seedgen_ror_count'], 'ror stage', s['seedgen_ror'])"
done
