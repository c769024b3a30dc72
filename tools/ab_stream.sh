#!/bin/bash
# A/B of ROR variants on the C4 stream bench (timing only: variant builds may skip work)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "" _a; do
  L=$PWD/active-orchard-slam_amd/libaos_gpu$v.so
  AOS_GPU_LIB=$L timeout -k 10 300 python bench.py --stream --steps 6 --warmup 2 > gpurun_out/abs$v.log 2>&1 || { tail -20 gpurun_out/abs$v.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/abs$v.log') if l.startswith('{')][0]); s=d['stages_ms']; print('variant[$v]', d['ms_per_step'], 'bin', s['seedgen_ror_bin'], 'scatter', s['seedgen_ror_scatter'], 'count', s['seedgen_ror_count'], 'ror', s['seedgen_ror'], 'thin', s['seedgen_thin'], 'cluster', s['seedgen_cluster'], 'total', s['seedgen_total'])"
done
