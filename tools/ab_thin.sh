#!/bin/bash
# A/B timing of k_thin_block variants (libaos_gpu_<v>.so built with DEFS=-DAOS_THIN_TB=... / -DAOS_THIN_TH=...):
# C2 bench, thinning stage ms from the HIP events (opening + the temporal-block launches + one read-back).
set -e
mkdir -p gpurun_out
for v in "" ${VARIANTS-_t512 _t1024 _h128}; do
  L=$PWD/active-orchard-slam_amd/libaos_gpu$v.so
  AOS_GPU_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --device-io --no-device-rate --steps 10 --warmup 3 > gpurun_out/ab_thin$v.log 2> gpurun_out/ab_thin$v.err || { tail -20 gpurun_out/ab_thin$v.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab_thin$v.log') if l.startswith('{')][0]); s=d['stages_ms']; print('variant[$v]', 'thin', s['seedgen_thin'], 'T', d['frame']['T'], 'seedgen', s['seedgen_total'])"
done
