#!/bin/bash
# A/B timing of ROR tile-walk variants (libaos_gpu_<v>.so built with DEFS=-DAOS_RT_VARIANT=<v>):
# device-resident C2 bench, ROR sub-stage times from the HIP events. Timing only: variants 1/2 are wrong.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "" ${VARIANTS:-_1 _2}; do
  L=$PWD/active-orchard-slam_amd/libaos_gpu$v.so
  AOS_GPU_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --device-io --no-device-rate --steps 10 --warmup 3 > gpurun_out/ab_rt$v.log 2> gpurun_out/ab_rt$v.err || { tail -20 gpurun_out/ab_rt$v.err; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab_rt$v.log') if l.startswith('{')][0]); s=d['stages_ms']; print('variant[$v]', d['median_ms'], 'count', s['seedgen_ror_bin'], 'scatter', s['seedgen_ror_scatter'], 'tiles', s['seedgen_ror_count'], 'ror stage', s['seedgen_ror'])"
done
