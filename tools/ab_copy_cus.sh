#!/bin/bash
# A/B of the CU-masked copy stream (AOS_COPY_CUS): alternating bench processes on one box, then a kernel trace
# of each setting; the lines go to gpurun_out/${TAG}_ab.txt
set -e
TAG=${TAG:-r05e}
mkdir -p gpurun_out
out=gpurun_out/${TAG}_ab.txt
: > $out
for v in 0 16 0 16; do
  AOS_COPY_CUS=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate \
    --steps 30 --warmup 5 > gpurun_out/${TAG}_ab_$v.log 2> gpurun_out/${TAG}_ab_$v.err
  python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/${TAG}_ab_$v.log') if l.startswith('{')][-1])
s=d['stages_ms_p50']
print('AOS_COPY_CUS=$v frame p50', d['frame_ms']['p50'], 'cluster p50', s['seedgen_cluster'], 'seeds', s['seedgen_seeds'], 'seedgen', s['seedgen_total'])
" | tee -a $out
done
for v in 0 16; do
  rm -rf gpurun_out/${TAG}_kt$v
  (cd /tmp && AOS_COPY_CUS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/gpurun_out/${TAG}_kt$v -o kt \
    -- python3 $OLDPWD/bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 10 --warmup 2 > $OLDPWD/gpurun_out/${TAG}_kt$v.log 2>&1)
  echo "== AOS_COPY_CUS=$v: k_fg beside the copies" | tee -a $out
  python3 tools/kt_overlap.py gpurun_out/${TAG}_kt$v/kt_kernel_trace.csv "aos::k_fg(" | head -6 | tee -a $out
  python3 tools/kt_summary.py gpurun_out/${TAG}_kt$v 12 > gpurun_out/${TAG}_kt${v}_summary.txt
  head -8 gpurun_out/${TAG}_kt${v}_summary.txt | tee -a $out
done
