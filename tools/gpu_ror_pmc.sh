#!/bin/bash
# ROR-stage counters from the standalone microbenchmark (tools/rorbench, built in-tree beforehand):
# kernel trace + two SQ passes (each pass its own run and time limit) on the packed 12-B C2 cloud.
# usage: TAG=r03t bash tools/gpu_ror_pmc.sh [rorbench binaries...]
set -e
R=$PWD
TAG=${TAG:-r03t}
export TMPDIR=/tmp
mkdir -p gpurun_out
BINS=${*:-tools/rorbench/rorbench}
for b in $BINS; do
  n=$(basename $b)
  echo "== $n"
  timeout -k 10 120 $R/$b 4096 10000000 10 12 > gpurun_out/${TAG}_${n}.log 2>&1 || { tail -5 gpurun_out/${TAG}_${n}.log; exit 1; }
  tail -2 gpurun_out/${TAG}_${n}.log
  [ "${PMC:-1}" = "1" ] || continue
  rm -rf gpurun_out/${TAG}_${n}_kt gpurun_out/${TAG}_${n}_sq1 gpurun_out/${TAG}_${n}_sq2
  cd /tmp
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${n}_kt -o kt -- $R/$b 4096 10000000 4 12 > $R/gpurun_out/${TAG}_${n}_kt.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/gpurun_out/${TAG}_${n}_sq1 -o sq1 -- $R/$b 4096 10000000 2 12 > $R/gpurun_out/${TAG}_${n}_sq1.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/${TAG}_${n}_sq2 -o sq2 -- $R/$b 4096 10000000 2 12 > $R/gpurun_out/${TAG}_${n}_sq2.log 2>&1 || echo "sq2 pass failed (counter names?)"
  cd $R
  python3 tools/pmc_summary.py gpurun_out/${TAG}_${n}_sq1 gpurun_out/${TAG}_${n}_sq2 || true
done
echo "[ror_pmc] done"
