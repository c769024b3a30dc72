#!/bin/bash
# C3 through aos_group at 1x1 / 2x1 / 2x2 / 4x2 on one GPU under rocprofv3 --kernel-trace, then the summary
# (tools/tiling_overhead.py). usage: TAG=r06b tools/tiling_overhead.sh   -> gpurun_out/TAG_tiling.json
set -e
R=$PWD
TAG=${TAG:-r06x}
FR=${FRAMES:-4}
WU=${WARMUP:-2}
export TMPDIR=/tmp
export AOS_GROUP_SERIAL=${AOS_GROUP_SERIAL:-1}
mkdir -p gpurun_out
dirs=""
for t in "1 1" "2 1" "2 2" "4 2"; do
  set -- $t
  d=$R/gpurun_out/${TAG}_tile_$1x$2
  rm -rf $d
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt \
    -- python3 $R/tools/tiling_overhead.py run $1 $2 $FR $WU > $d.log 2>&1) || { tail -20 $d.log; exit 1; }
  grep '^{' $d.log | tail -1 > $d/run.json
  cat $d/run.json
  dirs="$dirs $d"
done
python3 tools/tiling_overhead.py summarize gpurun_out/${TAG}_tiling.json $dirs
