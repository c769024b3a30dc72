#!/bin/bash
# Replay timing on the box's host CPU: builds tools/sdcheck/sdprof against the product's subdiv2d.cpp (plain and
# with the -DAOS_SD_PROF phase counters) and against each variant source named in SD_VARIANTS (paths of
# subdiv2d.cpp variants), then runs them alternating, pinned to one core, ROUNDS times.
set -e
D=$(cd "$(dirname "$0")" && pwd)
C=$D/../../active-orchard-slam_amd/csrc
mkdir -p $D/../../gpurun_out
B=/tmp/sdprof_bins; mkdir -p $B
build() {   # name source [defs]   (a variant directory may hold its own subdiv2d.h: it is searched first)
  /opt/rocm/bin/hipcc -x c++ -O3 -std=c++17 -ffp-contract=off -fno-fast-math -march=x86-64-v3 -mtune=znver5 $3 \
    -I$(dirname $2) -I$C $D/sdprof.cpp $2 -o $B/$1
}
build base $C/subdiv2d.cpp
build prof $C/subdiv2d.cpp -DAOS_SD_PROF
names="base prof"
for v in ${SD_VARIANTS:-}; do n=$(basename $(dirname $v))_$(basename $v .cpp); n=${n#exp_}; build $n $v; build ${n}_prof $v -DAOS_SD_PROF; names="$names $n ${n}_prof"; done
for r in $(seq 1 ${ROUNDS:-3}); do
  for n in $names; do
    echo "$n: $(timeout -k 5 300 taskset -c 2 $B/$n ${SD_SEEDS:-$D/c2_seeds.bin} ${SD_REPS:-5})"
  done
done
