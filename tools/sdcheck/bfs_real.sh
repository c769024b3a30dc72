#!/bin/bash
# BFS-replay A/B on real skeleton clusters (the oracle's C1 rows), on the box's host CPU pinned to core 2: the product's
# cluster_host.cpp against the round-6 start (exp/cluster_host_r06.cpp) and the exp/ forms named in BFS_OLD. Prints ns per cell: the walk alone, then the
# whole replay with the endpoint search; the check sums must agree.
set -e
D=$(cd "$(dirname "$0")" && pwd)
C=$D/../../active-orchard-slam_amd/csrc
W=$(mktemp -d)
python3 $D/dump_clusters.py $W/c1.bin ${BFS_GPU_CONFIG:+--gpu $BFS_GPU_CONFIG}   # (BFS_GPU_CONFIG=C3: the GPU frame's clusters)
# variants: the product (new), the round-6 start (old), and BFS_OLD's other exp/ forms (name:file pairs)
VARS="new old ${BFS_OLD:-}"
for v in $VARS; do
  name=${v%%:*}
  I=$W/$name; mkdir -p $I
  case $v in
    new) cp $C/cluster_host.cpp $I/cluster_host.cpp ;;
    old) sed 's/namespace aos_old { using namespace aos;/namespace aos {/' $D/exp/cluster_host_r06.cpp > $I/cluster_host.cpp ;;
    *) sed 's/namespace aos_old { using namespace aos;/namespace aos {/' $D/exp/${v#*:} > $I/cluster_host.cpp ;;
  esac
  cp $D/bfsbench_real.cpp $I/bench.cpp
  /opt/rocm/bin/hipcc -x c++ -O3 -std=c++17 -ffp-contract=off -fno-fast-math -march=x86-64-v3 -mtune=znver5 -D__HIP_PLATFORM_AMD__ \
    -I/opt/rocm/include -I$C -I$D/../../include $I/bench.cpp -o $W/bench_$name -lpthread
done
for r in 1 2; do
  for v in $VARS; do name=${v%%:*}; echo "== $name"; taskset -c 2 timeout -k 5 120 $W/bench_$name $W/c1.bin | tail -3; done
done
rm -rf $W
