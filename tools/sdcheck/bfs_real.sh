#!/bin/bash
# BFS-replay A/B on real skeleton clusters (the oracle's C1 rows), on the box's host CPU pinned to core 2: the product's
# cluster_host.cpp against the round-6 start (exp/cluster_host_r06.cpp). Prints ns per cell: the walk alone, then the
# whole replay with the endpoint search; the check sums must agree.
set -e
D=$(cd "$(dirname "$0")" && pwd)
C=$D/../../active-orchard-slam_amd/csrc
W=$(mktemp -d)
python3 $D/dump_clusters.py $W/c1.bin
cp $C/cluster_host.cpp $W/cluster_host.cpp
mkdir -p $W/old
sed 's/namespace aos_old { using namespace aos;/namespace aos {/' $D/exp/cluster_host_r06.cpp > $W/old/cluster_host.cpp
for v in new old; do
  I=$W; [ $v = old ] && I=$W/old
  cp $D/bfsbench_real.cpp $I/bench.cpp
  /opt/rocm/bin/hipcc -x c++ -O3 -std=c++17 -ffp-contract=off -fno-fast-math -march=x86-64-v3 -mtune=znver5 -D__HIP_PLATFORM_AMD__ \
    -I/opt/rocm/include -I$C -I$D/../../include $I/bench.cpp -o $W/bench_$v -lpthread
done
for v in new old new old; do echo "== $v"; taskset -c 2 timeout -k 5 120 $W/bench_$v $W/c1.bin | tail -3; done
rm -rf $W
