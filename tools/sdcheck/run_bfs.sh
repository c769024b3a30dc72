#!/bin/bash
# BFS-replay A/B on the box's host CPU (tools/sdcheck/bfsbench.cpp), pinned to core 2.
set -e
D=$(cd "$(dirname "$0")" && pwd)
C=$D/../../active-orchard-slam_amd/csrc
/opt/rocm/bin/hipcc -x c++ -O3 -std=c++17 -ffp-contract=off -fno-fast-math -march=x86-64-v3 -mtune=znver5 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -I$C -I$D/../../include \
  $D/bfsbench.cpp $C/cluster_host.cpp $D/exp/cluster_host_r06.cpp ${BFS_EXTRA:-} -o /tmp/bfsbench -lpthread
for mode in "STRAIGHT=1 NOROW=1" "STRAIGHT=1" "NOROW=1" ""; do
  echo "== $mode"; env $mode taskset -c 2 timeout -k 5 120 /tmp/bfsbench | tail -3
done
