#!/bin/bash
# Subdiv2D replay timing on the box's host CPU (no GPU), default malloc vs glibc's hugetlb tunable (THP for
# the replay's arrays), alternating.
cd $(dirname $0)
for i in 1 2 3; do
  echo -n "default: "; AOS_SDCHECK_REPS=0 timeout -k 5 60 ./sdcheck_bin c2_seeds.bin | tail -1 | cut -c20-110
  echo -n "thp:     "; GLIBC_TUNABLES=glibc.malloc.hugetlb=1 AOS_SDCHECK_REPS=0 timeout -k 5 60 ./sdcheck_bin c2_seeds.bin | tail -1 | cut -c20-110
done
grep -i huge /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag 2>/dev/null
