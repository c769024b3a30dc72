# Subdiv2D replay timing on the box's EPYC: compiler / ISA / PGO variants of csrc/subdiv2d.cpp (tools/sdcheck/var,
# built on the build host), alternating, best of 5 inserts of the C2 seeds each
set -e
cp tools/sdcheck/var/c2_seeds.bin tools/sdcheck/c2_seeds.bin
for r in 1 2 3 4; do
  for b in d0 d1; do
    echo "$b $(timeout -k 5 60 taskset -c 2 tools/sdcheck/var/tm_$b 5)"
  done
done
