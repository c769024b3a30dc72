# Subdiv2D replay variants on the box's EPYC (tools/sdcheck/var, built on the build host; VARIANTS), alternating,
# best of 5 per process
set -e
cp tools/sdcheck/var/c2_seeds.bin tools/sdcheck/c2_seeds.bin
for r in 1 2 3 4 5; do
  for b in ${VARIANTS:-f0 f1}; do
    echo "$b $(timeout -k 5 60 taskset -c 2 tools/sdcheck/var/tm_$b 5)"
  done
done
