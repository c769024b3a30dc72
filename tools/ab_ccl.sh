# Subdiv2D replay variants on the box's EPYC (tools/sdcheck/var), alternating, best of 5 per process
set -e
cp tools/sdcheck/var/c2_seeds.bin tools/sdcheck/c2_seeds.bin
for r in 1 2 3 4 5; do
  for b in ${VARIANTS:-g0 h1 h2}; do
    echo "$b $(timeout -k 5 60 taskset -c 2 tools/sdcheck/var/tm_$b 5)"
  done
done
