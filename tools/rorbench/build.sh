#!/bin/bash
# Builds tools/rorbench/rorbench[_<tag>] (DEFS passed through, e.g. DEFS=-DAOS_RT_VARIANT=1 TAG=_v1).
set -e
D=$(dirname "$0")
gcc -O2 -fPIC -ffp-contract=off -c "$D/../orchard_gen.c" -o /tmp/orchard_gen_rb.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize ${DEFS:-} \
  -I"$D/../../include" -c "$D/rorbench.hip" -o /tmp/rorbench${TAG:-}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/rorbench${TAG:-}.o /tmp/orchard_gen_rb.o -o "$D/rorbench${TAG:-}"
