#!/bin/bash
# Builds tools/sdcheck/sdcheck_bin with the product's host flags (active-orchard-slam_amd/Makefile).
set -e
D=$(cd "$(dirname "$0")" && pwd)
/opt/rocm/bin/hipcc -x c++ -O3 -std=c++17 -ffp-contract=off -fno-fast-math -march=x86-64-v3 -mtune=znver5 -I"$D/../../active-orchard-slam_amd/csrc" \
  "$D/sdcheck.cpp" "$D/../../active-orchard-slam_amd/csrc/subdiv2d.cpp" -o "$D/sdcheck_bin"
