#!/bin/bash
# Count-pass variants of the ROR partition (ror.hip compile-time knobs), built here and run on the box by
# run_count_variants.sh: packed 12-B cloud, warm (back to back) and cold (512 MB overwritten between frames).
set -e
D=$(dirname "$0")
build() { TAG=$1 DEFS="$2" "$D/build.sh" >/dev/null; echo "built rorbench$1: $2"; }
build _base ""
build _exp1 "-DAOS_RT_COUNT_EXP=1"
build _exp2 "-DAOS_RT_COUNT_EXP=2"
build _tb512 "-DAOS_RT_CTB=512"
build _tb1024 "-DAOS_RT_CTB=1024"
build _g1024 "-DAOS_RT_G=1024"
build _cper16 "-DAOS_RT_CPER=16"
build _tb512c4 "-DAOS_RT_CTB=512 -DAOS_RT_CPER=4"
