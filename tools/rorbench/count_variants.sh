#!/bin/bash
# Variants of the ROR partition (ror.hip compile-time knobs), built here and run on the box by
# run_count_variants.sh. Usage: tools/rorbench/count_variants.sh "_tag:-DKNOB=v -DKNOB2=w" ...
# (round 4 sets: count-pass block shapes — AOS_RT_CTB / AOS_RT_G / AOS_RT_CPER / AOS_RT_COUNT_EXP —, then
# nontemporal loads / stores, AOS_RT_NT)
set -e
D=$(dirname "$0")
rm -f "$D"/rorbench_*
for v in "$@"; do
  tag=${v%%:*}; defs=${v#*:}
  TAG=$tag DEFS="$defs" "$D/build.sh" >/dev/null
  echo "built rorbench$tag: $defs"
done
