#!/bin/bash
# Subdiv2D replay at C2 and C3 scale on the box's host CPU (needs a GPU for the seeds: dump_seeds.py): the phase
# split per insert (run_prof.sh), then the C3 replay alone and two at once on one CCD (cores 2, 3) and on two CCDs
# (cores 2, 10), as the frame runs its GVD and markers replays side by side.
set -e
D=$(cd "$(dirname "$0")" && pwd)
T=${TAG:-r06l}
O=$D/../../gpurun_out
mkdir -p $O
timeout -k 10 300 python3 $D/dump_seeds.py C2 /tmp/c2s.bin
timeout -k 10 300 python3 $D/dump_seeds.py C3 /tmp/c3s.bin
SD_SEEDS=/tmp/c2s.bin SD_REPS=3 ROUNDS=1 bash $D/run_prof.sh > $O/${T}_sdprof_c2.txt 2>&1
SD_SEEDS=/tmp/c3s.bin SD_REPS=2 ROUNDS=1 bash $D/run_prof.sh > $O/${T}_sdprof_c3.txt 2>&1
B=/tmp/sdprof_bins/base
{
  echo "alone core 2: $(taskset -c 2 timeout -k 5 120 $B /tmp/c3s.bin 2)"
  taskset -c 2 timeout -k 5 120 $B /tmp/c3s.bin 2 > /tmp/p1.txt & taskset -c 3 timeout -k 5 120 $B /tmp/c3s.bin 2 > /tmp/p2.txt; wait
  echo "same CCD 2+3: $(cat /tmp/p1.txt) || $(cat /tmp/p2.txt)"
  taskset -c 2 timeout -k 5 120 $B /tmp/c3s.bin 2 > /tmp/p1.txt & taskset -c 10 timeout -k 5 120 $B /tmp/c3s.bin 2 > /tmp/p2.txt; wait
  echo "two CCDs 2+10: $(cat /tmp/p1.txt) || $(cat /tmp/p2.txt)"
  lscpu | grep -E "L2|L3|Model name" || true
} > $O/${T}_sdprof_c3_pairs.txt 2>&1
cat $O/${T}_sdprof_c2.txt $O/${T}_sdprof_c3.txt $O/${T}_sdprof_c3_pairs.txt
