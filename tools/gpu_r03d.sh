#!/bin/bash
# r03d: the stream stall after a markers scan — cgroup throttling deltas, and the same stream without the
# Python-side copy of the markers
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
cat /sys/fs/cgroup/cpu.stat > gpurun_out/r03d_cpustat.txt
AOS_TRACE=1 timeout -k 10 300 python -u bench.py --stream --steps 12 --warmup 2 --trace > gpurun_out/r03d_stream.log 2> gpurun_out/r03d_stream.err
cat /sys/fs/cgroup/cpu.stat >> gpurun_out/r03d_cpustat.txt
AOS_TRACE=1 timeout -k 10 300 python -u bench.py --stream --steps 12 --warmup 2 --trace --markers-no-copy > gpurun_out/r03d_stream_nocopy.log 2> gpurun_out/r03d_stream_nocopy.err
cat /sys/fs/cgroup/cpu.stat >> gpurun_out/r03d_cpustat.txt
grep -c processor /proc/cpuinfo >> gpurun_out/r03d_cpustat.txt; cat /sys/fs/cgroup/cpu.max >> gpurun_out/r03d_cpustat.txt || true
grep "dedup" gpurun_out/r03d_stream.err | head -14
echo ---
grep "dedup" gpurun_out/r03d_stream_nocopy.err | head -14
cat gpurun_out/r03d_cpustat.txt
