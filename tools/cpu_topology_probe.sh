#!/bin/bash
# Host-CPU facts of the GPU box that decide where the two Subdiv2D replays (GVD + markers) run.
set -e
mkdir -p gpurun_out
{
nproc
grep -E "Cpus_allowed_list" /proc/self/status
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
lscpu | grep -E "Model name|Thread|Core|Socket|NUMA|L2|L3" || true
g++ -O3 -std=c++17 -ffp-contract=off -Iactive-orchard-slam_amd/csrc tools/sdbench/main.cpp active-orchard-slam_amd/csrc/subdiv2d.cpp -o /tmp/sdb
cd tools/sdbench
echo "one replay"; /tmp/sdb
echo "two concurrent replays (unpinned)"; /tmp/sdb & /tmp/sdb; wait
echo "two concurrent replays pinned to cpus 0 and 2"; taskset -c 0 /tmp/sdb & taskset -c 2 /tmp/sdb; wait
echo "two concurrent replays pinned to cpus 0 and 1"; taskset -c 0 /tmp/sdb & taskset -c 1 /tmp/sdb; wait
cat /sys/devices/system/cpu/cpu0/topology/thread_siblings_list
} > gpurun_out/cpu_probe.log 2>&1
cat gpurun_out/cpu_probe.log
