#!/bin/bash
# tools/copyprobe: the standalone binary (the HIP runtime of /opt/rocm) and the same code loaded into a Python
# process after torch (torch's bundled HIP runtime, as aos_gpu loads libaos_gpu.so), each under a short limit;
# GAPS: streams created between the copy stream and the kernel stream
set -e
pyrun() { echo "== python+torch gap $1"; timeout -k 5 120 python3 -c "
import ctypes, torch
L = ctypes.CDLL('tools/copyprobe.so')
argv = (ctypes.c_char_p * 4)(b'p', b'16777216', b'0', b'$1')
L.copyprobe_main(4, argv)" | grep -v "kernel copy G"; }
for g in ${GAPS:-0 3}; do echo "== standalone gap $g"; timeout -k 5 60 tools/copyprobe 16777216 0 $g | grep -v "kernel copy G"; pyrun $g; done
