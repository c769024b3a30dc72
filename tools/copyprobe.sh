#!/bin/bash
# tools/copyprobe: the standalone binary (the HIP runtime of /opt/rocm) and the same code loaded into a Python
# process after torch (torch's bundled HIP runtime, as aos_gpu loads libaos_gpu.so), each under a short limit
set -e
run() { echo "== $*"; env "$@" timeout -k 5 60 tools/copyprobe 16777216 0; }
pyrun() { echo "== python+torch $*"; env "$@" timeout -k 5 120 python3 -c "
import ctypes, torch
L = ctypes.CDLL('tools/copyprobe.so')
argv = (ctypes.c_char_p * 3)(b'p', b'16777216', b'0')
L.copyprobe_main(3, argv)"; }
run X=0
pyrun X=0


