#!/bin/bash
# the driver's --gpus 2 flow rehearsed on one GPU over gloo (independent maps + the tiled key), then the
# tiled C3 bench at 1 and 2 ranks with the distributed cluster stage
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[r03q] --gpus 2 over gloo (ranks share the GPU)"
AOS_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/r03q_gpus2_gloo.log 2>&1 || { tail -30 gpurun_out/r03q_gpus2_gloo.log; exit 1; }
grep '^{' gpurun_out/r03q_gpus2_gloo.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'tiled', json.dumps(d.get('tiled'))[:600])"
TAG=r03q RANKS="1 2" STEPS=8 bash tools/gpu_tiled_scale.sh
