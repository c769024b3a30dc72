#!/bin/bash
# Tiled C4 stream (bench.py --tiled --stream) at 1 rank, then the driver's --gpus 2 flow over gloo (ranks share
# the box's GPU) with the tiled and tiled_stream keys. Each GPU step has its own time limit.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03ts}
echo "[$TAG] --tiled --stream, 1 rank"
timeout -k 10 300 python -u bench.py --tiled --stream --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_1.log 2> gpurun_out/${TAG}_1.err || { tail -30 gpurun_out/${TAG}_1.err; exit 1; }
grep '^{' gpurun_out/${TAG}_1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], json.dumps(d['stream'])[:300])"
echo "[$TAG] --gpus 2 over gloo"
AOS_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_2.log 2>&1 || { tail -30 gpurun_out/${TAG}_2.log; exit 1; }
grep '^{' gpurun_out/${TAG}_2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value']); print('tiled', json.dumps(d.get('tiled'))[:300]); print('tiled_stream', json.dumps(d.get('tiled_stream'))[:600])"
echo "[$TAG] done"
