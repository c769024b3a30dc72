#!/bin/bash
# GPU rehearsal of the tiled C3 schedule on the box's one GPU: the rotating-root test,
# then bench.py --tiled at 1, 2 and 4 ranks (2 and 4 ranks share the GPU over gloo; every rank has its
# own host cores), and optionally the C4 stream over STREAM_STEPS scans. Every GPU step has its own
# time limit and the chain stops at the first failure.
set -e
export TMPDIR=/tmp
TAG=${TAG:-r02h}
STEPS=${STEPS:-8}
mkdir -p gpurun_out
echo "[tiled] rotating-root test"
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiled.py -x -v --timeout 400 --timeout-method thread -k "rotating" > gpurun_out/${TAG}_pytest_rot.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_rot.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_rot.log
for n in ${RANKS:-1 2 4}; do
  echo "[tiled] bench --tiled, $n rank(s)"
  if [ "$n" = 1 ]; then
    timeout -k 10 400 python -u bench.py --tiled --steps $STEPS --warmup 2 --depth ${DEPTH1:-4} --no-cpu-baseline > gpurun_out/${TAG}_tiled_c3_${n}.log 2>&1 || { tail -20 gpurun_out/${TAG}_tiled_c3_${n}.log; exit 1; }
  else
    AOS_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --tiled --steps $STEPS --warmup 2 --depth ${DEPTHN:-2} --no-cpu-baseline > gpurun_out/${TAG}_tiled_c3_${n}.log 2>&1 || { tail -30 gpurun_out/${TAG}_tiled_c3_${n}.log; exit 1; }
  fi
  grep '^{' gpurun_out/${TAG}_tiled_c3_${n}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ranks', $n, 'value', d['value'], 'ms/frame', d['ms_per_step'], 'latency', d['frame_latency_ms'], 'delaunay', d['stages_ms'].get('gvd_delaunay'))"
done
if [ -n "$STREAM_STEPS" ]; then
  echo "[stream] bench --stream, $STREAM_STEPS scans"
  timeout -k 10 500 python -u bench.py --stream --steps $STREAM_STEPS --warmup 2 > gpurun_out/${TAG}_stream.log 2>&1 || { tail -20 gpurun_out/${TAG}_stream.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_stream.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('stream', d['stream'], d['ms_per_step'])"
fi
echo "[tiled] done"
