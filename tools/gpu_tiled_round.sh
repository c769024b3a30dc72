#!/bin/bash
# GPU round for the tiled frame: full gpu test suite, smoke, the default bench, and the tiled bench
# at 1 rank (whole C3 map) and 2 ranks sharing the box's GPU (gloo rehearsal of the --gpus N flow).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[round] pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
echo "[round] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "[round] bench"
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log | cut -c1-600
echo "[round] bench --tiled (1 rank, C3)"
timeout -k 10 400 python bench.py --tiled --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_tiled1.log 2>&1 || { tail -20 gpurun_out/bench_tiled1.log; exit 1; }
grep '^{' gpurun_out/bench_tiled1.log | cut -c1-600
echo "[round] bench --tiled (2 ranks on one GPU, gloo)"
AOS_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --tiled --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_tiled2.log 2>&1 || { tail -30 gpurun_out/bench_tiled2.log; exit 1; }
grep '^{' gpurun_out/bench_tiled2.log | cut -c1-600
echo "[round] done"
