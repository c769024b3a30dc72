#!/bin/bash
# Re-entry check of the restored tree: GPU parity tests, smoke, the default bench line, then the
# driver's --gpus 2 flow rehearsed over gloo (ranks share the one GPU) with the tiled key.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[r03s] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r03s_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03s_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r03s_pytest_gpu.log
echo "[r03s] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03s_smoke.log 2>&1 || { tail -20 gpurun_out/r03s_smoke.log; exit 1; }
tail -1 gpurun_out/r03s_smoke.log
echo "[r03s] bench"
timeout -k 10 400 python -u bench.py > gpurun_out/r03s_bench.log 2> gpurun_out/r03s_bench.err || { tail -20 gpurun_out/r03s_bench.err; exit 1; }
grep '^{' gpurun_out/r03s_bench.log | cut -c1-600
echo "[r03s] --gpus 2 over gloo"
AOS_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 8 --warmup 3 --no-cpu-baseline > gpurun_out/r03s_gpus2_gloo.log 2>&1 || { tail -30 gpurun_out/r03s_gpus2_gloo.log; exit 1; }
grep '^{' gpurun_out/r03s_gpus2_gloo.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'tiled', json.dumps(d.get('tiled'))[:800])"
echo "[r03s] done"
