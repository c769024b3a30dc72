#!/bin/bash
# One GPU round on the MI355X box: parity tests, smoke, bench, rocprofv3 kernel stats and the two
# PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950). Every GPU step has its own
# time limit and the chain stops at the first failure.
set -e
R=$PWD
TAG=${TAG:-r01}
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[gpu_round] pytest -m gpu"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
echo "[gpu_round] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "[gpu_round] bench"
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
if [ "${DIST:-0}" = "1" ]; then
echo "[gpu_round] 2-rank rehearsal of the --gpus N flow (gloo timing reduction, ranks share the GPU)"
AOS_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_dist.log 2>&1 || { tail -30 gpurun_out/bench_dist.log; exit 1; }
grep '^{' gpurun_out/bench_dist.log | cut -c1-400
fi
echo "[gpu_round] rocprofv3 kernel trace"
rm -rf gpurun_out/prof_kt gpurun_out/prof_fetch gpurun_out/prof_write
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_kt -o ${TAG}_kt -- python3 $R/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/gpurun_out/prof_kt.log 2>&1
if [ "${PMC:-1}" = "1" ]; then
echo "[gpu_round] pmc FETCH_SIZE"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o ${TAG}_fetch -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/prof_fetch.log 2>&1
echo "[gpu_round] pmc WRITE_SIZE"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o ${TAG}_write -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/prof_write.log 2>&1
fi
cd $R
find gpurun_out -name "*.csv" -path "*prof_*" | sort
echo "[gpu_round] done"
