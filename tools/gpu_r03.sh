#!/bin/bash
# GPU round helper (round 3). STEPS picks what runs, in this order; every GPU step has its own time
# limit and the chain stops at the first failure.
#   test   pytest -m gpu          smoke   __graft_entry__.smoke()
#   bench  bench.py (BENCH_ARGS)  sd      Subdiv2D cavity-insert checker + timing on the box's CPU
#   prof   rocprofv3 kernel stats pmc     FETCH_SIZE / WRITE_SIZE passes
#   probe  tools/thin_graph_probe.py (hipGraph thinning shapes)   stream  bench.py --stream (C4)
set -e
R=$PWD
TAG=${TAG:-r03}
STEPS=${STEPS:-"test bench"}
export TMPDIR=/tmp
mkdir -p gpurun_out
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has sd; then
  echo "[gpu] sdcheck (CPU)"
  g++ -O2 -std=c++17 -ffp-contract=off -Iactive-orchard-slam_amd/csrc tools/sdcheck/sdcheck.cpp active-orchard-slam_amd/csrc/subdiv2d.cpp -o /tmp/sdcheck
  timeout -k 10 300 /tmp/sdcheck tools/sdcheck/c2_seeds.bin > gpurun_out/${TAG}_sdcheck.log 2>&1 || { tail -20 gpurun_out/${TAG}_sdcheck.log; exit 1; }
  tail -3 gpurun_out/${TAG}_sdcheck.log
fi
if has probe; then
  echo "[gpu] thin graph probe"
  timeout -k 10 400 python -u tools/thin_graph_probe.py ${PROBE_SCANS:-8} > gpurun_out/${TAG}_probe.log 2>&1 || { tail -30 gpurun_out/${TAG}_probe.log; exit 1; }
  tail -12 gpurun_out/${TAG}_probe.log
fi
if has test; then
  echo "[gpu] pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_OPTS:-} ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/${TAG}_pytest_gpu.log
fi
if has smoke; then
  echo "[gpu] smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
fi
if has bench; then
  echo "[gpu] bench ${BENCH_ARGS:-}"
  timeout -k 10 500 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_bench.log
fi
if has stream; then
  echo "[gpu] bench --stream ${STREAM_ARGS:-}"
  timeout -k 10 400 python -u bench.py --stream --steps 40 --warmup 3 ${STREAM_ARGS:-} > gpurun_out/${TAG}_stream.log 2> gpurun_out/${TAG}_stream.err || { tail -30 gpurun_out/${TAG}_stream.err; exit 1; }
  grep '^{' gpurun_out/${TAG}_stream.log | cut -c1-600
fi
cd /tmp
if has prof; then
  echo "[gpu] rocprofv3 kernel trace"
  rm -rf $R/gpurun_out/prof_kt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_kt -o ${TAG}_kt -- python3 $R/bench.py --no-cpu-baseline --no-device-rate --no-pipelined-rate --steps 7 --warmup 2 > $R/gpurun_out/${TAG}_prof_kt.log 2>&1
fi
if has pmc; then
  echo "[gpu] pmc FETCH_SIZE"
  rm -rf $R/gpurun_out/prof_fetch $R/gpurun_out/prof_write
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_fetch -o ${TAG}_fetch -- python3 $R/bench.py --no-cpu-baseline --no-device-rate --no-pipelined-rate --steps 3 --warmup 1 > $R/gpurun_out/${TAG}_prof_fetch.log 2>&1
  echo "[gpu] pmc WRITE_SIZE"
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_write -o ${TAG}_write -- python3 $R/bench.py --no-cpu-baseline --no-device-rate --no-pipelined-rate --steps 3 --warmup 1 > $R/gpurun_out/${TAG}_prof_write.log 2>&1
  cd $R && python3 tools/pmc_traffic.py $(ls gpurun_out/prof_fetch/*counter_collection.csv | head -1) $(ls gpurun_out/prof_write/*counter_collection.csv | head -1) gpurun_out/${TAG}_pmc_traffic.json; cd /tmp
fi
cd $R
echo "[gpu] done"
