#!/bin/bash
# One GPU check of the current build: parity tests, smoke, the default bench line (optionally the C4 stream
# and a kernel-trace profile). TAG names the outputs under gpurun_out/. Every GPU step has its own limit and
# the chain stops at the first failure.
set -e
export TMPDIR=/tmp
R=$PWD
TAG=${TAG:-chk}
mkdir -p gpurun_out
echo "[$TAG] pytest -m gpu ${PYTEST_K:+-k $PYTEST_K}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
if [ "${SMOKE:-1}" = "1" ]; then
  echo "[$TAG] smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  echo "[$TAG] bench ${BENCH_ARGS:-}"
  timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  grep '^{' gpurun_out/${TAG}_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms']; r=d['roofline']
print('value', d['value'], 'p50', d['frame_ms']['p50'], 'pipelined', d.get('pipelined',{}).get('value'), 'device', d.get('device_resident',{}).get('value'))
print('ror', s.get('seedgen_ror'), 'count', s.get('seedgen_ror_count'), 'bin', s.get('seedgen_ror_bin'), 'scatter', s.get('seedgen_ror_scatter'), 'seedgen', s.get('seedgen_total'), 'delaunay', s.get('gvd_delaunay'), 'graph', s.get('gvd_graph'))
print('roofline frac', r['frac'], 'achieved', r['achieved'], r.get('kernels'))"
fi
if [ -n "$STREAM_STEPS" ]; then
  echo "[$TAG] bench --stream $STREAM_STEPS"
  timeout -k 10 500 python -u bench.py --stream --steps $STREAM_STEPS --warmup 2 > gpurun_out/${TAG}_stream.log 2> gpurun_out/${TAG}_stream.err || { tail -20 gpurun_out/${TAG}_stream.err; exit 1; }
  grep '^{' gpurun_out/${TAG}_stream.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('stream', json.dumps(d.get('stream'))[:400], 'ror', d['stages_ms'].get('seedgen_ror'))"
fi
if [ "${KT:-0}" = "1" ]; then
  echo "[$TAG] rocprofv3 kernel trace"
  rm -rf gpurun_out/${TAG}_kt
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kt -o kt -- python3 $R/bench.py --no-cpu-baseline --no-pipelined-rate --steps 9 --warmup 2 > $R/gpurun_out/${TAG}_kt.log 2>&1
  cd $R
fi
echo "[$TAG] done"
