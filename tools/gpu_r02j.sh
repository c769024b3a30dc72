#!/bin/bash
# round-2 check: GPU suite, default bench, C4 stream over STREAM_STEPS scans
set -e
export TMPDIR=/tmp
TAG=${TAG:-r02j}
mkdir -p gpurun_out
echo "[gpu] pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_gpu.log
if [ -n "$BENCH" ]; then
  echo "[gpu] bench"
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step'], 'lat', d['frame_latency_ms'], 'ror', d['roofline']['ms_per_launch'], 'thin', d['stages_ms']['seedgen_thin'])"
fi
if [ -n "$STREAM_STEPS" ]; then
  echo "[gpu] stream $STREAM_STEPS"
  timeout -k 10 500 python -u bench.py --stream --steps $STREAM_STEPS --warmup 2 > gpurun_out/${TAG}_stream.log 2>&1 || { tail -20 gpurun_out/${TAG}_stream.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_stream.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stream']; print('p50', s['scan_latency_ms_p50'], 'max', s['scan_latency_ms_max'], s['scan_latency_ms'], 'ror', d['stages_ms']['seedgen_ror'], 'thin', d['stages_ms']['seedgen_thin'])"
fi
echo "[gpu] done"
