#!/bin/bash
# markers policy A/B at depth 6 (throttled vs every frame), stream with every-frame markers, GPU suite
set -e
export TMPDIR=/tmp
TAG=${TAG:-r02p}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
for m in "" "--markers-every-frame"; do
  for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device-rate --steps 20 --warmup 5 $m > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('markers[$m]', 'value', d['value'], 'median', d['value_median'], 'ms', d['ms_per_step'], 'lat', d['frame_latency_ms'], 'mk', d['markers']['timed_frames_with_markers'])"
  done
done
timeout -k 10 300 python -u bench.py --stream --steps 40 --warmup 2 --markers-every-frame > gpurun_out/${TAG}_stream.log 2>&1 || { tail -20 gpurun_out/${TAG}_stream.log; exit 1; }
grep '^{' gpurun_out/${TAG}_stream.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stream']; print('stream every-frame markers p50', s['scan_latency_ms_p50'], 'max', s['scan_latency_ms_max'], s['scan_latency_ms'])"
