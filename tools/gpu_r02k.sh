#!/bin/bash
# markers at the publish throttle: the pipeline / parity markers tests, then the bench at several depths
# and once with markers every frame
set -e
export TMPDIR=/tmp
TAG=${TAG:-r02k}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "markers or pipeline" > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for d in ${DEPTHS:-4 6 8}; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device-rate --steps 20 --warmup 5 --depth $d > gpurun_out/${TAG}_bench_d$d.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_d$d.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_bench_d$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('depth', $d, 'value', d['value'], 'median', d['value_median'], 'ms', d['ms_per_step'], 'lat', d['frame_latency_ms'], 'mk', d['markers']['timed_frames_with_markers'], 'delaunay', d['stages_ms']['gvd_delaunay'], 'graph', d['stages_ms']['gvd_graph'])"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device-rate --steps 20 --warmup 5 --markers-every-frame > gpurun_out/${TAG}_bench_mkall.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_mkall.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_mkall.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('every-frame markers: value', d['value'], 'ms', d['ms_per_step'], 'mk', d['markers']['timed_frames_with_markers'])"
