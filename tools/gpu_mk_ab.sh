# pipelined bench: markers throttled vs none (diagnostic for the post-markers stall), two runs each
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do for m in "" "--no-markers"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-device-rate --steps 20 --warmup 5 $m > gpurun_out/mkab.log 2>&1 || { tail -20 gpurun_out/mkab.log; exit 1; }
  grep '^{' gpurun_out/mkab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$m]', 'value', d['value'], 'median', d['value_median'], 'lat', d['frame_latency_ms'], 'delaunay', d['stages_ms']['gvd_delaunay'], 'graph', d['stages_ms']['gvd_graph'], 'merge', d['stages_ms']['gvd_merge'])"
done; done
