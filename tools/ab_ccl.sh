# GPU-side splits of the cluster stage (AOS_TRACE) over consecutive bench processes
set -e
mkdir -p gpurun_out
for k in 1 2 3 4; do
  AOS_TRACE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 6 --warmup 2 > gpurun_out/r04o_trace_$k.log 2> gpurun_out/r04o_trace_$k.err
  echo "== process $k: $(grep '^{' gpurun_out/r04o_trace_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['frame_ms']['p50'], d['stages_ms']['seedgen_cluster'])")"
  grep "aos trace events\|aos trace cluster" gpurun_out/r04o_trace_$k.err | tail -4
done
