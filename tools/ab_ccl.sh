# grid D2H by kernel (AOS_GRID_COPY_KERNEL=1, default) vs hipMemcpyAsync (0): host-held frames over processes
set -e
mkdir -p gpurun_out
TAG=r04p STEPS="pytest" PYTEST_K="golden or c1 or tiled" tools/gpu_run.sh
for v in 1 0 1 0 1 0; do
  AOS_GRID_COPY_KERNEL=$v AOS_TRACE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 16 --warmup 2 > gpurun_out/r04p_$v.log 2> gpurun_out/r04p_$v.err
  echo "AOS_GRID_COPY_KERNEL=$v: $(grep '^{' gpurun_out/r04p_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms']; print(d['frame_ms'], s['seedgen_cluster'], s['seedgen_seeds'], s['seedgen_total'])") | copy_issued > 1 ms in $(grep 'aos trace finish' gpurun_out/r04p_$v.err | awk '{if ($5 > 1.0) n++} END {print n+0}') of $(grep -c 'aos trace finish' gpurun_out/r04p_$v.err) frames; max $(grep 'aos trace finish' gpurun_out/r04p_$v.err | awk 'BEGIN{m=0} {if ($5 > m) m=$5} END {print m}')"
done
