set -e
# A/B timing of alternative builds of libaos_gpu.so (AOS_GPU_LIB), e.g. make BUILD=build_a LIB=libaos_gpu_a.so DEFS=...
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for v in "" _a _b; do
  L=$PWD/active-orchard-slam_amd/libaos_gpu$v.so
  AOS_GPU_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 8 --warmup 2 > gpurun_out/ab$v.log 2>&1
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab$v.log') if l.startswith('{')][0]); print('$v', d['ms_per_step'], d['roofline']['ms_per_launch'], d['stages_ms']['seedgen_ror'])"
done
