# (1) Subdiv2D replay variants on the box's EPYC; (2) GPU tests touching the upload; (3) bench with the upload trace
set -e
cp tools/sdcheck/var/c2_seeds.bin tools/sdcheck/c2_seeds.bin
for r in 1 2 3 4; do
  for b in e0 e1; do
    echo "$b $(timeout -k 5 60 taskset -c 2 tools/sdcheck/var/tm_$b 5)"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04p2_pytest.log 2>&1 || { tail -30 gpurun_out/r04p2_pytest.log; exit 1; }
tail -1 gpurun_out/r04p2_pytest.log
AOS_TRACE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 10 --warmup 3 > gpurun_out/r04p2_bench.log 2> gpurun_out/r04p2_bench.err
grep '^{' gpurun_out/r04p2_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('frame p50', d['frame_ms']['p50'], 'delaunay', d['stages_ms_p50']['gvd_delaunay'])"
grep 'aos trace upload' gpurun_out/r04p2_bench.err | tail -5
