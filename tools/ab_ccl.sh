# host cloud split (AOS_UP_SPLIT) A/B with 4 / 8 / 16 gather threads, after the GPU tests
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04v_pytest.log 2>&1 || { tail -30 gpurun_out/r04v_pytest.log; exit 1; }
tail -2 gpurun_out/r04v_pytest.log
for v in "1 4" "0 4" "1 8" "0 8" "1 16" "0 16" "1 8" "0 8" "1 4" "0 4"; do
  set -- $v
  AOS_UP_SPLIT=$1 AOS_UP_THREADS=$2 AOS_TRACE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 8 --warmup 3 > gpurun_out/r04v_$1_$2.log 2> gpurun_out/r04v_$1_$2.err
  echo "split=$1 threads=$2: $(grep '^{' gpurun_out/r04v_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_p50']; print(d['frame_ms']['p50'], s['seedgen_ror'], s['seedgen_ror_bin'], s['seedgen_ror_scatter'], s['gvd_delaunay'])") | $(grep 'aos trace upload' gpurun_out/r04v_$1_$2.err | tail -3 | sed 's/.*: //' | tr '\n' ';')"
done
