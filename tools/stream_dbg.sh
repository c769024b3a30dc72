# per-step breakdown of the C4 stream (bench --stream --trace)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
AOS_DEBUG_GVD_TIMING=1 timeout -k 10 300 python -u bench.py --stream --steps 6 --warmup 2 --trace > gpurun_out/sdbg.log 2> gpurun_out/sdbg.err || { tail -20 gpurun_out/sdbg.err; exit 1; }
grep -E "trace|gvd-dbg" gpurun_out/sdbg.err | tail -60
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q --timeout 300 -k "markers" > gpurun_out/sdbg_pytest.log 2>&1 || { tail -30 gpurun_out/sdbg_pytest.log; exit 1; }
tail -1 gpurun_out/sdbg_pytest.log
