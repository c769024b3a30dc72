# pipeline tests (collected markers), then the markers A/B with one-step-later collection
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 300 -k "markers or pipeline or collected" > gpurun_out/r02r_pytest.log 2>&1 || { tail -30 gpurun_out/r02r_pytest.log; exit 1; }
tail -1 gpurun_out/r02r_pytest.log
bash tools/gpu_mk_ab.sh
