#!/bin/bash
# A/B of the Subdiv2D export straight into pinned memory (profiles/r03k_gvd_trace_export_ab.log): the base is
# the previous commit built beside the product (git stash; make BUILD=build_base LIB=libaos_gpu_base.so)
set -e
mkdir -p gpurun_out
for i in 1 2; do
  echo "== base"; AOS_GPU_LIB=$PWD/active-orchard-slam_amd/libaos_gpu_base.so timeout -k 10 200 python -u tools/gvd_trace.py > gpurun_out/r03k_trace_base_$i.log 2>&1; cat gpurun_out/r03k_trace_base_$i.log
  echo "== new"; timeout -k 10 200 python -u tools/gvd_trace.py > gpurun_out/r03k_trace_new_$i.log 2>&1; cat gpurun_out/r03k_trace_new_$i.log
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "gvd or full_frame or markers" > gpurun_out/r03k_pytest.log 2>&1; tail -2 gpurun_out/r03k_pytest.log
