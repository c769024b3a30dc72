# read-backs through kernel stores (AOS_ZC_READBACK=1, default) vs hipMemcpyAsync (0), in an order that separates
# the setting from the process-to-process alternation of the cluster-stage figure (each GPU step its own limit)
set -e
mkdir -p gpurun_out
for v in 1 0 0 1 1 0 0 1; do
  AOS_ZC_READBACK=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 12 --warmup 3 > gpurun_out/r04n_zc.log 2>&1
  echo "AOS_ZC_READBACK=$v: $(grep '^{' gpurun_out/r04n_zc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms']; print(d['frame_ms']['p50'], s['seedgen_cluster'], s['seedgen_seeds'], s['seedgen_total'])")"
done
