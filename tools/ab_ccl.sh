# staged read-ahead placement: during the upload (1, default), on the stage's clock before the count pass (3), none (0)
set -e
mkdir -p gpurun_out
for v in 1 3 0 3 1; do
  AOS_STAGED_TOUCH=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 16 --warmup 3 > gpurun_out/r04t.log 2>&1
  echo "AOS_STAGED_TOUCH=$v: $(grep '^{' gpurun_out/r04t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_p50']; r=d['roofline']; print(d['frame_ms']['p50'], 'ror', s['seedgen_ror_bin'], s['seedgen_ror_scatter'], s['seedgen_ror_count'], 'stage', r['ms_per_launch'], 'frac', r['frac'])")"
done
