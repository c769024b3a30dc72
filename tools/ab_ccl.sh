# A/B runs of round 4's copy and upload switches (each GPU step under its own limit)
set -e
mkdir -p gpurun_out
tools/copyprobe.sh
for v in "AOS_UP_THREADS=4" "AOS_UP_THREADS=8" "AOS_UP_THREADS=12" "AOS_UP_THREADS=4" "AOS_UP_THREADS=8"; do
  env $v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 12 --warmup 3 > gpurun_out/r04k_${v/=/_}.log 2>&1
  echo "$v: $(grep '^{' gpurun_out/r04k_${v/=/_}.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['frame_ms'], d['stages_ms']['seedgen_cluster'], d['stages_ms']['seedgen_total'])")"
done
