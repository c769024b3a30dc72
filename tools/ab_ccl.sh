set -e
mkdir -p gpurun_out
AOS_CCL_CHUNK=512 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "golden" > gpurun_out/r04j_golden_chunk512.log 2>&1 && tail -1 gpurun_out/r04j_golden_chunk512.log
for v in "2048 256" "2048 1024" "1024 256" "512 256" "4096 1024"; do
  set -- $v
  AOS_CCL_CHUNK=$1 AOS_CCL_TB=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 12 --warmup 3 > gpurun_out/r04j_ccl_$1_$2.log 2>&1
  echo "chunk $1 tb $2: $(grep '^{' gpurun_out/r04j_ccl_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['frame_ms']['p50'], d['stages_ms']['seedgen_cluster'], d['stages_ms']['seedgen_seeds'])")"
done
