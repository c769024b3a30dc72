#!/bin/bash
# markers returned as views (default) vs copies (--markers-copy): the sequential C2 loop, alternating
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "markers" > gpurun_out/r03m_pytest.log 2>&1 || { tail -30 gpurun_out/r03m_pytest.log; exit 1; }
tail -1 gpurun_out/r03m_pytest.log
for i in 1 2; do
  for v in "" "--markers-copy"; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate $v > gpurun_out/r03m_bench.log 2> gpurun_out/r03m_bench.err || { tail -20 gpurun_out/r03m_bench.err; exit 1; }
    grep '^{' gpurun_out/r03m_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${v:-views}', d['value'], d['frame_ms'], d['markers']['timed_frames_with_markers'])"
  done
done
