#!/bin/bash
# Round-3 evidence run on the final build: GPU parity tests, smoke, the default bench line (with the CPU
# baseline), the C4 stream, a kernel-trace profile and the two PMC passes (FETCH_SIZE, WRITE_SIZE: separate
# runs on gfx950) whose per-kernel bytes feed bench.py's roofline.traffic. Each GPU step has its own limit.
set -e
R=$PWD
TAG=${TAG:-r03fin}
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[$TAG] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_gpu.log
echo "[$TAG] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
echo "[$TAG] bench (default)"
timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.log 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
grep '^{' gpurun_out/${TAG}_bench.log | cut -c1-300
echo "[$TAG] stream"
timeout -k 10 400 python -u bench.py --stream --steps 20 --warmup 2 > gpurun_out/${TAG}_stream.log 2> gpurun_out/${TAG}_stream.err || { tail -20 gpurun_out/${TAG}_stream.err; exit 1; }
echo "[$TAG] rocprofv3 kernel trace"
rm -rf gpurun_out/${TAG}_kt gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kt -o kt -- python3 $R/bench.py --no-cpu-baseline --no-pipelined-rate --steps 9 --warmup 2 > $R/gpurun_out/${TAG}_kt.log 2>&1
echo "[$TAG] pmc FETCH_SIZE"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_fetch -o fetch -- python3 $R/bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 3 --warmup 1 > $R/gpurun_out/${TAG}_fetch.log 2>&1
echo "[$TAG] pmc WRITE_SIZE"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_write -o write -- python3 $R/bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 3 --warmup 1 > $R/gpurun_out/${TAG}_write.log 2>&1
cd $R
python3 tools/pmc_traffic.py $(ls gpurun_out/${TAG}_fetch/*counter_collection.csv | head -1) $(ls gpurun_out/${TAG}_write/*counter_collection.csv | head -1) gpurun_out/${TAG}_pmc_traffic.json
echo "[$TAG] done"
