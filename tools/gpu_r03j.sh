#!/bin/bash
# counted candidates + old/new sub-bins in big ROR tiles: stream tests, stream bench, kernel stats
set -e
TAG=${TAG:-r03j}
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_tiled.py -x -v --timeout 300 --timeout-method thread -k "stream" > gpurun_out/${TAG}_pytest_stream.log 2>&1 || { tail -60 gpurun_out/${TAG}_pytest_stream.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest_stream.log
timeout -k 10 300 python -u bench.py --stream --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_stream.log 2> gpurun_out/${TAG}_stream.err || { tail -20 gpurun_out/${TAG}_stream.err; exit 1; }
grep '^{' gpurun_out/${TAG}_stream.log | cut -c1-300
cd /tmp
rm -rf $R/gpurun_out/prof_${TAG}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_${TAG} -o stream -- python3 $R/bench.py --stream --steps 20 --warmup 2 --no-cpu-baseline > $R/gpurun_out/${TAG}_stream_prof.log 2>&1 || { tail -20 $R/gpurun_out/${TAG}_stream_prof.log; exit 1; }
cd $R
f=$(ls gpurun_out/prof_${TAG}/*kernel_stats.csv | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{r["Name"][:80]:80s} calls {r["Calls"]:>6} tot {float(r["TotalDurationNs"])/1e6:9.2f} ms avg {float(r["AverageNs"])/1e3:9.1f} us')
PY
rm -f gpurun_out/prof_${TAG}/*kernel_trace.csv
