#!/bin/bash
# kernel trace of the C4 stream (per-kernel time of the incremental ROR on big tiles)
set -e
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
rm -rf $R/gpurun_out/prof_stream3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_stream3 -o stream -- python3 $R/bench.py --stream --steps 20 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r03i_stream_prof.log 2>&1 || { tail -20 $R/gpurun_out/r03i_stream_prof.log; exit 1; }
cd $R
f=$(ls gpurun_out/prof_stream3/*kernel_stats.csv | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{r["Name"][:80]:80s} calls {r["Calls"]:>6} tot {float(r["TotalDurationNs"])/1e6:9.2f} ms avg {float(r["AverageNs"])/1e3:9.1f} us')
PY
rm -f gpurun_out/prof_stream3/*kernel_trace.csv
