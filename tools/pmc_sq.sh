set -e
# SQ counters of the seed-gen kernels (one pass, SQ block has 8 slots)
R=$PWD; export TMPDIR=/tmp; rm -rf gpurun_out/prof_sq; cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/prof_sq -o sq -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/gpurun_out/prof_sq.log 2>&1
cd $R; python - <<'PY'
import csv,collections,glob
f=glob.glob('gpurun_out/prof_sq/*counter_collection.csv')[0]
d=collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    d[r['Kernel_Name'].split('(')[0]][r['Counter_Name']].append(float(r['Counter_Value']))
for k in ('aos::k_ror_sweep','aos::k_ror_bin','aos::k_ror_scatter','aos::k_thin_block','aos::k_conflicts'):
    if k in d: print(k, {c: round(sum(v)/len(v)) for c,v in d[k].items()})
PY
