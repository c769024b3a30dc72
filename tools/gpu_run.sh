#!/bin/bash
# One parameterised GPU evidence run (replaces round 3's one-off gpu_r03*.sh launchers). Steps are named
# in STEPS (space separated, run in order; each GPU step has its own time limit and the chain stops at the
# first failure):
#   pytest   the -m gpu parity suite (PYTEST_K: a -k expression)
#   smoke    __graft_entry__.smoke()
#   bench    the default bench line (BENCH_ARGS, default --no-cpu-baseline)
#   stream   the C4 streaming bench
#   kt       rocprofv3 --kernel-trace --stats of the sequential C2 loop
#   ktc3     the same on one C3 frame set (bench --config C3 on one GPU)
#   pmc      FETCH_SIZE and WRITE_SIZE passes (separate runs) -> TAG_pmc_traffic.json
#   pmcc3    the same on C3 (bench --config C3, one GPU) -> TAG_c3_pmc_traffic.json
#   tiled    the rotating-root test, then bench.py --tiled at RANKS (default "1 2 4"; 2 and 4 ranks share the
#            box's GPU over gloo)
#   tiledstream  bench.py --tiled --stream at 1 rank, then the driver's --gpus 2 flow over gloo
#   rorpmc   tools/rorbench binaries (RORBENCH, built in-tree beforehand): kernel trace + two SQ passes
#   bfsreal  the host BFS replay A/B on real skeleton clusters (tools/sdcheck/bfs_real.sh; CPU only)
#   trace    AOS_TRACE=1 host timelines (per stage: ms at each host sync) of a short C2 run
#   pmcsq    two SQ counter passes over the C2 bench for the kernels matching PMC_KERNELS
# Usage: TAG=r04a STEPS="pytest smoke bench kt" tools/gpu_run.sh
set -e
R=$PWD
TAG=${TAG:-r04x}
STEPS=${STEPS:-"pytest smoke bench kt"}
export TMPDIR=/tmp
mkdir -p gpurun_out
for step in $STEPS; do
  echo "[$TAG] $step $(date +%T)"
  case $step in
    pytest)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
        > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
      tail -1 gpurun_out/${TAG}_pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
        || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
      tail -1 gpurun_out/${TAG}_smoke.log ;;
    bench)
      timeout -k 10 600 python -u bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/${TAG}_bench.log \
        2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
      grep '^{' gpurun_out/${TAG}_bench.log | cut -c1-400 ;;
    stream)
      timeout -k 10 400 python -u bench.py --stream --steps 20 --warmup 2 > gpurun_out/${TAG}_stream.log \
        2> gpurun_out/${TAG}_stream.err || { tail -20 gpurun_out/${TAG}_stream.err; exit 1; }
      grep '^{' gpurun_out/${TAG}_stream.log | cut -c1-300 ;;
    kt)
      rm -rf gpurun_out/${TAG}_kt
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kt -o kt \
        -- python3 $R/bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 10 --warmup 2 \
        > $R/gpurun_out/${TAG}_kt.log 2>&1)
      python3 tools/kt_summary.py gpurun_out/${TAG}_kt 12 > gpurun_out/${TAG}_kt_summary.txt
      head -30 gpurun_out/${TAG}_kt_summary.txt ;;
    ktc3)
      rm -rf gpurun_out/${TAG}_ktc3
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_ktc3 -o kt \
        -- python3 $R/bench.py --config C3 --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 3 --warmup 1 \
        > $R/gpurun_out/${TAG}_ktc3.log 2>&1)
      python3 tools/kt_summary.py gpurun_out/${TAG}_ktc3 4 > gpurun_out/${TAG}_ktc3_summary.txt
      head -30 gpurun_out/${TAG}_ktc3_summary.txt ;;
    kttiled)
      rm -rf gpurun_out/${TAG}_kttiled
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_kttiled -o kt \
        -- python3 $R/bench.py --tiled --steps 4 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${TAG}_kttiled.log 2>&1)
      python3 tools/kt_summary.py gpurun_out/${TAG}_kttiled 5 > gpurun_out/${TAG}_kttiled_summary.txt
      head -40 gpurun_out/${TAG}_kttiled_summary.txt ;;
    pmc)
      rm -rf gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_fetch -o fetch \
        -- python3 $R/bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 3 --warmup 1 \
        > $R/gpurun_out/${TAG}_fetch.log 2>&1)
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_write -o write \
        -- python3 $R/bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 3 --warmup 1 \
        > $R/gpurun_out/${TAG}_write.log 2>&1)
      python3 tools/pmc_traffic.py $(ls gpurun_out/${TAG}_fetch/*counter_collection.csv | head -1) \
        $(ls gpurun_out/${TAG}_write/*counter_collection.csv | head -1) gpurun_out/${TAG}_pmc_traffic.json
      cp gpurun_out/${TAG}_pmc_traffic.json profiles/ ;;   # (a later bench step of this call reads it)
    pmcc3)
      rm -rf gpurun_out/${TAG}_c3fetch gpurun_out/${TAG}_c3write
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${TAG}_c3fetch -o fetch \
        -- python3 $R/bench.py --config C3 --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 2 --warmup 1 \
        > $R/gpurun_out/${TAG}_c3fetch.log 2>&1)
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${TAG}_c3write -o write \
        -- python3 $R/bench.py --config C3 --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 2 --warmup 1 \
        > $R/gpurun_out/${TAG}_c3write.log 2>&1)
      python3 tools/pmc_traffic.py $(ls gpurun_out/${TAG}_c3fetch/*counter_collection.csv | head -1) \
        $(ls gpurun_out/${TAG}_c3write/*counter_collection.csv | head -1) gpurun_out/${TAG}_c3_pmc_traffic.json ;;
    trace)   # AOS_TRACE host timelines of a short C2 run -> TAG_trace.err
      AOS_TRACE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 6 \
        --warmup 2 > gpurun_out/${TAG}_trace.log 2> gpurun_out/${TAG}_trace.err || { tail -20 gpurun_out/${TAG}_trace.err; exit 1; }
      grep -c "aos trace" gpurun_out/${TAG}_trace.err ;;
    tracec3)   # the same on C3 -> TAG_tracec3.err
      AOS_TRACE=1 timeout -k 10 400 python -u bench.py --config C3 --no-cpu-baseline --no-pipelined-rate --no-device-rate \
        --steps 4 --warmup 1 > gpurun_out/${TAG}_tracec3.log 2> gpurun_out/${TAG}_tracec3.err || { tail -20 gpurun_out/${TAG}_tracec3.err; exit 1; }
      grep -c "aos trace" gpurun_out/${TAG}_tracec3.err ;;
    pmcsq)   # two SQ passes over the C2 bench for the kernels in PMC_KERNELS (a regex) -> TAG_pmcsq.txt
      K=${PMC_KERNELS:-k_occupancy|k_lfmis|k_ccl_local|k_scan_1p|k_rt_ror}
      rm -rf gpurun_out/${TAG}_sq1 gpurun_out/${TAG}_sq2
      (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "$K" --output-format csv \
        -d $R/gpurun_out/${TAG}_sq1 -o sq1 -- python3 $R/bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate \
        --steps 3 --warmup 1 > $R/gpurun_out/${TAG}_sq1.log 2>&1)
      (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
        SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "$K" --output-format csv \
        -d $R/gpurun_out/${TAG}_sq2 -o sq2 -- python3 $R/bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate \
        --steps 3 --warmup 1 > $R/gpurun_out/${TAG}_sq2.log 2>&1)
      python3 tools/pmc_summary.py gpurun_out/${TAG}_sq1 gpurun_out/${TAG}_sq2 > gpurun_out/${TAG}_pmcsq.txt
      cat gpurun_out/${TAG}_pmcsq.txt ;;
    tiled)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_tiled.py -x -v --timeout 400 --timeout-method thread -k rotating \
        > gpurun_out/${TAG}_pytest_rot.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_rot.log; exit 1; }
      tail -1 gpurun_out/${TAG}_pytest_rot.log
      for n in ${RANKS:-1 2 4}; do
        log=gpurun_out/${TAG}_tiled_${n}.log
        if [ "$n" = 1 ]; then
          timeout -k 10 400 python -u bench.py --tiled --steps 8 --warmup 2 --no-cpu-baseline > $log 2>&1 || { tail -20 $log; exit 1; }
        else
          AOS_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
            --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --tiled --steps 8 --warmup 2 \
            --no-cpu-baseline > $log 2>&1 || { tail -30 $log; exit 1; }
        fi
        grep '^{' $log | cut -c1-300
      done ;;
    tiledstream)
      timeout -k 10 300 python -u bench.py --tiled --stream --steps 10 --warmup 2 --no-cpu-baseline \
        > gpurun_out/${TAG}_ts1.log 2> gpurun_out/${TAG}_ts1.err || { tail -30 gpurun_out/${TAG}_ts1.err; exit 1; }
      grep '^{' gpurun_out/${TAG}_ts1.log | cut -c1-300
      AOS_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29631 bench.py --gpus 2 --steps 8 --warmup 3 --no-cpu-baseline \
        > gpurun_out/${TAG}_ts2.log 2>&1 || { tail -30 gpurun_out/${TAG}_ts2.log; exit 1; }
      grep '^{' gpurun_out/${TAG}_ts2.log | cut -c1-300 ;;
    rccl2)   # the driver's --gpus 2 flow over RCCL itself on the one GPU (AOS_BENCH_RCCL_SHARED_GPU: a NCCL_HOSTID per
             # rank, RCCL's socket transport on loopback): the independent maps, then the tiled C3 / C4 extras
      AOS_BENCH_RCCL_SHARED_GPU=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29651 bench.py --gpus 2 --steps 8 --warmup 2 --no-cpu-baseline \
        > gpurun_out/${TAG}_rccl2.log 2>&1 || { tail -30 gpurun_out/${TAG}_rccl2.log; exit 1; }
      grep '^{' gpurun_out/${TAG}_rccl2.log | cut -c1-400 ;;
    rccl6)   # the tiled C3 frame over 6 RCCL ranks on the one GPU (3 x 2 tiles: halo strips to neighbours only)
      AOS_BENCH_RCCL_SHARED_GPU=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 6 \
        --master-addr 127.0.0.1 --master-port 29652 bench.py --gpus 6 --tiled --steps 6 --warmup 2 --no-cpu-baseline \
        > gpurun_out/${TAG}_rccl6.log 2>&1 || { tail -30 gpurun_out/${TAG}_rccl6.log; exit 1; }
      grep '^{' gpurun_out/${TAG}_rccl6.log | cut -c1-400 ;;
    bfsreal)   # the host BFS replay A/B on real C1 row clusters (tools/sdcheck/bfs_real.sh) on the box's EPYC
      timeout -k 10 300 bash tools/sdcheck/bfs_real.sh > gpurun_out/${TAG}_bfs_real.txt 2>&1 || { tail -20 gpurun_out/${TAG}_bfs_real.txt; exit 1; }
      tail -14 gpurun_out/${TAG}_bfs_real.txt ;;
    c3bench)
      timeout -k 10 600 python -u bench.py --config C3 --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 6 \
        --warmup 2 > gpurun_out/${TAG}_c3_bench.log 2> gpurun_out/${TAG}_c3_bench.err || { tail -20 gpurun_out/${TAG}_c3_bench.err; exit 1; }
      grep '^{' gpurun_out/${TAG}_c3_bench.log | cut -c1-300 ;;
    rorpmc)
      for b in ${RORBENCH:-tools/rorbench/rorbench}; do
        n=$(basename $b)
        timeout -k 10 120 $R/$b 4096 10000000 10 12 > gpurun_out/${TAG}_${n}.log 2>&1 || { tail -5 gpurun_out/${TAG}_${n}.log; exit 1; }
        tail -2 gpurun_out/${TAG}_${n}.log
        rm -rf gpurun_out/${TAG}_${n}_kt gpurun_out/${TAG}_${n}_sq1 gpurun_out/${TAG}_${n}_sq2
        (cd /tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${TAG}_${n}_kt -o kt \
          -- $R/$b 4096 10000000 4 12 > $R/gpurun_out/${TAG}_${n}_kt.log 2>&1)
        (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
          SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $R/gpurun_out/${TAG}_${n}_sq1 -o sq1 \
          -- $R/$b 4096 10000000 2 12 > $R/gpurun_out/${TAG}_${n}_sq1.log 2>&1)
        (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
          SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/${TAG}_${n}_sq2 -o sq2 \
          -- $R/$b 4096 10000000 2 12 > $R/gpurun_out/${TAG}_${n}_sq2.log 2>&1)
        python3 tools/pmc_summary.py gpurun_out/${TAG}_${n}_sq1 gpurun_out/${TAG}_${n}_sq2 || true
      done ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$TAG] done $(date +%T)"
