# grid D2H variants beside the cluster stage: DMA (default), DMA with the runtime's blit kernels limited to N
# workgroups (DEBUG_CLR_LIMIT_BLIT_WG), our copy kernel with N workgroups (AOS_GRID_COPY_KERNEL=1 AOS_GRID_COPY_BLOCKS=N)
set -e
mkdir -p gpurun_out
run() {   # tag, env...
  local tag=$1; shift
  env "$@" AOS_TRACE=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pipelined-rate --no-device-rate --steps 10 --warmup 3 > gpurun_out/r04gc_$tag.log 2> gpurun_out/r04gc_$tag.err
  echo "$tag: $(grep '^{' gpurun_out/r04gc_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_p50']; print('frame', d['frame_ms']['p50'], 'cluster', s['seedgen_cluster'], 'seeds', s['seedgen_seeds'], 'total', s['seedgen_total'])") | fg $(grep 'aos trace cluster' gpurun_out/r04gc_$tag.err | tail -5 | sed 's/.*fg \([0-9.]*\).*/\1/' | tr '\n' ' ')| synced $(grep 'aos trace finish' gpurun_out/r04gc_$tag.err | tail -5 | sed 's/.*copies_synced \([0-9.]*\).*/\1/' | tr '\n' ' ')"
}
for r in 1 2; do
  run dma A=1
  run blitwg8 DEBUG_CLR_LIMIT_BLIT_WG=8
  run blitwg32 DEBUG_CLR_LIMIT_BLIT_WG=32
  run k8 AOS_GRID_COPY_KERNEL=1 AOS_GRID_COPY_BLOCKS=8
  run k16 AOS_GRID_COPY_KERNEL=1 AOS_GRID_COPY_BLOCKS=16
  run k32 AOS_GRID_COPY_KERNEL=1 AOS_GRID_COPY_BLOCKS=32
done
