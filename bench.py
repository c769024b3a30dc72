#!/usr/bin/env python3
"""bench.py — Mcells/s of the AOS seed-gen + GVD hot path on MI355X (BASELINE.json metric).

One step = one full frame of the path on one GPU, measured as SURVEY §8d defines it: the
PointCloud2 bytes in host memory -> ROR / clip / raster -> inflation -> opening + Zhang-Suen ->
clusters / tree rows / seeds -> GVD graph (seed merge, Delaunay replay, boundary points, edges,
labels) -> host GvdGraph, seeds / rows arrays and both OccupancyGrids in host memory.
`value` = W*H x K / the timed region (pipelined GVD jobs, --depth; the frame latency beside it), or
W*H / median frame time with --sequential. The device-resident rate (cloud already in HBM, grids left in
HBM) is reported beside it (`device_resident`). Workload: config C2 (10 M points, 4096^2 cells @
0.1 m, BASELINE.json configs[2]).

Multi-GPU (--gpus N, launched by torch.distributed.run): weak scaling — every rank processes its
own independent 4096^2 map tile (scene seed 3 + rank); no data-path collective; the barrier and
the max-over-ranks time use torch.distributed (RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for sub in ("tools", "active-orchard-slam_amd"):
    sys.path.insert(0, os.path.join(ROOT, sub))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PMC_FILE = os.path.join(ROOT, "profiles", "r02q_pmc_traffic.json")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default=None, help="C2 (default), or C3 with --tiled")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-config", default="C2", help="config of the CPU baseline frame (default: the bench's C2)")
    ap.add_argument("--stream", action="store_true",
                    help="C4 (BASELINE configs[4]): 1 M-point 20 Hz scans appended to the device-resident C2 map")
    ap.add_argument("--device-io", action="store_true",
                    help="time the device-resident frame (cloud in HBM, grids left in HBM) instead of SURVEY §8d's "
                         "host-in / host-out frame")
    ap.add_argument("--no-device-rate", action="store_true", help="skip the extra device-resident loop")
    ap.add_argument("--trace", action="store_true", help="per-step timeline of the pipelined loop on stderr")
    ap.add_argument("--depth", type=int, default=8,
                    help="pipelined GVD jobs in flight (aos_gvd_pipeline_depth): frames are independent, so frame "
                         "k's GVD runs beside the GVDs of frames k-1 .. k-depth+1, each Subdiv2D replay on its own core")
    ap.add_argument("--sequential", action="store_true",
                    help="run seed-gen and GVD of a frame back to back instead of the default pipeline (frame k's "
                         "seed-gen overlaps frame k-1's GVD, as the reference's two nodes do)")
    ap.add_argument("--tiled", action="store_true",
                    help="one map split into tiles over the ranks (SURVEY §8e, BASELINE configs[3]); strong scaling")
    ap.add_argument("--markers-every-frame", action="store_true",
                    help="publishMarkers' cells (a second Subdiv2D) for every frame; default: for the frames the "
                         "node publishes, at most max_graph_publish_rate (10 Hz) as the reference does (gvd:306-314)")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="upload each frame's PointCloud2 inside its own seed-gen call (no aos_cloud_prefetch)")
    ap.add_argument("--no-markers", action="store_true",
                    help="(diagnostic) no publishMarkers cells at all; not the reference's work")
    ap.add_argument("--fixed-root", action="store_true",
                    help="--tiled: rank 0 finishes every frame (default: frame k's root is rank k mod N, so the "
                         "whole-map stages and the GVD jobs rotate over the ranks)")
    a = ap.parse_args(argv)
    if a.config is None:
        a.config = "C3" if a.tiled else "C2"
    return a


def timed_region(step, steps: int, warmup: int, world: int, sync, dist=None, device=None):
    """The contract's timed region: W untimed steps, barrier + sync, EXACTLY K timed steps, sync +
    barrier, then the max over ranks. Every step ends with its outputs in host memory, so the host
    clock between steps is a frame time. Returns (seconds, per-step results, per-step seconds, max
    over ranks per step)."""
    last = None
    for _ in range(warmup):
        last = step()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    results, marks = [], [t0]
    for _ in range(steps):
        results.append(step())
        marks.append(time.perf_counter())
    sync()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    per = [b - a for a, b in zip(marks[:-1], marks[1:])]
    if world > 1:
        import torch
        t = torch.tensor([dt] + per, dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, per = float(t[0].item()), [float(x) for x in t[1:].tolist()]
    return dt, results or [last], per


def throughput(units_per_step: float, world: int, steps: int, dt: float) -> float:
    """Whole-job rate: units processed by all ranks / max-over-ranks wall time."""
    return units_per_step * world * steps / dt


def cpu_baseline(cfg_name: str) -> dict:
    """The oracle (single-threaded CPU restatement of the reference path) on a bounded sample."""
    import orchard
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as O
    cfg = orchard.CONFIGS[cfg_name]
    cloud = orchard.generate(cfg)
    poly = orchard.polygon(cfg)
    p = O.default_params(grid_resolution=cfg.res, faithful_dead_work=1, markers=1)
    t0 = time.perf_counter()
    r = O.seedgen(cloud, poly, p)
    t1 = time.perf_counter()
    O.gvd(r["voronoi_seeds"], r["rows_info"], r, p)
    t2 = time.perf_counter()
    cells = r["width"] * r["height"]
    return {"value": round(cells / (t2 - t0) / 1e6, 4), "unit": "Mcells/s", "cores": 1, "kind": "port",
            "sample": f"oracle/ CPU restatement, 1 thread, one full frame of config {cfg_name} "
                      f"({cfg.n_points} pts, {r['width']}x{r['height']} cells): seed-gen {t1 - t0:.2f} s + "
                      f"GVD {t2 - t1:.2f} s (incl. the reference's never-read vertex dedup and publishMarkers' cell "
                      f"boundaries)" + ("" if cfg_name == "C2" else "; not the bench config (the CPU GVD is super-linear in the "
                                                                    "map size, so a smaller config over-states the CPU rate)"),
            "cpu": _cpu_model()}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc passes (FETCH_SIZE x2 on
    gfx950 for 16 B/lane streaming reads + WRITE_SIZE, MI355X_MICROARCH.md 'HBM'), or None."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        k = d["kernels"][kernel]
        return k["bytes_per_launch"], d.get("source", PMC_FILE)
    except (OSError, KeyError, ValueError):
        return None, None


def _progress(msg: str) -> None:
    """Phase markers on stderr (a long silent run looks hung to the GPU harness)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    a = parse()
    _progress("importing torch")
    import torch  # (import before libaos_gpu: shared HIP runtime, see aos_gpu.lib)
    import torch.distributed as dist

    import aos_gpu
    import orchard
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # AOS_BENCH_BACKEND=gloo rehearses the N > 1 flow on fewer GPUs than ranks (ranks share devices;
    # the timing all-reduce runs on the host). The default, and the driver's run, is RCCL.
    backend = os.environ.get("AOS_BENCH_BACKEND", "nccl")
    gpu = local % torch.cuda.device_count() if backend == "gloo" else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    cfg = orchard.CONFIGS[a.config]
    _progress(f"generating {a.config}")
    poly = orchard.polygon(cfg)
    params = aos_gpu.default_params(grid_resolution=cfg.res)
    ctx = aos_gpu.Ctx(params, device=gpu)
    ctx.set_polygon(poly)
    if a.tiled:
        # one map: every rank holds the points of its tile's box (tile + ROR margin), resident in HBM
        import aos_tiles
        tx, ty = aos_tiles.tiling_for(world)
        plan = aos_tiles.tile_plan(params, poly, tx, ty, rank)
        cloud = aos_tiles.shard(orchard.generate(cfg), plan["points_box"])
        if world > 1 and backend == "nccl":   # the library's C++ RCCL communicator (no Python callbacks)
            comm = aos_tiles.RcclComm(plan["exchange_bytes"], gpu, rank, world)
        elif world > 1:                        # gloo rehearsal (ranks sharing a GPU)
            comm = aos_tiles.TorchDistComm(plan["exchange_bytes"], dev)
        else:
            comm = aos_tiles.ThreadGroup(1).comm(0, plan["exchange_bytes"], dev)
    else:
        cloud = orchard.generate(cfg, seed=cfg.seed + rank)
    d_cloud = torch.from_numpy(cloud).to(dev)
    n = cloud.shape[0]
    # the frame starts from the PointCloud2 bytes in host memory (a ROS message) and ends
    # with the OccupancyGrids in host memory. Stream / tiled modes start from their own HBM-resident maps.
    host_io = not (a.device_io or a.stream or a.tiled)
    mode = {"host": host_io}
    h_cloud = cloud if host_io else None
    del cloud
    if a.stream:
        # the map so far (the C2 cloud) is already device-resident; each step appends the next scan
        # from host memory (only the 16 MB scan crosses PCIe) and processes the whole map + GVD
        scans = [orchard.generate_scan(cfg, k) for k in range(a.warmup + a.steps)]
        ctx.map_reset(reserve_points=n + len(scans) * orchard.SCAN_POINTS)
        ctx.map_append(d_cloud.data_ptr(), n_points=n, on_device=True, want_host=False)
        latency, mk_latency = [], []
    # The reference builds the graph on every callback and publishes it, with the markers (publishMarkers:
    # a second Subdiv2D for the Voronoi cells), only when 1 / max_graph_publish_rate (0.1 s) has passed
    # since the last publish (gvd:306-314). The bench does the same work: every frame's graph, and the
    # markers of the frames that would be published (decided when the frame's GVD starts); with
    # --markers-every-frame, the markers of every frame. The markers' cells of a frame finish in the
    # background after its graph (publishGraph before publishMarkers, gvd:310-313) and are collected
    # with it, so each timed frame includes its markers.
    # --sequential: step k = seed-gen k, the markers of frame k - 1, then the GVD of frame k.
    # Pipelined (default): the reference's seed-gen and GVD are two nodes, so frame k's seed-gen runs while
    # frame k - 1's graph is built (aos_gvd_from_seedgen_async on the handle's GVD worker). Step k =
    # seed-gen k, collect graph + markers of frame k - 1, start the GVD of frame k; the last step also
    # collects its own frame, so every frame of the timed region completes inside it.
    n_calls = a.warmup + a.steps
    pend = {"k": 0, "t0": {}, "mt0": None, "ms": 0.0, "fifo": [], "lat": {}, "mk": {}, "last_pub": -1e9}
    pub_period = 1.0 / params.max_graph_publish_rate

    def markers_for(k):   # the publish throttle of processGraph (gvd:306-314)
        now = time.perf_counter()
        # (--stream keeps the markers on every scan: with the throttle, the scan after a markers scan
        # showed a ~25 ms stall of its first stream sync with the GPU idle, not understood)
        every = a.markers_every_frame or (a.stream and not os.environ.get("AOS_BENCH_STREAM_THROTTLE"))
        mk = not a.no_markers and (every or now - pend["last_pub"] >= pub_period)
        if mk:
            pend["last_pub"] = now
        pend["mk"][k] = mk
        ctx.gvd_set_markers(mk)
        return mk
    pipeline = not (a.sequential or a.stream)
    rotate = a.tiled and world > 1 and not a.fixed_root
    depth = max(1, a.depth) if pipeline else 1
    if pipeline:
        ctx.gvd_pipeline_depth(depth)

    def collect(collected=False):
        m = ctx.gvd_markers(collected=collected)
        if pend["mt0"] is not None and a.stream:
            mk_latency.append(time.perf_counter() - pend["mt0"])
        pend["ms"] = m["ms_cells"]
        pend["mt0"] = None
        return m

    def flush_markers():
        # the markers of the last frame collected with markers: its cells job finishes on its own core
        # after the graph, so it is collected one step later (before the next aos_gvd_wait makes another
        # frame the handle's current result) instead of holding the pipeline at once
        j = pend.pop("mk_frame", None)
        if j is not None:
            pend["mt0"] = pend["t0"][j]
            collect(collected=True)
            pend["lat"][j] = time.perf_counter() - pend["t0"][j]   # PointCloud2 in -> graph + markers out

    def finish(j):   # pipelined: frame j's graph; its markers at the next finish (or the drain)
        flush_markers()
        gg = ctx.gvd_wait()
        if a.stream:
            latency.append(time.perf_counter() - pend["t0"][j])
        if pend["mk"].get(j):
            pend["mk_frame"] = j
        else:
            pend["ms"] = 0.0
            pend["lat"][j] = time.perf_counter() - pend["t0"][j]
        gg["ms"]["cells"] = pend["ms"]
        return gg

    def step():
        k = pend["k"]
        pend["k"] += 1
        t0 = time.perf_counter()
        pend["t0"][k] = t0
        if a.stream:
            g = ctx.map_append(scans[k], want_host=False)
        elif a.tiled:
            # every rank receives the gathered skeleton and inflated tiles, so any rank can finish a frame:
            # frame k's root (a6, a8-a16 and its GVD job) is rank k mod N, which spreads the whole-map
            # stages and the GVD replays over the ranks' GPUs and host cores
            root_k = (k % world) if rotate else 0
            g = ctx.tiled_seedgen(comm, tx, ty, d_cloud.data_ptr(), root=root_k, n_points=n, on_device=True,
                                  want_host=False)
            if not g["root"]:
                gg = None
                if pipeline and k == n_calls - 1:   # drain this rank's GVD jobs (its earlier root frames)
                    while pend["fifo"]:
                        gg = finish(pend["fifo"].pop(0))
                    flush_markers()
                elif not pipeline and k == n_calls - 1 and pend.get("mk_pending"):
                    collect()
                return g, gg
        else:
            if mode["host"]:   # PointCloud2 bytes from host memory in, both OccupancyGrids to host out
                # (the grids are returned as views of the library's pinned buffers: the ABI's ownership rule)
                g = ctx.seedgen(h_cloud, want_host=True, copy_grids=False)
                if pipeline and not a.no_prefetch:
                    # the next frame's PointCloud2 crosses PCIe while this frame's GVD starts and the next
                    # step begins (aos_cloud_prefetch); the last step waits for its (unused) upload, so the
                    # timed region holds one upload per frame
                    ctx.cloud_prefetch(h_cloud)
                    if k == n_calls - 1:
                        ctx.cloud_prefetch_wait()
            else:
                g = ctx.seedgen(d_cloud.data_ptr(), n_points=n, on_device=True, want_host=False)
        if pipeline:
            # at most `depth` GVD jobs in flight: collect the oldest (graph + markers), start this frame's;
            # the last step drains every job, so each frame started in the timed region ends inside it
            t1 = time.perf_counter()
            gg = finish(pend["fifo"].pop(0)) if len(pend["fifo"]) >= depth else None
            t2 = time.perf_counter()
            markers_for(k)
            ctx.gvd_async()
            pend["fifo"].append(k)
            t3 = time.perf_counter()
            if k == n_calls - 1:
                while pend["fifo"]:
                    gg = finish(pend["fifo"].pop(0))
                flush_markers()
            if a.trace:
                ms = gg["ms"] if gg is not None else {}
                print(f"[trace] step {k}: seed-gen {1e3 * (t1 - t0):.2f} ms, wait oldest graph+markers "
                      f"{1e3 * (t2 - t1):.2f} ms, start GVD {1e3 * (t3 - t2):.2f} ms | collected frame: delaunay "
                      f"{ms.get('delaunay', 0):.1f} total {ms.get('total', 0):.1f} cells {ms.get('cells', 0):.1f}",
                      file=sys.stderr, flush=True)
            return g, gg
        ta = time.perf_counter()
        if k > 0 and pend.get("mk_pending", False):
            collect()
        tb = time.perf_counter()
        mk = markers_for(k)
        gg = ctx.gvd_from_seedgen()
        pend["mk_pending"] = mk
        if a.trace:
            print(f"[trace] step {k}: seed-gen {1e3 * (ta - t0):.2f} ms, collect previous markers {1e3 * (tb - ta):.2f} ms "
                  f"(cells {pend['ms']:.1f} ms), GVD {1e3 * (time.perf_counter() - tb):.2f} ms (delaunay "
                  f"{gg['ms'].get('delaunay', 0):.1f}, all {gg['ms']}), markers {int(mk)}", file=sys.stderr, flush=True)
        if a.stream:
            latency.append(time.perf_counter() - t0)
        pend["mt0"] = t0
        if k == n_calls - 1 and mk:
            collect()
        pend["lat"][k] = time.perf_counter() - t0
        gg["ms"]["cells"] = pend["ms"]   # the previous frame's (the last step: its own)
        return g, gg

    _progress(f"{a.warmup} warmup + {a.steps} timed frames")
    dt, res, per = timed_region(step, a.steps, a.warmup, world, torch.cuda.synchronize, dist, red_dev)
    mk_frames = sum(1 for k in range(a.warmup, a.warmup + a.steps) if pend["mk"].get(k))
    g, gg = res[-1]
    if a.tiled:   # the frame statistics of this rank's last root frame (its seeds, rows and graph)
        roots = [(gs, ggs) for gs, ggs in res if gs.get("root") and ggs is not None] or \
                [(gs, ggs) for gs, ggs in res if ggs is not None]
        if roots:
            g, gg = roots[-1]
    frame_lat = sorted(1e3 * pend["lat"][k] for k in range(a.warmup, a.warmup + a.steps) if k in pend["lat"])
    dev_rate = None
    if host_io and not a.no_device_rate:
        # the same frame with the cloud already in HBM and the grids left there (no PCIe)
        mode["host"] = False
        pend["k"], n_calls = 0, 2 + a.steps
        ddt, _, dper = timed_region(step, a.steps, 2, world, torch.cuda.synchronize, dist, red_dev)
        dmed = sorted(dper)[len(dper) // 2]
        dval = (throughput(g["width"] * g["height"] / 1e6, world, a.steps, ddt) if pipeline
                else (g["width"] * g["height"] / 1e6) * world / dmed)
        dev_rate = {"value": round(dval, 3), "median_ms": round(dmed * 1e3, 3),
                    "ms_per_step": round(ddt / a.steps * 1e3, 3),
                    "io": "cloud already in HBM, OccupancyGrids left in HBM, GvdGraph + seeds to host"}
    stage = {}
    n_gvd = sum(1 for _, ggs in res if ggs is not None)
    for gs, ggs in res:
        for k, v in gs["ms"].items():
            stage["seedgen_" + k] = stage.get("seedgen_" + k, 0.0) + v / len(res)
        for k, v in (ggs["ms"].items() if ggs is not None else ()):
            stage["gvd_" + k] = stage.get("gvd_" + k, 0.0) + v / n_gvd
    cells = g["width"] * g["height"]
    # weak: every rank processes its own map; tiled: the ranks share one map (strong scaling).
    # value = cells / median frame time (median of the warm frames), the contract's
    # timed-region mean beside it (value_mean).
    # pipelined (default): frames overlap, so a step's wall time is not a frame time; value = the
    # contract's timed-region throughput (K frames, the drain of the last jobs included), and the
    # frame latency (PointCloud2 in -> graph + markers out) is reported beside it
    med = sorted(per)[len(per) // 2]
    value_median = (cells / 1e6) * (1 if a.tiled else world) / med
    value_mean = throughput(cells / 1e6, 1 if a.tiled else world, len(res), dt)
    value = value_mean if pipeline else value_median
    avg = stage

    # Roofline (SURVEY §8d algorithmic bytes, HBM-bound; no MFMA). Per frame B_alg = 12 N + C (6 + 4 T):
    # 12 B per input point to read the cloud once and C for the raster write (the ROR stage), 2 C
    # inflation, 2 C opening, 4 C T thinning, C labelling. The ROR stage (a1-a4) is the dominant GPU
    # stage and is reported as `roofline`: its §8d bytes 12 N + C over the device time of its four
    # launches (count, tile scan, scatter, per-tile neighbour count), timed live with HIP events on the
    # handle's stream (aos_seedgen_out.ms_ror_*), averaged over the timed frames. `kernels` gives each
    # launch's time and the count pass's own figure (it is the one launch that reads the cloud: 12 N).
    n_all = float(n)   # the points this rank's ROR kernels read (tiled: its tile's shard)
    T = g["thin_iters"]
    t_cnt, t_scat, t_ror = avg["seedgen_ror_bin"], avg["seedgen_ror_scatter"], avg["seedgen_ror_count"]
    t_stage = avg.get("seedgen_ror_kernels", t_cnt + t_scat + t_ror)
    b_ror = 12.0 * n_all + cells
    ach = b_ror / (t_stage * 1e-3) / 1e9 if t_stage > 0 else 0.0
    traffic, src = pmc_traffic("ror_stage")
    kern = {"k_rt_part<count>": {"ms": round(t_cnt, 4), "alg_bytes": 12.0 * n_all,
                                  "achieved_GBs": round(12.0 * n_all / (t_cnt * 1e-3) / 1e9, 1) if t_cnt > 0 else 0.0},
            "k_rt_part<scatter>": {"ms": round(t_scat, 4)}, "k_rt_ror": {"ms": round(t_ror, 4)}}
    kern["k_rt_part<count>"]["frac"] = round(kern["k_rt_part<count>"]["achieved_GBs"] / HBM_PEAK_GBS, 4)
    roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": "ROR stage a1-a4 (k_rt_part<count>, tile scan, k_rt_part<scatter>, k_rt_ror)",
            "alg_bytes_per_launch": b_ror, "alg_bytes_model": "SURVEY §8d: 12 B per input point + 1 B per cell (raster)",
            "ms_per_launch": round(t_stage, 4), "units_per_launch": n_all, "traffic_source": src, "kernels": kern}
    # thinning: 4 C T bytes over the thinning stage (opening + temporal blocks, one read-back)
    b_thin = 4.0 * cells * T
    t_thin = avg.get("seedgen_thin", 0.0)
    thin_roof = {"alg_bytes": b_thin, "ms": round(t_thin, 4),
                 "achieved_GBs": round(b_thin / (t_thin * 1e-3) / 1e9, 1) if t_thin > 0 else 0.0}
    thin_roof["frac"] = round(thin_roof["achieved_GBs"] / HBM_PEAK_GBS, 4)
    # BASELINE.md frame-level figure: B_alg = 12 N + C (6 + 4 T) over the whole frame wall-clock
    b_frame = 12.0 * n_all + cells * (6.0 + 4.0 * T)
    frame_roof = {"alg_bytes": b_frame, "achieved_GBs": round(b_frame / med / 1e9, 2),
                  "frac": round(b_frame / med / 1e9 / HBM_PEAK_GBS, 5),
                  "note": "whole frame (median) incl. PCIe and the host Subdiv2D replay (DESIGN.md)"}

    if rank == 0:
        if a.stream:
            workload = (f"C4: 1 M-point scans at {orchard.SCAN_HZ:g} Hz appended to the device-resident {a.config} map "
                        f"({n} pts at start, {g['n_input']} after the last step), {g['width']}x{g['height']} cells "
                        f"@ {cfg.res} m, full seed-gen + GVD of the whole map per scan")
        elif a.tiled:
            workload = (f"{a.config}: {cfg.n_points} pts, {g['width']}x{g['height']} cells @ {cfg.res} m, one map in "
                        f"{tx}x{ty} tiles (rank 0 holds {n} pts), halo all-gathers, "
                        + (f"frame k finished (a6, a8-a16, GVD) by rank k mod {world}" if rotate else "GVD on rank 0"))
        else:
            workload = (f"{a.config}: {n} pts, {g['width']}x{g['height']} cells @ {cfg.res} m, "
                        f"full seed-gen + GVD per frame, one independent tile per GPU")
        out = {
            "metric": "Mcells/s skeleton+GVD (seed-gen + GVD frame) on 4096^2 grid",
            "value": round(value, 3), "unit": "Mcells/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(dt / len(res) * 1e3, 3), "higher_is_better": True,
            "value_mean": round(value_mean, 3), "value_median": round(value_median, 3), "median_ms": round(med * 1e3, 3),
            "frame_latency_ms": {"p50": round(frame_lat[len(frame_lat) // 2], 2), "max": round(frame_lat[-1], 2)}
            if frame_lat else None,
            "scaling": "strong" if a.tiled else "weak",
            "vs_baseline": None, "dtype": "f32/f64 (reference float/double arithmetic), u8/bit grids",
            "data": ("synthetic orchard (tools/orchard_gen.c, SplitMix64; 1 % in-clip outliers, not SURVEY §8d's 10 %, "
                     "which bridge every row at 0.1 m: DESIGN.md §8), "
                     + ("PointCloud2 bytes in host memory" if host_io else
                        "scans from host memory into the HBM-resident map" if a.stream else
                        "HBM-resident PointCloud2 shards" if a.tiled else "HBM-resident PointCloud2")),
            "config": {"workload": workload, "global_batch": 1 if a.tiled else world,
                       "parallelism": f"tiled{tx}x{ty}" if a.tiled else f"tiles{world}"},
            "io": "host PointCloud2 in, host OccupancyGrids + GvdGraph out (SURVEY §8d)" if host_io else
                  "device-resident cloud, device-resident grids, host GvdGraph",
            "device_resident": dev_rate,
            "pipeline": (f"depth {depth}: frame k's seed-gen overlaps the GVDs of frames k-1 .. k-{depth} (the "
                         f"reference's two nodes; frames are independent, each GVD's Subdiv2D replay on its own core)"
                         + ("; frame k+1's PointCloud2 upload (aos_cloud_prefetch) overlaps frame k's GVD start, one "
                            "upload per frame inside the timed region" if host_io and not a.no_prefetch else ""))
                        if pipeline else "sequential",
            "markers": {"policy": "every frame" if a.markers_every_frame or a.stream else
                        f"the frames the node publishes: at most max_graph_publish_rate = {params.max_graph_publish_rate:g} Hz "
                        f"of wall time (gvd:306-314); every frame's graph is built and returned",
                        "timed_frames_with_markers": mk_frames},
            "stages_ms": {k: round(v, 3) for k, v in avg.items()},
            "frame": {"T": T, "rows": len(g["row_length"]), "seeds": len(g["voronoi_seeds"]),
                      "nodes": len(gg["nodes"]), "edges": len(gg["edges"]), "n_binned": g["n_binned"],
                      "n_clipped": g["n_clipped"]},
            "roofline": roof,
            "thin_roofline": thin_roof,
            "frame_roofline": frame_roof,
        }
        if a.stream:
            lat = sorted(x * 1e3 for x in latency[a.warmup:])
            mlat = sorted(x * 1e3 for x in mk_latency[a.warmup:])
            out["stream"] = {"scan_latency_ms_p50": round(lat[len(lat) // 2], 2), "scan_latency_ms_max": round(lat[-1], 2),
                             "markers_latency_ms_p50": round(mlat[len(mlat) // 2], 2),
                             "markers_latency_ms_max": round(mlat[-1], 2),
                             "scan_latency_ms": [round(x * 1e3, 1) for x in latency[a.warmup:]],
                             "scan_markers": [int(bool(pend["mk"].get(k))) for k in range(a.warmup, a.warmup + a.steps)],
                             "scan_delaunay_ms": [round(gs[1]["ms"].get("delaunay", 0.0), 1) for gs in res],
                             "budget_ms": 1e3 / orchard.SCAN_HZ,
                             "keeps_up": max(lat[-1], dt / len(res) * 1e3) <= 1e3 / orchard.SCAN_HZ,
                             "note": "scan latency = scan H2D + pack + whole-map seed-gen + GVD graph (host clock); "
                                     "markers latency = until that scan's /gvd/markers cells are collected; "
                                     "keeps_up: graph latency and time per scan (markers included) within the budget"}
        if world == 1 and not a.no_cpu_baseline and not a.stream:
            _progress(f"CPU baseline (oracle, 1 thread) on {a.cpu_config}")
            out["cpu_baseline"] = cpu_baseline(a.cpu_config)
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
