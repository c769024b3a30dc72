#!/usr/bin/env python3
"""bench.py — Mcells/s of the AOS seed-gen + GVD hot path on MI355X (BASELINE.json metric).

One step = one full frame of the path on one GPU, measured as SURVEY §8d / BASELINE.md:32 define it:
the PointCloud2 bytes in host memory -> ROR / clip / raster -> inflation -> opening + Zhang-Suen ->
clusters / tree rows / seeds -> GVD graph (seed merge, Delaunay replay, boundary points, edges,
labels) -> host GvdGraph, seeds / rows arrays and both OccupancyGrids in host memory.

`value` = W*H / the median per-frame wall-clock of the sequential loop (one frame at a time, no overlap
between frames: the timed region of the contract), i.e. BASELINE.md's "W.H / (seed-gen + GVD
wall-clock per frame), median of >= 5 warm runs". Beside it, in the same run:
  pipelined       frames overlapped as the reference's two nodes overlap (seed-gen of frame k while
                  the GVDs of earlier frames run, --depth jobs in flight, next cloud prefetched):
                  throughput and frame latency;
  device_resident the sequential frame with the cloud already in HBM and the grids left there.
Workload: config C2 (10 M points, 4096^2 cells @ 0.1 m, BASELINE.json configs[2]).

Multi-GPU (--gpus N, launched by torch.distributed.run): weak scaling — every rank processes its
own independent 4096^2 map (scene seed 3 + rank); no data-path collective; the barrier and the
max-over-ranks time use torch.distributed (RCCL). --tiled: one map split into tiles over the ranks
(SURVEY §8e, strong scaling). --tiled --stream: C4 over the ranks (BASELINE configs[4], 8 x MI355X
streaming): every rank receives each scan and keeps its tile's points box in its own HBM map. With N > 1
the same launch also reports the tiled C3 map (`tiled`) and the tiled C4 stream (`tiled_stream`).
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
WATCHDOG_EXIT = 3      # exit status of a run whose tiled section hung (its watchdog fired)
TILED_ERROR_EXIT = 4   # exit status of a run whose tiled / tiled_stream section raised (after the main line)
# rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE summaries (tools/pmc_traffic.py) of the ROR stage, per config,
# for the kernels of this build's ROR design. A config or design without a committed PMC run gets null.
ROR_DESIGN = "r06"    # (r04v: the host cloud split at upload; the partition passes read the front only. r05: + the tile
                      # pass's batched loads and branch on the exact division: the same kernels and bytes. r06: the
                      # column scan also max-reduces the tile totals; passes re-collected at the round-6 build)
PMC_FILES = {("C2", "r02"): os.path.join(ROOT, "profiles", "r02q_pmc_traffic.json"),
             ("C2", "r03"): os.path.join(ROOT, "profiles", "r03fin_pmc_traffic.json"),
             ("C2", "r04"): os.path.join(ROOT, "profiles", "r04i_pmc_traffic.json"),
             ("C2", "r04v"): os.path.join(ROOT, "profiles", "r04w_pmc_traffic.json"),
             ("C3", "r04v"): os.path.join(ROOT, "profiles", "r05_c3_pmc_traffic.json"),
             ("C2", "r05"): os.path.join(ROOT, "profiles", "r05zc_pmc_traffic.json"),
             ("C3", "r05"): os.path.join(ROOT, "profiles", "r05_c3_pmc_traffic.json"),
             ("C2", "r06"): os.path.join(ROOT, "profiles", "r06", "r06o_pmc_traffic.json"),
             ("C3", "r06"): os.path.join(ROOT, "profiles", "r06", "r06o_c3_pmc_traffic.json")}
# rocprofv3 --kernel-trace --stats summaries (tools/kt_summary.py) of the sequential loop at this build: the median
# trace frame's kernel time (every kernel of a frame, copies included), beside the live stage spans
KT_FILES = {"C2": os.path.join(ROOT, "profiles", "r06", "r06zs_kt_summary.txt")}


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
    ap.add_argument("--no-pipelined-rate", action="store_true", help="skip the extra pipelined loop")
    ap.add_argument("--no-tiled-rate", action="store_true",
                    help="--gpus N > 1: skip the extra tiled C3 / tiled C4 measurements (tiled, tiled_stream keys)")
    ap.add_argument("--trace", action="store_true", help="per-step timeline on stderr")
    ap.add_argument("--depth", type=int, default=4,
                    help="pipelined loop: GVD jobs in flight (aos_gvd_pipeline_depth): frames are independent, so "
                         "frame k's GVD runs beside the GVDs of frames k-1 .. k-depth+1, each replay on its own core. "
                         "4 keeps the frame latency near the sequential frame's; 8 adds ~10 %% throughput for "
                         "~20 ms of latency (DESIGN.md §5)")
    ap.add_argument("--pipelined", action="store_true",
                    help="make the pipelined loop the timed region (value = its throughput) instead of the "
                         "sequential per-frame loop")
    ap.add_argument("--sequential", action="store_true", help="(default) kept for older scripts")
    ap.add_argument("--tiled", action="store_true",
                    help="one map split into tiles over the ranks (SURVEY §8e, BASELINE configs[3]); strong scaling")
    ap.add_argument("--markers-every-frame", action="store_true",
                    help="publishMarkers' cells (a second Subdiv2D) for every frame; default: for the frames the "
                         "node publishes, at most max_graph_publish_rate (10 Hz) as the reference does (gvd:306-314)")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="pipelined loop: upload each frame's PointCloud2 inside its own seed-gen call")
    ap.add_argument("--no-markers", action="store_true",
                    help="(diagnostic) no publishMarkers cells at all; not the reference's work")
    ap.add_argument("--markers-no-copy", action="store_true",
                    help="(diagnostic) wait for the markers' cells but do not copy them into Python arrays")
    ap.add_argument("--markers-copy", action="store_true",
                    help="copy the markers into fresh Python arrays (default: views of the library-owned arrays, "
                         "as the grids are returned)")
    ap.add_argument("--cpu-baseline-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--sustain-s", type=float, default=None,
                    help="seconds of the sustained device-resident seed-gen leg before the CPU baseline's frame "
                         "(default 20; the baseline then runs in its child beside an idle bench process)")
    ap.add_argument("--fixed-root", action="store_true",
                    help="--tiled: rank 0 finishes every frame (default: frame k's root is rank k mod N, so the "
                         "whole-map stages and the GVD jobs rotate over the ranks)")
    a = ap.parse_args(argv)
    if a.config is None:
        a.config = "C3" if a.tiled and not a.stream else "C2"
    return a


def timed_region(step, steps: int, warmup: int, world: int, sync, dist=None, device=None):
    """The contract's timed region: W untimed steps, barrier + sync, EXACTLY K timed steps, sync +
    barrier, then the max over ranks. Every step ends with its outputs in host memory, so the host
    clock between steps is a frame time. Returns (seconds, per-step results, per-step seconds, the
    max over ranks per step)."""
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


def ror_points_read(res, n_default: int) -> float:
    """Mean over the timed frames of the points the ROR stage's partition passes read (aos_seedgen_out.n_ror_read);
    a frame that skipped the stage (a tiled streaming rank the scan missed) counts 0. n_default only for results
    that carry no such field."""
    vals = [gs.get("n_ror_read") for gs, _ in res]
    vals = [float(v) if v is not None else float(n_default) for v in vals]
    return sum(vals) / len(vals) if vals else float(n_default)


def _median(xs):
    s = sorted(xs)
    return s[len(s) // 2]


def cpu_baseline(cfg_name: str) -> dict:
    """The oracle (single-threaded CPU restatement of the reference path), one frame, with this thread
    pinned to one core (BASELINE.md:21's taskset -c; sched_setaffinity(0) pins the calling thread)."""
    import orchard
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as O
    cfg = orchard.CONFIGS[cfg_name]
    cloud = orchard.generate(cfg)
    poly = orchard.polygon(cfg)
    p = O.default_params(grid_resolution=cfg.res, faithful_dead_work=1, markers=1)
    allowed = sorted(os.sched_getaffinity(0))
    core = allowed[0]
    os.sched_setaffinity(0, {core})
    try:
        t0 = time.perf_counter()
        r = O.seedgen(cloud, poly, p)
        t1 = time.perf_counter()
        O.gvd(r["voronoi_seeds"], r["rows_info"], r, p)
        t2 = time.perf_counter()
    finally:
        os.sched_setaffinity(0, set(allowed))
    cells = r["width"] * r["height"]
    return {"value": round(cells / (t2 - t0) / 1e6, 4), "unit": "Mcells/s", "cores": 1, "kind": "port",
            "pinned_core": core,
            "sample": f"oracle/ CPU restatement, 1 thread pinned to core {core}, one full frame of config {cfg_name} "
                      f"({cfg.n_points} pts, {r['width']}x{r['height']} cells): seed-gen {t1 - t0:.2f} s + "
                      f"GVD {t2 - t1:.2f} s (incl. the reference's never-read vertex dedup and publishMarkers' cell "
                      f"boundaries)" + ("" if cfg_name == "C2" else "; not the bench config (the CPU GVD is super-linear in the "
                                                                    "map size, so a smaller config over-states the CPU rate)"),
            "ms_per_frame": round((t2 - t0) * 1e3, 1), "cpu": _cpu_model(), "host_cpus": os.cpu_count()}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pmc_traffic(config: str, kernel: str = "ror_stage"):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc passes of this config and ROR
    design (FETCH_SIZE x2 on gfx950 for 16 B/lane streaming reads + WRITE_SIZE, MI355X_MICROARCH.md
    'HBM'), or (None, None) when no such run is committed."""
    path = PMC_FILES.get((config, ROR_DESIGN))
    if path is None:
        return None, None
    try:
        with open(path) as f:
            d = json.load(f)
        src = os.path.relpath(path, ROOT) + " (summary of rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes; " + \
            "their raw counter CSVs are not committed)"
        return d["kernels"][kernel]["bytes_per_launch"], src
    except (OSError, KeyError, ValueError):
        return None, None


def kt_kernel_ms(config: str):
    """(median kernel ms per trace frame, source) from the committed kernel-trace summary of `config`, or (None, None)."""
    path = KT_FILES.get(config)
    try:
        with open(path) as f:
            for line in f:
                if line.startswith("trace frames"):   # "trace frames (10): median 76 launches, 1434.3 us kernel time, ..."
                    us = float(line.split("launches,")[1].split("us kernel time")[0])
                    return us * 1e-3, os.path.relpath(path, ROOT)
    except (OSError, TypeError, ValueError, IndexError):
        pass
    return None, None


def _progress(msg: str) -> None:
    """Phase markers on stderr (a long silent run looks hung to the GPU harness)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def spawn_cpu_baseline(a):
    """The CPU baseline runs in a child process pinned to one core of this process's CPU set; this process keeps
    the other cores (set before torch and the library start any thread, so every later thread inherits it). The
    child builds its cloud at once and starts the timed oracle frame when told to (after the main timed region and
    this process's sustained seed-gen leg; this process then waits). Started before anything touches the GPU (no
    exec from a process that has initialised it). Returns the Popen, or None (then the baseline runs inline)."""
    import subprocess
    allowed = sorted(os.sched_getaffinity(0))
    if len(allowed) < 2:
        return None
    core = allowed[0]
    try:
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--cpu-config",
                              a.cpu_config], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                             preexec_fn=lambda: os.sched_setaffinity(0, {core}))
    except OSError:
        return None
    os.sched_setaffinity(0, set(allowed) - {core})
    p.core = core
    return p


def cpu_baseline_child(a) -> None:
    """--cpu-baseline-child: wait for 'go' on stdin, time the oracle frame, print its JSON line."""
    import orchard
    orchard.generate(orchard.CONFIGS[a.cpu_config])   # (page in the generator and numpy before the clock)
    if sys.stdin.readline().strip() != "go":
        return
    print(json.dumps(cpu_baseline(a.cpu_config)), flush=True)


def start_cpu_baseline(child) -> None:
    try:
        child.stdin.write("go\n")
        child.stdin.flush()
        child.stdin.close()
    except (BrokenPipeError, OSError, ValueError):
        pass


def finish_cpu_baseline(child) -> dict:
    """The child's result (waits for it; its frame started after the sustained leg)."""
    if child.stdin and not child.stdin.closed:
        start_cpu_baseline(child)
    so = child.stdout.read()
    child.wait(timeout=1800)
    lines = [x for x in (so or "").splitlines() if x.startswith("{")]
    if child.returncode != 0 or not lines:
        return {"error": f"CPU baseline child exited {child.returncode}"}
    r = json.loads(lines[-1])
    r["sample"] += "; timed in a child process pinned to its own core while the bench process waited idle"
    return r


def main():
    a = parse()
    if a.cpu_baseline_child:
        cpu_baseline_child(a)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    cpu_child = None
    if world == 1 and not (a.no_cpu_baseline or a.stream or a.tiled) and os.environ.get("AOS_BENCH_CPU_INLINE") != "1":
        cpu_child = spawn_cpu_baseline(a)
    _progress("importing torch")
    import torch  # (import before libaos_gpu: shared HIP runtime, see aos_gpu.lib)
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # AOS_BENCH_BACKEND=gloo rehearses the N > 1 flow on fewer GPUs than ranks (ranks share devices;
    # the timing all-reduce runs on the host). The default, and the driver's run, is RCCL.
    backend = os.environ.get("AOS_BENCH_BACKEND", "nccl")
    # AOS_BENCH_RCCL_SHARED_GPU=1 rehearses it over RCCL itself on fewer GPUs than ranks: RCCL refuses two ranks
    # on one device of one host, so each rank takes its own NCCL_HOSTID and RCCL links the ranks over its socket
    # transport on loopback (the collectives are the production ones; only the wire differs from xGMI)
    shared_rccl = backend == "nccl" and os.environ.get("AOS_BENCH_RCCL_SHARED_GPU") == "1"
    if shared_rccl:
        os.environ["NCCL_HOSTID"] = f"aos-bench-rank-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    gpu = local % torch.cuda.device_count() if (backend == "gloo" or shared_rccl) else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    red_dev = dev if backend == "nccl" else torch.device("cpu")
    E = {"world": world, "rank": rank, "gpu": gpu, "dev": dev, "red_dev": red_dev, "backend": backend,
         "cpu_child": cpu_child}
    out = run(a, E, dist)
    sys.exit(report(a, E, dist, out))


def report(a, E, dist, out) -> int:
    """After the main measurement: the --gpus N launch's tiled extras, rank 0's JSON line, the process group's
    end. Returns the exit status: non-zero when a tiled section raised (the line is printed regardless)."""
    world, rank = E["world"], E["rank"]
    extras = {}
    if world > 1 and not (a.tiled or a.stream or a.no_tiled_rate):
        # the multi-GPU launch also measures the one-map design (BASELINE configs[3]): C3 split
        # into tiling_for(N) tiles over the same ranks, halos and flags over the library's RCCL communicator
        extras["tiled"] = tiled_extra(a, E, dist, out)
        if out is not None:
            out["tiled"] = extras["tiled"]
        extras["tiled_stream"] = tiled_extra(a, E, dist, out, stream=True)
        if out is not None:
            out["tiled_stream"] = extras["tiled_stream"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    code = exit_status(extras)   # (every rank: a rank whose tiled section raised exits non-zero)
    if code:
        print(f"bench: a tiled section failed (exit {code}); the main line above holds the single-map measurement",
              file=sys.stderr, flush=True)
    return code


def exit_status(out) -> int:
    """Non-zero when the --gpus N launch's tiled / tiled_stream section raised: the line is still printed (the
    single-map measurement is valid), but the run did not complete what it was asked to measure."""
    if not isinstance(out, dict):
        return 0
    for key in ("tiled", "tiled_stream"):
        t = out.get(key)
        if isinstance(t, dict) and "error" in t:
            return TILED_ERROR_EXIT
    return 0


def tiled_extra(a, E, dist, main_out, stream: bool = False) -> dict:
    """One map (C3, 8192^2, 40 M points) in tiling_for(N) tiles over the N ranks, rotating roots with
    background GVD jobs: Mcells/s, frame latency and the root's serial whole-map finish. stream: C4 over the
    ranks instead (the C2 map, then 1 M-point scans; each rank keeps its tile's points box; frame k's root is
    rank k mod N): per-scan latency. Guarded by a watchdog: if the collectives do not finish in time every
    rank reports the timeout and exits."""
    import copy
    import threading
    b = copy.copy(a)
    b.tiled, b.stream, b.no_cpu_baseline = True, stream, True
    b.config = "C2" if stream else "C3"
    b.steps, b.warmup = (max(4, min(a.steps, 16)), 2) if stream else (max(4, min(a.steps, 12)), 3)
    key = "tiled_stream" if stream else "tiled"
    limit = float(os.environ.get("AOS_BENCH_TILED_TIMEOUT", "300"))
    res = {"main_out": main_out}

    def watchdog():
        res["error"] = f"{key} section did not finish within {limit:.0f} s (collective hang?)"
        if E["rank"] == 0 and res["main_out"] is not None:
            res["main_out"][key] = {"error": res["error"]}
            print(json.dumps(res["main_out"]), flush=True)
        print(f"bench: {res['error']}", file=sys.stderr, flush=True)
        # every rank's own watchdog fires: none is left waiting in a collective; the exit status says the run
        # did not complete (the main line above still carries the single-map measurement)
        os._exit(WATCHDOG_EXIT)
    timer = threading.Timer(limit, watchdog)
    timer.daemon = True
    timer.start()
    try:
        o = run(b, E, dist, quiet=True)
    except Exception as e:   # a failing communicator must not cost the main result
        timer.cancel()
        return {"error": f"{type(e).__name__}: {e}"}
    timer.cancel()
    if o is None:
        return None
    keep = ("value", "unit", "ms_per_step", "frame_latency_ms", "root_serial_ms", "root_serial_split_ms", "per_rank",
            "config", "frame", "stages_ms", "stream")
    return {k: o[k] for k in keep if k in o}


def pick_tiled_frames(res, g, gg):
    """The frame statistics a tiled rank reports: its last root frame (seeds, rows) and its last collected
    graph, picked separately (pipelined: a step returns an older frame's graph; with rotating roots a rank's
    steps mostly return non-root results). A rank whose timed steps held no root frame keeps (g, gg)."""
    gr = [gs for gs, _ in res if gs.get("root")]
    gq = [ggs for _, ggs in res if ggs is not None]
    return (gr[-1] if gr else g), (gq[-1] if gq else gg)


def tiled_breakdown(res, pend, warmup: int, world: int, rank: int, dist):
    """Per rank, the timed tiled frames' averages of aos_tiled_stats (host clock): the whole call, the time
    inside the all-gather / all-reduce callbacks (a collective includes the wait for the slowest rank), and
    the rest (compute); and, over the root frames of all ranks, the root's serial part split into the
    cluster stage (of which the exact BFS replays run on the root), rows + seeds and the GVD's GPU prefix
    (the seed merge, before its job goes to the background). Returns (per-rank list, split) on rank 0."""
    keys = ("ms_frame", "ms_comm_gather", "ms_comm_reduce", "ms_ror", "ms_thin", "ms_cluster_local",
            "ms_cluster_global", "ms_replay")
    sts = [gs["tiled_stats"] for gs, _ in res if "tiled_stats" in gs]
    mine = {"rank": rank, "frames": len(sts)}
    for k in keys:
        mine[k] = round(sum(t[k] for t in sts) / max(1, len(sts)), 3)
    mine["ms_compute"] = round(mine["ms_frame"] - mine["ms_comm_gather"] - mine["ms_comm_reduce"], 3)
    mine["collectives_per_frame"] = round(sum(t["n_gather"] + t["n_reduce"] for t in sts) / max(1, len(sts)), 1)
    mine["gather_MB_per_frame"] = round(sum(t["bytes_gather"] for t in sts) / max(1, len(sts)) / 1e6, 3)
    mine["recv_MB_per_frame"] = round(sum(t.get("bytes_recv", 0) for t in sts) / max(1, len(sts)) / 1e6, 3)
    nonroot = [t for t in sts if not t["is_root"]]
    mine["recv_MB_nonroot_frame"] = round(sum(t.get("bytes_recv", 0) for t in nonroot) / max(1, len(nonroot)) / 1e6, 3)
    mine["ror_skipped_frames"] = sum(t["ror_skipped"] for t in sts)
    root_frames = [(k, t) for k, (gs, _) in enumerate(res) if gs.get("root") for t in [gs.get("tiled_stats")] if t]
    gstart = pend.get("gvd_start", {})
    mine_root = [(t["ms_cluster"], t["ms_replay"], t["ms_seeds"], 1e3 * gstart.get(warmup + k, 0.0)) for k, t in root_frames]
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, (mine, mine_root))
    else:
        allr = [(mine, mine_root)]
    if rank != 0:
        return None, None
    per_rank = [m for m, _ in allr]
    roots = [r for _, rr in allr for r in rr]
    split = None
    if roots:
        n = len(roots)
        split = {"cluster_stage": round(sum(r[0] for r in roots) / n, 3),
                 "of_which_replays_on_root": round(sum(r[1] for r in roots) / n, 3),
                 "rows_and_seeds": round(sum(r[2] for r in roots) / n, 3),
                 "gvd_prefix": round(sum(r[3] for r in roots) / n, 3), "root_frames": n}
    return per_rank, split


def run(a, E, dist, quiet=False):
    """One timed configuration; returns rank 0's result dict (None on other ranks)."""
    import torch

    import aos_gpu
    import orchard
    if os.environ.get("AOS_NUMPY_HUGEPAGE") != "1":
        aos_gpu.disable_numpy_hugepage()   # (the markers copies: DESIGN §7b; AOS_NUMPY_HUGEPAGE=1 keeps numpy's default)
    if os.environ.get("AOS_BENCH_REPLAY_GPU"):   # A/B runs: the exact BFS replays from this many clusters on the GPU
        aos_gpu.debug_replay(int(os.environ["AOS_BENCH_REPLAY_GPU"]))
    world, rank, gpu, dev, red_dev, backend = E["world"], E["rank"], E["gpu"], E["dev"], E["red_dev"], E["backend"]

    cfg = orchard.CONFIGS[a.config]
    _progress(f"generating {a.config}")
    poly = orchard.polygon(cfg)
    params = aos_gpu.default_params(grid_resolution=cfg.res)
    ctx = aos_gpu.Ctx(params, device=gpu)
    ctx.set_polygon(poly)
    if a.tiled:
        # one map: every rank holds the points of its tile's box (tile + ROR margin), resident in HBM (a
        # tiled stream: every rank receives the whole map and each whole scan; the library keeps the box)
        import aos_tiles
        tx, ty = aos_tiles.tiling_for(world)
        plan = aos_tiles.tile_plan(params, poly, tx, ty, rank)
        cloud = orchard.generate(cfg) if a.stream else aos_tiles.shard(orchard.generate(cfg), plan["points_box"])
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
    h_cloud = cloud if host_io else None
    del cloud
    if a.stream:
        # the map so far (the C2 cloud) is already device-resident; each step appends the next scan
        # from host memory (only the 16 MB scan crosses PCIe) and processes the whole map + GVD
        scans = [orchard.generate_scan(cfg, k) for k in range(a.warmup + a.steps)]
        ctx.map_reset(reserve_points=n + len(scans) * orchard.SCAN_POINTS)
        if a.tiled:   # the map's first tiled frame (every rank keeps its box; rank 0 finishes it)
            ctx.tiled_map_append(comm, tx, ty, d_cloud.data_ptr(), root=0, n_points=n, on_device=True, want_host=False)
        else:
            ctx.map_append(d_cloud.data_ptr(), n_points=n, on_device=True, want_host=False)
    latency, mk_latency = [], []
    # The reference builds the graph on every callback and publishes it, with the markers (publishMarkers:
    # a second Subdiv2D for the Voronoi cells), only when 1 / max_graph_publish_rate (0.1 s) has passed
    # since the last publish (gvd:306-314). The bench does the same work: every frame's graph, and the
    # markers of the frames that would be published (decided when the frame's GVD starts); with
    # --markers-every-frame, the markers of every frame. The markers' cells of a frame finish in the
    # background after its graph (publishGraph before publishMarkers, gvd:310-313) and are collected
    # one step later.
    # sequential (the default timed region): step k = seed-gen k, the markers of frame k - 1, then the GVD
    # of frame k — one frame at a time, PointCloud2 in host memory -> GvdGraph + grids in host memory.
    # pipelined: the reference's seed-gen and GVD are two nodes, so frame k's seed-gen runs while frame
    # k - 1's graph is built (aos_gvd_from_seedgen_async). Step k = seed-gen k, collect graph + markers of
    # the oldest frame when `depth` are in flight, start the GVD of frame k; the last step drains every
    # job, so every frame of the timed region completes inside it.
    mode = {"host": host_io, "pipeline": False, "depth": 1, "prefetch": False, "n_calls": a.warmup + a.steps}
    pend = {"k": 0, "t0": {}, "mt0": None, "ms": 0.0, "fifo": [], "lat": {}, "mk": {}, "last_pub": -1e9}
    pub_period = 1.0 / params.max_graph_publish_rate
    rotate = a.tiled and world > 1 and not a.fixed_root

    def reset(pipeline: bool, host: bool, steps: int, warmup: int):
        mode.update(host=host, pipeline=pipeline, depth=max(1, a.depth) if pipeline else 1,
                    prefetch=pipeline and host and not a.no_prefetch, n_calls=warmup + steps)
        pend.update(k=0, t0={}, mt0=None, ms=0.0, fifo=[], lat={}, mk={}, last_pub=-1e9)
        pend.pop("mk_frame", None)
        pend.pop("mk_pending", None)
        if pipeline:
            ctx.gvd_pipeline_depth(mode["depth"])

    def markers_for(k):   # the publish throttle of processGraph (gvd:306-314)
        now = time.perf_counter()
        mk = not a.no_markers and (a.markers_every_frame or now - pend["last_pub"] >= pub_period)
        if mk:
            pend["last_pub"] = now
        pend["mk"][k] = mk
        ctx.gvd_set_markers(mk)
        return mk

    def collect(collected=False):
        m = ctx.gvd_markers(collected=collected, copy=not a.markers_no_copy, view=not a.markers_copy)
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
        gg = ctx.gvd_wait(copy=False)
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
        last = k == mode["n_calls"] - 1
        t0 = time.perf_counter()
        pend["t0"][k] = t0
        if a.stream and a.tiled:
            # C4 over the ranks: every rank appends the whole scan to its box's map and runs its tiles; the
            # frame's root (rank k mod N) finishes it and builds the graph
            root_k = k % world
            g = ctx.tiled_map_append(comm, tx, ty, scans[k], root=root_k, want_host=False)
            if not g["root"]:
                if last and pend.get("mk_pending"):
                    collect()
                    pend["mk_pending"] = False
                return g, None
        elif a.stream:
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
                if mode["pipeline"] and last:   # drain this rank's GVD jobs (its earlier root frames)
                    while pend["fifo"]:
                        gg = finish(pend["fifo"].pop(0))
                    flush_markers()
                elif not mode["pipeline"] and last and pend.get("mk_pending"):
                    collect()
                return g, gg
        elif mode["host"]:   # PointCloud2 bytes from host memory in, both OccupancyGrids to host out
            # (the grids are returned as views of the library's pinned buffers: the ABI's ownership rule)
            g = ctx.seedgen(h_cloud, want_host=True, copy_grids=False)
            if mode["prefetch"]:
                # pipelined: the next frame's PointCloud2 crosses PCIe while this frame's GVD starts and the
                # next step begins (aos_cloud_prefetch); the last step waits for its (unused) upload, so the
                # timed region holds one upload per frame
                ctx.cloud_prefetch(h_cloud)
                if last:
                    ctx.cloud_prefetch_wait()
        else:
            g = ctx.seedgen(d_cloud.data_ptr(), n_points=n, on_device=True, want_host=False)
        if mode["pipeline"]:
            # at most `depth` GVD jobs in flight: collect the oldest (graph + markers), start this frame's;
            # the last step drains every job, so each frame started in the timed region ends inside it
            t1 = time.perf_counter()
            gg = finish(pend["fifo"].pop(0)) if len(pend["fifo"]) >= mode["depth"] else None
            t2 = time.perf_counter()
            markers_for(k)
            ctx.gvd_async()
            pend["fifo"].append(k)
            t3 = time.perf_counter()
            pend.setdefault("gvd_start", {})[k] = t3 - t2   # the GVD's GPU prefix (seed merge) before it goes async
            if last:
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
        gg = ctx.gvd_from_seedgen(copy=False)   # (views of the library's arrays, as the seed-gen grids)
        pend["mk_pending"] = mk
        if a.trace:
            print(f"[trace] step {k}: seed-gen {1e3 * (ta - t0):.2f} ms (device {g['ms']['total']:.2f}), collect "
                  f"previous markers {1e3 * (tb - ta):.2f} ms (cells {pend['ms']:.1f} ms), GVD "
                  f"{1e3 * (time.perf_counter() - tb):.2f} ms (merge {gg['ms'].get('merge', 0):.2f}, delaunay "
                  f"{gg['ms'].get('delaunay', 0):.1f}, graph {gg['ms'].get('graph', 0):.2f}), markers {int(mk)}",
                  file=sys.stderr, flush=True)
        if a.stream:
            latency.append(time.perf_counter() - t0)
        pend["mt0"] = t0
        if last and mk:
            collect()
        pend["lat"][k] = time.perf_counter() - t0
        gg["ms"]["cells"] = pend["ms"]   # the previous frame's (the last step: its own)
        return g, gg

    sync = torch.cuda.synchronize
    # the timed region: sequential frames (default), the tiled map's rotating-root pipeline, or --pipelined
    main_pipe = a.pipelined or (a.tiled and not a.sequential and not a.stream)
    reset(main_pipe, host_io, a.steps, a.warmup)
    _progress(f"{a.warmup} warmup + {a.steps} timed frames ({'pipelined' if main_pipe else 'sequential'})")
    dt, res, per = timed_region(step, a.steps, a.warmup, world, sync, dist, red_dev)
    mk_frames = sum(1 for k in range(a.warmup, a.warmup + a.steps) if pend["mk"].get(k))
    frame_lat = sorted(1e3 * pend["lat"][k] for k in range(a.warmup, a.warmup + a.steps) if k in pend["lat"])
    if a.tiled and a.stream:
        # every step is one scan's frame, finished by its root (rank k mod N): the root's own latency (its
        # seed-gen call start -> GvdGraph), gathered by a max over ranks (the other ranks report 0)
        root_lat = [pend["lat"].get(k, 0.0) for k in range(a.warmup, a.warmup + a.steps)]
        if world > 1:
            t = torch.tensor(root_lat, dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            root_lat = [float(x) for x in t.tolist()]
        frame_lat = sorted(1e3 * x for x in root_lat)
    g, gg = res[-1]
    if a.tiled:
        g, gg = pick_tiled_frames(res, g, gg)
    cells = g["width"] * g["height"]
    units = (cells / 1e6) * (1 if a.tiled else world)   # Mcells per step over all ranks
    med = _median(per)
    value_mean = units * len(res) / dt
    # sequential: every step is one whole frame, so the median step is the median per-frame wall-clock
    # (the max over ranks at N > 1); pipelined: frames overlap and the timed-region throughput is the rate
    value = value_mean if main_pipe else units / med

    tiled_ranks = tiled_split = None
    if a.tiled:
        tiled_ranks, tiled_split = tiled_breakdown(res, pend, a.warmup, world, rank, dist)

    stage = {}
    per_stage = {}   # every timed frame's value per stage: stages_ms_p50 beside the means
    n_gvd = sum(1 for _, ggs in res if ggs is not None)
    for gs, ggs in res:
        for key, v in gs["ms"].items():
            stage["seedgen_" + key] = stage.get("seedgen_" + key, 0.0) + v / len(res)
            per_stage.setdefault("seedgen_" + key, []).append(v)
        for key, v in (ggs["ms"].items() if ggs is not None else ()):
            stage["gvd_" + key] = stage.get("gvd_" + key, 0.0) + v / n_gvd
            per_stage.setdefault("gvd_" + key, []).append(v)
    stage_p50 = {k: round(_median(v), 3) for k, v in per_stage.items()}

    extra = {}
    if not a.stream and not a.tiled and not main_pipe and not a.no_pipelined_rate:
        # the same frames overlapped as the reference's two nodes overlap (throughput, latency beside it)
        reset(True, host_io, a.steps, 3)
        _progress(f"pipelined loop (depth {mode['depth']})")
        pdt, pres, pper = timed_region(step, a.steps, 3, world, sync, dist, red_dev)
        plat = sorted(1e3 * pend["lat"][k] for k in range(3, 3 + a.steps) if k in pend["lat"])
        extra["pipelined"] = {
            "value": round(units * len(pres) / pdt, 3), "unit": "Mcells/s", "depth": mode["depth"],
            "ms_per_step": round(pdt / len(pres) * 1e3, 3), "step_median_ms": round(_median(pper) * 1e3, 3),
            "frame_latency_ms": {"p50": round(_median(plat), 2), "max": round(plat[-1], 2)} if plat else None,
            "what": (f"frame k's seed-gen overlaps the GVDs of frames k-1 .. k-{mode['depth']} (the reference's two "
                     f"nodes; frames are independent, each GVD's Subdiv2D replay on its own core)"
                     + ("; frame k+1's PointCloud2 upload (aos_cloud_prefetch) overlaps frame k's GVD start, one "
                        "upload per frame inside the timed region" if mode["prefetch"] else "")
                     + "; value = frames x W.H / timed region incl. the drain of the last jobs")}
    if host_io and not main_pipe and not a.no_device_rate:
        # the same sequential frame with the cloud already in HBM and the grids left there (no PCIe)
        reset(False, False, a.steps, 2)
        _progress("device-resident sequential loop")
        ddt, _, dper = timed_region(step, a.steps, 2, world, sync, dist, red_dev)
        dmed = _median(dper)
        extra["device_resident"] = {"value": round(units / dmed, 3), "median_ms": round(dmed * 1e3, 3),
                                    "ms_per_step": round(ddt / a.steps * 1e3, 3),
                                    "io": "cloud already in HBM, OccupancyGrids left in HBM, GvdGraph + seeds to host"}
    if not (a.stream or a.tiled):
        # SURVEY §8d's GVD figure: the graph phase's "pair evaluations" (one counted frame outside the timed
        # region: the counts are a function of the frame's inputs; rates over the timed frames' graph phase)
        ctx.gvd_set_count_evals(True)
        ctx.seedgen(d_cloud.data_ptr(), n_points=n, on_device=True, want_host=False)
        ctx.gvd_set_markers(False)
        ctx.gvd_from_seedgen(copy=False)
        ev = ctx.gvd_evals()
        ctx.gvd_set_count_evals(False)
        t_graph = stage_p50.get("gvd_graph", 0.0)
        ref = ev["ref_nearest"] + ev["ref_pairs"] + ev["ref_labels"]
        gpu = ev["gpu_nearest"] + ev["gpu_pairs"] + ev["gpu_labels"]
        extra["gvd_evals"] = {
            **ev, "graph_ms_p50": t_graph,
            "ref_pair_evals_per_s": round(ref / (t_graph * 1e-3), 1) if t_graph > 0 else None,
            "gpu_pair_evals_per_s": round(gpu / (t_graph * 1e-3), 1) if t_graph > 0 else None,
            "gpu_samples_per_s": round(ev["gpu_samples"] / (t_graph * 1e-3), 1) if t_graph > 0 else None,
            "what": "the GVD graph phase's searches (g6 nearest boundary point per edge end, gvd:812-824; pairs "
                    "<= 0.5 m, gvd:861-894; occupancy samples, gvd:320-359; label points, gvd:686-790): ref_* = the "
                    "distance evaluations the reference makes on this frame, gpu_* = the candidates the kernels "
                    "examined (cell-index neighbourhoods); rates over the timed frames' graph phase (p50, all "
                    "of its kernels); per-kernel times in the committed kernel trace"}
    child = E.get("cpu_child") if (world == 1 and not quiet) else None
    if child is not None:
        # a sustained device-resident seed-gen leg (cloud in HBM, grids left there, no GVD) for a bounded time, THEN
        # the CPU baseline's frame in its child (pinned to its own core) while this process only waits: the
        # baseline is timed beside an idle parent (no GPU-driving threads competing with it)
        limit = a.sustain_s if a.sustain_s is not None else 20.0
        _progress(f"sustained device-resident seed-gen leg ({limit:.0f} s)")
        t_s0, s_frames, s_gpu = time.perf_counter(), 0, []
        while True:
            gs = ctx.seedgen(d_cloud.data_ptr(), n_points=n, on_device=True, want_host=False)
            s_frames += 1
            s_gpu.append(gs["ms"]["total"])
            if time.perf_counter() - t_s0 >= limit:
                break
        sync()
        el = time.perf_counter() - t_s0
        extra["sustained_seedgen"] = {
            "value": round(cells / 1e6 * s_frames / el, 3), "unit": "Mcells/s", "frames": s_frames,
            "seconds": round(el, 2), "gpu_stages_ms_p50": round(_median(s_gpu), 3),
            "what": "device-resident seed-gen frames (a1-a16, cloud in HBM, grids left in HBM, no GVD) back to back"}
        _progress(f"CPU baseline (oracle, child process pinned to core {child.core}; this process idle)")
        start_cpu_baseline(child)
    avg = stage

    # Roofline (SURVEY §8d algorithmic bytes, HBM-bound; no MFMA). Per frame B_alg = 12 N + C (6 + 4 T):
    # 12 B per input point to read the cloud once and C for the raster write (the ROR stage), 2 C
    # inflation, 2 C opening, 4 C T thinning, C labelling. The ROR stage (a1-a4) is the dominant GPU
    # stage and is reported as `roofline`: its §8d bytes 12 N + C over the device time of its launches
    # (count, tile scan, scatter, per-tile neighbour count), timed live with HIP events on the handle's
    # stream (aos_seedgen_out.ms_ror_*), averaged over the timed frames. `kernels` gives each launch's
    # time and the count pass's own figure (it is the one launch that reads the cloud: 12 N).
    # the points this frame's ROR partition passes read: a host cloud's split front (the points inside the binned
    # box: the upload keeps the others in host memory), a streaming append's scan, a tiled rank's shard
    # (averaged over the same timed frames as the stage times; a frame that skipped the stage read 0 points)
    n_all = ror_points_read(res, n)
    T = g["thin_iters"]
    t_cnt, t_scat, t_ror = avg["seedgen_ror_bin"], avg["seedgen_ror_scatter"], avg["seedgen_ror_count"]
    t_stage = avg.get("seedgen_ror_kernels", t_cnt + t_scat + t_ror)
    b_ror = 12.0 * n_all + cells
    ach = b_ror / (t_stage * 1e-3) / 1e9 if t_stage > 0 else 0.0
    traffic, src = (None, None) if (a.stream or a.tiled) else pmc_traffic(a.config)
    # (the count pass is two launches, k_rt_part<count> + k_rt_colscan, timed together by the events around
    # them; the count kernel's own duration is in the committed kernel trace, profiles/r04*_kt_summary.txt)
    kern = {"k_rt_part<count>+k_rt_colscan": {"ms": round(t_cnt, 4), "alg_bytes": 12.0 * n_all,
                                  "achieved_GBs": round(12.0 * n_all / (t_cnt * 1e-3) / 1e9, 1) if t_cnt > 0 else 0.0},
            "k_rt_part<scatter>": {"ms": round(t_scat, 4)}, "k_rt_ror": {"ms": round(t_ror, 4)}}
    kern["k_rt_part<count>+k_rt_colscan"]["frac"] = round(kern["k_rt_part<count>+k_rt_colscan"]["achieved_GBs"] / HBM_PEAK_GBS, 4)
    roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": "ROR stage a1-a4 (k_rt_part<count>, k_rt_colscan, k_rt_part<scatter>, k_rt_ror)",
            "alg_bytes_per_launch": b_ror,
            "alg_bytes_model": ("SURVEY §8d: 12 B per point the stage reads + 1 B per cell (raster); a host cloud's "
                                "upload sends only the points inside the binned box (units_per_launch of n_input)"),
            "ms_per_launch": round(t_stage, 4), "units_per_launch": n_all,
            "traffic_source": src if traffic is not None else
            f"no rocprofv3 --pmc run committed for config {a.config} / ROR design {ROR_DESIGN}",
            "kernels": kern,
            "readahead": "k_rt_touch reads the last frame's staged array (~90 MB at C2) while the cloud's upload DMAs "
                         "run, so the scatter's partial-line writes hit the Infinity Cache; it is not on the stage's "
                         "clock (the GPU idles during the upload) but its bytes are in `traffic`"}
    # thinning: 4 C T bytes over the thinning stage (opening + temporal blocks, one read-back)
    b_thin = 4.0 * cells * T
    t_thin = avg.get("seedgen_thin", 0.0)
    thin_roof = {"alg_bytes": b_thin, "ms": round(t_thin, 4),
                 "achieved_GBs": round(b_thin / (t_thin * 1e-3) / 1e9, 1) if t_thin > 0 else 0.0}
    thin_roof["frac"] = round(thin_roof["achieved_GBs"] / HBM_PEAK_GBS, 4)
    # the model above counts SURVEY §8d's 1 B per cell per sub-iteration; the bit-packed, temporally blocked kernel
    # moves far less: its measured HBM bytes (the committed PMC passes) over the same stage time
    t_pmc, t_src = (None, None) if (a.stream or a.tiled) else pmc_traffic(a.config, "k_thin_block")
    if t_pmc is not None:
        nl = g.get("thin_launches") or 0
        thin_roof.update({"what": "achieved/frac: SURVEY §8d's model bytes (4 C T) over the stage; hbm_*: the kernel's "
                                  "measured HBM bytes (FETCH x2 + WRITE, per launch x this frame's launches) over it; the "
                                  "kernel is LDS / VALU bound",
                          "hbm_bytes_per_frame": round(t_pmc * nl, 1), "launches": nl,
                          "hbm_GBs": round(t_pmc * nl / (t_thin * 1e-3) / 1e9, 1) if t_thin > 0 else None,
                          "hbm_source": t_src})
    # BASELINE.md:35-37 frame-level figure: B_alg = 12 N + C (6 + 4 T) over the per-frame wall-clock
    b_frame = 12.0 * float(n) + cells * (6.0 + 4.0 * T)   # (every input point is read once on the host)
    t_frame = med if not main_pipe else (_median(frame_lat) * 1e-3 if frame_lat else med)
    frame_roof = {"alg_bytes": b_frame, "frame_ms": round(t_frame * 1e3, 3),
                  "achieved_GBs": round(b_frame / t_frame / 1e9, 2),
                  "frac": round(b_frame / t_frame / 1e9 / HBM_PEAK_GBS, 5),
                  "note": "whole frame (median per-frame wall-clock) incl. PCIe and the host Subdiv2D replay"}

    # how much of the headline frame the GPU works (verdict r05 weak 3): the frame's GPU stage spans (HIP events on
    # the handle's streams: seed-gen a1-a16 incl. the cluster stage's short host waits, the GVD's merge and graph
    # phases; not the host Subdiv2D replay between them), and the committed kernel trace's kernel time per frame
    gpu_spans = sum(stage_p50.get(k, 0.0) for k in ("seedgen_total", "gvd_merge", "gvd_graph"))
    kt_ms, kt_src = kt_kernel_ms(a.config) if not (a.stream or a.tiled or main_pipe) else (None, None)
    f_ms = _median(frame_lat) if frame_lat else med * 1e3
    gpu_util = {"gpu_stage_ms_per_frame": round(gpu_spans, 3), "frame_ms_p50": round(f_ms, 3),
                "gpu_stage_frac": round(gpu_spans / f_ms, 4) if f_ms > 0 else None,
                "gpu_kernel_ms_per_frame": round(kt_ms, 3) if kt_ms is not None else None,
                "gpu_kernel_frac": round(kt_ms / f_ms, 4) if kt_ms is not None and f_ms > 0 else None,
                "kernel_source": kt_src,
                "what": "stage spans: HIP-event device time of seed-gen (a1-a16) + the GVD merge and graph phases per "
                        "frame (p50); kernel ms: the median frame of the committed rocprofv3 kernel trace (sum of its "
                        "kernel durations); the rest of the frame is the host Subdiv2D replay, upload and read-backs"}

    if rank == 0:
        if a.stream and a.tiled:
            workload = (f"C4 on {world} GPU(s): 1 M-point scans at {orchard.SCAN_HZ:g} Hz appended to the {a.config} map, "
                        f"one map in {tx}x{ty} tiles (each rank keeps its tile's points box), {g['width']}x{g['height']} "
                        f"cells @ {cfg.res} m, full seed-gen + GVD per scan, root rotating")
        elif a.stream:
            workload = (f"C4: 1 M-point scans at {orchard.SCAN_HZ:g} Hz appended to the device-resident {a.config} map "
                        f"({n} pts at start, {g['n_input']} after the last step), {g['width']}x{g['height']} cells "
                        f"@ {cfg.res} m, full seed-gen + GVD of the whole map per scan")
        elif a.tiled:
            workload = (f"{a.config}: {cfg.n_points} pts, {g['width']}x{g['height']} cells @ {cfg.res} m, one map in "
                        f"{tx}x{ty} tiles (rank 0 holds {n} pts), halo all-gathers, "
                        + (f"frame k finished (a6, a8-a16, GVD) by rank k mod {world}" if rotate else "GVD on rank 0"))
        else:
            workload = (f"{a.config}: {n} pts, {g['width']}x{g['height']} cells @ {cfg.res} m, "
                        f"full seed-gen + GVD per frame, one independent map per GPU")
        out = {
            "metric": "Mcells/s skeleton+GVD (seed-gen + GVD frame) on 4096^2 grid",
            "value": round(value, 3), "unit": "Mcells/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(dt / len(res) * 1e3, 3), "higher_is_better": True,
            "value_definition": ("frames x W.H / timed region (pipelined)" if main_pipe else
                                 "W.H / median per-frame wall-clock of the sequential loop (BASELINE.md:32)"),
            "frame_ms": {"p50": round(_median(frame_lat), 2), "min": round(frame_lat[0], 2),
                         "max": round(frame_lat[-1], 2), "mean": round(sum(frame_lat) / len(frame_lat), 2)}
            if frame_lat else None,
            "value_mean": round(value_mean, 3), "step_median_ms": round(med * 1e3, 3),
            "scaling": "strong" if a.tiled else "weak",
            "vs_baseline": None, "dtype": "f32/f64 (reference float/double arithmetic), u8/bit grids",
            "data": ("synthetic orchard (tools/orchard_gen.c, SplitMix64; 1 % in-clip outliers, not SURVEY §8d's 10 %, "
                     "which bridge every row at 0.1 m: DESIGN.md §8), "
                     + ("PointCloud2 bytes in host memory" if host_io else
                        "scans from host memory into the HBM-resident map" if a.stream else
                        "HBM-resident PointCloud2 shards" if a.tiled else "HBM-resident PointCloud2")),
            "config": {"workload": workload, "global_batch": 1 if a.tiled else world,
                       "parallelism": f"tiled{tx}x{ty}" if a.tiled else f"maps{world}"},
            "io": "host PointCloud2 in, host OccupancyGrids + GvdGraph out (SURVEY §8d)" if host_io else
                  "device-resident cloud, device-resident grids, host GvdGraph",
            **extra,
            "markers": {"policy": "every frame" if a.markers_every_frame else
                        f"the frames the node publishes: at most max_graph_publish_rate = {params.max_graph_publish_rate:g} Hz "
                        f"of wall time (gvd:306-314); every frame's graph is built and returned",
                        "timed_frames_with_markers": mk_frames,
                        "returned_as": "copies" if a.markers_copy else "views of the library-owned arrays (ABI ownership rule)"},
            "stages_ms": {k: round(v, 3) for k, v in avg.items()},
            # (medians: a frame in which the host was held, e.g. 3-7 ms inside hipMemcpyAsync of the grids,
            # moves a stage's mean by ~0.5 ms over 12-20 frames)
            "stages_ms_p50": stage_p50,
            "frame": {"T": T, "rows": len(g.get("row_length", ())), "seeds": len(g.get("voronoi_seeds", ())),
                      "nodes": len(gg["nodes"]) if gg else 0, "edges": len(gg["edges"]) if gg else 0,
                      "n_binned": g.get("n_binned"), "n_clipped": g.get("n_clipped"),
                      # the last frame's exact BFS replays (clusters without the order-free certificate) by where they ran
                      "bfs_replays": None if a.tiled else ctx.replay_counts()},
            "gpu_utilisation": gpu_util,
            "roofline": roof,
            "thin_roofline": thin_roof,
            "frame_roofline": frame_roof,
        }
        if a.stream and a.tiled:
            out["stream"] = {"scan_latency_ms_p50": round(_median(frame_lat), 2), "scan_latency_ms_max": round(frame_lat[-1], 2),
                             "scan_latency_ms": [round(x * 1e3, 1) for x in root_lat],
                             "step_ms_max_over_ranks": [round(x * 1e3, 1) for x in per],
                             "budget_ms": 1e3 / orchard.SCAN_HZ,
                             "keeps_up": frame_lat[-1] <= 1e3 / orchard.SCAN_HZ,
                             "map_points": g["n_input"],
                             "note": f"C4 over {world} rank(s) in {tx}x{ty} tiles: every rank appends each whole scan "
                                     f"to its tile's points box (aos_tiled_map_append); frame k's root (rank k mod "
                                     f"{world}) finishes it and builds the GvdGraph; scan latency = the root's wall-clock "
                                     f"from its append call to the GvdGraph; value = W.H / the median step (max over ranks)"}
        elif a.stream:
            lat = sorted(x * 1e3 for x in latency[a.warmup:])
            mlat = sorted(x * 1e3 for x in mk_latency[a.warmup:]) or [0.0]
            out["stream"] = {"scan_latency_ms_p50": round(_median(lat), 2), "scan_latency_ms_max": round(lat[-1], 2),
                             "markers_latency_ms_p50": round(_median(mlat), 2),
                             "markers_latency_ms_max": round(mlat[-1], 2),
                             "scan_latency_ms": [round(x * 1e3, 1) for x in latency[a.warmup:]],
                             "scan_markers": [int(bool(pend["mk"].get(k))) for k in range(a.warmup, a.warmup + a.steps)],
                             "scan_delaunay_ms": [round(gs[1]["ms"].get("delaunay", 0.0), 1) for gs in res],
                             "scan_thin_iters": [gs[0]["thin_iters"] for gs in res],
                             "budget_ms": 1e3 / orchard.SCAN_HZ,
                             "keeps_up": max(lat[-1], dt / len(res) * 1e3) <= 1e3 / orchard.SCAN_HZ,
                             "note": "scan latency = scan H2D + pack + whole-map seed-gen + GVD graph (host clock); "
                                     "markers latency = until that scan's /gvd/markers cells are collected; "
                                     "keeps_up: graph latency and time per scan (markers included) within the budget"}
        if a.tiled:
            roots = [gs for gs, _ in res if gs.get("root")]
            if roots:
                out["root_serial_ms"] = round(sum(gs["ms"].get("cluster", 0.0) + gs["ms"].get("seeds", 0.0)
                                                  for gs in roots) / len(roots), 3)
            if tiled_ranks is not None:
                out["per_rank"] = tiled_ranks
                out["root_serial_split_ms"] = tiled_split
            if frame_lat:
                out["frame_latency_ms"] = {"p50": round(_median(frame_lat), 2), "max": round(frame_lat[-1], 2)}
        if child is not None:
            out["cpu_baseline"] = finish_cpu_baseline(child)
        elif world == 1 and not a.no_cpu_baseline and not a.stream:
            _progress(f"CPU baseline (oracle, 1 thread pinned) on {a.cpu_config}")
            out["cpu_baseline"] = cpu_baseline(a.cpu_config)
    ctx.close()
    if a.tiled and hasattr(comm, "close"):
        comm.close()
    return out if rank == 0 else None


if __name__ == "__main__":
    main()
