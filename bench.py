#!/usr/bin/env python3
"""bench.py — Mcells/s of the AOS seed-gen + GVD hot path on MI355X (BASELINE.json metric).

One step = one full frame of the path on one GPU: PointCloud2 (already resident in HBM) ->
ROR / clip / raster -> inflation -> opening + Zhang-Suen -> clusters / tree rows / seeds ->
GVD graph (seed merge, Delaunay replay, boundary points, edges, labels) -> host GvdGraph +
seeds/rows arrays; the OccupancyGrid outputs stay device-resident (their D2H is PCIe, see DESIGN).
Workload: config C2 (10 M points, 4096^2 cells @ 0.1 m, BASELINE.json configs[2]).

Multi-GPU (--gpus N, launched by torch.distributed.run): weak scaling — every rank processes its
own independent 4096^2 map tile (scene seed 3 + rank); no data-path collective; the barrier and
the max-over-ranks time use torch.distributed.
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

import torch  # noqa: E402  (import before libaos_gpu: shared HIP runtime, see aos_gpu.lib)
import torch.distributed as dist  # noqa: E402

import aos_gpu  # noqa: E402
import orchard  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-config", default="C1")
    return ap.parse_args()


def cpu_baseline(cfg_name: str) -> dict:
    """The oracle (single-threaded CPU restatement of the reference path) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_py as O
    cfg = orchard.CONFIGS[cfg_name]
    cloud = orchard.generate(cfg)
    poly = orchard.polygon(cfg)
    p = O.default_params(grid_resolution=cfg.res, faithful_dead_work=1)
    t0 = time.perf_counter()
    r = O.seedgen(cloud, poly, p)
    t1 = time.perf_counter()
    O.gvd(r["voronoi_seeds"], r["rows_info"], r, p)
    t2 = time.perf_counter()
    cells = r["width"] * r["height"]
    return {"value": cells / (t2 - t0) / 1e6, "unit": "Mcells/s", "cores": 1, "kind": "port",
            "sample": f"oracle/ CPU restatement, 1 thread, one full frame of config {cfg_name} "
                      f"({cfg.n_points} pts, {r['width']}x{r['height']} cells): seed-gen {t1 - t0:.2f} s + "
                      f"GVD {t2 - t1:.2f} s (incl. the reference's never-read vertex dedup); the CPU GVD is "
                      f"super-linear, so this over-states the CPU rate at the 4096^2 bench size",
            "cpu": _cpu_model()}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    cfg = orchard.CONFIGS[a.config]
    cloud = orchard.generate(cfg, seed=cfg.seed + rank)
    poly = orchard.polygon(cfg)
    d_cloud = torch.from_numpy(cloud).to(f"cuda:{local}")
    n = cloud.shape[0]
    ctx = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res), device=local)
    ctx.set_polygon(poly)

    def step():
        g = ctx.seedgen(d_cloud.data_ptr(), n_points=n, on_device=True, want_host=False)
        gg = ctx.gvd_from_seedgen()
        return g, gg

    for _ in range(a.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stage = {}
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g, gg = step()
        for k, v in g["ms"].items():
            stage["seedgen_" + k] = stage.get("seedgen_" + k, 0.0) + v
        for k, v in gg["ms"].items():
            stage["gvd_" + k] = stage.get("gvd_" + k, 0.0) + v
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    cells = g["width"] * g["height"]
    value = cells * world * a.steps / dt / 1e6
    avg = {k: v / a.steps for k, v in stage.items()}

    # roofline of the dominant kernel group, timed live with HIP events on the handle's stream
    # (aos_seedgen_out.ms_*): Zhang-Suen thinning, algorithmic bytes (SURVEY §8d, 1 B/cell):
    # 2 sub-iterations x (read + write) per iteration = 4 * C * T bytes per frame.
    T = g["thin_iters"]
    alg_bytes = 4.0 * cells * T
    thin_ms = avg["seedgen_thin"]
    achieved = alg_bytes / (thin_ms * 1e-3) / 1e9
    roof = {"bound": "hbm", "kernel": "k_open + k_thin_block (Zhang-Suen, T iterations)", "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "alg_bytes_per_frame": alg_bytes, "ms_per_frame": round(thin_ms, 4), "T": T}

    if rank == 0:
        out = {
            "metric": "Mcells/s skeleton+GVD (seed-gen + GVD frame) on 4096^2 grid",
            "value": round(value, 3), "unit": "Mcells/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32/f64 (reference float/double arithmetic), u8/bit grids",
            "data": "synthetic orchard (tools/orchard_gen.c, SplitMix64), device-resident PointCloud2",
            "config": {"workload": f"{a.config}: {n} pts, {g['width']}x{g['height']} cells @ {cfg.res} m, "
                                   f"full seed-gen + GVD per frame, one independent tile per GPU",
                       "global_batch": world, "parallelism": f"tiles{world}"},
            "stages_ms": {k: round(v, 3) for k, v in avg.items()},
            "frame": {"T": T, "rows": len(g["row_length"]), "seeds": len(g["voronoi_seeds"]),
                      "nodes": len(gg["nodes"]), "edges": len(gg["edges"])},
            "roofline": roof,
        }
        if world == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(a.cpu_config)
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
