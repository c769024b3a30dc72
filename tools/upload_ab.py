"""Seed-gen wall time with host PointCloud2 input (upload included) for the current AOS_UP_THREADS,
C2 cloud, grids to host (diagnostics for the uploader's thread count; bench.py is the contract).
Prints the median over --reps frames of the whole aos_seedgen_process call and its device stages."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "active-orchard-slam_amd")]

import aos_gpu  # noqa: E402
import orchard  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--reps", type=int, default=15)
    args = ap.parse_args()
    cfg = orchard.CONFIGS[args.config]
    cloud = orchard.generate(cfg)
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(orchard.polygon(cfg))
    wall, dev = [], []
    for r in range(args.reps + 3):
        t0 = time.perf_counter()
        g = c.seedgen(cloud, want_host=True, copy_grids=False)
        t1 = time.perf_counter()
        if r >= 3:
            wall.append((t1 - t0) * 1e3)
            dev.append(g["ms"]["total"])
    wall.sort()
    dev.sort()
    print(json.dumps({"up_threads": os.environ.get("AOS_UP_THREADS", "default"), "seedgen_wall_ms_p50": round(wall[len(wall) // 2], 3),
                      "min": round(wall[0], 3), "device_ms_p50": round(dev[len(dev) // 2], 3)}), flush=True)
    c.close()


if __name__ == "__main__":
    main()
