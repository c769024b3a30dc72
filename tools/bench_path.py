"""Planning latency over the GvdGraph (aos_path_plan) at a bench config.

Runs one seed-gen + GVD frame on the GPU, then plans to every waypoint of the sequence from the
previous one (the node's steady state) through aos_path_plan, and times the oracle restatement of
aos_path_gen_node (the reference's O(E) edge scan per A* relaxation) on a bounded sample of the same
queries, checking each sampled plan for bit-exact equality. Prints one JSON line.

    python tools/bench_path.py [--config C2] [--oracle-queries 12]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("tools", "oracle", "active-orchard-slam_amd"):
    sys.path.insert(0, os.path.join(ROOT, sub))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--oracle-queries", type=int, default=12)
    a = ap.parse_args()
    import torch  # noqa: F401  (shared HIP runtime first)
    import numpy as np

    import aos_gpu
    import oracle_py as O
    import orchard

    cfg = orchard.CONFIGS[a.config]
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(orchard.polygon(cfg))
    f = c.seedgen(orchard.generate(cfg))
    gg = c.gvd_from_seedgen()
    grid = {"origin": f["origin"], "resolution": f["resolution"], "width": f["width"], "height": f["height"],
            "skeleton_framed": f["skeleton_framed"]}
    first = c.path_plan(aos_gpu.path_query(target=0))
    n_wp = len(first["waypoints"])
    qs = [dict(target=t, previous=t - 1) for t in range(n_wp)]
    ms, poses, ok = [], 0, 0
    for kw in qs:
        t0 = time.perf_counter()
        r = c.path_plan(aos_gpu.path_query(**kw))
        ms.append((time.perf_counter() - t0) * 1e3)
        poses += len(r["poses"])
        ok += r["status"]
    step = max(1, n_wp // max(1, a.oracle_queries))
    sample = qs[::step][: a.oracle_queries]
    oms, equal = [], 0
    keys = ("status", "target", "waypoint_nodes", "node_path", "poses", "trimmed_from")
    for kw in sample:
        t0 = time.perf_counter()
        ro = O.path_plan(gg, grid, **kw)
        oms.append((time.perf_counter() - t0) * 1e3)
        rg = c.path_plan(aos_gpu.path_query(**kw))
        equal += all(np.array_equal(rg[k], ro[k]) if isinstance(ro[k], np.ndarray) else rg[k] == ro[k] for k in keys)
    ms_s = sorted(ms)
    out = {"metric": "ms per waypoint plan (graphCallback + planAndPublishPath)", "config": a.config,
           "nodes": len(gg["nodes"]), "edges": len(gg["edges"]), "waypoints": n_wp, "plans_ok": ok,
           "poses_total": poses, "ms_p50": round(ms_s[len(ms_s) // 2], 3), "ms_max": round(ms_s[-1], 3),
           "ms_mean": round(sum(ms) / len(ms), 3),
           "oracle": {"queries": len(sample), "ms_mean": round(sum(oms) / len(oms), 2),
                      "ms_max": round(max(oms), 2), "bit_exact": f"{equal}/{len(sample)}",
                      "note": "CPU restatement, 1 thread, the reference's O(E) edge scan per A* relaxation"},
           "speedup_mean": round((sum(oms) / len(oms)) / (sum(ms[i] for i in range(0, len(ms), step)[: len(sample)])
                                                         / len(sample)), 1)}
    print(json.dumps(out), flush=True)
    c.close()
    if equal != len(sample):
        sys.exit(1)


if __name__ == "__main__":
    main()
