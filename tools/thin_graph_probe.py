"""Diagnosis of round 2's hipGraph thinning failure (commit d6ea4a7, tools/dbg_stream7.py).

Replays round 2's failing frame sequence — the C2 map, then the map plus 1 M-point scans, each frame
reprocessed whole (device-resident cloud, and host cloud) — on one handle per graph shape of the first
thinning batch (AOS_THIN_GRAPH, seedgen.hip thin_first_batch):
  0 plain launches (reference), 1 kernels only (clearing kernel, flags read back outside the graph),
  2 round 1's shape (memset node + kernels + D2H copy node), 3 memset node + kernels,
  4 clearing kernel + kernels + D2H copy node,
with AOS_THIN_GRAPH_CHECK=1 (the library compares the host flags with a fresh device read after every
read-back and reports to stderr). Prints per shape the T sequence, whether every frame's grids equal
shape 0's, and the graph use per frame. usage: python tools/thin_graph_probe.py [n_scans]
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "active-orchard-slam_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import aos_gpu  # noqa: E402
import orchard  # noqa: E402


def h(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def run(shape, n_scans, host):
    os.environ["AOS_THIN_GRAPH"] = str(shape)
    os.environ["AOS_THIN_GRAPH_CHECK"] = "1"
    cfg = orchard.CONFIGS["C2"]
    ctx = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ctx.set_polygon(orchard.polygon(cfg))
    full = torch.from_numpy(orchard.generate(cfg)).to("cuda:0")
    rows = []
    for k in range(n_scans + 1):
        if k:
            full = torch.cat([full, torch.from_numpy(orchard.generate_scan(cfg, 40 * (k - 1))).to("cuda:0")])
        torch.cuda.synchronize()
        if host:
            g = ctx.seedgen(full.cpu().numpy())
        else:
            g = ctx.seedgen(full.data_ptr(), n_points=full.shape[0], on_device=True)
            g["occupancy"], g["skeleton_framed"] = ctx.grids_copy((g["height"], g["width"]))
        rows.append({"T": g["thin_iters"], "graph": g["thin_graph"], "launches": g["thin_launches"],
                     "occ": h(g["occupancy"]), "skel": h(g["skeleton_framed"])})
    ctx.close()
    return rows


def main():
    n_scans = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    out = {}
    for host in (False, True):
        ref = None
        for shape in (0, 1, 2, 3, 4):
            try:
                rows = run(shape, n_scans, host)
            except RuntimeError as e:   # the failing shapes run the thinning to its iteration cap
                key = f"{'host' if host else 'device'}_shape{shape}"
                out[key] = {"error": str(e), "equal_to_plain": [False]}
                print(key, json.dumps(out[key]), flush=True)
                continue
            if shape == 0:
                ref = rows
            same = [r["T"] == q["T"] and r["occ"] == q["occ"] and r["skel"] == q["skel"] for r, q in zip(rows, ref)]
            key = f"{'host' if host else 'device'}_shape{shape}"
            out[key] = {"T": [r["T"] for r in rows], "graph": [r["graph"] for r in rows],
                        "launches": [r["launches"] for r in rows], "equal_to_plain": same}
            print(key, json.dumps(out[key]), flush=True)
    print(json.dumps({"summary": {k: all(v["equal_to_plain"]) for k, v in out.items()}}), flush=True)


if __name__ == "__main__":
    main()
