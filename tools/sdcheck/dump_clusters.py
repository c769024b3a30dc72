"""The largest 8-connected clusters of a skeleton (tools/sdcheck/bfsbench_real.cpp's input): cell ids in shuffled
order, as int32 (W, H, count, then per cluster its size and cells). Default: the 48 largest of the oracle's C1
skeleton (CPU). --gpu CONFIG: the frameless skeleton of the GPU frame of that config (needs a GPU), every cluster of
at least 1000 cells (C3: the 215 row clusters the frame replays).
usage: dump_clusters.py OUT [--gpu CONFIG]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in ("oracle", "tools", "tests", "active-orchard-slam_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402
from scipy import ndimage  # noqa: E402

import orchard  # noqa: E402

if len(sys.argv) > 3 and sys.argv[2] == "--gpu":
    import aos_gpu
    cfg = orchard.CONFIGS[sys.argv[3]]
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(orchard.polygon(cfg))
    g = c.seedgen(orchard.generate(cfg))
    sk = c.debug_grid("skeleton_frameless", (g["height"], g["width"])) != 0
    c.close()
    min_n, top = 1000, None
else:
    import oracle_py as O
    cfg = orchard.CONFIGS["C1"]
    o = O.seedgen(orchard.generate(cfg), orchard.polygon(cfg), O.default_params(grid_resolution=cfg.res))
    sk = o["skeleton"] != 0
    min_n, top = 0, 48
H, W = sk.shape
lab, n = ndimage.label(sk, structure=np.ones((3, 3)))
sizes = ndimage.sum(sk, lab, range(1, n + 1))
order = np.argsort(-sizes)
big = [int(L) + 1 for L in (order[:top] if top else order[sizes[order] >= min_n])]
boxes = ndimage.find_objects(lab)
out = []
for L in big:
    sl = boxes[L - 1]
    ys, xs = np.nonzero(lab[sl] == L)
    cells = ((ys + sl[0].start).astype(np.int64) * W + xs + sl[1].start).astype(np.int32)
    np.random.default_rng(L).shuffle(cells)
    out.append(cells)
with open(sys.argv[1], "wb") as f:
    np.array([W, H, len(out)], np.int32).tofile(f)
    for cl in out:
        np.array([len(cl)], np.int32).tofile(f)
        cl.tofile(f)
print(W, H, len(out), sum(map(len, out)))
