"""The 48 largest 8-connected clusters of the oracle's C1 skeleton (tools/sdcheck/bfsbench_real.cpp's input): cell ids
in shuffled order, as int32 (W, H, count, then per cluster its size and cells). usage: dump_clusters.py OUT"""
import sys
sys.path[:0] = ["oracle", "tools", "tests"]
import numpy as np
import oracle_py as O, orchard
from scipy import ndimage
cfg = orchard.CONFIGS["C1"]
cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
o = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res))
sk = o["skeleton"] != 0
H, W = sk.shape
lab, n = ndimage.label(sk, structure=np.ones((3, 3)))
sizes = ndimage.sum(sk, lab, range(1, n + 1))
big = [L + 1 for L in np.argsort(-sizes)[:48]]
out = []
for L in big:
    ys, xs = np.nonzero(lab == L)
    cells = (ys * W + xs).astype(np.int32)
    np.random.default_rng(L).shuffle(cells)
    out.append(cells)
with open(sys.argv[1], "wb") as f:
    np.array([W, H, len(out)], np.int32).tofile(f)
    for c in out:
        np.array([len(c)], np.int32).tofile(f); c.tofile(f)
print(W, H, len(out), sum(map(len, out)))
