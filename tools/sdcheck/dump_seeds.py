"""The GPU seed-gen frame's /voronoi_seeds of a config (the Subdiv2D replay's input before the 0.5 m merge) in
sdcheck / sdprof's seed-file format (int n, n double pairs, 4 double bounds: min x, max x, min y, max y), for
replay timing at other scales than the committed c2_seeds.bin. usage: dump_seeds.py CONFIG OUT (needs a GPU)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "tools"), os.path.join(ROOT, "active-orchard-slam_amd")):
    sys.path.insert(0, p)
import aos_gpu  # noqa: E402
import orchard  # noqa: E402

cfg = orchard.CONFIGS[sys.argv[1]]
c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
c.set_polygon(orchard.polygon(cfg))
g = c.seedgen(orchard.generate(cfg))
s = np.asarray(g["voronoi_seeds"], np.float64).reshape(-1, 2)
s = s[np.isfinite(s).all(axis=1)]
c.close()
with open(sys.argv[2], "wb") as f:
    np.array([len(s)], np.int32).tofile(f)
    s.reshape(-1).tofile(f)
    np.array([s[:, 0].min(), s[:, 0].max(), s[:, 1].min(), s[:, 1].max()], np.float64).tofile(f)
print(sys.argv[1], len(s), "seeds")
