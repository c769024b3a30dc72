"""Diagnostics: GPU raster vs oracle raster on one config (cells only in one of them)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("tools", "oracle", "active-orchard-slam_amd")]
import numpy as np
import aos_gpu, orchard, oracle_py as O
name = sys.argv[1] if len(sys.argv) > 1 else "C0"
cfg = orchard.CONFIGS[name]
cloud = orchard.generate(cfg); poly = orchard.polygon(cfg)
c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res)); c.set_polygon(poly)
g = c.seedgen(cloud)
o = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res))
r = c.debug_grid("raster", (g["height"], g["width"])) == 100
ro = np.asarray(o["raster"]).reshape(g["height"], g["width"]) != 0
print("n_binned", g["n_binned"], "n_clipped", g["n_clipped"], "oracle keys", [k for k in o if k.startswith("n_")])
for k in o:
    if k.startswith("n_"): print(" oracle", k, o[k])
print("gpu cells", r.sum(), "oracle cells", ro.sum(), "gpu-only", (r & ~ro).sum(), "oracle-only", (ro & ~r).sum())
ys, xs = np.nonzero(r ^ ro)
print("first diffs (y,x):", list(zip(ys[:20].tolist(), xs[:20].tolist())))
