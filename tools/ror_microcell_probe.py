"""How many ROR candidates the verdict's dense micro-cell shortcut would decide: the C2 cloud's points
inside the clip box, binned into 3-D micro-cells of side s (s = r / sqrt(3) and finer, so any two points of one cell are
within r); a candidate whose micro-cell holds >= need = min_neighbors + 1 = 3 points is kept without a neighbour walk.
usage: python tools/ror_microcell_probe.py [CONFIG]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import orchard  # noqa: E402

cfg = orchard.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C2"]
xyz = orchard.xyz(orchard.generate(cfg)).astype(np.float64)
poly = orchard.polygon(cfg)
inside = ((xyz[:, 2] >= -0.4) & (xyz[:, 2] <= 0.5) & (xyz[:, 0] >= poly[:, 0].min()) & (xyz[:, 0] <= poly[:, 0].max())
          & (xyz[:, 1] >= poly[:, 1].min()) & (xyz[:, 1] <= poly[:, 1].max()))
p = xyz[inside]
print(cfg.name, "candidates (clip box)", len(p))
for s in (0.2 / np.sqrt(3) * 0.999, 0.1, 0.08):
    k = np.floor(p / s).astype(np.int64)
    key = (k[:, 0] * 100003 + k[:, 1]) * 1000 + k[:, 2]
    _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    print(f"micro-cell side {s:.4f} m: {(cnt[inv] >= 3).mean():.3f} of the candidates decided; "
          f"{cnt.mean():.2f} points per occupied micro-cell")
