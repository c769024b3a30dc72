"""Independent pin of the oracle's a8-a9 cluster stage (clusterOccupiedCells seed_gen:970-1083 +
isPointInPolygon :1231-1255; SURVEY §8c suggests scipy's 8-connected labelling): on a C0 frame the oracle's
clusters must be the 8-connected components of (frameless skeleton ∩ polygon) from scipy.ndimage.label,
numbered in raster order of their first cell (the reference's discovery order); each cluster's cells must be
in the FIFO-BFS order of a separate Python BFS with the reference's neighbour order, its centre the float32
sum in that order divided by n, and its length float(sqrt(double(max pairwise d^2)) * res). The reference
ships no fixtures for this path, so this and test_oracle_grid.py are the oracle's pins."""
from collections import deque

import numpy as np
from scipy import ndimage

import oracle_py as O
import orchard

NB = ((-1, -1), (-1, 0), (-1, 1), (0, -1), (0, 1), (1, -1), (1, 0), (1, 1))   # (dx, dy), seed_gen:986-987


def inside(px: float, py: float, poly: np.ndarray) -> bool:
    """isPointInPolygon: even-odd ray test in double, horizontal edges (|dy| <= 1e-9) skipped."""
    n, c, j = len(poly), False, len(poly) - 1
    for i in range(n):
        xi, yi, xj, yj = poly[i][0], poly[i][1], poly[j][0], poly[j][1]
        dy = yj - yi
        if abs(dy) > 1e-9 and ((yi > py) != (yj > py)) and px < (xj - xi) * (py - yi) / dy + xi:
            c = not c
        j = i
    return c


def test_oracle_clusters_match_independent_labelling_and_bfs():
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg)
    poly = orchard.polygon(cfg).astype(np.float64)
    r = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res))
    sk = r["skeleton"] == 100
    H, W = sk.shape
    ox, oy = r["origin"]
    res = np.float32(r["resolution"])
    # world point of a cell: origin + float(i) * res (float product, double add), stored as float
    wx = (ox + (np.arange(W, dtype=np.float32) * res).astype(np.float64)).astype(np.float32).astype(np.float64)
    wy = (oy + (np.arange(H, dtype=np.float32) * res).astype(np.float64)).astype(np.float32).astype(np.float64)
    ys, xs = np.nonzero(sk)
    fg = np.zeros_like(sk)
    for y, x in zip(ys, xs):
        fg[y, x] = inside(wx[x], wy[y], poly)
    lab, n = ndimage.label(fg, structure=np.ones((3, 3), bool))
    off = r["cluster_offsets"]
    assert n == len(off) - 1 and n > 0
    # raster order of first cells (row-major: y outer, x inner) = discovery order
    first = ndimage.minimum(np.arange(H * W).reshape(H, W), lab, index=np.arange(1, n + 1)).astype(np.int64)
    order = np.argsort(first, kind="stable") + 1
    cells = r["cluster_cells"]
    for k, comp in enumerate(order):
        ref_cells = cells[off[k]:off[k + 1]]                        # (x, y) in the oracle's BFS order
        cy, cx = np.nonzero(lab == comp)
        assert len(ref_cells) == len(cx)
        assert set(map(tuple, ref_cells.tolist())) == set(zip(cx.tolist(), cy.tolist()))
        # FIFO BFS from the first raster cell with the reference's neighbour order
        s = int(first[comp - 1])
        start = (s % W, s // W)
        seen, q, bfs = {start}, deque([start]), []
        while q:
            x, y = q.popleft()
            bfs.append((x, y))
            for dx, dy in NB:
                nx, ny = x + dx, y + dy
                if 0 <= nx < W and 0 <= ny < H and lab[ny, nx] == comp and (nx, ny) not in seen:
                    seen.add((nx, ny))
                    q.append((nx, ny))
        assert bfs == list(map(tuple, ref_cells.tolist())), k
        sx = sy = np.float32(0)
        for x, y in bfs:   # float sums in BFS order
            sx = np.float32(sx + np.float32(x))
            sy = np.float32(sy + np.float32(y))
        cnt = np.float32(len(bfs))
        np.testing.assert_array_equal(r["cluster_center"][k], np.array([sx / cnt, sy / cnt], np.float32))
        pts = np.array(bfs, np.int64)
        d2 = ((pts[:, None, :] - pts[None, :, :]) ** 2).sum(-1).max()
        assert r["cluster_length"][k] == np.float32(np.float32(np.sqrt(np.float64(d2))) * res)


def test_oracle_tree_rows_match_independent_restatement():
    """convertClustersToTreeRows (seed_gen:1309-1406) restated independently on the oracle's own clusters:
    the length filter (>= cluster_min_length, float), the centre-in-polygon filter, start = the first cell
    with a strictly larger squared distance from the centre, end = the first strictly farthest cell with a
    negative dot(normalized diff, first direction), else the farthest from the start (Eigen: normalized() =
    v / sqrt(x*x + y*y), all in double from float world points)."""
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg)
    poly = orchard.polygon(cfg).astype(np.float64)
    p = O.default_params(grid_resolution=cfg.res)
    r = O.seedgen(cloud, poly, p)
    ox, oy = r["origin"]
    res = np.float32(r["resolution"])
    off, cells = r["cluster_offsets"], r["cluster_cells"]

    def norm(v):
        z = v[0] * v[0] + v[1] * v[1]
        return (v[0] / np.sqrt(z), v[1] / np.sqrt(z)) if z > 0 else v

    rows = []
    for k in range(len(off) - 1):
        if not r["cluster_length"][k] >= np.float32(p.cluster_min_length):
            continue
        cxf, cyf = r["cluster_center"][k]
        center = (float(np.float32(ox + float(np.float32(cxf * res)))), float(np.float32(oy + float(np.float32(cyf * res)))))
        if not inside(center[0], center[1], poly):
            continue
        wp = [(float(np.float32(ox + float(np.float32(np.float32(x) * res)))),
               float(np.float32(oy + float(np.float32(np.float32(y) * res))))) for x, y in cells[off[k]:off[k + 1]]]
        best, first, fdir = 0.0, 0, (0.0, 0.0)
        for i, (x, y) in enumerate(wp):
            d = (x - center[0], y - center[1])
            d2 = d[0] * d[0] + d[1] * d[1]
            if d2 > best:
                best, first, fdir = d2, i, norm(d)
        best2, second = 0.0, 0
        for i, (x, y) in enumerate(wp):
            if i == first:
                continue
            d = (x - center[0], y - center[1])
            d2 = d[0] * d[0] + d[1] * d[1]
            nd = norm(d)
            if nd[0] * fdir[0] + nd[1] * fdir[1] < 0.0 and d2 > best2:
                best2, second = d2, i
        if best2 == 0.0:
            for i, (x, y) in enumerate(wp):
                if i == first:
                    continue
                d = (x - wp[first][0], y - wp[first][1])
                d2 = d[0] * d[0] + d[1] * d[1]
                if d2 > best2:
                    best2, second = d2, i
        rows.append((center, wp[first], wp[second], float(r["cluster_length"][k])))
    assert len(rows) == len(r["row_length"]) > 0
    for i, (c, s, e, ln) in enumerate(rows):
        assert tuple(r["row_center"][i]) == c and tuple(r["row_start"][i]) == s and tuple(r["row_end"][i]) == e, i
        assert r["row_length"][i] == ln
