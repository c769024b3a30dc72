"""Independent pins of the oracle's GVD front (the reference ships no fixtures for this path): on a C0 frame
the oracle's merged seeds must equal a separate Python restatement of voronoiSeedsCallback (gvd:84-128:
greedy, non-transitive merge within 0.5 m, Eigen norm and mean in double, index order), and its boundary
points must equal a restatement of VoronoiDiagram::extractBoundaryPoints (voronoi_diagram.cpp:149-207: per
edge start then end, the 1 cm integer key set of kept points and a 5 cm squared-distance test against every
kept point, in edge order)."""
import math

import numpy as np

import oracle_py as O
import orchard


def _frame():
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg)
    poly = orchard.polygon(cfg).astype(np.float64)
    p = O.default_params(grid_resolution=cfg.res)
    r = O.seedgen(cloud, poly, p)
    return r, O.gvd(r["voronoi_seeds"], r["rows_info"], r, p)


def _merge(raw):
    used = [False] * len(raw)
    merged = []
    for i, (xi, yi) in enumerate(raw):
        if used[i]:
            continue
        used[i] = True
        members = [i]
        for j in range(i + 1, len(raw)):
            if used[j]:
                continue
            dx, dy = xi - raw[j][0], yi - raw[j][1]
            if math.sqrt(dx * dx + dy * dy) <= 0.5:
                members.append(j)
                used[j] = True
        sx = sy = 0.0
        for k in members:
            sx += raw[k][0]
            sy += raw[k][1]
        merged.append((sx / float(len(members)), sy / float(len(members))))
    return np.array(merged)


def test_merge_matches_restatement():
    r, g = _frame()
    raw = [tuple(map(float, s)) for s in r["voronoi_seeds"]]
    np.testing.assert_array_equal(g["merged"], _merge(raw))


def test_merge_matches_restatement_with_near_duplicates():
    """C0's seeds are >= 0.5 m apart, so the merge is exercised on the same frame with jittered copies of
    every third seed interleaved (0.1-0.45 m away: chains where the greedy, non-transitive order matters)."""
    r, _ = _frame()
    rng = np.random.default_rng(7)
    base = np.asarray(r["voronoi_seeds"], np.float64)
    seeds = []
    for i, s in enumerate(base):
        seeds.append(s)
        if i % 3 == 0:
            a, d = rng.uniform(0, 2 * np.pi), rng.uniform(0.1, 0.45)
            seeds.append(s + d * np.array([np.cos(a), np.sin(a)]))
    seeds = np.array(seeds)
    p = O.default_params(grid_resolution=orchard.CONFIGS["C0"].res)
    g = O.gvd(seeds, r["rows_info"], r, p)
    ref = _merge([tuple(map(float, s)) for s in seeds])
    assert len(ref) < len(seeds)
    np.testing.assert_array_equal(g["merged"], ref)


def test_boundary_points_match_restatement():
    _, g = _frame()
    edges = g["vor_edges"]
    assert len(edges) > 0
    keys, kept = set(), []
    arr = np.zeros((0, 2))
    thr2 = 0.05 * 0.05
    for x0, y0, x1, y1 in edges:
        for x, y in ((x0, y0), (x1, y1)):
            key = (int(x * 100), int(y * 100))   # static_cast<int>: truncation toward zero
            if key in keys:
                continue
            if len(kept):
                d = arr - (x, y)
                if np.any(d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] < thr2):
                    continue
            keys.add(key)
            kept.append((x, y))
            arr = np.array(kept)
    np.testing.assert_array_equal(g["boundary_raw"], np.array(kept))
