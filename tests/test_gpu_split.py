"""Host cloud split at upload (seedgen.hip upload_pack, aos_ctx::CloudSplit).

Only the points inside the ROR stage's binned box for the polygon current at upload time cross PCIe on the
frame's path; the others stay in pinned host memory and are copied behind them when a later frame's box is
not inside that one (aos_seedgen_reprocess after a polygon change, a prefetched cloud whose polygon changed
before the frame). Every frame must equal the oracle (or an unsplit upload), and the points the partition
passes read (n_ror_read) must be exactly the cloud's points inside the box, by the same float compares.
"""
import numpy as np
import pytest

import aos_gpu
import oracle_py as O
import orchard
from parity_util import assert_seedgen_parity

pytestmark = pytest.mark.gpu


def binned_box(poly, ror_radius=0.2, minz=-0.4, maxz=0.5):
    """seedgen.hip binned_box / ror_stage: frame_geom's float bounds (polygon +- 2.5 m, double -> float)
    minus / plus ror_margin, in float32 as on the host."""
    f = np.float32
    m = f(f(ror_radius * 1.01) + f(1e-4))
    minx, maxx = f(poly[:, 0].min() - 2.5), f(poly[:, 0].max() + 2.5)
    miny, maxy = f(poly[:, 1].min() - 2.5), f(poly[:, 1].max() + 2.5)
    return [f(minx - m), f(maxx + m), f(miny - m), f(maxy + m), f(f(minz) - m), f(f(maxz) + m)]


def inside(cloud, box):
    p = orchard.xyz(cloud).astype(np.float32)
    x, y, z = p[:, 0], p[:, 1], p[:, 2]
    with np.errstate(invalid="ignore"):
        return int(np.count_nonzero((x >= box[0]) & (x <= box[1]) & (y >= box[2]) & (y <= box[3]) &
                                    (z >= box[4]) & (z <= box[5])))


def shrunk(poly, k):
    c = poly.mean(axis=0)
    return c + (poly - c) * k


def with_far_points(cloud, frac=0.3, seed=5):
    """A copy with a fraction of the points moved out of the box (far in x, high in z, NaN / inf)."""
    out = cloud.copy()
    p = out.view(np.float32).reshape(-1, 4)
    rng = np.random.default_rng(seed)
    idx = rng.choice(len(p), int(frac * len(p)), replace=False)
    q = len(idx) // 4
    p[idx[:q], 0] += 500.0
    p[idx[q:2 * q], 2] = 3.0
    p[idx[2 * q:3 * q], 1] = np.nan
    p[idx[3 * q:3 * q + 7], 0] = np.inf
    return out


def test_split_front_is_the_binned_box_and_frames_match_the_oracle():
    cfg = orchard.CONFIGS["C0"]
    poly = orchard.polygon(cfg)
    cloud = with_far_points(orchard.generate(cfg))
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    g = c.seedgen(cloud, is_dense=False)
    o = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res), is_dense=False)
    assert_seedgen_parity(g, o)
    assert g["n_input"] == len(cloud)
    assert g["n_ror_read"] == inside(cloud, binned_box(poly)) < len(cloud)
    assert g["n_binned"] <= g["n_ror_read"]
    c.close()


def test_split_reprocess_with_a_larger_polygon_copies_the_rest():
    """Frame under a small polygon (front only), reprocess under the whole one (the rest is copied behind
    the front), back to the small one (the whole cloud is resident now), then a new cloud (its upload waits
    for the rest copy's reads of the pinned buffer)."""
    cfg = orchard.CONFIGS["C0"]
    big = orchard.polygon(cfg)
    small = shrunk(big, 0.45)
    cloud = orchard.generate(cfg)
    P = aos_gpu.default_params(grid_resolution=cfg.res)
    OP = O.default_params(grid_resolution=cfg.res)
    c = aos_gpu.Ctx(P)
    c.set_polygon(small)
    g = c.seedgen(cloud)
    o_small = O.seedgen(cloud, small, OP)
    assert_seedgen_parity(g, o_small)
    assert g["n_ror_read"] == inside(cloud, binned_box(small)) < len(cloud)
    c.set_polygon(big)
    g = c.reprocess()
    assert_seedgen_parity(g, O.seedgen(cloud, big, OP))
    assert g["n_ror_read"] == len(cloud)
    c.set_polygon(small)
    g = c.reprocess()
    assert_seedgen_parity(g, o_small)
    assert g["n_ror_read"] == len(cloud)
    cloud2 = orchard.generate(cfg, seed=cfg.seed + 1)
    g = c.seedgen(cloud2)
    assert_seedgen_parity(g, O.seedgen(cloud2, small, OP))
    assert g["n_ror_read"] == inside(cloud2, binned_box(small))
    c.close()


def test_split_prefetch_under_an_older_polygon():
    """A cloud prefetched under one polygon and processed under a larger one equals the plain upload."""
    cfg = orchard.CONFIGS["C1"]
    big = orchard.polygon(cfg)
    small = shrunk(big, 0.5)
    a = orchard.generate(cfg, n_points=2_500_000)                    # 40 MB: above the prefetch floor
    b = orchard.generate(cfg, seed=cfg.seed + 3, n_points=2_500_000)
    keys = ("occupancy", "skeleton_framed", "voronoi_seeds", "rows_info")
    ref = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ref.set_polygon(big)
    rb = ref.seedgen(b)
    ref.close()
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(small)
    c.seedgen(a)
    c.cloud_prefetch(b)             # split under the small polygon's box
    c.set_polygon(big)
    g = c.seedgen(b)                # the box grew: the rest is copied behind the front
    assert g["n_ror_read"] == len(b)
    assert g["thin_iters"] == rb["thin_iters"]
    for k in keys:
        assert np.array_equal(g[k], rb[k]), k
    c.close()
