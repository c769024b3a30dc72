"""Oracle checks for the grid stages (a1 ROR, a5 inflation, a7 opening + Zhang-Suen) against
independent implementations available here (numpy brute force, scipy.ndimage / cKDTree) and
hand-derived known answers. The reference ships no fixtures for this path, so these
are the pins of oracle/ (parity vs the reference binary itself: unpinned)."""
import numpy as np
import pytest
from scipy import ndimage
from scipy.spatial import cKDTree

import oracle_py as O

CROSS = np.array([[0, 1, 0], [1, 1, 1], [0, 1, 0]], bool)


def ror_bruteforce(xyz, is_dense=True, radius=0.2, min_pts=2):
    """Independent numpy restatement: float32 ((dx*dx)+dy*dy)+dz*dz, PCL dense (<= r^2 in double,
    kNN k=min_pts+1) / non-dense (< float(r^2), count > min_pts) branches."""
    x = xyz.astype(np.float32)
    fin = np.isfinite(x).all(1)
    keep = np.zeros(len(x), np.uint8)
    idx = np.nonzero(fin)[0]
    if is_dense and len(idx) < min_pts + 1:
        return keep
    for i in idx:
        d = x[idx] - x[i]
        d2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
        d2 = d2.astype(np.float32)
        if is_dense:
            cnt = np.count_nonzero(d2.astype(np.float64) <= radius * radius)
        else:
            cnt = np.count_nonzero(d2 < np.float32(radius * radius))
        keep[i] = cnt >= min_pts + 1
    return keep


@pytest.mark.parametrize("dense", [True, False])
def test_ror_matches_bruteforce(dense):
    rng = np.random.default_rng(7)
    pts = rng.uniform(0, 2.0, size=(1500, 3)).astype(np.float32)
    pts[:, 2] *= 0.3
    pts[100] = pts[101]                          # duplicates
    pts[200] = pts[201] + np.float32([0.2, 0, 0])  # exactly-at-radius along x
    if not dense:
        pts[300] = np.nan
    assert np.array_equal(O.ror(pts, dense), ror_bruteforce(pts, dense))


def test_ror_vs_ckdtree_counts():
    rng = np.random.default_rng(3)
    pts = rng.uniform(0, 5.0, size=(20000, 3)).astype(np.float32)
    keep = O.ror(pts, True)
    cnt = cKDTree(pts.astype(np.float64)).query_ball_point(pts.astype(np.float64), r=0.2, return_length=True)
    ref = (cnt >= 3).astype(np.uint8)
    # float32 vs float64 distance only differs on measure-zero boundary cases
    assert np.count_nonzero(keep != ref) <= 2


def test_ror_tiny_clouds():
    p2 = np.zeros((2, 3), np.float32)
    assert O.ror(p2, True).sum() == 0          # k < mean_k -> removed
    p3 = np.zeros((3, 3), np.float32)
    assert O.ror(p3, True).sum() == 3


@pytest.mark.parametrize("R", [1, 4, 8])
def test_inflation_is_thresholded_edt(R):
    rng = np.random.default_rng(R)
    g = np.zeros((97, 131), np.int8)
    g[rng.random(g.shape) < 0.01] = 100
    g[0, 0] = 100
    g[-1, 60] = 100
    out = O.inflate(g, R)
    d = ndimage.distance_transform_edt(g != 100)
    ref = np.where(np.rint(d * d) <= R * R, 100, 0).astype(np.int8)
    assert np.array_equal(out, ref)


def test_opening_matches_ndimage():
    rng = np.random.default_rng(11)
    img = (rng.random((120, 90)) < 0.55).astype(np.uint8)
    img[:3, :] = 1
    out = O.open_cross(img)
    er = ndimage.binary_erosion(img.astype(bool), structure=CROSS, border_value=1)
    ref = ndimage.binary_dilation(er, structure=CROSS, border_value=0)
    assert np.array_equal(out.astype(bool), ref)


def zs_numpy(img):
    """Independent vectorised Zhang-Suen (ximgproc semantics: Jacobi sub-iterations, borders untouched)."""
    a = img.astype(np.uint8).copy()
    it = 0
    prev = np.zeros_like(a)
    while True:
        for sub in (0, 1):
            p = np.pad(a, 1)
            P2, P3, P4 = p[:-2, 1:-1], p[:-2, 2:], p[1:-1, 2:]
            P5, P6, P7 = p[2:, 2:], p[2:, 1:-1], p[2:, :-2]
            P8, P9 = p[1:-1, :-2], p[:-2, :-2]
            seq = [P2, P3, P4, P5, P6, P7, P8, P9, P2]
            A = sum(((seq[k] == 0) & (seq[k + 1] == 1)).astype(int) for k in range(8))
            B = sum(s.astype(int) for s in seq[:8])
            if sub == 0:
                m1, m2 = P2 * P4 * P6, P4 * P6 * P8
            else:
                m1, m2 = P2 * P4 * P8, P2 * P6 * P8
            mark = (A == 1) & (B >= 2) & (B <= 6) & (m1 == 0) & (m2 == 0)
            mark[0, :] = mark[-1, :] = False
            mark[:, 0] = mark[:, -1] = False
            a = a & ~mark.astype(np.uint8) & 1
        it += 1
        if np.array_equal(a, prev):
            return a, it
        prev = a.copy()


def test_thinning_matches_independent_numpy():
    rng = np.random.default_rng(5)
    img = np.zeros((80, 110), np.uint8)
    for _ in range(25):
        y, x = rng.integers(0, 80), rng.integers(0, 110)
        img[max(0, y - 4):y + 5, max(0, x - 12):x + 13] = 1
    img[:, :2] = 1
    out, it = O.thin(img)
    ref, rit = zs_numpy(img)
    assert np.array_equal(out, ref) and it == rit


def test_thinning_known_answers():
    # a single pixel is a fixed point; ximgproc's `prev` starts as zeros, so a non-empty fixed
    # point still costs T = 2 iterations (the first differs from the zero image)
    img = np.zeros((9, 9), np.uint8)
    img[4, 4] = 1
    out, it = O.thin(img)
    assert np.array_equal(out, img) and it == 2
    # 3-px thick horizontal bar -> its centre line (ends eroded) in one pass, confirmed by a second: T = 2
    bar = np.zeros((9, 20), np.uint8)
    bar[3:6, 2:18] = 1
    out, it = O.thin(bar)
    assert out[[3, 5], :].sum() == 0 and out[4, 3:16].all() and out[4].sum() == 13 and it == 2
    # image-border pixels are never examined
    full = np.ones((6, 6), np.uint8)
    out, _ = O.thin(full)
    assert out[0].all() and out[-1].all() and out[:, 0].all() and out[:, -1].all()
    # empty image: T = 1
    out, it = O.thin(np.zeros((5, 5), np.uint8))
    assert it == 1 and out.sum() == 0


def test_thinning_idempotent():
    rng = np.random.default_rng(9)
    img = ndimage.binary_dilation(rng.random((64, 64)) < 0.02, iterations=3).astype(np.uint8)
    out, _ = O.thin(img)
    out2, it2 = O.thin(out)
    assert np.array_equal(out, out2) and it2 == (2 if out.any() else 1)
    assert not (out & ~img).any()
