"""The C-ABI's error contract (SURVEY §8b "Errors"), called raw through ctypes: bad arguments return
AOS_E_INVALID, calls out of order AOS_E_STATE, each with a message in aos_last_error(); nothing is thrown
across the ABI, and the handle serves the next good frame exactly as a fresh one (parity with the oracle).
Non-finite seeds are not an error: processGraph filters them (gvd:255-318), so the GVD of seeds with NaN /
inf rows interleaved equals the oracle's on the same list.
"""
import ctypes

import numpy as np
import pytest

import aos_gpu
import oracle_py as O
import orchard
from parity_util import assert_gvd_parity, assert_seedgen_parity

pytestmark = pytest.mark.gpu

E_INVALID, E_STATE = -1, -4


def _err():
    return aos_gpu.lib().aos_last_error().decode()


def _view(arr, step=16, ox=0, oy=4, oz=8, n=None):
    return aos_gpu.CloudView(arr.ctypes.data if arr is not None else None, arr.shape[0] if n is None else n, step,
                             ox, oy, oz, 1, 0)


def test_bad_arguments_and_call_order_then_recovery():
    L = aos_gpu.lib()
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg)
    ctx = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ctx.set_polygon(orchard.polygon(cfg))
    h, out, gout = ctx.h, aos_gpu.SeedGenOut(), aos_gpu.GvdOut()

    # before any frame: the calls that read the last frame are out of order
    assert L.aos_gvd_from_seedgen(h, ctypes.byref(gout)) == E_STATE and "no seed-gen frame" in _err()
    assert L.aos_gvd_from_seedgen_async(h) == E_STATE and "no seed-gen frame" in _err()
    occ = np.empty(4, np.int8)
    assert L.aos_seedgen_grids_copy(h, occ.ctypes.data, None) == E_STATE
    assert L.aos_gvd_wait(h, ctypes.byref(gout)) == E_STATE and "no GVD job" in _err()

    # PointCloud2 layouts the reference's fromROSMsg could not read as float32 x / y / z
    bad_views = [
        _view(cloud, step=8),                      # point_step < 12
        _view(cloud, ox=2),                        # misaligned field
        _view(cloud, oz=16),                       # field past the record
        _view(cloud, step=18),                     # step not a multiple of 4
        _view(None, n=10),                         # no data for 10 points
    ]
    for v in bad_views:
        assert L.aos_seedgen_process(h, ctypes.byref(v), 1, ctypes.byref(out)) == E_INVALID
        assert "invalid PointCloud2 layout" in _err()
        assert L.aos_map_append(h, ctypes.byref(v), 1, ctypes.byref(out)) == E_INVALID
    v = _view(cloud)
    assert L.aos_seedgen_process(h, None, 1, ctypes.byref(out)) == E_INVALID and "null argument" in _err()
    assert L.aos_seedgen_process(h, ctypes.byref(v), 1, None) == E_INVALID
    assert L.aos_seedgen_process(None, ctypes.byref(v), 1, ctypes.byref(out)) == E_INVALID
    for depth in (0, 17, -3):
        assert L.aos_gvd_pipeline_depth(h, depth) == E_INVALID and "[1, 16]" in _err()

    # aos_gvd_process: negative counts, null arrays behind non-empty lists
    info = aos_gpu.GridInfo(0.0, 0.0, 0.1, 64, 64)
    sk = np.zeros(64 * 64, np.int8)
    seeds = np.zeros(8, np.float64)
    P = ctypes.POINTER
    dp = lambda a: a.ctypes.data_as(P(ctypes.c_double))   # noqa: E731
    skp = sk.ctypes.data_as(P(ctypes.c_int8))
    bad_in = [
        aos_gpu.GvdIn(None, 4, None, 0, info, skp),
        aos_gpu.GvdIn(dp(seeds), -1, None, 0, info, skp),
        aos_gpu.GvdIn(dp(seeds), 4, None, 2, info, skp),
        aos_gpu.GvdIn(dp(seeds), 4, dp(seeds), -2, info, skp),
        aos_gpu.GvdIn(dp(seeds), 4, None, 0, info, None),
    ]
    for gi in bad_in:
        assert L.aos_gvd_process(h, ctypes.byref(gi), ctypes.byref(gout)) == E_INVALID
        assert "aos_gvd_process" in _err()
    # empty inputs are the callbacks' early returns: status 0, nothing published
    gi = aos_gpu.GvdIn(None, 0, None, 0, aos_gpu.GridInfo(0.0, 0.0, 0.1, 0, 0), None)
    assert L.aos_gvd_process(h, ctypes.byref(gi), ctypes.byref(gout)) == 0
    assert gout.published == 0 and gout.num_nodes == 0 and gout.num_edges == 0

    # the handle serves the next good frame like a fresh one
    g = ctx.seedgen(cloud)
    o = O.seedgen(cloud, orchard.polygon(cfg), O.default_params(grid_resolution=cfg.res))
    assert_seedgen_parity(g, o)
    assert_gvd_parity(ctx.gvd_from_seedgen(), O.gvd(o["voronoi_seeds"], o["rows_info"], o))
    ctx.close()


def test_gvd_non_finite_seeds_are_filtered_like_the_reference():
    """NaN / inf seeds interleaved with the C0 seeds: g1's greedy merge never absorbs them (every distance
    test with a NaN is false), g3's finite filter drops them from the bounds and the inserts, and the
    markers' second Subdiv2D takes only the finite merged seeds (voronoi_diagram.cpp:209-311)."""
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg)
    ctx = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ctx.set_polygon(orchard.polygon(cfg))
    ctx.seedgen(cloud)
    o = O.seedgen(cloud, orchard.polygon(cfg), O.default_params(grid_resolution=cfg.res))
    base = np.asarray(o["voronoi_seeds"], np.float64)
    bad = np.array([[np.nan, 1.0], [2.0, np.inf], [-np.inf, np.nan], [np.nan, np.nan]])
    seeds = []
    for i, s in enumerate(base):
        seeds.append(s)
        if i % 17 == 5:
            seeds.append(bad[(i // 17) % len(bad)])
    seeds = np.array(seeds)
    assert (~np.isfinite(seeds)).any(axis=1).sum() >= 4
    go = O.gvd(seeds, o["rows_info"], o, O.default_params(grid_resolution=cfg.res, markers=1))
    gg = ctx.gvd(seeds, o["rows_info"], o)
    assert_gvd_parity(gg, go)
    assert len(gg["nodes"]) == len(go["nodes"]) > 0
    # the graph is the finite seeds' graph: the non-finite ones change nothing
    gf = ctx.gvd(base, o["rows_info"], o)
    assert_gvd_parity(gf, O.gvd(base, o["rows_info"], o))
    for k in ("nodes", "edges", "edge_lengths", "node_labels", "node_label_clusters"):
        assert np.array_equal(gg[k], gf[k]), k
    ctx.gvd(seeds, o["rows_info"], o)
    m = ctx.gvd_markers()
    assert np.array_equal(m["seeds"], go["merged"], equal_nan=True)   # the merged list, non-finite rows kept
    for k in ("cell_offsets", "cell_xy", "cell_center", "cell_rgba"):   # the cells: finite merged seeds only
        assert np.array_equal(m[k], go[k]), k
    ctx.close()

    # all seeds non-finite: processGraph returns before the graph (gvd:273-275), nothing published
    ctx = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    r = ctx.gvd(bad, o["rows_info"], o)
    gb = O.gvd(bad, o["rows_info"], o)
    assert not gb["published"] and not r["published"] and len(r["nodes"]) == 0
    assert_gvd_parity(r, gb)
    ctx.close()
