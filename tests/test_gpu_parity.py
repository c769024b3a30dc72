"""GPU parity tests: libaos_gpu.so (through its C-ABI) vs the CPU oracle on the same seeded inputs.

Bar (north_star): grids / skeleton / GvdGraph topology bit-exact, seeds within 1e-6.
"""
import numpy as np
import pytest

import aos_gpu
import oracle_py as O
import orchard
from parity_util import assert_golden_hashes, assert_gvd_parity, assert_seedgen_parity, grid_diff

pytestmark = pytest.mark.gpu


def run_both(cfg, poly=None, cloud=None, res=None, **kw):
    cloud = orchard.generate(cfg) if cloud is None else cloud
    poly = orchard.polygon(cfg) if poly is None else poly
    res = cfg.res if res is None else res
    g_ctx = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=res))
    g_ctx.set_polygon(poly)
    g = g_ctx.seedgen(cloud, **kw)
    o = O.seedgen(cloud, poly, O.default_params(grid_resolution=res), is_dense=kw.get("is_dense", True))
    return g_ctx, g, o


def test_grids_copy_into_caller_memory():
    """aos_seedgen_grids_copy (the node's publish path: a frame with want_host = 0, both OccupancyGrids
    copied from HBM straight into the outgoing messages' data) equals the frame's host grids and the
    oracle's."""
    cfg = orchard.CONFIGS["C0"]
    c, g, o = run_both(cfg)
    c2 = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    with pytest.raises(RuntimeError, match="no seed-gen frame"):
        c2.grids_copy((g["height"], g["width"]))
    c2.set_polygon(orchard.polygon(cfg))
    g2 = c2.seedgen(orchard.generate(cfg), want_host=False)
    occ, skel = c2.grids_copy((g2["height"], g2["width"]))
    assert np.array_equal(occ, g["occupancy"]) and np.array_equal(skel, g["skeleton_framed"])
    assert np.array_equal(occ, o["occupancy"]) and np.array_equal(skel, o["skeleton_framed"])
    c.close()
    c2.close()


def test_c0_full_frame():
    cfg = orchard.CONFIGS["C0"]
    c, g, o = run_both(cfg)
    assert_seedgen_parity(g, o)
    for which, ref in (("raster", o["raster"]), ("inflated", o["inflated"]), ("skeleton_frameless", o["skeleton"])):
        got = c.debug_grid(which, (g["height"], g["width"]))
        assert grid_diff(got, ref) == 0, which
    opened = c.debug_grid("opened", (g["height"], g["width"]))
    assert grid_diff(opened == 100, o["opened"] == 1) == 0
    gg = c.gvd_from_seedgen()
    go = O.gvd(o["voronoi_seeds"], o["rows_info"], o)
    assert_gvd_parity(gg, go)
    # the same GVD through the external-input entry point (drop-in aos_gvd_node path)
    ge = c.gvd(o["voronoi_seeds"], o["rows_info"], o)
    assert_gvd_parity(ge, go)
    c.close()


def test_gvd_external_near_duplicate_seeds():
    """voronoiSeedsCallback's greedy 0.5 m merge (gvd:84-128) actually firing: the C0 seeds with jittered
    copies of every third seed interleaved (0.1-0.45 m away) through the external-input entry point."""
    cfg = orchard.CONFIGS["C0"]
    c, g, o = run_both(cfg)
    rng = np.random.default_rng(7)
    seeds = []
    for i, s in enumerate(np.asarray(o["voronoi_seeds"], np.float64)):
        seeds.append(s)
        if i % 3 == 0:
            a, d = rng.uniform(0, 2 * np.pi), rng.uniform(0.1, 0.45)
            seeds.append(s + d * np.array([np.cos(a), np.sin(a)]))
    seeds = np.array(seeds)
    go = O.gvd(seeds, o["rows_info"], o, O.default_params(grid_resolution=cfg.res, markers=1))
    assert len(go["merged"]) < len(seeds)
    assert_gvd_parity(c.gvd(seeds, o["rows_info"], o), go)
    _assert_markers(c.gvd_markers(), go)      # markers' seeds = the merged seeds
    c.close()


def test_c1_full_frame():
    cfg = orchard.CONFIGS["C1"]
    c, g, o = run_both(cfg)
    assert_seedgen_parity(g, o)
    gg = c.gvd_from_seedgen()
    go = O.gvd(o["voronoi_seeds"], o["rows_info"], o)
    assert_gvd_parity(gg, go)
    c.close()


def test_default_polygon_and_resolution():
    """Reference defaults: hard-coded polygon (seed_gen:196-199), 0.05 m grid (R = 16), exclusion discs."""
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg, n_points=60000)
    xyz = orchard.xyz(cloud)
    xyz[:, 0] = xyz[:, 0] * 0.75 - 2.0   # squeeze the orchard into the default polygon's box
    xyz[:, 1] = xyz[:, 1] * 0.12
    c = aos_gpu.Ctx(aos_gpu.default_params())
    g = c.seedgen(cloud)
    o = O.seedgen(cloud, None, O.default_params())
    assert (g["width"], g["height"]) == (1546, 296)
    assert_seedgen_parity(g, o)
    assert_gvd_parity(c.gvd_from_seedgen(), O.gvd(o["voronoi_seeds"], o["rows_info"], o))
    c.close()


def test_polygon_change_reprocess():
    """explorationAreaCallback: new polygon -> reprocess the last (ROR-filtered) cloud."""
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg)
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(orchard.polygon(cfg))
    c.seedgen(cloud)
    poly2 = np.array([[5.0, 3.0], [60.0, 1.0], [70.0, 14.0], [8.0, 18.0]])
    c.set_polygon(poly2)
    g = c.reprocess()
    o = O.seedgen(cloud, poly2, O.default_params(grid_resolution=cfg.res))
    assert_seedgen_parity(g, o)
    c.set_polygon(np.zeros((2, 2)))   # < 3 points: ignored (seed_gen:253)
    g2 = c.reprocess()
    assert_seedgen_parity(g2, o)
    c.close()


def test_non_dense_cloud_with_nans_and_custom_layout():
    """is_dense = false -> PCL radius-search branch; NaNs dropped; point_step 32 with y/x swapped offsets."""
    cfg = orchard.CONFIGS["C0"]
    base = orchard.generate(cfg, n_points=50000)
    f = base.view(np.float32).reshape(-1, 4)
    rec = np.zeros((len(f), 8), np.float32)
    rec[:, 3], rec[:, 1], rec[:, 5] = f[:, 0], f[:, 1], f[:, 2]   # x @12, y @4, z @20
    rec[::97, 3] = np.nan
    cloud = rec.view(np.uint8).reshape(len(f), 32)
    poly = orchard.polygon(cfg)
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    g = c.seedgen(cloud, point_step=32, offs=(12, 4, 20), is_dense=False)
    o = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res), is_dense=False, point_step=32, offs=(12, 4, 20))
    assert_seedgen_parity(g, o)
    c.close()


@pytest.mark.parametrize("n", [0, 2])
def test_empty_and_tiny_clouds(n):
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg, n_points=max(n, 1))[:n]
    poly = orchard.polygon(cfg)
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    g = c.seedgen(cloud)
    o = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res))
    assert_seedgen_parity(g, o)
    gg = c.gvd_from_seedgen()
    assert not gg["published"] and not O.gvd(o["voronoi_seeds"], o["rows_info"], o)["published"]
    c.close()


def test_device_resident_input_matches_host_input():
    import torch
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg)
    poly = orchard.polygon(cfg)
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    h = c.seedgen(cloud)
    t = torch.from_numpy(cloud).cuda()
    torch.cuda.synchronize()
    d = c.seedgen(t.data_ptr(), n_points=cloud.shape[0], on_device=True)
    assert_seedgen_parity(d, {**h, "cluster_length": np.zeros(h["n_clusters_all"])})
    c.close()


def _line_cloud(segments, step=0.05):
    """Dense points along horizontal segments (x0, x1, y): thin bands whose skeletons are straight
    lines, symmetric about their centre (argmax ties on both ends)."""
    pts = []
    for x0, x1, y in segments:
        xs = np.arange(x0, x1 + 1e-9, step)
        for dy in (-0.05, 0.0, 0.05):
            pts.append(np.stack([xs, np.full_like(xs, y + dy), np.zeros_like(xs)], 1))
    p = np.concatenate(pts).astype(np.float32)
    rec = np.zeros((len(p), 4), np.float32)
    rec[:, :3] = p
    return rec.view(np.uint8).reshape(len(p), 16)


@pytest.fixture(params=["host", "gpu"])
def replay_where(request):
    """Where the frame's exact BFS replays run: host threads, or the GPU walk (replay_gpu.hip) for every flagged
    cluster however few (the library's default sends a frame there from 32 flagged clusters on)."""
    aos_gpu.debug_replay(0 if request.param == "gpu" else 1 << 30)
    yield request.param
    aos_gpu.debug_replay()


def _check_replay_counts(c, g, where):
    rc = c.replay_counts()
    assert rc["all"] == g["n_bfs_replayed"]
    assert rc["gpu"] + rc["host_bits"] + rc["host_cells"] == rc["all"], rc
    if where == "gpu":
        assert rc["gpu"] == rc["all"], rc
    else:
        assert rc["gpu"] == 0, rc
    return rc


def test_argmax_ties_force_exact_bfs_replay(replay_where):
    # origin 0 (polygon bbox starts at 2.5) and res 0.25: world coordinates are exact in float, so a
    # straight skeleton bar symmetric about its centre has exactly tied end distances
    cloud = _line_cloud([(10.0, 60.0, 20.0), (15.0, 55.25, 40.0), (5.0, 5.0, 60.0)])
    poly = np.array([[2.5, 2.5], [90.0, 2.5], [90.0, 90.0], [2.5, 90.0]])
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=0.25))
    c.set_polygon(poly)
    g = c.seedgen(cloud)
    o = O.seedgen(cloud, poly, O.default_params(grid_resolution=0.25))
    assert g["n_bfs_replayed"] >= 1
    _check_replay_counts(c, g, replay_where)
    assert_seedgen_parity(g, o)
    assert_gvd_parity(c.gvd_from_seedgen(), O.gvd(o["voronoi_seeds"], o["rows_info"], o))
    c.close()


def test_c2_seedgen_parity_with_large_sums(replay_where):
    """4096^2: two merged-row clusters have coordinate sums > 2^24 (float sums order-dependent)."""
    cfg = orchard.CONFIGS["C2"]
    c, g, o = run_both(cfg)
    assert g["n_bfs_replayed"] >= 1
    _check_replay_counts(c, g, replay_where)
    assert_seedgen_parity(g, o)
    c.close()


@pytest.mark.parametrize("ring_cap", [0, 2])
def test_gpu_replay_of_every_cluster_equals_certified_records(ring_cap):
    """Every C1 cluster replayed by the GPU walk (aos_debug_replay replay_all), certified or not: the rows, seeds
    and GvdGraph equal the frame whose certified clusters kept the order-free statistics (k_cluster_stats) and the
    oracle. ring_cap 2: a walk with more than 2 queued cells gives its cluster up to the host threads (the
    fallback), so both paths serve one frame."""
    cfg = orchard.CONFIGS["C1"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    base = c.seedgen(cloud)
    gg_base = c.gvd_from_seedgen()
    try:
        aos_gpu.debug_replay(0, ring_cap, replay_all=True)
        g = c.seedgen(cloud)
        rc = c.replay_counts()
        gg = c.gvd_from_seedgen()
    finally:
        aos_gpu.debug_replay()
    assert rc["all"] == g["n_clusters_all"] == base["n_clusters_all"] > 10, rc
    if ring_cap == 0:
        assert rc["gpu"] == rc["all"], rc
    else:
        assert 0 < rc["gpu"] < rc["all"], rc
    assert_seedgen_parity(g, {**base, "cluster_length": np.zeros(base["n_clusters_all"])})
    for k in ("nodes", "edges", "edge_lengths", "edge_clearances", "node_labels"):
        assert np.array_equal(gg[k], gg_base[k]), k
    c.close()


# ---------------------------------------------------------------- against the committed fixtures
def _golden(name):
    import os
    return np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name), allow_pickle=False)


def test_c0_against_golden_fixtures():
    """GPU C0 frame vs tests/golden (oracle outputs frozen by tools/make_golden.py), no oracle call."""
    import json
    gs, gg = _golden("c0_seedgen.npz"), _golden("c0_gvd.npz")
    meta = json.loads(str(gs["meta"]))
    h, w = meta["height"], meta["width"]

    def grid(k):
        return np.where(np.unpackbits(gs[f"grid_{k}"])[: h * w].reshape(h, w) != 0, 100, 0).astype(np.int8)

    o = {k: gs[k] for k in gs.files if not k.startswith("grid_") and k not in ("meta", "origin", "resolution")}
    o.update(meta, origin=tuple(gs["origin"]), resolution=float(gs["resolution"]),
             occupancy=grid("occupancy"), skeleton_framed=grid("skeleton_framed"))
    og = {k: gg[k] for k in gg.files}
    og["published"] = bool(gg["published"])
    cfg = orchard.CONFIGS["C0"]
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(orchard.polygon(cfg))
    g = c.seedgen(orchard.generate(cfg))
    assert g["n_clipped"] == meta["n_clipped"]
    assert_seedgen_parity(g, o)
    assert grid_diff(c.debug_grid("raster", (h, w)) == 100, grid("raster") == 100) == 0
    assert grid_diff(c.debug_grid("skeleton_frameless", (h, w)), grid("skeleton")) == 0
    assert_gvd_parity(c.gvd_from_seedgen(), og)
    c.close()


@pytest.mark.parametrize("name", ["C1", "C2"])
def test_against_golden_hashes(name):
    """Full frame (seed gen + GVD) vs the SHA-256 of the oracle's outputs (tests/golden/<name>_sha256.json);
    C2 is the bench frame, so this pins bench.py's workload bit-exactly without running the oracle."""
    import json
    import os
    hs = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", f"{name.lower()}_sha256.json")))
    cfg = orchard.CONFIGS[name]
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(orchard.polygon(cfg))
    g = c.seedgen(orchard.generate(cfg))
    gg = c.gvd_from_seedgen()
    assert_golden_hashes(g, gg, hs)
    c.close()


# ---------------------------------------------------------------- paths the orchard scenes rarely hit
def _full_frame_parity(cloud, poly, res, **kw):
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=res))
    c.set_polygon(poly)
    g = c.seedgen(cloud, **kw)
    o = O.seedgen(cloud, poly, O.default_params(grid_resolution=res), is_dense=kw.get("is_dense", True))
    assert_seedgen_parity(g, o)
    assert_gvd_parity(c.gvd_from_seedgen(), O.gvd(o["voronoi_seeds"], o["rows_info"], o))
    c.close()
    return g


def test_dense_patches_overflow_the_lds_row_ring():
    """Bin rows with more than 512 staged points are scanned from global memory (k_ror_sweep)."""
    cfg = orchard.CONFIGS["C0"]
    base = orchard.generate(cfg)
    rng = np.random.default_rng(11)
    extra = []
    for cx, cy in ((20.0, 2.0), (40.3, 5.5), (71.9, 12.5), (10.0, 30.0)):   # on rows and between them
        n = 4000
        p = np.zeros((n, 4), np.float32)
        p[:, 0] = cx + rng.uniform(-0.25, 0.25, n)
        p[:, 1] = cy + rng.uniform(-0.25, 0.25, n)
        p[:, 2] = rng.uniform(-0.3, 0.4, n)
        extra.append(p)
    cloud = np.concatenate([base.view(np.float32).reshape(-1, 4)] + extra).view(np.uint8).reshape(-1, 16)
    _full_frame_parity(cloud, orchard.polygon(cfg), cfg.res)


def test_big_tile_after_frames_without_one_on_the_same_handle():
    """The big-tile ROR kernels are skipped on frames whose largest tile fits LDS (seedgen.hip ror_stage: the
    peeked tile maximum) and on guessed frames of a handle that never needed them; a guessed frame that then
    finds a big tile sets overflow bit 2 and is redone with them (ror_collect). Sequence on one handle:
    spread extra points (no big tile, fixes the staging guess) -> dense patches (the guessed frame's redo)
    -> spread -> dense again (big kernels on from then on), each frame vs the oracle."""
    cfg = orchard.CONFIGS["C0"]
    base = orchard.generate(cfg).view(np.float32).reshape(-1, 4)
    poly = orchard.polygon(cfg)
    rng = np.random.default_rng(12)

    def with_extra(dense):
        n = 16000
        p = np.zeros((n, 4), np.float32)
        if dense:
            c = np.repeat(np.array([[20.0, 2.0], [40.3, 5.5], [71.9, 12.5], [10.0, 30.0]]), n // 4, axis=0)
            p[:, :2] = c + rng.uniform(-0.25, 0.25, (n, 2))
        else:
            p[:, 0] = rng.uniform(2.0, 95.0, n)
            p[:, 1] = rng.uniform(2.0, 40.0, n)
        p[:, 2] = rng.uniform(-0.3, 0.4, n)
        return np.concatenate([base, p]).view(np.uint8).reshape(-1, 16)

    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    for dense in (False, True, False, True):
        cloud = with_extra(dense)
        g = c.seedgen(cloud)
        o = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res))
        assert_seedgen_parity(g, o)
        assert_gvd_parity(c.gvd_from_seedgen(), O.gvd(o["voronoi_seeds"], o["rows_info"], o))
    c.close()


def test_rotated_orchard_concave_polygon_and_odd_resolution():
    """Rows at 30 degrees, an L-shaped exploration polygon, 0.15 m cells (R = 5)."""
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg, n_points=80000).copy()
    f = cloud.view(np.float32).reshape(-1, 4)
    a = np.deg2rad(30.0)
    x, y = f[:, 0].astype(np.float64) - 50.0, f[:, 1].astype(np.float64) - 10.0
    f[:, 0] = (x * np.cos(a) - y * np.sin(a) + 50.0).astype(np.float32)
    f[:, 1] = (x * np.sin(a) + y * np.cos(a) + 30.0).astype(np.float32)
    poly = np.array([[5.0, 5.0], [95.0, 5.0], [95.0, 40.0], [55.0, 40.0], [55.0, 75.0], [5.0, 75.0]])
    g = _full_frame_parity(cloud, poly, 0.15)
    assert len(g["row_length"]) > 0


def test_grid_resolution_0_3_and_non_dense():
    cfg = orchard.CONFIGS["C0"]
    _full_frame_parity(orchard.generate(cfg, n_points=70000), orchard.polygon(cfg), 0.3, is_dense=False)


# ---------------------------------------------------------------- /gvd/markers
def _assert_markers(m, og):
    assert np.array_equal(m["seeds"], og["merged"])
    assert np.array_equal(m["row_label_valid"], og["row_label_valid"])
    v = og["row_label_valid"].astype(bool)
    assert np.array_equal(m["row_label_pts"][v], og["row_label_pts"][v])
    assert np.array_equal(m["cell_offsets"], og["cell_offsets"])
    assert np.array_equal(m["cell_xy"], og["cell_xy"]), "cell boundaries differ"
    assert np.array_equal(m["cell_center"], og["cell_center"])
    assert np.array_equal(m["cell_rgba"], og["cell_rgba"])


@pytest.mark.parametrize("name", ["C0", "C1"])
def test_gvd_markers_cells_vs_oracle(name):
    """publishMarkers' Voronoi cells: extractCellBoundaries' second Subdiv2D (seed bounding box),
    computed on a worker thread next to the main replay, plus the merged seeds and label points."""
    cfg = orchard.CONFIGS[name]
    c, g, o = run_both(cfg)
    gg = c.gvd_from_seedgen()
    m = c.gvd_markers()
    og = O.gvd(o["voronoi_seeds"], o["rows_info"], o, O.default_params(grid_resolution=cfg.res, markers=1))
    assert_gvd_parity(gg, og)
    assert len(m["cell_offsets"]) > 100
    _assert_markers(m, og)
    _assert_markers(c.gvd_markers(view=True), og)   # zero-copy views of the same arrays (bench.py's way)
    c.close()


@pytest.mark.parametrize("name", ["C0", "C1"])
def test_gvd_rect_mode_1_vs_oracle(name):
    """The unpinned Subdiv2D constructor choice: subdiv_rect_mode = 1 (the Rect2f -> Rect
    conversion) on full frames — graph and markers' cells vs the oracle in the same mode."""
    cfg = orchard.CONFIGS[name]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res, subdiv_rect_mode=1))
    c.set_polygon(poly)
    g = c.seedgen(cloud)
    gg = c.gvd_from_seedgen()
    m = c.gvd_markers()
    o = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res))
    op = O.default_params(grid_resolution=cfg.res, markers=1, subdiv_rect_mode=1)
    og = O.gvd(o["voronoi_seeds"], o["rows_info"], o, op)
    assert_seedgen_parity(g, o)
    assert_gvd_parity(gg, og)
    _assert_markers(m, og)
    c.close()


def test_gvd_markers_external_input_and_disabled():
    cfg = orchard.CONFIGS["C0"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    o = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res))
    og = O.gvd(o["voronoi_seeds"], o["rows_info"], o, O.default_params(grid_resolution=cfg.res, markers=1))
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.gvd(o["voronoi_seeds"], o["rows_info"], o)
    _assert_markers(c.gvd_markers(), og)
    c.close()
    # markers off (a frame the node does not publish, gvd:306-314): nothing is computed with the graph;
    # asking for them computes them on demand, equal to the eager job
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res, gvd_markers=0))
    with pytest.raises(RuntimeError, match="no markers"):
        c.gvd_markers()                     # no GVD frame yet
    c.gvd(o["voronoi_seeds"], o["rows_info"], o)
    _assert_markers(c.gvd_markers(), og)
    c.gvd_set_markers(True)
    c.gvd(o["voronoi_seeds"], o["rows_info"], o)
    _assert_markers(c.gvd_markers(), og)
    c.close()


def test_gvd_markers_background_job_overlaps_next_frame():
    """The cells finish in the background after the graph (publishGraph before publishMarkers,
    gvd:310-313): a seed-gen frame may run before they are collected, a GVD call that nobody
    collected is superseded by the next one, and closing a handle with a job in flight joins it."""
    cfg = orchard.CONFIGS["C0"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    o = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res))
    og = O.gvd(o["voronoi_seeds"], o["rows_info"], o, O.default_params(grid_resolution=cfg.res, markers=1))
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    c.seedgen(cloud)
    c.gvd_from_seedgen()
    c.gvd_from_seedgen()          # the first call's job is joined and replaced
    c.seedgen(cloud)              # overlaps the second job
    m = c.gvd_markers()
    assert m["ms_cells"] > 0
    _assert_markers(m, og)
    c.gvd_from_seedgen()
    c.close()                     # job still in flight


def test_ccl_link_list_overflow_fallback(monkeypatch):
    """k_ccl_local hands its cross-chunk links to k_ccl_cross through a list; when the list overflows, the same
    launch unions every link of every cell instead. A C1 frame with a 2-entry list (AOS_DEBUG_CCL_ECAP) equals
    the default frame, clusters and seeds included."""
    cfg = orchard.CONFIGS["C1"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    ctx = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ctx.set_polygon(poly)
    a = ctx.seedgen(cloud)
    monkeypatch.setenv("AOS_DEBUG_CCL_ECAP", "2")
    b = ctx.seedgen(cloud)
    monkeypatch.delenv("AOS_DEBUG_CCL_ECAP")
    ctx.close()
    assert a["n_clusters_all"] == b["n_clusters_all"] and a["n_bfs_replayed"] == b["n_bfs_replayed"]
    for k in ("row_center", "row_start", "row_end", "row_length", "voronoi_seeds", "cluster_info", "rows_info"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k


def test_cluster_stats_global_memory_path(monkeypatch):
    """k_cluster_stats keeps a cluster's cells in LDS when it fits (kStatLds cells, grids below 65536 columns and
    rows) and otherwise reads global memory in every pass. A C1 frame with the LDS copy off (AOS_DEBUG_STATS_LDS=0)
    equals the default frame: records, replays, rows and seeds."""
    cfg = orchard.CONFIGS["C1"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    ctx = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ctx.set_polygon(poly)
    a = ctx.seedgen(cloud)
    monkeypatch.setenv("AOS_DEBUG_STATS_LDS", "0")
    b = ctx.seedgen(cloud)
    monkeypatch.delenv("AOS_DEBUG_STATS_LDS")
    ctx.close()
    assert a["n_clusters_all"] == b["n_clusters_all"] and a["n_bfs_replayed"] == b["n_bfs_replayed"]
    for k in ("row_center", "row_start", "row_end", "row_length", "voronoi_seeds", "cluster_info", "rows_info"):
        assert np.array_equal(np.asarray(a[k]), np.asarray(b[k])), k
