"""Pipelined GVD (aos_gvd_from_seedgen_async / aos_gvd_wait): the next seed-gen frame runs while the
previous frame's graph is built, as the reference's two nodes do. The graph, the markers and the
path planner must equal the sequential calls on the same frames."""
import numpy as np
import pytest

import aos_gpu
import orchard

pytestmark = pytest.mark.gpu

GRAPH_KEYS = ("nodes", "node_labels", "node_cluster_indices", "node_label_counts", "node_label_clusters",
              "node_label_types", "edges", "edge_lengths", "edge_clearances")


def assert_same_graph(a, b, what):
    assert a["published"] == b["published"], what
    for k in GRAPH_KEYS:
        assert np.array_equal(a[k], b[k]), f"{what}: {k}"


def assert_same_markers(a, b, what):
    for k in ("seeds", "row_label_valid", "cell_offsets", "cell_xy", "cell_center", "cell_rgba"):
        assert np.array_equal(a[k], b[k]), f"{what}: markers {k}"


def frames():
    cfg = orchard.CONFIGS["C1"]
    poly = orchard.polygon(cfg)
    return cfg, poly, [orchard.generate(cfg), orchard.generate(cfg, seed=cfg.seed + 7)]


def test_pipelined_graph_equals_sequential():
    cfg, poly, clouds = frames()
    ref = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ref.set_polygon(poly)
    seq = []
    for cl in clouds:
        ref.seedgen(cl, want_host=False)
        seq.append((ref.gvd_from_seedgen(), ref.gvd_markers(), ref.path_plan(aos_gpu.path_query(target=3, previous=2))))
    ref.close()

    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    c.seedgen(clouds[0], want_host=False)
    c.gvd_async()
    c.seedgen(clouds[1], want_host=False)      # overlaps frame 0's graph
    g0 = c.gvd_wait()
    assert_same_graph(g0, seq[0][0], "frame 0")
    assert_same_markers(c.gvd_markers(), seq[0][1], "frame 0")
    # frame 0's skeleton was snapshotted: planning on its graph still works after frame 1's seed-gen
    p0 = c.path_plan(aos_gpu.path_query(target=3, previous=2))
    assert np.array_equal(p0["poses"], seq[0][2]["poses"]) and np.array_equal(p0["node_path"], seq[0][2]["node_path"])
    c.gvd_async()                              # frame 1
    m_first = None
    try:
        m_first = c.gvd_markers()              # waits for the job without collecting it
    finally:
        g1 = c.gvd_wait()
    assert_same_graph(g1, seq[1][0], "frame 1")
    assert_same_markers(m_first, seq[1][1], "frame 1")
    c.close()


def test_pipeline_state_rules():
    cfg, poly, clouds = frames()
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    with pytest.raises(RuntimeError, match="no seed-gen frame"):
        c.gvd_async()
    c.seedgen(clouds[0], want_host=False)
    with pytest.raises(RuntimeError, match="no GVD job"):
        c.gvd_wait()
    c.gvd_async()
    g_sync = c.gvd_from_seedgen()               # supersedes the job's result
    with pytest.raises(RuntimeError, match="no GVD job"):
        c.gvd_wait()
    c.gvd_async()
    assert_same_graph(c.gvd_wait(), g_sync, "re-run")
    c.gvd_async()
    c.close()                                  # a job in flight is joined


def test_pipeline_markers_per_frame():
    """The bench's publish throttle: aos_gvd_set_markers switches the cells on for some jobs only (a job
    keeps the setting it started with); the graphs are unaffected, the frames with markers carry them,
    and asking a frame without them computes them on demand — all equal to the sequential calls."""
    cfg, poly, clouds = frames()
    ref = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ref.set_polygon(poly)
    seq = []
    for cl in clouds:
        ref.seedgen(cl, want_host=False)
        seq.append((ref.gvd_from_seedgen(), ref.gvd_markers()))
    ref.close()
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    c.gvd_pipeline_depth(len(clouds))
    on = [k % 2 == 0 for k in range(len(clouds))]
    for k, cl in enumerate(clouds):
        c.seedgen(cl, want_host=False)
        c.gvd_set_markers(on[k])
        c.gvd_async()
    for k in range(len(clouds)):
        assert_same_graph(c.gvd_wait(), seq[k][0], f"frame {k}")
        m = c.gvd_markers()
        assert_same_markers(m, seq[k][1], f"frame {k}")
    c.close()


def test_collected_markers_while_next_job_runs():
    """aos_gvd_collected_markers_get: the markers of the frame last returned by aos_gvd_wait, collected
    after the next frame's job has started (the bench's one-step-later collection), equal the
    sequential markers; aos_gvd_markers_get would address the newest job instead."""
    cfg, poly, clouds = frames()
    ref = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ref.set_polygon(poly)
    seq = []
    for cl in clouds:
        ref.seedgen(cl, want_host=False)
        seq.append((ref.gvd_from_seedgen(), ref.gvd_markers()))
    ref.close()
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    c.gvd_pipeline_depth(2)
    c.seedgen(clouds[0], want_host=False)
    c.gvd_async()
    assert_same_graph(c.gvd_wait(), seq[0][0], "frame 0")
    c.seedgen(clouds[1], want_host=False)
    c.gvd_async()                                   # frame 1's job runs
    assert_same_markers(c.gvd_markers(collected=True), seq[0][1], "frame 0 collected")
    assert_same_markers(c.gvd_markers(), seq[1][1], "frame 1 (newest)")
    assert_same_graph(c.gvd_wait(), seq[1][0], "frame 1")
    c.close()


def test_cloud_prefetch():
    """aos_cloud_prefetch: the next frame's PointCloud2 uploaded in the background is used by the next
    seed-gen of the same view, a mismatching view discards it, NULL waits and drops it; every frame equals
    the plain upload's."""
    cfg = orchard.CONFIGS["C1"]
    poly = orchard.polygon(cfg)
    a = orchard.generate(cfg, n_points=2_500_000)                    # 40 MB: above the 32 MB floor
    b = orchard.generate(cfg, seed=cfg.seed + 3, n_points=2_500_000)
    keys = ("occupancy", "skeleton_framed", "voronoi_seeds", "rows_info")
    ref = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ref.set_polygon(poly)
    ra, rb = ref.seedgen(a), ref.seedgen(b)
    ref.close()

    def same(g, r, what):
        assert g["thin_iters"] == r["thin_iters"], what
        for k in keys:
            assert np.array_equal(g[k], r[k]), (what, k)

    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    same(c.seedgen(a), ra, "plain a")
    c.cloud_prefetch(b)
    same(c.seedgen(b), rb, "prefetched b")
    c.cloud_prefetch(a)
    same(c.seedgen(b), rb, "b while a was prefetched")
    c.cloud_prefetch(a)
    c.cloud_prefetch_wait()
    same(c.seedgen(a), ra, "a after a dropped prefetch")
    c.cloud_prefetch(b)
    c.close()                                                        # a prefetch in flight at close


def test_pipeline_depth_frames_in_flight():
    """aos_gvd_pipeline_depth(3): three frames' GVDs run at once, collected in start order; each graph,
    its markers and a plan on it equal the sequential calls. One start past the depth supersedes the
    oldest job."""
    cfg, poly, clouds = frames()
    clouds = clouds + [orchard.generate(cfg, seed=cfg.seed + 11), orchard.generate(cfg, seed=cfg.seed + 13)]
    ref = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ref.set_polygon(poly)
    seq = []
    for cl in clouds:
        ref.seedgen(cl, want_host=False)
        seq.append((ref.gvd_from_seedgen(), ref.gvd_markers(), ref.path_plan(aos_gpu.path_query(target=3, previous=2))))
    ref.close()

    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    with pytest.raises(RuntimeError, match="depth"):
        c.gvd_pipeline_depth(0)
    c.gvd_pipeline_depth(3)
    for k in range(3):                         # frames 0-2 in flight together
        c.seedgen(clouds[k], want_host=False)
        c.gvd_async()
    c.seedgen(clouds[3], want_host=False)
    for k in range(4):
        if k == 1:
            c.gvd_async()                      # frame 3 starts while frames 1 and 2 are in flight
        g = c.gvd_wait()
        assert_same_graph(g, seq[k][0], f"frame {k}")
        assert_same_markers(c.gvd_markers(), seq[k][1], f"frame {k}")
        p = c.path_plan(aos_gpu.path_query(target=3, previous=2))
        assert np.array_equal(p["poses"], seq[k][2]["poses"]), f"frame {k} plan"
    with pytest.raises(RuntimeError, match="no GVD job"):
        c.gvd_wait()
    # depth 2: a third start supersedes the oldest job
    c.gvd_pipeline_depth(2)
    for k in (1, 2, 3):
        c.seedgen(clouds[k], want_host=False)
        c.gvd_async()
    assert_same_graph(c.gvd_wait(), seq[2][0], "superseded: frame 2 first")
    assert_same_graph(c.gvd_wait(), seq[3][0], "superseded: frame 3")
    with pytest.raises(RuntimeError, match="no GVD job"):
        c.gvd_wait()
    c.seedgen(clouds[0], want_host=False)
    c.gvd_async()
    c.gvd_async()                              # (the same frame twice: both jobs run)
    c.close()                                  # jobs in flight are joined
