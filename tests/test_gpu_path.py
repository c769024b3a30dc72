"""Path planning over the GvdGraph (aos_path_plan) vs the oracle restatement of
aos_path_gen_node (oracle/oracle_path.cpp). Bar: bit-exact waypoints, A* node path, /path poses
(x, y, qz, qw), trim index, status and indices."""
import json
import os

import numpy as np
import pytest

import aos_gpu
import oracle_py as O
import orchard

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

KEYS = ("status", "target", "cluster_index", "cluster_ids", "cluster_nodes", "waypoints", "waypoint_nodes",
        "node_path", "poses", "trimmed_from")


def assert_path_equal(got, ref, what=""):
    for k in KEYS:
        a, b = got[k], ref[k]
        if isinstance(b, np.ndarray):
            assert a.shape == b.shape, f"{what}: {k} shape {a.shape} vs {b.shape}"
            bad = np.argwhere(a != b)
            assert len(bad) == 0, f"{what}: {k} differs at {bad[:4].tolist()}: " + \
                ", ".join(f"{a[tuple(i)]!r} vs {b[tuple(i)]!r}" for i in bad[:4])
        else:
            assert a == b, f"{what}: {k} {a} != {b}"


def c0_fixture():
    g = dict(np.load(os.path.join(GOLDEN, "c0_gvd.npz")))
    s = np.load(os.path.join(GOLDEN, "c0_seedgen.npz"))
    meta = json.loads(str(s["meta"]))
    W, H = meta["width"], meta["height"]
    sk = np.unpackbits(s["grid_skeleton_framed"])[: W * H].astype(np.int8) * 100
    grid = {"origin": tuple(float(v) for v in s["origin"]), "resolution": float(s["resolution"]), "width": W,
            "height": H, "skeleton_framed": sk}
    return g, grid


def queries(n_wp):
    """The node states the reference goes through: every target from the previous waypoint, the
    initial straight line (also across a tree row, which the trim cuts), a service call from the
    robot's position, the target restore rules and the origin return."""
    q = [dict(initial_waypoint_reached=False),
         dict(initial_waypoint_reached=False, initial_waypoint=(8.0, 9.0)),
         dict(initial_waypoint_reached=False, initial_waypoint=(30.0, 3.0))]
    for t in range(n_wp):
        q.append(dict(target=t, previous=t - 1))
    q += [dict(target=2, current=(11.3, 4.1)), dict(target=1, current=(60.0, 12.0)),
          dict(target=3, saved_target=(1.0, 1.0)), dict(target=50, saved_target=(1.0, 1.0)),
          dict(target=-1), dict(target=50), dict(target=-1, saved_target=(40.0, 9.0)),
          dict(target=n_wp, previous=n_wp - 1, exploration_completed=True),
          dict(target=99, previous=2, exploration_completed=True),
          dict(target=n_wp, current=(20.0, 20.0), exploration_completed=True)]
    return q


def test_path_c0_fixture_external_graph():
    """External GvdGraph + host skeleton (the drop-in aos_path_gen_node inputs)."""
    g, grid = c0_fixture()
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=grid["resolution"]))
    n_wp = len(O.path_plan(g, grid, target=0)["waypoints"])
    assert n_wp >= 10
    trims = 0
    for kw in queries(n_wp):
        ref = O.path_plan(g, grid, **kw)
        got = c.path_plan(aos_gpu.path_query(**kw), graph=g, skeleton=grid["skeleton_framed"], info=grid)
        assert_path_equal(got, ref, str(kw))
        trims += ref["trimmed_from"] >= 0
    assert trims >= 1, "no query exercised the trim"
    c.close()


def test_path_fallback_labels_and_empty_graph():
    """No node_label_* entries: the bitmask fallback of buildClusterWaypointMapping (:711-736);
    an empty graph: Failed."""
    g, grid = c0_fixture()
    g2 = dict(g)
    g2["node_label_clusters"] = np.zeros(0, np.int32)
    g2["node_label_types"] = np.zeros(0, np.int32)
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=grid["resolution"]))
    for kw in (dict(target=0), dict(target=3, previous=2)):
        assert_path_equal(c.path_plan(aos_gpu.path_query(**kw), graph=g2, skeleton=grid["skeleton_framed"], info=grid),
                          O.path_plan(g2, grid, **kw), "fallback")
    empty = {k: np.zeros((0, 2) if k in ("nodes", "edges") else 0, np.float64 if k == "nodes" else np.int32)
             for k in ("nodes", "node_labels", "node_cluster_indices", "node_label_counts", "node_label_clusters",
                       "node_label_types", "edges")}
    empty["edge_lengths"] = np.zeros(0, np.float32)
    got = c.path_plan(aos_gpu.path_query(target=0), graph=empty, skeleton=grid["skeleton_framed"], info=grid)
    ref = O.path_plan(empty, grid, target=0)
    assert ref["status"] == 0
    assert_path_equal(got, ref, "empty")
    c.close()


def test_path_c1_own_graph_and_device_skeleton():
    """The handle's own GVD graph and skeleton (graph = NULL, skeleton = NULL), and the seed-gen
    frame's device skeleton passed explicitly; a later frame makes the implicit skeleton stale."""
    cfg = orchard.CONFIGS["C1"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    c.set_polygon(poly)
    f = c.seedgen(cloud)
    gg = c.gvd_from_seedgen()
    grid = {"origin": f["origin"], "resolution": f["resolution"], "width": f["width"], "height": f["height"],
            "skeleton_framed": f["skeleton_framed"]}
    n_wp = len(O.path_plan(gg, grid, target=0)["waypoints"])
    assert n_wp >= 50
    for kw in [dict(target=t, previous=t - 1) for t in range(0, n_wp, 7)] + [
            dict(target=n_wp, previous=n_wp - 1, exploration_completed=True),
            dict(initial_waypoint_reached=False, initial_waypoint=(30.0, 12.0))]:
        ref = O.path_plan(gg, grid, **kw)
        assert_path_equal(c.path_plan(aos_gpu.path_query(**kw)), ref, f"own {kw}")
        got = c.path_plan(aos_gpu.path_query(**kw), graph=gg, skeleton=f["d_skeleton"], info=grid, on_device=True)
        assert_path_equal(got, ref, f"device skeleton {kw}")
    c.seedgen(cloud)
    with pytest.raises(RuntimeError, match="replaced by a later seed-gen frame"):
        c.path_plan(aos_gpu.path_query(target=0))
    c.close()
