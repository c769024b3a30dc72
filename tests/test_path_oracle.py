"""Known-answer tests of the oracle's aos_path_gen_node restatement (oracle/oracle_path.cpp),
derived by hand from src/aos_path_gen_node.cpp. CPU only."""
import math

import numpy as np

import oracle_py as O


def graph(nodes, edges, lengths, labels):
    """labels: list of (node, cluster, type) in node order (the new GvdGraph label arrays)."""
    n = len(nodes)
    counts = np.zeros(n, np.int32)
    cl, ty = [], []
    for node, c, t in sorted(labels):
        counts[node] += 1
        cl.append(c)
        ty.append(t)
    return {"nodes": np.array(nodes, np.float64), "node_labels": np.zeros(n, np.int32),
            "node_cluster_indices": np.full(n, -1, np.int32), "node_label_counts": counts,
            "node_label_clusters": np.array(cl, np.int32), "node_label_types": np.array(ty, np.int32),
            "edges": np.array(edges, np.int32).reshape(-1, 2), "edge_lengths": np.array(lengths, np.float32)}


def empty_grid(w=200, h=200, res=0.1, origin=(-5.0, -5.0)):
    return {"origin": origin, "resolution": res, "width": w, "height": h, "skeleton_framed": np.zeros(w * h, np.int8)}


def test_line_graph_path_and_orientations():
    # cluster 0 (even, last, max id even): BR -> BL -> TR (:615-637)
    g = graph([(0, 10), (1, 10), (2, 10), (3, 10)], [0, 1, 1, 2, 2, 3], [1, 1, 1],
              [(3, 0, 3), (0, 0, 2), (1, 0, 1)])
    r = O.path_plan(g, empty_grid(), target=1, previous=0)
    assert r["status"] == 1
    assert r["waypoint_nodes"].tolist() == [3, 0, 1]
    assert r["cluster_ids"].tolist() == [0] and r["cluster_nodes"].tolist() == [[-1, 1, 0, 3]]
    # start = WP[0] = node 3; candidates 3, 2, 1 all cost 3: the first (node 3) wins (strict <)
    assert r["node_path"].tolist() == [3, 2, 1, 0]
    p = r["poses"]
    assert p[:, 0].tolist() == [3.0, 2.0, 1.0, 0.0] and np.all(p[:, 1] == 10.0)
    # each pose faces the next (yaw = pi); the last faces the next waypoint, node 1 (yaw = 0)
    assert np.all(p[:3, 2] == math.sin(math.pi / 2)) and np.all(p[:3, 3] == math.cos(math.pi / 2))
    assert p[3, 2] == 0.0 and p[3, 3] == 1.0
    assert r["trimmed_from"] == -1 and r["cluster_index"] == 0


def test_sequence_two_clusters_and_min_distance():
    # cluster 0 (even): BR, BL; cluster 1 (odd, last, max id odd): TL, TR, BL (:638-661).
    nodes = [(0, 0), (5, 0), (5, 3.5), (0, 3.5), (0.1, 3.5), (9, 9)]
    g = graph(nodes, [0, 1, 1, 2, 2, 3, 3, 4, 0, 3], [5, 3.5, 5, 0.1, 3.5],
              [(1, 0, 3), (0, 0, 2), (3, 1, 0), (2, 1, 1), (4, 1, 2)])
    r = O.path_plan(g, empty_grid(), target=0)
    # BR(1), BL(0), TL(3), TR(2), BL(4): node 4 is 0.1 m from node 3, but the filter compares with
    # the last kept waypoint (node 2, 4.9 m away), so it stays
    assert r["waypoint_nodes"].tolist() == [1, 0, 3, 2, 4]
    # calculateClusterIndex: 2 waypoints for cluster 0, 3 for the last
    assert [O.path_plan(g, empty_grid(), target=t)["cluster_index"] for t in range(5)] == [0, 0, 1, 1, 1]
    # the 0.2 m filter drops a waypoint next to the previous kept one: TL(4), TR(2), BL(3)
    g2 = graph(nodes, [0, 1, 1, 2, 2, 3, 3, 4, 0, 3], [5, 3.5, 5, 0.1, 3.5],
               [(1, 0, 3), (0, 0, 2), (4, 1, 0), (2, 1, 1), (3, 1, 2)])
    assert O.path_plan(g2, empty_grid(), target=0)["waypoint_nodes"].tolist() == [1, 0, 4, 2, 3]
    g3 = graph(nodes, [0, 1], [5], [(1, 0, 3), (0, 0, 2), (3, 1, 0), (4, 1, 1)])
    assert O.path_plan(g3, empty_grid(), target=0)["waypoint_nodes"].tolist() == [1, 0, 3]


def test_initial_straight_line_trimmed():
    # (0, 0) -> (8, 0) in 0.2 m steps (41 poses); a 3 x 3 occupied block, cells x 59-61, y 49-51.
    # OccupancyGrid resolution is float32: res = 0.1f = 0.10000000149, so rc = ceil(0.2 / res) = 2
    # but the dx = 2 samples are 2 res = 0.200000003 > 0.2 away and skipped. Pose 4 (x = 0.8)
    # reaches x = 0.9 only (cell 58); pose 5 (x = 1.0, cell 59) is the first too close, so the
    # path keeps poses 0..4 (:1591-1627).
    grid = empty_grid()
    sk = grid["skeleton_framed"].reshape(200, 200)
    sk[49:52, 59:62] = 100
    r = O.path_plan(graph([(0, 0)], [], [], []), grid, initial_waypoint_reached=False)
    assert r["status"] == 1 and r["trimmed_from"] == 41
    assert r["poses"].shape == (5, 4)
    assert np.allclose(r["poses"][:, 0], [0.0, 0.2, 0.4, 0.6, 0.8], rtol=0, atol=1e-12)
    assert np.all(r["poses"][:, 3] == 1.0) and np.all(r["poses"][:, 2] == 0.0)


def test_failures():
    g = graph([(0, 0), (1, 0)], [0, 1], [1], [(1, 0, 3), (0, 0, 2)])
    assert O.path_plan(g, empty_grid(), target=5)["status"] == 0    # target outside the sequence
    g_none = graph([(0, 0), (1, 0)], [0, 1], [1], [])
    r = O.path_plan(g_none, empty_grid(), target=0)                   # no labels: no waypoints
    assert r["status"] == 0 and r["poses"].shape == (0, 4)
    g_cut = graph([(0, 0), (1, 0), (5, 5)], [0, 1], [1], [(2, 0, 3), (0, 0, 2)])
    # goal node 2 has no edges: every candidate's A* fails (:813-821)
    assert O.path_plan(g_cut, empty_grid(), target=0)["status"] == 0
    # from node 2's position the candidates are 2 (no edges), 1 and 0: 1 -> 0 succeeds
    assert O.path_plan(g_cut, empty_grid(), target=1, previous=0)["node_path"].tolist() == [1, 0]
