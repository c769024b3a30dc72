"""Shared comparison helpers for GPU-vs-oracle parity (test infrastructure)."""
import numpy as np

SEED_TOL = 1e-6  # north_star: seeds within 1e-6; grids/skeleton/topology bit-exact


def grid_diff(a, b):
    return int(np.count_nonzero(np.asarray(a) != np.asarray(b)))


def assert_seedgen_parity(g: dict, o: dict, check_grids=True):
    assert (g["width"], g["height"]) == (o["width"], o["height"])
    assert g["origin"] == o["origin"] and np.float32(g["resolution"]) == np.float32(o["resolution"])
    if check_grids:
        assert grid_diff(g["occupancy"], o["occupancy"]) == 0, "occupancy grid differs"
        assert grid_diff(g["skeleton_framed"], o["skeleton_framed"]) == 0, "skeleton grid differs"
    assert g["thin_iters"] == o["thin_iters"], (g["thin_iters"], o["thin_iters"])
    assert g["n_clusters_all"] == len(o["cluster_length"])
    assert g["row_center"].shape == o["row_center"].shape, (g["row_center"].shape, o["row_center"].shape)
    for k in ("row_center", "row_start", "row_end", "row_length"):
        assert np.array_equal(g[k], o[k]), k
    for k in ("virtual_seeds", "ray_seeds", "endpoint_seeds", "voronoi_seeds", "rows_info", "cluster_info"):
        assert g[k].shape == o[k].shape, (k, g[k].shape, o[k].shape)
        if g[k].size:
            assert np.max(np.abs(g[k] - o[k])) <= SEED_TOL, k
    # the implementation is bit-exact by construction; report it as well
    return all(np.array_equal(g[k], o[k]) for k in ("voronoi_seeds", "rows_info", "cluster_info"))


def assert_gvd_parity(g: dict, o: dict):
    assert g["published"] == o["published"]
    if not o["published"]:
        return
    assert g["n_merged"] == len(o["merged"]), (g["n_merged"], len(o["merged"]))
    assert g["n_vor_edges"] == len(o["vor_edges"]), (g["n_vor_edges"], len(o["vor_edges"]))
    assert g["n_boundary_raw"] == len(o["boundary_raw"]), (g["n_boundary_raw"], len(o["boundary_raw"]))
    assert g["nodes"].shape == o["nodes"].shape, (g["nodes"].shape, o["nodes"].shape)
    assert np.array_equal(g["nodes"], o["nodes"]), "node coordinates / order differ"
    assert g["edges"].shape == o["edges"].shape, (g["edges"].shape, o["edges"].shape)
    assert np.array_equal(g["edges"], o["edges"]), "edge topology differs"
    assert np.array_equal(g["edge_lengths"], o["edge_lengths"])
    assert np.array_equal(g["edge_clearances"], o["edge_clearances"])
    for k in ("node_labels", "node_cluster_indices", "node_label_counts", "node_label_clusters", "node_label_types"):
        assert np.array_equal(g[k], o[k]), k


def sha_of(a, dt):
    """SHA-256 of an array as tools/make_golden.py hashes it (dtype, shape, bytes)."""
    import hashlib
    a = np.ascontiguousarray(np.asarray(a, dtype=dt))
    return hashlib.sha256(a.dtype.str.encode() + str(a.shape).encode() + a.tobytes()).hexdigest()


def assert_golden_hashes(g: dict, gg: dict, hs: dict, check_grids=True):
    """A GPU frame (seed-gen dict g, GVD dict gg) vs the oracle's SHA-256 fixture hs (make_golden.py)."""
    assert g["thin_iters"] == hs["meta"]["thin_iters"], (g["thin_iters"], hs["meta"]["thin_iters"])
    assert g["n_clipped"] == hs["meta"]["n_clipped"], (g["n_clipped"], hs["meta"]["n_clipped"])
    if check_grids:
        for k in ("occupancy", "skeleton_framed"):
            assert sha_of(g[k], np.int8) == hs["seedgen"][k], k
    for k in ("row_center", "row_start", "row_end", "row_length", "virtual_seeds", "ray_seeds", "endpoint_seeds",
              "voronoi_seeds", "rows_info", "cluster_info"):
        assert sha_of(g[k], np.float64) == hs["seedgen"][k], k
    for k, dt in (("nodes", np.float64), ("edges", np.int32), ("edge_lengths", np.float32),
                  ("edge_clearances", np.float32), ("node_labels", np.int32), ("node_cluster_indices", np.int32),
                  ("node_label_counts", np.int32), ("node_label_clusters", np.int32), ("node_label_types", np.int32)):
        assert sha_of(gg[k], dt) == hs["gvd"][k], k
