"""ctypes binding of the ORACLE (test infrastructure only; see oracle/oracle.h).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")

c_f = ctypes.c_float
c_d = ctypes.c_double
c_i = ctypes.c_int32
c_u = ctypes.c_uint32
c_u64 = ctypes.c_uint64
P = ctypes.POINTER


class Params(ctypes.Structure):
    _fields_ = [("clip_minz", c_f), ("clip_maxz", c_f), ("clip_minx", c_f), ("clip_maxx", c_f),
                ("clip_miny", c_f), ("clip_maxy", c_f), ("grid_resolution", c_f), ("inflation_radius", c_f),
                ("cluster_min_length", c_d), ("ror_radius", c_d), ("ror_min_neighbors", c_i),
                ("subdiv_rect_mode", c_i), ("faithful_dead_work", c_i), ("markers", c_i)]


class SeedGenOut(ctypes.Structure):
    _fields_ = [("origin_x", c_d), ("origin_y", c_d), ("resolution", c_f), ("width", c_u), ("height", c_u),
                ("thin_iters", c_i), ("n_input", c_u64), ("n_ror_kept", c_u64), ("n_clipped", c_u64),
                ("raster", P(ctypes.c_int8)), ("inflated", P(ctypes.c_int8)), ("occupancy", P(ctypes.c_int8)),
                ("opened", P(ctypes.c_uint8)), ("skeleton", P(ctypes.c_int8)), ("skeleton_framed", P(ctypes.c_int8)),
                ("ror_keep", P(ctypes.c_uint8)), ("n_clusters", c_i), ("cluster_offsets", P(c_i)),
                ("cluster_cells", P(c_i)), ("cluster_center", P(c_f)), ("cluster_length", P(c_f)),
                ("n_rows", c_i), ("row_center", P(c_d)), ("row_start", P(c_d)), ("row_end", P(c_d)),
                ("row_length", P(c_d)), ("n_virtual", c_i), ("n_ray", c_i), ("n_endpoint", c_i), ("n_voronoi", c_i),
                ("virtual_xy", P(c_d)), ("ray_xy", P(c_d)), ("endpoint_xy", P(c_d)), ("voronoi_xy", P(c_d)),
                ("rows_info_xy", P(c_d)), ("n_cluster_info", c_i), ("cluster_info_xy", P(c_d))]


class GvdIn(ctypes.Structure):
    _fields_ = [("seeds_xy", P(c_d)), ("n_seeds", c_i), ("rows_info_xy", P(c_d)), ("n_rows_poses", c_i),
                ("origin_x", c_d), ("origin_y", c_d), ("resolution", c_f), ("width", c_u), ("height", c_u),
                ("skeleton", P(ctypes.c_int8))]


class GvdOut(ctypes.Structure):
    _fields_ = [("published", c_i), ("resolution", c_d), ("origin_x", c_d), ("origin_y", c_d),
                ("n_merged", c_i), ("merged_xy", P(c_d)), ("n_vor_edges", c_i), ("vor_edges", P(c_d)),
                ("n_boundary_raw", c_i), ("boundary_raw", P(c_d)), ("n_vertices_dead", c_i),
                ("num_nodes", c_i), ("nodes_xy", P(c_d)), ("node_labels", P(c_i)),
                ("node_cluster_indices", P(c_i)), ("node_label_counts", P(c_i)), ("n_label_entries", c_i),
                ("node_label_clusters", P(c_i)), ("node_label_types", P(c_i)), ("num_edges", c_i),
                ("edges", P(c_i)), ("edge_lengths", P(c_f)), ("edge_clearances", P(c_f)),
                ("n_label_rows", c_i), ("row_label_pts", P(c_d)), ("row_label_valid", P(c_i)),
                ("n_cells", c_i), ("cell_offsets", P(c_i)), ("cell_xy", P(c_d)), ("cell_center_xy", P(c_d)),
                ("cell_rgba", P(c_f))]


class PathGraph(ctypes.Structure):
    _fields_ = [("num_nodes", c_i), ("nodes_xy", P(c_d)), ("node_labels", P(c_i)), ("node_cluster_indices", P(c_i)),
                ("node_label_counts", P(c_i)), ("n_label_entries", c_i), ("node_label_clusters", P(c_i)),
                ("node_label_types", P(c_i)), ("num_edges", c_i), ("edges", P(c_i)), ("edge_lengths", P(c_f))]


class PathQuery(ctypes.Structure):
    _fields_ = [("initial_waypoint_reached", c_i), ("initial_waypoint_xy", c_d * 2), ("target_waypoint_index", c_i),
                ("have_saved_target", c_i), ("saved_target_xy", c_d * 2), ("previous_waypoint_index", c_i),
                ("use_current_position", c_i), ("current_xy", c_d * 2), ("exploration_completed", c_i)]


class PathOut(ctypes.Structure):
    _fields_ = [("status", c_i), ("target_waypoint_index", c_i), ("cluster_index", c_i), ("n_clusters", c_i),
                ("cluster_ids", P(c_i)), ("cluster_nodes", P(c_i)), ("n_waypoints", c_i), ("waypoints_xy", P(c_d)),
                ("waypoint_nodes", P(c_i)), ("n_node_path", c_i), ("node_path", P(c_i)), ("n_poses", c_i),
                ("poses", P(c_d)), ("trimmed_from", c_i)]


def build_lib() -> str:
    srcs = [os.path.join(_HERE, f) for f in ("oracle_seedgen.cpp", "oracle_gvd.cpp", "oracle_path.cpp", "oracle_capi.cpp",
                                               "oracle.h", "oracle_internal.h")]
    if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < max(os.path.getmtime(s) for s in srcs):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build_lib()
        L = ctypes.CDLL(_LIB)
        L.orc_default_params.argtypes = [P(Params)]
        L.orc_seedgen_run.restype = ctypes.c_void_p
        L.orc_seedgen_run.argtypes = [P(Params), ctypes.c_void_p, c_u64, c_u, c_u, c_u, c_u, c_i, ctypes.c_void_p,
                                      c_i, P(SeedGenOut)]
        L.orc_gvd_run.restype = ctypes.c_void_p
        L.orc_gvd_run.argtypes = [P(Params), P(GvdIn), P(GvdOut)]
        L.orc_path_plan.restype = ctypes.c_void_p
        L.orc_path_plan.argtypes = [P(PathGraph), ctypes.c_void_p, c_d, c_d, c_f, c_u, c_u, P(PathQuery), P(PathOut)]
        L.orc_subdiv_state.restype = ctypes.c_void_p
        L.orc_subdiv_state.argtypes = [ctypes.c_void_p, c_i, ctypes.c_void_p, c_i, P(c_i), P(P(c_i)), P(c_i), P(P(c_i)),
                                       P(P(c_i)), P(P(c_f)), P(P(c_i)), P(c_i), P(P(c_i)), P(P(c_f))]
        for f in ("orc_free_seedgen", "orc_free_gvd", "orc_free_facets", "orc_free_path", "orc_free_subdiv_state"):
            getattr(L, f).argtypes = [ctypes.c_void_p]
        L.orc_ror.argtypes = [ctypes.c_void_p, c_u64, c_i, c_d, c_i, ctypes.c_void_p]
        L.orc_inflate.argtypes = [ctypes.c_void_p, c_u, c_u, c_i, ctypes.c_void_p]
        L.orc_open_cross.argtypes = [ctypes.c_void_p, c_u, c_u, ctypes.c_void_p]
        L.orc_thin.restype = c_i
        L.orc_thin.argtypes = [ctypes.c_void_p, c_u, c_u, ctypes.c_void_p]
        L.orc_subdiv_facets.restype = ctypes.c_void_p
        L.orc_subdiv_facets.argtypes = [ctypes.c_void_p, c_i, c_d, c_d, c_d, c_d, c_i, P(c_i), P(P(c_i)),
                                        P(P(c_f)), P(P(c_f))]
        _lib = L
    return _lib


def default_params(**kw) -> Params:
    p = Params()
    lib().orc_default_params(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _arr(ptr, n, dtype):
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


def seedgen(cloud: np.ndarray, polygon: np.ndarray | None, params: Params | None = None, is_dense: bool = True,
            point_step: int = 16, offs=(0, 4, 8)) -> dict:
    """Runs the oracle seed-gen frame; returns a dict of numpy copies."""
    p = params or default_params()
    cloud = np.ascontiguousarray(cloud)
    n = cloud.shape[0] if cloud.ndim == 2 else cloud.size // point_step
    out = SeedGenOut()
    poly = None if polygon is None else np.ascontiguousarray(polygon, dtype=np.float64).reshape(-1)
    h = lib().orc_seedgen_run(ctypes.byref(p), cloud.ctypes.data, n, point_step, offs[0], offs[1], offs[2],
                              int(is_dense), None if poly is None else poly.ctypes.data,
                              0 if poly is None else poly.size // 2, ctypes.byref(out))
    try:
        W, H = out.width, out.height
        C = W * H
        nc = out.n_clusters
        off = _arr(out.cluster_offsets, nc + 1, np.int32)
        r = {
            "origin": (out.origin_x, out.origin_y), "resolution": out.resolution, "width": W, "height": H,
            "thin_iters": out.thin_iters, "n_input": out.n_input, "n_ror_kept": out.n_ror_kept,
            "n_clipped": out.n_clipped,
            "raster": _arr(out.raster, C, np.int8).reshape(H, W),
            "inflated": _arr(out.inflated, C, np.int8).reshape(H, W),
            "occupancy": _arr(out.occupancy, C, np.int8).reshape(H, W),
            "opened": _arr(out.opened, C, np.uint8).reshape(H, W),
            "skeleton": _arr(out.skeleton, C, np.int8).reshape(H, W),
            "skeleton_framed": _arr(out.skeleton_framed, C, np.int8).reshape(H, W),
            "ror_keep": _arr(out.ror_keep, n, np.uint8),
            "cluster_offsets": off,
            "cluster_cells": _arr(out.cluster_cells, 2 * int(off[-1]) if nc else 0, np.int32).reshape(-1, 2),
            "cluster_center": _arr(out.cluster_center, 2 * nc, np.float32).reshape(-1, 2),
            "cluster_length": _arr(out.cluster_length, nc, np.float32),
            "row_center": _arr(out.row_center, 2 * out.n_rows, np.float64).reshape(-1, 2),
            "row_start": _arr(out.row_start, 2 * out.n_rows, np.float64).reshape(-1, 2),
            "row_end": _arr(out.row_end, 2 * out.n_rows, np.float64).reshape(-1, 2),
            "row_length": _arr(out.row_length, out.n_rows, np.float64),
            "virtual_seeds": _arr(out.virtual_xy, 2 * out.n_virtual, np.float64).reshape(-1, 2),
            "ray_seeds": _arr(out.ray_xy, 2 * out.n_ray, np.float64).reshape(-1, 2),
            "endpoint_seeds": _arr(out.endpoint_xy, 2 * out.n_endpoint, np.float64).reshape(-1, 2),
            "voronoi_seeds": _arr(out.voronoi_xy, 2 * out.n_voronoi, np.float64).reshape(-1, 2),
            "rows_info": _arr(out.rows_info_xy, 4 * out.n_rows, np.float64).reshape(-1, 2),
            "cluster_info": _arr(out.cluster_info_xy, 2 * out.n_cluster_info, np.float64).reshape(-1, 2),
        }
    finally:
        lib().orc_free_seedgen(h)
    return r


def gvd(seeds: np.ndarray, rows_info: np.ndarray, grid: dict, params: Params | None = None) -> dict:
    """Runs the oracle GVD on the settled seed-gen state. grid: origin/resolution/width/height/skeleton_framed."""
    p = params or default_params()
    seeds = np.ascontiguousarray(seeds, dtype=np.float64).reshape(-1)
    rows = np.ascontiguousarray(rows_info, dtype=np.float64).reshape(-1)
    sk = np.ascontiguousarray(grid["skeleton_framed"], dtype=np.int8).reshape(-1)
    gin = GvdIn(seeds.ctypes.data_as(P(c_d)), seeds.size // 2, rows.ctypes.data_as(P(c_d)), rows.size // 2,
                grid["origin"][0], grid["origin"][1], grid["resolution"], grid["width"], grid["height"],
                sk.ctypes.data_as(P(ctypes.c_int8)))
    out = GvdOut()
    h = lib().orc_gvd_run(ctypes.byref(p), ctypes.byref(gin), ctypes.byref(out))
    try:
        r = {
            "published": bool(out.published), "resolution": out.resolution, "origin": (out.origin_x, out.origin_y),
            "merged": _arr(out.merged_xy, 2 * out.n_merged, np.float64).reshape(-1, 2),
            "vor_edges": _arr(out.vor_edges, 4 * out.n_vor_edges, np.float64).reshape(-1, 4),
            "boundary_raw": _arr(out.boundary_raw, 2 * out.n_boundary_raw, np.float64).reshape(-1, 2),
            "n_vertices_dead": out.n_vertices_dead,
            "nodes": _arr(out.nodes_xy, 2 * out.num_nodes, np.float64).reshape(-1, 2),
            "node_labels": _arr(out.node_labels, out.num_nodes, np.int32),
            "node_cluster_indices": _arr(out.node_cluster_indices, out.num_nodes, np.int32),
            "node_label_counts": _arr(out.node_label_counts, out.num_nodes, np.int32),
            "node_label_clusters": _arr(out.node_label_clusters, out.n_label_entries, np.int32),
            "node_label_types": _arr(out.node_label_types, out.n_label_entries, np.int32),
            "edges": _arr(out.edges, 2 * out.num_edges, np.int32).reshape(-1, 2),
            "edge_lengths": _arr(out.edge_lengths, out.num_edges, np.float32),
            "edge_clearances": _arr(out.edge_clearances, out.num_edges, np.float32),
            "row_label_pts": _arr(out.row_label_pts, 8 * out.n_label_rows, np.float64).reshape(-1, 4, 2),
            "row_label_valid": _arr(out.row_label_valid, 4 * out.n_label_rows, np.int32).reshape(-1, 4),
        }
        nc = out.n_cells
        off = _arr(out.cell_offsets, nc + 1, np.int32) if nc else np.zeros(1, np.int32)
        r.update(cell_offsets=off, cell_xy=_arr(out.cell_xy, 2 * int(off[-1]), np.float64).reshape(-1, 2),
                 cell_center=_arr(out.cell_center_xy, 2 * nc, np.float64).reshape(-1, 2),
                 cell_rgba=_arr(out.cell_rgba, 4 * nc, np.float32).reshape(-1, 4))
    finally:
        lib().orc_free_gvd(h)
    return r


def ror(xyz: np.ndarray, is_dense=True, radius=0.2, min_pts=2) -> np.ndarray:
    xyz = np.ascontiguousarray(xyz, dtype=np.float32)
    keep = np.zeros(xyz.shape[0], np.uint8)
    lib().orc_ror(xyz.ctypes.data, xyz.shape[0], int(is_dense), radius, min_pts, keep.ctypes.data)
    return keep


def inflate(grid: np.ndarray, cells: int) -> np.ndarray:
    g = np.ascontiguousarray(grid, dtype=np.int8)
    out = np.zeros_like(g)
    lib().orc_inflate(g.ctypes.data, g.shape[1], g.shape[0], cells, out.ctypes.data)
    return out


def open_cross(img01: np.ndarray) -> np.ndarray:
    g = np.ascontiguousarray(img01, dtype=np.uint8)
    out = np.zeros_like(g)
    lib().orc_open_cross(g.ctypes.data, g.shape[1], g.shape[0], out.ctypes.data)
    return out


def thin(img01: np.ndarray):
    g = np.ascontiguousarray(img01, dtype=np.uint8)
    out = np.zeros_like(g)
    it = lib().orc_thin(g.ctypes.data, g.shape[1], g.shape[0], out.ctypes.data)
    return out, it


def subdiv_facets(seeds: np.ndarray, bounds, rect_mode=0):
    s = np.ascontiguousarray(seeds, dtype=np.float64).reshape(-1)
    nf = c_i()
    off = P(c_i)()
    pts = P(c_f)()
    cen = P(c_f)()
    h = lib().orc_subdiv_facets(s.ctypes.data, s.size // 2, bounds[0], bounds[1], bounds[2], bounds[3], rect_mode,
                                ctypes.byref(nf), ctypes.byref(off), ctypes.byref(pts), ctypes.byref(cen))
    try:
        n = nf.value
        o = _arr(off, n + 1, np.int32)
        facets = _arr(pts, 2 * int(o[-1]) if n else 0, np.float32).reshape(-1, 2)
        centers = _arr(cen, 2 * n, np.float32).reshape(-1, 2)
    finally:
        lib().orc_free_facets(h)
    return [facets[o[i]:o[i + 1]] for i in range(n)], centers


def subdiv_state(points, rect, rect_mode=0) -> dict:
    """Test hook: the raw OpenCV-layout state of a Subdiv2D(rect) after inserting `points` (float32 pairs)
    in order: next / pt per quad-edge (pt[1] = pt[3] = 0: before calcVoronoi), firstEdge / type / point per
    vertex, whether each insert succeeded, and getVoronoiFacetList's facets (in vertex order)."""
    xy = np.ascontiguousarray(points, dtype=np.float32).reshape(-1)
    r = np.ascontiguousarray(rect, dtype=np.float32)
    nq, nv, nf = c_i(), c_i(), c_i()
    qe, vf, vt, ins, off = P(c_i)(), P(c_i)(), P(c_i)(), P(c_i)(), P(c_i)()
    vxy, pts = P(c_f)(), P(c_f)()
    h = lib().orc_subdiv_state(xy.ctypes.data, xy.size // 2, r.ctypes.data, rect_mode, ctypes.byref(nq), ctypes.byref(qe),
                               ctypes.byref(nv), ctypes.byref(vf), ctypes.byref(vt), ctypes.byref(vxy), ctypes.byref(ins),
                               ctypes.byref(nf), ctypes.byref(off), ctypes.byref(pts))
    try:
        q = _arr(qe, 8 * nq.value, np.int32)
        o = _arr(off, nf.value + 1, np.int32)
        f = _arr(pts, 2 * int(o[-1]) if nf.value else 0, np.float32).reshape(-1, 2)
        out = {"next": q[:4 * nq.value].reshape(-1, 4), "pt": q[4 * nq.value:].reshape(-1, 4),
               "first_edge": _arr(vf, nv.value, np.int32), "type": _arr(vt, nv.value, np.int32),
               "vxy": _arr(vxy, 2 * nv.value, np.float32).reshape(-1, 2), "inserted": _arr(ins, xy.size // 2, np.int32),
               "facets": [f[o[i]:o[i + 1]] for i in range(nf.value)]}
    finally:
        lib().orc_free_subdiv_state(h)
    return out


def path_plan(graph: dict, grid: dict, initial_waypoint_reached=True, initial_waypoint=(8.0, 0.0), target=-1,
              saved_target=None, previous=-1, current=None, exploration_completed=False) -> dict:
    """aos_path_gen_node graphCallback + planAndPublishPath on a GvdGraph dict and the
    /skeletonized_occupancy_grid (grid: origin/resolution/width/height/skeleton_framed)."""
    nodes = np.ascontiguousarray(graph["nodes"], dtype=np.float64).reshape(-1)
    a = {k: np.ascontiguousarray(graph[k], dtype=np.int32).reshape(-1)
         for k in ("node_labels", "node_cluster_indices", "node_label_counts", "node_label_clusters",
                   "node_label_types", "edges")}
    lens = np.ascontiguousarray(graph["edge_lengths"], dtype=np.float32).reshape(-1)
    ip = lambda x: x.ctypes.data_as(P(c_i))  # noqa: E731
    g = PathGraph(nodes.size // 2, nodes.ctypes.data_as(P(c_d)), ip(a["node_labels"]), ip(a["node_cluster_indices"]),
                  ip(a["node_label_counts"]), a["node_label_clusters"].size, ip(a["node_label_clusters"]),
                  ip(a["node_label_types"]), a["edges"].size // 2, ip(a["edges"]), lens.ctypes.data_as(P(c_f)))
    q = PathQuery()
    q.initial_waypoint_reached = int(bool(initial_waypoint_reached))
    q.initial_waypoint_xy[:] = list(initial_waypoint)
    q.target_waypoint_index = target
    if saved_target is not None:
        q.have_saved_target = 1
        q.saved_target_xy[:] = list(saved_target)
    q.previous_waypoint_index = previous
    if current is not None:
        q.use_current_position = 1
        q.current_xy[:] = list(current)
    q.exploration_completed = int(bool(exploration_completed))
    sk = np.ascontiguousarray(grid["skeleton_framed"], dtype=np.int8).reshape(-1)
    out = PathOut()
    h = lib().orc_path_plan(ctypes.byref(g), sk.ctypes.data, grid["origin"][0], grid["origin"][1], grid["resolution"],
                            grid["width"], grid["height"], ctypes.byref(q), ctypes.byref(out))
    try:
        nc = out.n_clusters
        return {"status": out.status, "target": out.target_waypoint_index, "cluster_index": out.cluster_index,
                "cluster_ids": _arr(out.cluster_ids, nc, np.int32),
                "cluster_nodes": _arr(out.cluster_nodes, 4 * nc, np.int32).reshape(-1, 4),
                "waypoints": _arr(out.waypoints_xy, 2 * out.n_waypoints, np.float64).reshape(-1, 2),
                "waypoint_nodes": _arr(out.waypoint_nodes, out.n_waypoints, np.int32),
                "node_path": _arr(out.node_path, out.n_node_path, np.int32),
                "poses": _arr(out.poses, 4 * out.n_poses, np.float64).reshape(-1, 4),
                "trimmed_from": out.trimmed_from}
    finally:
        lib().orc_free_path(h)
