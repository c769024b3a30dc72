"""ctypes binding of libaos_gpu.so (include/aos_gpu.h) — the MI355X seed-gen + GVD hot path.

Mirrors the reference nodes' interface (AosSeedGenNode / AosGvdNode callbacks) for Python
harnesses (tests, bench). There is no fallback: if libaos_gpu.so is missing or no gfx950 device
is visible, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np



def disable_numpy_hugepage() -> bool:
    """Turn off numpy's madvise(MADV_HUGEPAGE) of allocations >= 4 MB for this process.

    Copying the /gvd/markers arrays out of the library into fresh numpy arrays stalled the next GPU
    synchronisation of the process by 10-30 ms (measured on the MI355X box: profiles/r03d_stream*.json
    with the copies, r03f with the switch), most likely the transparent-huge-page work on
    those pages invalidating the device's view of the address space. This changes numpy's behaviour for
    every user in the process, so it is opt-in: the bench (a long-running loop that copies the markers)
    calls it; importing the binding does not. Returns whether the switch exists in this numpy.
    """
    try:
        core = getattr(np, "_core", None) or getattr(np, "core", None)
        mod = getattr(core, "multiarray", None)
        fn = getattr(mod, "_set_madvise_hugepage", None)
        if fn is None:
            return False
        fn(False)
        return True
    except Exception:  # a private numpy API: absent or changed -> leave numpy's default
        return False


HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# AOS_GPU_LIB: alternative build of the same library (A/B experiments, tools/)
LIB_PATH = os.environ.get("AOS_GPU_LIB") or os.path.join(HERE, "libaos_gpu.so")
HEADER = os.path.join(ROOT, "include", "aos_gpu.h")

c_f, c_d, c_i, c_u, c_u64, c_vp = (ctypes.c_float, ctypes.c_double, ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64,
                                   ctypes.c_void_p)
P = ctypes.POINTER


class Params(ctypes.Structure):
    _fields_ = [("clipping_minz", c_f), ("clipping_maxz", c_f), ("clipping_minx", c_f), ("clipping_maxx", c_f),
                ("clipping_miny", c_f), ("clipping_maxy", c_f), ("grid_resolution", c_f), ("inflation_radius", c_f),
                ("cluster_min_length", c_d), ("ror_radius", c_d), ("ror_min_neighbors", c_i),
                ("subdiv_rect_mode", c_i), ("max_graph_publish_rate", c_d), ("gvd_markers", c_i), ("thin_graph", c_i),
                ("gvd_count_evals", c_i)]


class GvdEvals(ctypes.Structure):
    _fields_ = [("counted", c_i), ("n_label_jobs", c_i), ("edge_ends", c_u64), ("boundary_points", c_u64),
                ("filtered_nodes", c_u64), ("ref_nearest", c_u64), ("ref_pairs", c_u64), ("ref_labels", c_u64),
                ("gpu_nearest", c_u64), ("gpu_pairs", c_u64), ("gpu_samples", c_u64), ("gpu_labels", c_u64)]


class GvdMarkers(ctypes.Structure):
    _fields_ = [("n_seeds", c_i), ("seeds_xy", P(c_d)), ("n_rows", c_i), ("row_label_xy", P(c_d)),
                ("row_label_valid", P(c_i)), ("n_cells", c_i), ("cell_offsets", P(c_i)), ("cell_xy", P(c_d)),
                ("cell_center_xy", P(c_d)), ("cell_rgba", P(c_f)), ("ms_cells", c_f)]


class CloudView(ctypes.Structure):
    _fields_ = [("data", c_vp), ("n_points", c_u64), ("point_step", c_u), ("off_x", c_u), ("off_y", c_u),
                ("off_z", c_u), ("is_dense", c_i), ("on_device", c_i)]


class GridInfo(ctypes.Structure):
    _fields_ = [("origin_x", c_d), ("origin_y", c_d), ("resolution", c_f), ("width", c_u), ("height", c_u)]


class SeedGenOut(ctypes.Structure):
    _fields_ = [("info", GridInfo), ("thin_iters", c_i), ("n_input", c_u64), ("n_ror_kept", c_u64),
                ("n_clipped", c_u64), ("occupancy", P(ctypes.c_int8)), ("skeleton", P(ctypes.c_int8)),
                ("d_occupancy", c_vp), ("d_skeleton", c_vp), ("n_clusters_all", c_i), ("n_bfs_replayed", c_i),
                ("n_rows", c_i),
                ("row_center", P(c_d)), ("row_start", P(c_d)), ("row_end", P(c_d)), ("row_length", P(c_d)),
                ("n_virtual", c_i), ("n_ray", c_i), ("n_endpoint", c_i), ("n_voronoi", c_i), ("voronoi_xy", P(c_d)),
                ("rows_info_xy", P(c_d)), ("n_cluster_info", c_i), ("cluster_info_xy", P(c_d)),
                ("ms_ror", c_f), ("ms_grid", c_f), ("ms_thin", c_f), ("ms_cluster", c_f), ("ms_seeds", c_f),
                ("ms_total", c_f), ("n_binned", ctypes.c_uint64), ("ms_ror_count", c_f),
                ("ms_ror_bin", c_f), ("ms_ror_scatter", c_f), ("thin_graph", c_i), ("thin_launches", c_i),
                ("n_ror_read", c_u64)]


class GvdIn(ctypes.Structure):
    _fields_ = [("seeds_xy", P(c_d)), ("n_seeds", c_i), ("rows_info_xy", P(c_d)), ("n_rows_poses", c_i),
                ("info", GridInfo), ("skeleton", P(ctypes.c_int8))]


class GvdOut(ctypes.Structure):
    _fields_ = [("published", c_i), ("resolution", c_d), ("origin_x", c_d), ("origin_y", c_d), ("num_nodes", c_i),
                ("num_edges", c_i), ("nodes_xy", P(c_d)), ("node_labels", P(c_i)), ("node_cluster_indices", P(c_i)),
                ("node_label_counts", P(c_i)), ("n_label_entries", c_i), ("node_label_clusters", P(c_i)),
                ("node_label_types", P(c_i)), ("edges", P(c_i)), ("edge_lengths", P(c_f)),
                ("edge_clearances", P(c_f)), ("n_merged_seeds", c_i), ("n_voronoi_edges", c_i),
                ("n_boundary_points", c_i), ("ms_merge", c_f), ("ms_delaunay", c_f), ("ms_graph", c_f),
                ("ms_total", c_f), ("ms_cells", c_f)]


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
                ("poses", P(c_d)), ("trimmed_from", c_i), ("ms_plan", c_f)]


def path_query(initial_waypoint_reached=True, initial_waypoint=(8.0, 0.0), target=-1, saved_target=None, previous=-1,
               current=None, exploration_completed=False) -> PathQuery:
    """aos_path_gen_node state when a graph arrives (aos_path_query)."""
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
    return q


def path_graph(g: dict):
    """aos_path_graph view of a GvdGraph dict (Ctx.gvd / oracle gvd keys); returns (struct, keep-alive)."""
    nodes = np.ascontiguousarray(g["nodes"], dtype=np.float64).reshape(-1)
    arrs = {k: np.ascontiguousarray(g[k], dtype=np.int32).reshape(-1)
            for k in ("node_labels", "node_cluster_indices", "node_label_counts", "node_label_clusters",
                      "node_label_types", "edges")}
    lens = np.ascontiguousarray(g["edge_lengths"], dtype=np.float32).reshape(-1)
    ip = lambda a: a.ctypes.data_as(P(c_i))  # noqa: E731
    s = PathGraph(nodes.size // 2, nodes.ctypes.data_as(P(c_d)), ip(arrs["node_labels"]),
                  ip(arrs["node_cluster_indices"]), ip(arrs["node_label_counts"]), arrs["node_label_clusters"].size,
                  ip(arrs["node_label_clusters"]), ip(arrs["node_label_types"]), arrs["edges"].size // 2,
                  ip(arrs["edges"]), lens.ctypes.data_as(P(c_f)))
    return s, (nodes, arrs, lens)


def _path_dict(o: PathOut) -> dict:
    nc = o.n_clusters
    return {"status": o.status, "target": o.target_waypoint_index, "cluster_index": o.cluster_index,
            "cluster_ids": _arr(o.cluster_ids, nc, np.int32),
            "cluster_nodes": _arr(o.cluster_nodes, 4 * nc, np.int32).reshape(-1, 4),
            "waypoints": _arr(o.waypoints_xy, 2 * o.n_waypoints, np.float64).reshape(-1, 2),
            "waypoint_nodes": _arr(o.waypoint_nodes, o.n_waypoints, np.int32),
            "node_path": _arr(o.node_path, o.n_node_path, np.int32),
            "poses": _arr(o.poses, 4 * o.n_poses, np.float64).reshape(-1, 4),
            "trimmed_from": o.trimmed_from, "ms": o.ms_plan}


AllGatherFn = ctypes.CFUNCTYPE(c_i, c_vp, c_u64)
AllReduceMaxFn = ctypes.CFUNCTYPE(c_i, c_vp, P(c_i), c_i)
AllToAllFn = ctypes.CFUNCTYPE(c_i, c_vp, P(c_u64))


class Comm(ctypes.Structure):
    _fields_ = [("user", c_vp), ("rank", c_i), ("world", c_i), ("send_buf", c_vp), ("recv_buf", c_vp),
                ("buf_bytes", c_u64), ("all_gather", AllGatherFn), ("all_reduce_max", AllReduceMaxFn),
                ("all_to_all", AllToAllFn)]


class TilePlan(ctypes.Structure):
    _fields_ = [("tiles_x", c_i), ("tiles_y", c_i), ("rank", c_i), ("tile_x", c_i), ("tile_y", c_i),
                ("halo_rows", c_i), ("halo_words", c_i), ("row0", c_i), ("row1", c_i), ("word0", c_i),
                ("word1", c_i), ("win_row0", c_i), ("win_row1", c_i), ("win_word0", c_i), ("win_word1", c_i),
                ("points_box", c_d * 4), ("exchange_bytes", c_u64), ("info", GridInfo)]


class TiledStats(ctypes.Structure):
    _fields_ = [("ms_frame", c_f), ("ms_comm_gather", c_f), ("ms_comm_reduce", c_f), ("n_gather", c_i),
                ("n_reduce", c_i), ("bytes_gather", c_u64), ("ms_ror", c_f), ("ms_thin", c_f), ("ms_cluster", c_f),
                ("ms_seeds", c_f), ("ms_cluster_local", c_f), ("ms_cluster_global", c_f), ("ms_replay", c_f),
                ("n_replayed", c_i), ("ror_skipped", c_i), ("is_root", c_i), ("bytes_recv", c_u64)]


def build() -> str:
    subprocess.check_call(["make", "-s", "-C", HERE, "-j8"])
    return LIB_PATH


def header_functions() -> list[str]:
    """Function names declared in include/aos_gpu.h."""
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(aos_[a-z_]+)\s*\(", txt)))


_lib = None


def lib():
    global _lib
    if _lib is None:
        # torch (if present) bundles its own libamdhip64.so.7; load it first so this library binds
        # to the same HIP runtime (two runtimes in one process break torch's device init).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run `make -C {HERE}` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        L.aos_last_error.restype = ctypes.c_char_p
        L.aos_default_params.argtypes = [P(Params)]
        L.aos_create.argtypes = [P(Params), c_i, P(c_vp)]
        L.aos_destroy.argtypes = [c_vp]
        L.aos_set_polygon.argtypes = [c_vp, c_vp, c_u]
        L.aos_seedgen_process.argtypes = [c_vp, P(CloudView), c_i, P(SeedGenOut)]
        L.aos_seedgen_reprocess.argtypes = [c_vp, c_i, P(SeedGenOut)]
        L.aos_gvd_process.argtypes = [c_vp, P(GvdIn), P(GvdOut)]
        L.aos_gvd_from_seedgen.argtypes = [c_vp, P(GvdOut)]
        L.aos_cloud_prefetch.argtypes = [c_vp, c_vp]
        L.aos_seedgen_grids_copy.argtypes = [c_vp, c_vp, c_vp]
        L.aos_gvd_from_seedgen_async.argtypes = [c_vp]
        L.aos_gvd_wait.argtypes = [c_vp, P(GvdOut)]
        L.aos_gvd_pipeline_depth.argtypes = [c_vp, c_i]
        L.aos_gvd_set_markers.argtypes = [c_vp, c_i]
        L.aos_gvd_set_count_evals.argtypes = [c_vp, c_i]
        L.aos_gvd_evals_get.argtypes = [c_vp, P(GvdEvals)]
        L.aos_rccl_unique_id.argtypes = [c_vp]
        L.aos_rccl_create.argtypes = [c_vp, c_i, c_i, c_i, c_u64, P(c_vp)]
        L.aos_rccl_comm.argtypes = [c_vp]
        L.aos_rccl_comm.restype = c_vp
        L.aos_rccl_destroy.argtypes = [c_vp]
        L.aos_rccl_destroy.restype = None
        L.aos_debug_grid.argtypes = [c_vp, ctypes.c_char_p, c_vp, c_u64]
        L.aos_gvd_markers_get.argtypes = [c_vp, P(GvdMarkers)]
        L.aos_gvd_collected_markers_get.argtypes = [c_vp, P(GvdMarkers)]
        L.aos_map_reset.argtypes = [c_vp, c_u64]
        L.aos_map_append.argtypes = [c_vp, P(CloudView), c_i, P(SeedGenOut)]
        L.aos_tile_plan_compute.argtypes = [P(Params), c_vp, c_u, c_i, c_i, c_i, P(TilePlan)]
        L.aos_tiled_seedgen_process.argtypes = [c_vp, P(Comm), c_i, c_i, c_i, P(CloudView), c_i, P(SeedGenOut)]
        L.aos_tiled_stats_get.argtypes = [c_vp, P(TiledStats)]
        L.aos_path_plan.argtypes = [c_vp, P(PathGraph), c_vp, c_i, P(GridInfo), P(PathQuery), P(PathOut)]
        L.aos_group_create.argtypes = [P(Params), P(c_i), c_i, c_i, P(c_vp)]
        L.aos_group_destroy.argtypes = [c_vp]
        L.aos_group_set_polygon.argtypes = [c_vp, c_vp, c_u]
        L.aos_group_plan.argtypes = [c_vp, c_i, P(TilePlan)]
        L.aos_group_rank.restype = c_vp
        L.aos_group_rank.argtypes = [c_vp, c_i]
        L.aos_group_process.argtypes = [c_vp, P(CloudView), c_i, c_i, P(SeedGenOut)]
        L.aos_group_map_reset.argtypes = [c_vp, c_u64]
        L.aos_group_map_append.argtypes = [c_vp, P(CloudView), c_i, c_i, P(SeedGenOut)]
        L.aos_tiled_map_append.argtypes = [c_vp, P(Comm), c_i, c_i, c_i, P(CloudView), c_i, P(SeedGenOut)]
        L.aos_stream.restype = c_vp
        L.aos_stream.argtypes = [c_vp]
        L.aos_cluster_union.argtypes = [c_i, c_i, c_i, c_vp, c_i, c_vp, c_vp, c_vp, P(c_i)]
        L.aos_debug_scan.argtypes = [c_vp, c_vp, c_vp, c_i, c_i]
        L.aos_debug_faults.restype = None
        L.aos_debug_faults.argtypes = [c_i, c_u64]
        L.aos_debug_replay.restype = None
        L.aos_debug_replay.argtypes = [c_i, c_i, c_i]
        L.aos_replay_counts.argtypes = [c_vp, ctypes.POINTER(ctypes.c_int32)]
        L.aos_comm_init.restype = None
        L.aos_comm_init.argtypes = [c_vp]
        _lib = L
    return _lib


def _check(rc):
    if rc != 0:
        raise RuntimeError(f"libaos_gpu error {rc}: {lib().aos_last_error().decode()}")


def cluster_union(width: int, height: int, piece_root, border_cell, border_root):
    """aos_cluster_union (host code, no GPU): the border union-find of the tiled frame's distributed
    cluster stage. -> (cluster id per piece, clusters numbered in raster order of their first cell; count)."""
    pr = np.ascontiguousarray(piece_root, dtype=np.int32)
    bc = np.ascontiguousarray(border_cell, dtype=np.int32)
    br = np.ascontiguousarray(border_root, dtype=np.int32)
    if bc.shape != br.shape:
        raise ValueError("border_cell and border_root differ in length")
    out = np.empty(pr.size, np.int32)
    n = c_i(0)
    _check(lib().aos_cluster_union(int(width), int(height), pr.size, pr.ctypes.data, bc.size, bc.ctypes.data,
                                   br.ctypes.data, out.ctypes.data, ctypes.byref(n)))
    return out, n.value


def default_params(**kw) -> Params:
    p = Params()
    lib().aos_default_params(ctypes.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _arr(ptr, n, dtype):
    if n <= 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype, copy=True)


def _view_arr(ptr, n, dtype):
    """Zero-copy numpy view of a library-owned output (valid until the next call on the handle)."""
    if n <= 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).view(dtype)


def _seedgen_dict(o: SeedGenOut, want_host: bool, copy_grids: bool = True) -> dict:
    W, H = o.info.width, o.info.height
    nr = o.n_rows
    r = {
        "origin": (o.info.origin_x, o.info.origin_y), "resolution": o.info.resolution, "width": W, "height": H,
        "thin_iters": o.thin_iters, "n_input": o.n_input, "n_clipped": o.n_clipped, "n_clusters_all": o.n_clusters_all,
        "n_bfs_replayed": o.n_bfs_replayed,
        "row_center": _arr(o.row_center, 2 * nr, np.float64).reshape(-1, 2),
        "row_start": _arr(o.row_start, 2 * nr, np.float64).reshape(-1, 2),
        "row_end": _arr(o.row_end, 2 * nr, np.float64).reshape(-1, 2),
        "row_length": _arr(o.row_length, nr, np.float64),
        "n_virtual": o.n_virtual, "n_ray": o.n_ray, "n_endpoint": o.n_endpoint,
        "voronoi_seeds": _arr(o.voronoi_xy, 2 * o.n_voronoi, np.float64).reshape(-1, 2),
        "rows_info": _arr(o.rows_info_xy, 4 * nr, np.float64).reshape(-1, 2),
        "cluster_info": _arr(o.cluster_info_xy, 2 * o.n_cluster_info, np.float64).reshape(-1, 2),
        "d_occupancy": o.d_occupancy, "d_skeleton": o.d_skeleton,
        "ms": {"ror": o.ms_ror, "grid": o.ms_grid, "thin": o.ms_thin, "cluster": o.ms_cluster, "seeds": o.ms_seeds,
               "total": o.ms_total, "ror_count": o.ms_ror_count,
               "ror_bin": o.ms_ror_bin, "ror_scatter": o.ms_ror_scatter},
        "n_binned": o.n_binned, "thin_graph": o.thin_graph, "thin_launches": o.thin_launches, "n_ror_read": o.n_ror_read,
    }
    nv, nrr = o.n_virtual, o.n_ray
    seeds = r["voronoi_seeds"]
    r["virtual_seeds"], r["ray_seeds"], r["endpoint_seeds"] = seeds[:nv], seeds[nv:nv + nrr], seeds[nv + nrr:]
    if want_host:
        grid = _arr if copy_grids else _view_arr
        r["occupancy"] = grid(o.occupancy, W * H, np.int8).reshape(H, W)
        r["skeleton_framed"] = grid(o.skeleton, W * H, np.int8).reshape(H, W)
    return r


def _gvd_dict(o: GvdOut, copy: bool = True) -> dict:
    """copy=False: views of the library-owned arrays, valid until the next call on the handle (the ABI's
    ownership rule; what a node publishing from them sees)."""
    nn, ne = o.num_nodes, o.num_edges
    a = _arr if copy else _view_arr
    return {
        "published": bool(o.published), "resolution": o.resolution, "origin": (o.origin_x, o.origin_y),
        "nodes": a(o.nodes_xy, 2 * nn, np.float64).reshape(-1, 2),
        "node_labels": a(o.node_labels, nn, np.int32),
        "node_cluster_indices": a(o.node_cluster_indices, nn, np.int32),
        "node_label_counts": a(o.node_label_counts, nn, np.int32),
        "node_label_clusters": a(o.node_label_clusters, o.n_label_entries, np.int32),
        "node_label_types": a(o.node_label_types, o.n_label_entries, np.int32),
        "edges": a(o.edges, 2 * ne, np.int32).reshape(-1, 2),
        "edge_lengths": a(o.edge_lengths, ne, np.float32),
        "edge_clearances": a(o.edge_clearances, ne, np.float32),
        "n_merged": o.n_merged_seeds, "n_vor_edges": o.n_voronoi_edges, "n_boundary_raw": o.n_boundary_points,
        "ms": {"merge": o.ms_merge, "delaunay": o.ms_delaunay, "graph": o.ms_graph, "total": o.ms_total,
               "cells": o.ms_cells},
    }


class Ctx:
    """One handle = one GPU + one HIP stream (aos_create)."""

    def __init__(self, params: Params | None = None, device: int = 0):
        self.params = params or default_params()
        h = c_vp()
        _check(lib().aos_create(ctypes.byref(self.params), device, ctypes.byref(h)))
        self.h = h

    @classmethod
    def borrow(cls, handle: int, params: Params | None = None) -> "Ctx":
        """A non-owning view of a handle owned elsewhere (aos_group_rank): close() does not destroy it."""
        c = cls.__new__(cls)
        c.params = params or default_params()
        c.h = c_vp(handle)
        c._borrowed = True
        return c

    def close(self):
        if self.h:
            if not getattr(self, "_borrowed", False):
                lib().aos_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_polygon(self, poly_xy: np.ndarray):
        a = np.ascontiguousarray(poly_xy, dtype=np.float64).reshape(-1)
        _check(lib().aos_set_polygon(self.h, a.ctypes.data, a.size // 2))

    @staticmethod
    def _view(cloud, n_points, point_step, offs, is_dense, on_device):
        """(CloudView, keep-alive): cloud is a (n, point_step) uint8 array or, with on_device, a device pointer."""
        if on_device:
            ptr, n = int(cloud), int(n_points)
        else:
            cloud = np.ascontiguousarray(cloud)
            ptr = cloud.ctypes.data
            n = cloud.shape[0] if cloud.ndim == 2 else cloud.size // point_step
        return CloudView(ptr, n, point_step, offs[0], offs[1], offs[2], int(is_dense), int(on_device)), cloud

    def seedgen(self, cloud, n_points: int | None = None, point_step=16, offs=(0, 4, 8), is_dense=True,
                on_device=False, want_host=True, copy_grids=True) -> dict:
        """cloud: (n, point_step) uint8 numpy array, or an int device pointer with on_device=True.
        copy_grids=False returns the two OccupancyGrids as views of the library's pinned host buffers
        (the ABI's ownership rule: valid until the next call on this handle)."""
        v, _keep = self._view(cloud, n_points, point_step, offs, is_dense, on_device)
        o = SeedGenOut()
        _check(lib().aos_seedgen_process(self.h, ctypes.byref(v), int(want_host), ctypes.byref(o)))
        return _seedgen_dict(o, want_host, copy_grids)

    def map_reset(self, reserve_points: int = 0):
        """Empty the device-resident streaming map (aos_map_reset)."""
        _check(lib().aos_map_reset(self.h, int(reserve_points)))

    def map_append(self, scan, n_points: int | None = None, point_step=16, offs=(0, 4, 8), is_dense=True,
                   on_device=False, want_host=True) -> dict:
        """Append one scan to the streaming map and process the whole map (aos_map_append)."""
        v, _keep = self._view(scan, n_points, point_step, offs, is_dense, on_device)
        o = SeedGenOut()
        _check(lib().aos_map_append(self.h, ctypes.byref(v), int(want_host), ctypes.byref(o)))
        return _seedgen_dict(o, want_host)

    def tiled_stats(self) -> dict:
        """Where this rank's last tiled frame spent its time (aos_tiled_stats_get)."""
        t = TiledStats()
        _check(lib().aos_tiled_stats_get(self.h, ctypes.byref(t)))
        return {name: getattr(t, name) for name, _ in TiledStats._fields_}

    def _tiled_result(self, o, is_root: bool, want_host: bool) -> dict:
        if is_root:
            return {**_seedgen_dict(o, want_host), "root": True, "tiled_stats": self.tiled_stats()}
        return {"root": False, "width": o.info.width, "height": o.info.height, "thin_iters": o.thin_iters,
                "n_clipped": o.n_clipped, "n_input": o.n_input, "n_binned": o.n_binned, "n_ror_read": o.n_ror_read,
                "ms": {"ror": o.ms_ror, "grid": o.ms_grid, "thin": o.ms_thin, "total": o.ms_total,
                       "ror_count": o.ms_ror_count, "ror_bin": o.ms_ror_bin, "ror_scatter": o.ms_ror_scatter},
                "tiled_stats": self.tiled_stats()}

    def tiled_seedgen(self, comm, tiles_x: int, tiles_y: int, cloud, root: int = 0, n_points: int | None = None,
                      point_step=16, offs=(0, 4, 8), is_dense=True, on_device=False, want_host=True) -> dict:
        """One tiled frame on this rank (aos_tiled_seedgen_process); comm: a TorchDistComm / ThreadGroup comm.
        The root gets the whole frame; other ranks get the map info, T, n_clipped and their timings."""
        v, _keep = self._view(cloud, n_points, point_step, offs, is_dense, on_device)
        o = SeedGenOut()
        comm.error = None
        rc = lib().aos_tiled_seedgen_process(self.h, ctypes.byref(comm.c), tiles_x, tiles_y, root, ctypes.byref(v),
                                             int(want_host), ctypes.byref(o))
        if comm.error is not None:
            raise RuntimeError(f"communicator failed: {comm.error!r}") from comm.error
        _check(rc)
        return self._tiled_result(o, comm.rank == root, want_host)

    def tiled_map_append(self, comm, tiles_x: int, tiles_y: int, scan, root: int = 0, n_points: int | None = None,
                         point_step=16, offs=(0, 4, 8), is_dense=True, on_device=False, want_host=True) -> dict:
        """Append a scan to this rank's tiled streaming map (its points box) and run the tiled frame on it
        (aos_tiled_map_append). Returns like tiled_seedgen."""
        v, _keep = self._view(scan, n_points, point_step, offs, is_dense, on_device)
        o = SeedGenOut()
        comm.error = None
        rc = lib().aos_tiled_map_append(self.h, ctypes.byref(comm.c), tiles_x, tiles_y, root, ctypes.byref(v),
                                        int(want_host), ctypes.byref(o))
        if comm.error is not None:
            raise RuntimeError(f"communicator failed: {comm.error!r}") from comm.error
        _check(rc)
        return self._tiled_result(o, comm.rank == root, want_host)

    def reprocess(self, want_host=True) -> dict:
        o = SeedGenOut()
        _check(lib().aos_seedgen_reprocess(self.h, int(want_host), ctypes.byref(o)))
        return _seedgen_dict(o, want_host)

    def gvd_from_seedgen(self, copy: bool = True) -> dict:
        o = GvdOut()
        _check(lib().aos_gvd_from_seedgen(self.h, ctypes.byref(o)))
        return _gvd_dict(o, copy)

    def path_plan(self, query: PathQuery | None = None, graph: dict | None = None, skeleton=None, info: dict | None = None,
                  on_device: bool = False) -> dict:
        """aos_path_gen_node graphCallback + planAndPublishPath (aos_path_plan). graph None: this
        handle's last GVD graph; skeleton None: the skeleton that graph was built on."""
        q = query if query is not None else path_query()
        gs, keep = path_graph(graph) if graph is not None else (None, None)
        gi, sk = None, None
        if skeleton is not None:
            gi = GridInfo(info["origin"][0], info["origin"][1], info["resolution"], info["width"], info["height"])
            if on_device:
                sk = c_vp(int(skeleton))
            else:
                keep = (keep, np.ascontiguousarray(skeleton, dtype=np.int8).reshape(-1))
                sk = keep[1].ctypes.data_as(c_vp)
        o = PathOut()
        _check(lib().aos_path_plan(self.h, ctypes.byref(gs) if gs is not None else None, sk, int(on_device),
                                   ctypes.byref(gi) if gi is not None else None, ctypes.byref(q), ctypes.byref(o)))
        del keep
        return _path_dict(o)

    def cloud_prefetch(self, cloud, n_points: int | None = None, point_step=16, offs=(0, 4, 8), is_dense=True) -> None:
        """Start uploading a host PointCloud2 for the next seedgen() of the same array (aos_cloud_prefetch)."""
        v, keep = self._view(cloud, n_points, point_step, offs, is_dense, False)
        self._prefetch_keep = keep
        _check(lib().aos_cloud_prefetch(self.h, ctypes.byref(v)))

    def cloud_prefetch_wait(self) -> None:
        """Wait for the prefetch in flight and drop it (aos_cloud_prefetch(ctx, NULL))."""
        _check(lib().aos_cloud_prefetch(self.h, None))

    def grids_copy(self, shape) -> tuple:
        """The last frame's /occupancy_grid and /skeletonized_occupancy_grid straight from HBM into new
        arrays (aos_seedgen_grids_copy)."""
        occ, skel = np.empty(shape, np.int8), np.empty(shape, np.int8)
        _check(lib().aos_seedgen_grids_copy(self.h, occ.ctypes.data, skel.ctypes.data))
        return occ, skel

    def gvd_async(self) -> None:
        """Start the GVD of the last seed-gen frame in the background (aos_gvd_from_seedgen_async)."""
        _check(lib().aos_gvd_from_seedgen_async(self.h))

    def gvd_set_markers(self, on: bool) -> None:
        """publishMarkers' cells for the following GVD calls (aos_gvd_set_markers); off: on demand."""
        _check(lib().aos_gvd_set_markers(self.h, int(bool(on))))

    def gvd_set_count_evals(self, on: bool) -> None:
        """Count the GVD graph searches' work in the following GVD calls (aos_gvd_set_count_evals)."""
        _check(lib().aos_gvd_set_count_evals(self.h, int(bool(on))))

    def gvd_evals(self) -> dict:
        """SURVEY §8d's pair evaluations of the last counted GVD call (aos_gvd_evals_get): the reference's
        (ref_*) and the GPU kernels' (gpu_*) distance / sample evaluations."""
        e = GvdEvals()
        _check(lib().aos_gvd_evals_get(self.h, ctypes.byref(e)))
        return {k: int(getattr(e, k)) for k, _ in GvdEvals._fields_}

    def gvd_pipeline_depth(self, depth: int) -> None:
        """Up to `depth` background GVD jobs in flight (aos_gvd_pipeline_depth)."""
        _check(lib().aos_gvd_pipeline_depth(self.h, int(depth)))

    def gvd_wait(self, copy: bool = True) -> dict:
        """The graph of the background GVD (aos_gvd_wait)."""
        o = GvdOut()
        _check(lib().aos_gvd_wait(self.h, ctypes.byref(o)))
        return _gvd_dict(o, copy)

    def gvd_markers(self, collected: bool = False, copy: bool = True, view: bool = False) -> dict:
        """/gvd/markers content of the last GVD call (aos_gvd_markers_get); collected=True: of the frame
        last returned by gvd_wait, even with newer jobs in flight (aos_gvd_collected_markers_get).
        view=True: zero-copy views of the library-owned arrays (the ABI's ownership rule: valid until the
        next GVD call on the handle), as seedgen(copy_grids=False) returns the grids.
        copy=False (diagnostic): wait for the cells, return only their counts and time."""
        m = GvdMarkers()
        fn = lib().aos_gvd_collected_markers_get if collected else lib().aos_gvd_markers_get
        _check(fn(self.h, ctypes.byref(m)))
        nc = m.n_cells
        if not copy:
            return {"n_cells": nc, "n_seeds": m.n_seeds, "ms_cells": m.ms_cells}
        get = _view_arr if view else _arr
        off = get(m.cell_offsets, nc + 1, np.int32)
        return {"seeds": get(m.seeds_xy, 2 * m.n_seeds, np.float64).reshape(-1, 2),
                "row_label_pts": get(m.row_label_xy, 8 * m.n_rows, np.float64).reshape(-1, 4, 2),
                "row_label_valid": get(m.row_label_valid, 4 * m.n_rows, np.int32).reshape(-1, 4),
                "cell_offsets": off,
                "cell_xy": get(m.cell_xy, 2 * int(off[-1]) if nc else 0, np.float64).reshape(-1, 2),
                "cell_center": get(m.cell_center_xy, 2 * nc, np.float64).reshape(-1, 2),
                "cell_rgba": get(m.cell_rgba, 4 * nc, np.float32).reshape(-1, 4), "ms_cells": m.ms_cells}

    def gvd(self, seeds, rows_info, grid: dict) -> dict:
        s = np.ascontiguousarray(seeds, dtype=np.float64).reshape(-1)
        r = np.ascontiguousarray(rows_info, dtype=np.float64).reshape(-1)
        sk = np.ascontiguousarray(grid["skeleton_framed"], dtype=np.int8).reshape(-1)
        info = GridInfo(grid["origin"][0], grid["origin"][1], grid["resolution"], grid["width"], grid["height"])
        gi = GvdIn(s.ctypes.data_as(P(c_d)), s.size // 2, r.ctypes.data_as(P(c_d)), r.size // 2, info,
                   sk.ctypes.data_as(P(ctypes.c_int8)))
        o = GvdOut()
        _check(lib().aos_gvd_process(self.h, ctypes.byref(gi), ctypes.byref(o)))
        return _gvd_dict(o)

    def debug_grid(self, which: str, shape) -> np.ndarray:
        out = np.zeros(shape, dtype=np.int8)
        _check(lib().aos_debug_grid(self.h, which.encode(), out.ctypes.data, out.size))
        return out

    def debug_scan(self, d_in: int, d_out: int, n: int, zero_in: bool = False):
        """aos_debug_scan on device pointers: d_out[0..n] = the exclusive prefix sums of d_in[0..n)."""
        _check(lib().aos_debug_scan(self.h, d_in, d_out, int(n), int(zero_in)))

    def replay_counts(self) -> dict:
        """aos_replay_counts: the last seed-gen frame's exact BFS replays, in all and by where they ran."""
        out = (ctypes.c_int32 * 4)()
        _check(lib().aos_replay_counts(self.h, out))
        return {"all": out[0], "gpu": out[1], "host_bits": out[2], "host_cells": out[3]}

    def stream(self) -> int:
        return lib().aos_stream(self.h)


def debug_faults(ror_stuck_rank: int = -1, a2a_round_bytes: int = 0) -> None:
    """aos_debug_faults (test hooks, process-wide): a tiled rank that reports a stuck ROR look-back, and the
    cluster exchange's round-size cap; the defaults turn both off."""
    lib().aos_debug_faults(int(ror_stuck_rank), int(a2a_round_bytes))


def debug_replay(gpu_min_clusters: int = -1, ring_cap: int = 0, replay_all: bool = False) -> None:
    """aos_debug_replay (test hook, process-wide): the flagged-cluster count from which a seed-gen frame replays
    its clusters on the GPU (-1: the library default; 0: always), a smaller queue ring for the GPU walk (0: 64),
    and replay_all: every cluster replayed, certified or not. No arguments: the defaults."""
    lib().aos_debug_replay(int(gpu_min_clusters), int(ring_cap), int(bool(replay_all)))


class Group:
    """One map over several GPUs from one process (aos_group_*): one handle per tile, ranks driven by
    the library's own threads and an in-process communicator (peer copies, host max-reduction)."""

    def __init__(self, params: Params, devices, tiles_x: int, tiles_y: int):
        self.params = params
        self.tiles_x, self.tiles_y = tiles_x, tiles_y
        devices = list(devices)
        if len(devices) != tiles_x * tiles_y:   # aos_group_create reads devices[r] for every rank
            raise ValueError(f"Group: {len(devices)} devices for {tiles_x}x{tiles_y} tiles")
        d = (c_i * len(devices))(*devices)
        h = c_vp()
        _check(lib().aos_group_create(ctypes.byref(params), d, tiles_x, tiles_y, ctypes.byref(h)))
        self.h = h
        self.world = tiles_x * tiles_y

    def set_polygon(self, poly_xy: np.ndarray):
        a = np.ascontiguousarray(poly_xy, dtype=np.float64).reshape(-1)
        _check(lib().aos_group_set_polygon(self.h, a.ctypes.data, a.size // 2))

    def plan(self, rank: int) -> dict:
        t = TilePlan()
        _check(lib().aos_group_plan(self.h, rank, ctypes.byref(t)))
        return {"points_box": tuple(t.points_box), "exchange_bytes": t.exchange_bytes, "row0": t.row0, "row1": t.row1,
                "word0": t.word0, "word1": t.word1}

    def rank(self, r: int) -> Ctx:
        return Ctx.borrow(lib().aos_group_rank(self.h, r), self.params)

    def process(self, clouds, root: int = 0, want_host: bool = True, on_device: bool = False, n_points=None,
                point_step=16, offs=(0, 4, 8), is_dense=True) -> dict:
        """clouds[r]: rank r's points (host (n, point_step) uint8 arrays, or device pointers with
        on_device and n_points[r]). Returns the root's frame."""
        views, keep = [], []
        for r in range(self.world):
            v, k = Ctx._view(clouds[r], None if n_points is None else n_points[r], point_step, offs, is_dense,
                             on_device)
            views.append(v)
            keep.append(k)
        arr = (CloudView * self.world)(*views)
        o = SeedGenOut()
        _check(lib().aos_group_process(self.h, arr, root, int(want_host), ctypes.byref(o)))
        return _seedgen_dict(o, want_host)

    def map_reset(self, reserve_points: int = 0):
        """Empty every rank's tiled streaming map (aos_group_map_reset)."""
        _check(lib().aos_group_map_reset(self.h, int(reserve_points)))

    def map_append(self, scan, root: int = 0, want_host: bool = True, on_device: bool = False, n_points=None,
                   point_step=16, offs=(0, 4, 8), is_dense=True) -> dict:
        """One scan into the tiled streaming map (aos_group_map_append); returns the root's frame."""
        v, _keep = Ctx._view(scan, n_points, point_step, offs, is_dense, on_device)
        o = SeedGenOut()
        _check(lib().aos_group_map_append(self.h, ctypes.byref(v), root, int(want_host), ctypes.byref(o)))
        return _seedgen_dict(o, want_host)

    def close(self):
        if self.h:
            lib().aos_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
