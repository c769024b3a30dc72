"""Python front-end of the deterministic synthetic orchard generator (tools/orchard_gen.c).

Configs follow SURVEY.md §8d. Generation is split over threads (ctypes drops the GIL); every
point owns its own SplitMix64 stream, so the bytes do not depend on the thread count.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liborchard_gen.so")


class _Cfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("n_points", ctypes.c_uint64), ("grid_n", ctypes.c_int32),
                ("res", ctypes.c_float), ("max_rows", ctypes.c_int32), ("row_x_end", ctypes.c_double),
                ("outlier_frac", ctypes.c_double)]


@dataclass(frozen=True)
class OrchardConfig:
    name: str
    seed: int
    n_points: int
    grid_n: int
    res: float
    max_rows: int = 0
    row_x_end: float = 0.0
    outlier_frac: float = 0.01


CONFIGS = {
    "C0": OrchardConfig("C0", 1, 100_000, 512, 0.2, max_rows=5, row_x_end=95.0),
    "C1": OrchardConfig("C1", 2, 2_000_000, 2048, 0.1),
    "C2": OrchardConfig("C2", 3, 10_000_000, 4096, 0.1),
    "C3": OrchardConfig("C3", 4, 40_000_000, 8192, 0.1),
}

POINT_STEP = 16
OFF_X, OFF_Y, OFF_Z = 0, 4, 8


def build_lib() -> str:
    src = os.path.join(_HERE, "orchard_gen.c")
    if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-ffp-contract=off", "-shared", "-o", _LIB, src])
    return _LIB


_lib = None


def _load():
    global _lib
    if _lib is None:
        build_lib()
        _lib = ctypes.CDLL(_LIB)
        _lib.orchard_side_length.restype = ctypes.c_float
        _lib.orchard_side_length.argtypes = [ctypes.c_int32, ctypes.c_float]
        _lib.orchard_num_trees.restype = ctypes.c_int64
        _lib.orchard_num_trees.argtypes = [ctypes.POINTER(_Cfg)]
        _lib.orchard_tree_centres.restype = ctypes.c_int64
        _lib.orchard_tree_centres.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        _lib.orchard_polygon.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_void_p]
        _lib.orchard_generate_range.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                                ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        _lib.orchard_generate_scan.argtypes = [ctypes.POINTER(_Cfg), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                               ctypes.c_uint64, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                               ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    return _lib


def _cfg(c: OrchardConfig, seed: int | None = None, n_points: int | None = None) -> _Cfg:
    return _Cfg(c.seed if seed is None else seed, c.n_points if n_points is None else n_points, c.grid_n,
                c.res, c.max_rows, c.row_x_end, c.outlier_frac)


def polygon(c: OrchardConfig) -> np.ndarray:
    lib = _load()
    out = np.zeros(8, dtype=np.float64)
    cfg = _cfg(c)
    lib.orchard_polygon(ctypes.byref(cfg), out.ctypes.data)
    return out.reshape(4, 2)


def generate(c: OrchardConfig, seed: int | None = None, n_points: int | None = None, threads: int = 8) -> np.ndarray:
    """Returns the PointCloud2 data as a (n, 16) uint8 array (x, y, z, intensity float32)."""
    lib = _load()
    cfg = _cfg(c, seed, n_points)
    nt = lib.orchard_num_trees(ctypes.byref(cfg))
    tx = np.zeros(max(nt, 1), np.float64)
    ty = np.zeros(max(nt, 1), np.float64)
    lib.orchard_tree_centres(ctypes.byref(cfg), tx.ctypes.data, ty.ctypes.data, nt)
    n = cfg.n_points
    out = np.empty((n, POINT_STEP), dtype=np.uint8)
    threads = max(1, min(threads, n // 65536 + 1))
    bounds = [n * k // threads for k in range(threads + 1)]

    def work(k):
        lib.orchard_generate_range(ctypes.byref(cfg), tx.ctypes.data, ty.ctypes.data, nt, bounds[k], bounds[k + 1],
                                   out.ctypes.data)

    ts = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out


# ------------------------------------------------------------------ C4 streaming
SCAN_HZ, SPEED, SCAN_R, SCAN_POINTS = 20.0, 1.5, 30.0, 1_000_000


def scan_pose(c: OrchardConfig, k: int) -> tuple[float, float]:
    """Pose of scan k: 1.5 m/s at 20 Hz along a serpentine between the tree rows (lanes at y = 3.75 +
    3.5 j, x from 2 to L - 2 and back)."""
    L = float(_load().orchard_side_length(c.grid_n, c.res))
    run = (L - 2.0) - 2.0
    s = k * SPEED / SCAN_HZ
    lane = int(s // (run + 3.5))
    u = s - lane * (run + 3.5)
    y = 3.75 + 3.5 * lane
    if u > run:                      # turning to the next lane
        return (2.0 + run if lane % 2 == 0 else 2.0), y + (u - run)
    return (2.0 + u if lane % 2 == 0 else 2.0 + run - u), y


def generate_scan(c: OrchardConfig, k: int, n_points: int = SCAN_POINTS, seed: int | None = None,
                  threads: int = 8) -> np.ndarray:
    """Scan k of config c's scene (PointCloud2 bytes, point_step 16): n points within 30 m of scan_pose(k)."""
    lib = _load()
    cfg = _cfg(c, 5 if seed is None else seed, n_points)
    nt = lib.orchard_num_trees(ctypes.byref(cfg))
    tx = np.zeros(max(nt, 1), np.float64)
    ty = np.zeros(max(nt, 1), np.float64)
    lib.orchard_tree_centres(ctypes.byref(cfg), tx.ctypes.data, ty.ctypes.data, nt)
    px, py = scan_pose(c, k)
    near = (tx[:nt] - px) ** 2 + (ty[:nt] - py) ** 2 <= (SCAN_R + 0.5) ** 2
    tx, ty = np.ascontiguousarray(tx[:nt][near]), np.ascontiguousarray(ty[:nt][near])
    out = np.empty((n_points, POINT_STEP), dtype=np.uint8)
    threads = max(1, min(threads, n_points // 65536 + 1))
    bounds = [n_points * j // threads for j in range(threads + 1)]

    def work(j):
        lib.orchard_generate_scan(ctypes.byref(cfg), tx.ctypes.data, ty.ctypes.data, len(tx), k, px, py, SCAN_R,
                                  bounds[j], bounds[j + 1], out.ctypes.data)

    ts = [threading.Thread(target=work, args=(j,)) for j in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out


def xyz(cloud: np.ndarray) -> np.ndarray:
    return cloud.view(np.float32).reshape(-1, 4)[:, :3]
