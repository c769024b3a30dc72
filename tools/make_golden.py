"""Generate the committed golden fixtures under tests/golden/ from the oracle (test infrastructure).

The reference holds no fixtures for this path and cannot run here, so these vectors
freeze the oracle's outputs. The oracle itself is pinned by hand-derived known-answer tests and
scipy cross-checks (parity unpinned against the reference binary). They serve as:
  * regression pins for the oracle (tests/test_golden.py, CPU);
  * a second, oracle-free reference for the GPU parity tests (tests/test_gpu_parity.py).

Files:
  c0_seedgen.npz / c0_gvd.npz  config C0 (100 k points, 512^2 @ 0.2 m): every output, grids bit-packed
  c1_sha256.json               config C1 (2 M points, 2048^2 @ 0.1 m): SHA-256 of every output array
  c2_sha256.json               config C2 (10 M points, 4096^2 @ 0.1 m, the bench frame), with --c2
  c3_sha256.json               config C3 (40 M points, 8192^2 @ 0.1 m, the tiled config), with --c3
  c4_stream_sha256.json        config C4 (BASELINE configs[4]): the C2 map plus the scans
                               orchard.generate_scan(C2, 40 k), k = 0..n-1, after n = 5 and n = 20 scans
                               (the accumulated 15 M / 30 M-point clouds), with --c4
  subdiv_kat.npz               Subdiv2D micro known-answer cases: co-circular, collinear, duplicate,
                               near-duplicate and on-edge seeds (Voronoi facets per real vertex, both
                               rect modes)

usage: python tools/make_golden.py [--skip-c1] [--c2] [--c3] [--only-big]
"""
import argparse
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import oracle_py as O  # noqa: E402
import orchard  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
GRIDS = ("raster", "inflated", "occupancy", "opened", "skeleton", "skeleton_framed")
SEED_KEYS = ("cluster_offsets", "cluster_cells", "cluster_center", "cluster_length", "row_center", "row_start",
             "row_end", "row_length", "virtual_seeds", "ray_seeds", "endpoint_seeds", "voronoi_seeds", "rows_info",
             "cluster_info")
GVD_KEYS = ("merged", "vor_edges", "boundary_raw", "nodes", "node_labels", "node_cluster_indices", "node_label_counts",
            "node_label_clusters", "node_label_types", "edges", "edge_lengths", "edge_clearances", "row_label_pts",
            "row_label_valid")


def run(name):
    cfg = orchard.CONFIGS[name]
    cloud = orchard.generate(cfg)
    poly = orchard.polygon(cfg)
    p = O.default_params(grid_resolution=cfg.res)
    s = O.seedgen(cloud, poly, p)
    g = O.gvd(s["voronoi_seeds"], s["rows_info"], s, p)
    return s, g


def pack(grid):
    return np.packbits((np.asarray(grid) != 0).reshape(-1))


def sha(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.dtype.str.encode() + str(a.shape).encode() + a.tobytes()).hexdigest()


def subdiv_cases():
    """Degenerate Subdiv2D inputs (voronoi_diagram.cpp:63-94 path) as (seeds, bounds)."""
    sq = [(1.0, 1.0), (3.0, 1.0), (3.0, 3.0), (1.0, 3.0)]                       # 4 co-circular
    grid = [(float(x), float(y)) for y in range(4) for x in range(4)]            # many co-circular
    line = [(0.5 * i, 2.0) for i in range(8)]                                    # collinear
    dup = [(1.0, 1.0), (2.0, 1.5), (1.0, 1.0), (1.0 + 1e-8, 1.0), (3.0, 2.0)]    # duplicate / within FLT_EPSILON
    on_edge = [(0.0, 0.0), (4.0, 0.0), (2.0, 3.0), (2.0, 0.0), (1.0, 1.5)]       # later points on earlier edges
    hexa = [(np.cos(k * np.pi / 3), np.sin(k * np.pi / 3)) for k in range(6)] + [(0.0, 0.0)]
    return {"cocircular4": (sq, (0.0, 4.0, 0.0, 4.0)), "grid16": (grid, (-1.0, 4.0, -1.0, 4.0)),
            "collinear8": (line, (0.0, 4.0, 0.0, 4.0)), "duplicates": (dup, (0.0, 4.0, 0.0, 4.0)),
            "on_edge": (on_edge, (-1.0, 5.0, -1.0, 4.0)), "hexagon": (hexa, (-2.0, 2.0, -2.0, 2.0))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-c1", action="store_true")
    ap.add_argument("--c2", action="store_true", help="also hash config C2 (the bench frame; ~2-3 min of oracle time)")
    ap.add_argument("--c3", action="store_true", help="also hash config C3 (8192^2, 40 M points; ~30+ min of oracle time)")
    ap.add_argument("--c4", action="store_true", help="also hash the C4 stream frames after 5 and 20 scans")
    ap.add_argument("--only-big", action="store_true", help="skip C0 / KAT / C1 and write only the --c2 / --c3 / --c4 hashes")
    a = ap.parse_args()
    os.makedirs(GOLD, exist_ok=True)
    if a.only_big:
        a.skip_c1 = True
    else:
        small_fixtures()
    for name, want in (("C1", not a.skip_c1), ("C2", a.c2), ("C3", a.c3)):
        if not want:
            continue
        s1, g1 = run(name)
        h = frame_hashes(s1, g1)
        json.dump(h, open(os.path.join(GOLD, f"{name.lower()}_sha256.json"), "w"), indent=1, sort_keys=True)
        print(name, "hashed", flush=True)
    if a.c4:
        stream_hashes()
    print("golden fixtures written to", GOLD)


def frame_hashes(s1, g1):
    h = {"meta": {k: s1[k] for k in ("width", "height", "thin_iters", "n_input", "n_ror_kept", "n_clipped")}}
    h["seedgen"] = {k: sha(s1[k]) for k in GRIDS + SEED_KEYS}
    h["gvd"] = {k: sha(g1[k]) for k in GVD_KEYS}
    return h


def stream_hashes(counts=(5, 20)):
    """C4: the C2 map followed by scans generate_scan(C2, 40 k); the oracle reprocesses the whole
    accumulated cloud, as the reference's globalMapCallback does (seed_gen:230-248)."""
    cfg = orchard.CONFIGS["C2"]
    poly = orchard.polygon(cfg)
    p = O.default_params(grid_resolution=cfg.res)
    parts = [orchard.generate(cfg)]
    out = {"sequence": "C2 map, then orchard.generate_scan(C2, 40 * k) for k = 0 .. n - 1"}
    for k in range(max(counts)):
        parts.append(orchard.generate_scan(cfg, 40 * k))
        if k + 1 in counts:
            cloud = np.concatenate(parts)
            s1 = O.seedgen(cloud, poly, p)
            g1 = O.gvd(s1["voronoi_seeds"], s1["rows_info"], s1, p)
            out[f"scans_{k + 1}"] = frame_hashes(s1, g1)
            print("C4 after", k + 1, "scans hashed", flush=True)
    json.dump(out, open(os.path.join(GOLD, "c4_stream_sha256.json"), "w"), indent=1, sort_keys=True)


def small_fixtures():
    s, g = run("C0")
    meta = {k: s[k] for k in ("width", "height", "thin_iters", "n_input", "n_ror_kept", "n_clipped")}
    np.savez_compressed(os.path.join(GOLD, "c0_seedgen.npz"), origin=np.array(s["origin"]),
                        resolution=np.float32(s["resolution"]), meta=json.dumps(meta),
                        **{f"grid_{k}": pack(s[k]) for k in GRIDS}, **{k: s[k] for k in SEED_KEYS})
    np.savez_compressed(os.path.join(GOLD, "c0_gvd.npz"), published=np.int32(g["published"]),
                        **{k: g[k] for k in GVD_KEYS})
    kat = {}
    for name, (pts, b) in subdiv_cases().items():
        pts = np.asarray(pts, dtype=np.float64)
        kat[f"{name}_seeds"] = pts
        kat[f"{name}_bounds"] = np.asarray(b, dtype=np.float64)
        for mode in (0, 1):
            facets, centers = O.subdiv_facets(pts, b, rect_mode=mode)
            kat[f"{name}_m{mode}_facet_off"] = np.cumsum([0] + [len(f) for f in facets]).astype(np.int32)
            kat[f"{name}_m{mode}_facet_pts"] = (np.concatenate(facets) if facets else np.zeros((0, 2))).astype(np.float32)
            kat[f"{name}_m{mode}_centers"] = np.asarray(centers, dtype=np.float32)
    np.savez_compressed(os.path.join(GOLD, "subdiv_kat.npz"), **kat)


if __name__ == "__main__":
    main()
