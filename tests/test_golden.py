"""The oracle and the product's host Subdiv2D replay against the committed golden fixtures
(tests/golden/, made by tools/make_golden.py). CPU only. The reference holds no fixtures for this
path, so these pin the oracle against regressions. The oracle's own independent pins are
test_oracle_grid.py and test_subdiv_host.py."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_py as O
import orchard
from test_subdiv_host import product_edges

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
GRIDS = ("raster", "inflated", "occupancy", "opened", "skeleton", "skeleton_framed")


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def unpack(bits, h, w):
    return np.unpackbits(bits)[: h * w].reshape(h, w).astype(bool)


def _run(name):
    cfg = orchard.CONFIGS[name]
    cloud = orchard.generate(cfg)
    p = O.default_params(grid_resolution=cfg.res)
    s = O.seedgen(cloud, orchard.polygon(cfg), p)
    return s, O.gvd(s["voronoi_seeds"], s["rows_info"], s, p)


def _sha(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.dtype.str.encode() + str(a.shape).encode() + a.tobytes()).hexdigest()


def test_oracle_c0_matches_golden():
    s, g = _run("C0")
    gs, gg = load("c0_seedgen.npz"), load("c0_gvd.npz")
    meta = json.loads(str(gs["meta"]))
    for k, v in meta.items():
        assert s[k] == v, k
    assert tuple(gs["origin"]) == tuple(s["origin"])
    for k in GRIDS:
        assert np.array_equal(unpack(gs[f"grid_{k}"], meta["height"], meta["width"]), np.asarray(s[k]) != 0), k
    for k in gs.files:
        if k.startswith("grid_") or k in ("meta", "origin", "resolution"):
            continue
        assert np.array_equal(gs[k], s[k]), k
    assert bool(gg["published"]) == g["published"]
    for k in gg.files:
        if k != "published":
            assert np.array_equal(gg[k], g[k]), k


def test_oracle_c1_matches_golden_hashes():
    s, g = _run("C1")
    h = json.load(open(os.path.join(GOLD, "c1_sha256.json")))
    for k, v in h["meta"].items():
        assert s[k] == v, k
    for k, v in h["seedgen"].items():
        assert _sha(s[k]) == v, k
    for k, v in h["gvd"].items():
        assert _sha(g[k]) == v, k


def _kat_names():
    d = load("subdiv_kat.npz")
    return sorted({k[: -len("_seeds")] for k in d.files if k.endswith("_seeds")})


@pytest.mark.parametrize("name", _kat_names())
@pytest.mark.parametrize("mode", [0, 1])
def test_subdiv_known_answers(name, mode):
    d = load("subdiv_kat.npz")
    seeds, b = d[f"{name}_seeds"], tuple(d[f"{name}_bounds"])
    off, pts = d[f"{name}_m{mode}_facet_off"], d[f"{name}_m{mode}_facet_pts"]
    facets, centers = O.subdiv_facets(seeds, b, rect_mode=mode)
    assert len(facets) == len(off) - 1
    for i, f in enumerate(facets):
        assert np.array_equal(f, pts[off[i]:off[i + 1]]), (name, i)
    assert np.array_equal(np.asarray(centers, np.float32), d[f"{name}_m{mode}_centers"])
    # the product's host replay gives the same Voronoi edge list (voronoi_diagram.cpp:97-114)
    want = []
    for i in range(len(off) - 1):
        f = pts[off[i]:off[i + 1]]
        if len(f) >= 2:
            want += [np.concatenate([f[j], f[(j + 1) % len(f)]]) for j in range(len(f))]
    want = np.array(want, np.float32).reshape(-1, 4)
    assert np.array_equal(product_edges(seeds, b, mode), want)
