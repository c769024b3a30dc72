"""Parameter sweep: seeded random node parameters (ROR radius / min neighbours, PassThrough z range,
inflation radius, cluster_min_length, grid resolution, markers rectangle mode, dense / non-dense) and a jittered exploration
polygon on a C0-size cloud, each full frame (seed-gen a1-a16 + GVD g1-g9 + markers) bit-exact against
the oracle run with the same parameters. The other parity tests fix the node's defaults except the
resolution; this covers the parameter space the reference's YAML exposes."""
import numpy as np
import pytest

import aos_gpu
import oracle_py as O
import orchard
from parity_util import assert_gvd_parity, assert_seedgen_parity

pytestmark = pytest.mark.gpu

# field name in aos_params -> in the oracle's params
_ORACLE_NAME = {"clipping_minz": "clip_minz", "clipping_maxz": "clip_maxz"}


def case(seed: int):
    rng = np.random.default_rng(1000 + seed)
    kw = {
        "ror_radius": float(rng.choice([0.12, 0.2, 0.3])),
        "ror_min_neighbors": int(rng.choice([1, 2, 4, 6])),
        "inflation_radius": float(np.float32(rng.choice([0.4, 0.8, 1.2]))),
        "cluster_min_length": float(rng.choice([1.0, 2.0, 3.5])),
        "grid_resolution": float(np.float32(rng.choice([0.1, 0.15, 0.2, 0.25]))),
        "subdiv_rect_mode": int(rng.integers(0, 2)),
    }
    kw["clipping_minz"], kw["clipping_maxz"] = [(-0.4, 0.5), (-0.2, 0.3), (-1.0, 1.0)][int(rng.integers(0, 3))]
    poly = orchard.polygon(orchard.CONFIGS["C0"]) + rng.uniform(-3.0, 3.0, size=(4, 2))
    dense = bool(rng.integers(0, 4))   # a quarter of the cases: is_dense = false (PCL's radius-search branch)
    return kw, poly, dense


@pytest.mark.parametrize("seed", range(24))
def test_random_parameters_full_frame(seed):
    kw, poly, dense = case(seed)
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg, seed=20 + seed)
    c = aos_gpu.Ctx(aos_gpu.default_params(**kw))
    c.set_polygon(poly)
    g = c.seedgen(cloud, is_dense=dense)
    okw = {_ORACLE_NAME.get(k, k): v for k, v in kw.items()}
    o = O.seedgen(cloud, poly, O.default_params(**okw), is_dense=dense)
    assert_seedgen_parity(g, o)
    gg = c.gvd_from_seedgen()
    og = O.gvd(o["voronoi_seeds"], o["rows_info"], o, O.default_params(markers=1, **okw))
    assert_gvd_parity(gg, og)
    if og["published"]:
        m = c.gvd_markers()
        assert np.array_equal(m["seeds"], og["merged"])
        assert np.array_equal(m["cell_offsets"], og["cell_offsets"]) and np.array_equal(m["cell_xy"], og["cell_xy"])
    c.close()


@pytest.mark.parametrize("seed", range(6))
def test_random_parameters_stream(seed):
    """The streaming map (aos_map_append) under the same random parameters: its incremental
    ROR (tile store, kept marks, stored neighbour counts of the big tiles) and every later stage must equal
    the oracle's full reprocessing of the concatenated scans after every append."""
    kw, _, dense = case(100 + seed)
    kw["grid_resolution"] = 0.1   # (C1's grid)
    cfg = orchard.CONFIGS["C1"]
    poly = orchard.polygon(cfg)
    rng = np.random.default_rng(seed)
    poses = sorted(int(k) for k in rng.integers(0, 400, size=4))
    scans = [orchard.generate_scan(cfg, k, n_points=int(rng.integers(60_000, 200_000))) for k in poses]
    okw = {_ORACLE_NAME.get(k, k): v for k, v in kw.items()}
    s = aos_gpu.Ctx(aos_gpu.default_params(**kw))
    s.set_polygon(poly)
    s.map_reset(reserve_points=100_000)
    for k in range(len(scans)):
        g = s.map_append(scans[k], is_dense=dense)
        full = np.concatenate(scans[:k + 1])
        o = O.seedgen(full, poly, O.default_params(**okw), is_dense=dense)
        assert_seedgen_parity(g, o)
        assert g["n_clipped"] == o["n_clipped"] and g["n_input"] == o["n_input"] == full.shape[0]
        gg = s.gvd_from_seedgen()
        assert_gvd_parity(gg, O.gvd(o["voronoi_seeds"], o["rows_info"], o, O.default_params(**okw)))
    s.close()


@pytest.mark.parametrize("seed", range(6))
def test_random_parameters_tiled(seed):
    """The tiled frame (halo exchange, distributed cluster labelling and numbering, BFS
    replays split over the ranks) under random parameters, tilings and roots (ranks as threads on one
    GPU, aos_group_*): the root's frame and graph bit-exact vs the oracle."""
    import aos_tiles as T
    kw, poly, dense = case(200 + seed)
    kw["grid_resolution"] = float(np.float32([0.1, 0.15, 0.2][seed % 3]))
    rng = np.random.default_rng(300 + seed)
    tiles = [(2, 1), (1, 2), (2, 2), (3, 1), (4, 2), (2, 3)][seed]
    world = tiles[0] * tiles[1]
    root = int(rng.integers(0, world))
    cfg = orchard.CONFIGS["C1"]
    cloud = orchard.generate(cfg, seed=40 + seed, n_points=600_000)
    poly = orchard.polygon(cfg) + rng.uniform(-4.0, 4.0, size=(4, 2))
    grp = aos_gpu.Group(aos_gpu.default_params(**kw), [0] * world, *tiles)
    grp.set_polygon(poly)
    parts = [T.shard(cloud, grp.plan(r)["points_box"]) for r in range(world)]
    g = grp.process(parts, root=root, is_dense=dense)
    gg = grp.rank(root).gvd_from_seedgen()
    grp.close()
    okw = {_ORACLE_NAME.get(k, k): v for k, v in kw.items()}
    o = O.seedgen(cloud, poly, O.default_params(**okw), is_dense=dense)
    assert_seedgen_parity(g, o)
    assert g["n_clipped"] == o["n_clipped"]
    assert_gvd_parity(gg, O.gvd(o["voronoi_seeds"], o["rows_info"], o, O.default_params(**okw)))


@pytest.mark.parametrize("seed", range(6))
def test_random_parameters_path_queries(seed):
    """aos_path_plan on the graph of a random-parameter frame, for 24 seeded node states
    (targets in and out of range, previous waypoints, robot positions, the initial waypoint, saved targets,
    exploration completed): every output field bit-exact vs the oracle's aos_path_gen_node."""
    from test_gpu_path import assert_path_equal
    kw, poly, dense = case(400 + seed)
    cfg = orchard.CONFIGS["C0"] if seed % 2 else orchard.CONFIGS["C1"]
    cloud = orchard.generate(cfg, seed=60 + seed, n_points=None if seed % 2 else 800_000)
    if not seed % 2:
        kw["grid_resolution"] = 0.1
    c = aos_gpu.Ctx(aos_gpu.default_params(**kw))
    c.set_polygon(poly if seed % 2 else orchard.polygon(cfg))
    f = c.seedgen(cloud, is_dense=dense)
    gg = c.gvd_from_seedgen()
    grid = {"origin": f["origin"], "resolution": f["resolution"], "width": f["width"], "height": f["height"],
            "skeleton_framed": f["skeleton_framed"]}
    n_wp = len(O.path_plan(gg, grid, target=0)["waypoints"])
    rng = np.random.default_rng(500 + seed)
    W, H = f["width"] * f["resolution"], f["height"] * f["resolution"]
    ox, oy = f["origin"]
    for i in range(24):
        q = {"target": int(rng.integers(-1, n_wp + 3)), "previous": int(rng.integers(-1, n_wp + 1))}
        if rng.random() < 0.3:
            q["current"] = (float(ox + rng.uniform(0, W)), float(oy + rng.uniform(0, H)))
        if rng.random() < 0.2:
            q["initial_waypoint_reached"] = False
            q["initial_waypoint"] = (float(ox + rng.uniform(0, W)), float(oy + rng.uniform(0, H)))
        if rng.random() < 0.2:
            q["saved_target"] = (float(ox + rng.uniform(0, W)), float(oy + rng.uniform(0, H)))
        if rng.random() < 0.15:
            q["exploration_completed"] = True
        ref = O.path_plan(gg, grid, **q)
        assert_path_equal(c.path_plan(aos_gpu.path_query(**q)), ref, f"{seed}/{i} {q}")
    c.close()
