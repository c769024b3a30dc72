"""Tiled multi-GPU frame on the one GPU of a test box: the tiles of one map run as
threads (aos_tiles.ThreadGroup, one handle + stream each) or as processes over torch.distributed
(gloo). The root's outputs must be byte-identical to the oracle / the single-GPU frame of the whole
cloud, and the GVD graph built from them identical as well."""
import hashlib
import json
import os
import threading

import numpy as np
import pytest

import aos_gpu
import aos_tiles as T
import oracle_py as O
import orchard
from parity_util import assert_gvd_parity, assert_seedgen_parity

pytestmark = pytest.mark.gpu

GVD_KEYS = ("nodes", "edges", "edge_lengths", "edge_clearances", "node_labels", "node_cluster_indices",
            "node_label_counts", "node_label_clusters", "node_label_types")
GRIDS = ("inflated", "skeleton_frameless")


def _single(cloud, poly, res):
    c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=res))
    c.set_polygon(poly)
    g = c.seedgen(cloud)
    g["replay_counts"] = c.replay_counts()
    grids = {w: c.debug_grid(w, (g["height"], g["width"])) for w in GRIDS}
    gg = c.gvd_from_seedgen()
    c.close()
    return g, grids, gg


def _tiled_threads(cloud, poly, res, tiles_x, tiles_y, root, shard=True, a2a=True):
    world = tiles_x * tiles_y
    params = aos_gpu.default_params(grid_resolution=res)
    plans = [T.tile_plan(params, poly, tiles_x, tiles_y, r) for r in range(world)]
    group = T.ThreadGroup(world, timeout=120)
    ctxs = [aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=res)) for _ in range(world)]
    comms = [group.comm(r, plans[r]["exchange_bytes"], "cuda:0") for r in range(world)]
    if not a2a:
        comms = [c.without_all_to_all() for c in comms]
    out, errors = [None] * world, []

    def work(r):
        try:
            ctxs[r].set_polygon(poly)
            part = T.shard(cloud, plans[r]["points_box"]) if shard else cloud
            out[r] = ctxs[r].tiled_seedgen(comms[r], tiles_x, tiles_y, part, root=root)
        except BaseException as e:   # noqa: BLE001
            errors.append(e)
            group.abort()

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    if errors:
        raise errors[0]
    c = ctxs[root]
    g = out[root]
    assert g["root"] and all(not o["root"] for i, o in enumerate(out) if i != root)
    grids = {w: c.debug_grid(w, (g["height"], g["width"])) for w in GRIDS}
    gg = c.gvd_from_seedgen()
    for x in ctxs:
        x.close()
    return g, out, grids, gg


def _assert_same(single, tiled):
    g1, grids1, gg1 = single
    g, out, grids, gg = tiled
    assert_seedgen_parity(g, {**g1, "cluster_length": np.zeros(g1["n_clusters_all"])})
    assert (g["n_clipped"], g["n_bfs_replayed"]) == (g1["n_clipped"], g1["n_bfs_replayed"])
    for w in GRIDS:
        assert np.array_equal(grids[w], grids1[w]), w
    for o in out:
        assert (o["thin_iters"], o["n_clipped"]) == (g1["thin_iters"], g1["n_clipped"])
    assert gg["published"] == gg1["published"]
    for k in GVD_KEYS:
        assert np.array_equal(gg[k], gg1[k]), k


@pytest.mark.parametrize("tiles,root", [((1, 1), 0), ((2, 1), 1), ((1, 2), 0), ((2, 2), 3), ((3, 2), 2)])
def test_tiled_c1_equals_single_gpu(tiles, root):
    cfg = orchard.CONFIGS["C1"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    _assert_same(_single(cloud, poly, cfg.res), _tiled_threads(cloud, poly, cfg.res, *tiles, root))


@pytest.mark.parametrize("mode", ["all_gather", "rounds"])
def test_tiled_c1_cell_exchange_paths(mode):
    """The distributed cluster stage sends each long cluster's cells to its one owner rank. Both other routes
    give the same frame: a communicator without all_to_all (the cells travel by all_gather and each owner
    picks its blocks), and an exchange split into many small rounds (aos_debug_faults)."""
    cfg = orchard.CONFIGS["C1"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    if mode == "rounds":
        aos_gpu.debug_faults(a2a_round_bytes=4096)
    try:
        tiled = _tiled_threads(cloud, poly, cfg.res, 2, 2, 1, a2a=mode != "all_gather")
    finally:
        aos_gpu.debug_faults()
    _assert_same(_single(cloud, poly, cfg.res), tiled)


def test_tiled_rotating_roots_with_background_gvd():
    """The tiled bench's schedule (bench.py --tiled): frame k's root is rank k mod N, and the root starts
    the frame's GVD in the background (aos_gvd_from_seedgen_async) and goes on with the next frames'
    tile stages while it runs. Two C1 scenes alternate over 8 frames on 2 x 2 tiles, so every rank
    finishes two frames of different scenes with both jobs in flight; every graph must equal the
    single-GPU graph of its scene."""
    cfg = orchard.CONFIGS["C1"]
    poly = orchard.polygon(cfg)
    clouds = [orchard.generate(cfg), orchard.generate(cfg, seed=cfg.seed + 1)]
    singles = [_single(c, poly, cfg.res) for c in clouds]
    tiles_x, tiles_y, frames = 2, 2, 8
    world = tiles_x * tiles_y
    params = aos_gpu.default_params(grid_resolution=cfg.res)
    plans = [T.tile_plan(params, poly, tiles_x, tiles_y, r) for r in range(world)]
    group = T.ThreadGroup(world, timeout=120)
    ctxs = [aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res)) for _ in range(world)]
    comms = [group.comm(r, plans[r]["exchange_bytes"], "cuda:0") for r in range(world)]
    graphs, errors = {}, []

    def work(r):
        try:
            ctxs[r].set_polygon(poly)
            ctxs[r].gvd_pipeline_depth(2)
            parts = [T.shard(c, plans[r]["points_box"]) for c in clouds]
            mine = []
            for k in range(frames):
                g = ctxs[r].tiled_seedgen(comms[r], tiles_x, tiles_y, parts[k % 2], root=k % world, want_host=False)
                assert g["root"] == (k % world == r)
                if g["root"]:
                    ctxs[r].gvd_async()
                    mine.append(k)
            for k in mine:   # jobs complete in start order
                graphs[k] = ctxs[r].gvd_wait()
        except BaseException as e:   # noqa: BLE001
            errors.append(e)
            group.abort()

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(600)
    for x in ctxs:
        x.close()
    if errors:
        raise errors[0]
    assert sorted(graphs) == list(range(frames))
    for k, gg in graphs.items():
        gg1 = singles[k % 2][2]
        assert gg["published"] == gg1["published"]
        for key in GVD_KEYS:
            assert np.array_equal(gg[key], gg1[key]), (k, key)


def _sha(a, dt):
    a = np.ascontiguousarray(np.asarray(a, dtype=dt))
    return hashlib.sha256(a.dtype.str.encode() + str(a.shape).encode() + a.tobytes()).hexdigest()


def _assert_golden(name, g, gg):
    """The root's frame + GVD vs the SHA-256 of the oracle's outputs (tests/golden/<name>_sha256.json,
    tools/make_golden.py)."""
    here = os.path.dirname(os.path.abspath(__file__))
    hs = json.load(open(os.path.join(here, "golden", f"{name}_sha256.json")))
    assert g["thin_iters"] == hs["meta"]["thin_iters"] and g["n_clipped"] == hs["meta"]["n_clipped"]
    for k in ("occupancy", "skeleton_framed"):
        assert _sha(g[k], np.int8) == hs["seedgen"][k], k
    for k in ("row_center", "row_start", "row_end", "row_length", "voronoi_seeds", "rows_info", "cluster_info"):
        assert _sha(g[k], np.float64) == hs["seedgen"][k], k
    for k, dt in (("merged", np.float64), ("nodes", np.float64), ("edges", np.int32), ("edge_lengths", np.float32),
                  ("edge_clearances", np.float32), ("node_labels", np.int32), ("node_cluster_indices", np.int32),
                  ("node_label_counts", np.int32), ("node_label_clusters", np.int32), ("node_label_types", np.int32)):
        if k in gg:
            assert _sha(gg[k], dt) == hs["gvd"][k], k


def test_tiled_c1_against_golden_hashes():
    """2 x 2 tiles, every rank handed the whole cloud (points outside a tile's box are ignored)."""
    cfg = orchard.CONFIGS["C1"]
    g, _, _, gg = _tiled_threads(orchard.generate(cfg), orchard.polygon(cfg), cfg.res, 2, 2, 0, shard=False)
    _assert_golden("c1", g, gg)


def _blob_scene():
    """C0 orchard plus a 12 m x 12 m filled square across the map centre (~34 Zhang-Suen iterations:
    the thinning needs more than one halo period, so halos are refreshed mid-thinning)."""
    cfg = orchard.CONFIGS["C0"]
    base = orchard.generate(cfg).view(np.float32).reshape(-1, 4)
    rng = np.random.default_rng(5)
    n = 40000
    blob = np.zeros((n, 4), np.float32)
    blob[:, 0] = rng.uniform(42.6, 54.6, n)
    blob[:, 1] = rng.uniform(42.6, 54.6, n)
    blob[:, 2] = rng.uniform(-0.3, 0.4, n)
    return cfg, np.concatenate([base, blob]).view(np.uint8).reshape(-1, 16), orchard.polygon(cfg)


@pytest.mark.parametrize("tiles", [(2, 2), (4, 1), (1, 4)])
def test_tiled_blob_refreshes_halos_mid_thinning_vs_oracle(tiles):
    cfg, cloud, poly = _blob_scene()
    g, out, grids, gg = _tiled_threads(cloud, poly, cfg.res, *tiles, 0)
    o = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res))
    assert o["thin_iters"] > 29
    assert_seedgen_parity(g, o)
    assert np.array_equal(grids["skeleton_frameless"], o["skeleton"])
    assert np.array_equal(grids["inflated"], o["inflated"])
    assert g["n_clipped"] == o["n_clipped"]
    assert_gvd_parity(gg, O.gvd(o["voronoi_seeds"], o["rows_info"], o))


def _group(cloud, poly, res, tiles_x, tiles_y, root, shard=True, on_device=False):
    """The same frame through aos_group_* (the library's own rank threads and in-process comm)."""
    import torch
    world = tiles_x * tiles_y
    grp = aos_gpu.Group(aos_gpu.default_params(grid_resolution=res), [0] * world, tiles_x, tiles_y)
    grp.set_polygon(poly)
    parts = [T.shard(cloud, grp.plan(r)["points_box"]) if shard else cloud for r in range(world)]
    if on_device:
        dev = [torch.from_numpy(np.ascontiguousarray(p)).to("cuda:0") for p in parts]
        g = grp.process([d.data_ptr() for d in dev], root=root, on_device=True, n_points=[p.shape[0] for p in parts])
    else:
        g = grp.process(parts, root=root)
    c = grp.rank(root)
    grids = {w: c.debug_grid(w, (g["height"], g["width"])) for w in GRIDS}
    gg = c.gvd_from_seedgen()
    grp.close()
    return g, [g], grids, gg


@pytest.mark.parametrize("tiles,root,on_device", [((2, 1), 0, False), ((2, 2), 3, True), ((1, 3), 1, False)])
def test_group_c1_equals_single_gpu(tiles, root, on_device):
    cfg = orchard.CONFIGS["C1"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    _assert_same(_single(cloud, poly, cfg.res), _group(cloud, poly, cfg.res, *tiles, root, on_device=on_device))


def test_group_c1_tiling_for_8_equals_single_gpu():
    """The 8-rank split SURVEY §8e names (tiling_for(8) = 4 x 2 tiles) at C1 size, ranks on one GPU."""
    cfg = orchard.CONFIGS["C1"]
    tiles = T.tiling_for(8)
    assert tiles == (4, 2)
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    single = _single(cloud, poly, cfg.res)
    _assert_same(single, _group(cloud, poly, cfg.res, *tiles, 5))
    _assert_golden("c1", single[0], single[2])


@pytest.fixture(scope="module")
def c3_scene():
    cfg = orchard.CONFIGS["C3"]
    return cfg, orchard.generate(cfg), orchard.polygon(cfg)


@pytest.fixture(scope="module")
def c3_single(c3_scene):
    cfg, cloud, poly = c3_scene
    return _single(cloud, poly, cfg.res)


def test_c3_single_gpu_against_golden(c3_single):
    """BASELINE configs[3]'s map (40 M points, 8192^2 @ 0.1 m) as one frame on one GPU vs the oracle's
    hashes (tests/golden/c3_sha256.json)."""
    g, _, gg = c3_single
    assert (g["width"], g["height"]) == (8192, 8192)
    # every row cluster has coordinate sums > 2^24: exact BFS replays, on the host threads over the skeleton bits
    rc = g["replay_counts"]
    assert rc["all"] == g["n_bfs_replayed"] >= 200 and rc["host_bits"] == rc["all"], rc
    _assert_golden("c3", g, gg)


def test_c3_gpu_replays_equal_host(c3_scene, c3_single):
    """C3's ~215 row-cluster replays through the GPU walk (replay_gpu.hip, one wave per cluster; aos_debug_replay):
    the frame equals the host-replayed one."""
    cfg, cloud, poly = c3_scene
    aos_gpu.debug_replay(0)
    try:
        single = _single(cloud, poly, cfg.res)
    finally:
        aos_gpu.debug_replay()
    rc = single[0]["replay_counts"]
    assert rc["gpu"] == rc["all"] == c3_single[0]["n_bfs_replayed"], rc
    _assert_same(c3_single, (single[0], [], single[1], single[2]))


def test_group_c3_tiling_for_8_vs_single_and_golden(c3_scene, c3_single):
    """C3 through aos_group with the SURVEY §8e split (8 ranks, 4 x 2 tiles of 2048 columns x 4096 rows)
    on one GPU: the root's grids, seeds and GvdGraph equal the single-GPU frame and the oracle's hashes."""
    cfg, cloud, poly = c3_scene
    tiles = T.tiling_for(8)
    tiled = _group(cloud, poly, cfg.res, *tiles, 0)
    _assert_same(c3_single, tiled)
    g, _, _, gg = tiled
    _assert_golden("c3", g, gg)


def test_group_blob_vs_oracle_and_bad_cloud():
    cfg, cloud, poly = _blob_scene()
    g, _, grids, gg = _group(cloud, poly, cfg.res, 2, 2, 0)
    o = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res))
    assert_seedgen_parity(g, o)
    assert np.array_equal(grids["skeleton_frameless"], o["skeleton"])
    assert_gvd_parity(gg, O.gvd(o["voronoi_seeds"], o["rows_info"], o))
    # an invalid PointCloud2 layout fails the frame with the rank's own error, without hanging
    grp = aos_gpu.Group(aos_gpu.default_params(grid_resolution=cfg.res), [0, 0], 2, 1)
    grp.set_polygon(poly)
    with pytest.raises(RuntimeError, match=r"rank \d: .*invalid PointCloud2 layout"):
        grp.process([cloud, cloud], point_step=16, offs=(0, 4, 13))
    # and the group still works afterwards
    g2 = grp.process([cloud, cloud])
    assert g2["thin_iters"] == o["thin_iters"]
    grp.close()


def test_rccl_comm_single_rank_frame():
    """The library's C++ RCCL communicator (aos_rccl_*: ncclAllGather / ncclAllReduce(max) on its own
    HBM buffers, no Python callbacks) drives a 1 x 1 tiled C1 frame: the root's outputs equal the
    single-GPU frame. (One GPU per box: RCCL refuses two ranks on one device, so the multi-rank path is
    covered by the thread/gloo tests through the same aos_comm contract.)"""
    cfg = orchard.CONFIGS["C1"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    single = _single(cloud, poly, cfg.res)
    params = aos_gpu.default_params(grid_resolution=cfg.res)
    plan = T.tile_plan(params, poly, 1, 1, 0)
    comm = T.RcclComm(plan["exchange_bytes"], device=0, rank=0, world=1)
    c = aos_gpu.Ctx(params)
    c.set_polygon(poly)
    g = c.tiled_seedgen(comm, 1, 1, cloud, root=0)
    g2 = c.tiled_seedgen(comm, 1, 1, cloud, root=0)   # the communicator is reusable across frames
    assert g2["thin_iters"] == g["thin_iters"]
    grids = {w: c.debug_grid(w, (g["height"], g["width"])) for w in GRIDS}
    gg = c.gvd_from_seedgen()
    c.close()
    comm.close()
    _assert_same(single, (g, [g], grids, gg))
    with pytest.raises(RuntimeError, match="rank"):
        T.RcclComm(plan["exchange_bytes"], device=0, rank=1, world=1, unique_id=bytes(128))


def test_group_stream_4x2_equals_single_gpu_stream():
    """BASELINE configs[4] over 8 tiles (tiling_for(8) = 4 x 2, ranks on one GPU): the C2 map, then 10
    scans of 1 M points, into the group's tiled streaming map (aos_group_map_append: every rank keeps its
    points box of each scan in its own map and incremental ROR store) with the root rotating over the
    ranks; every frame equals the single-GPU aos_map_append frame (grids, T, counts, rows, seeds), the
    GvdGraph every third frame, and the last frame the oracle's hashes after 5 scans where they apply."""
    cfg = orchard.CONFIGS["C2"]
    poly = orchard.polygon(cfg)
    base = orchard.generate(cfg)
    params = aos_gpu.default_params(grid_resolution=cfg.res)
    single = aos_gpu.Ctx(params)
    single.set_polygon(poly)
    single.map_reset(reserve_points=base.shape[0] + 10 * orchard.SCAN_POINTS)
    tx, ty = T.tiling_for(8)
    grp = aos_gpu.Group(params, [0] * (tx * ty), tx, ty)
    grp.set_polygon(poly)
    grp.map_reset(reserve_points=base.shape[0] // 4)
    skipped = 0
    for k in range(11):
        cloud = base if k == 0 else orchard.generate_scan(cfg, 40 * (k - 1))
        g1 = single.map_append(cloud)
        root = (3 * k) % (tx * ty)
        gt = grp.map_append(cloud, root=root)
        # a rank whose box the scan missed keeps its committed ROR store without re-partitioning
        skipped += sum(grp.rank(r).tiled_stats()["ror_skipped"] for r in range(tx * ty)) if k else 0
        assert_seedgen_parity(gt, {**g1, "cluster_length": np.zeros(g1["n_clusters_all"])})
        assert (gt["n_clipped"], gt["n_input"], gt["thin_iters"]) == (g1["n_clipped"], g1["n_input"], g1["thin_iters"]), k
        if k % 3 == 2 or k == 10:
            gg1, ggt = single.gvd_from_seedgen(), grp.rank(root).gvd_from_seedgen()
            for key in GVD_KEYS:
                assert np.array_equal(gg1[key], ggt[key]), (k, key)
    assert skipped > 0   # ... and the frames above still equal the single-GPU map's
    # changing the polygon changes the tiles' boxes: the tiled map refuses until it is reset
    grp.set_polygon(poly + 1.0)
    with pytest.raises(RuntimeError, match="points box changed"):
        grp.map_append(orchard.generate_scan(cfg, 400))
    grp.close()
    single.close()


def test_tiled_stuck_lookback_fails_every_rank():
    """A tiled rank whose ROR column scan reports a stuck look-back (bit 4 of its overflow word, injected with
    aos_debug_faults) must not leave the frame alone: the bit travels with the kept counts in the
    max-reduction, so every rank raises the same error and none is left inside a collective.
    The group is never aborted here: a rank that left early would show as a barrier timeout instead."""
    cfg = orchard.CONFIGS["C1"]
    cloud, poly = orchard.generate(cfg, n_points=400_000), orchard.polygon(cfg)
    world = 2
    params = aos_gpu.default_params(grid_resolution=cfg.res)
    plans = [T.tile_plan(params, poly, 2, 1, r) for r in range(world)]
    group = T.ThreadGroup(world, timeout=60)
    ctxs = [aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res)) for _ in range(world)]
    comms = [group.comm(r, plans[r]["exchange_bytes"], "cuda:0") for r in range(world)]
    for c in ctxs:
        c.set_polygon(poly)
    errs = [None] * world

    def work(r):
        try:
            ctxs[r].tiled_seedgen(comms[r], 2, 1, T.shard(cloud, plans[r]["points_box"]), root=0)
        except BaseException as e:   # noqa: BLE001
            errs[r] = e

    aos_gpu.debug_faults(ror_stuck_rank=1)
    try:
        ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(180)
    finally:
        aos_gpu.debug_faults()
    for r in range(world):
        assert isinstance(errs[r], RuntimeError) and "bits 4" in str(errs[r]) and "look-back" in str(errs[r]), (r, errs[r])
    # both handles still work on the next frame
    out = [None] * world

    def again(r):
        out[r] = ctxs[r].tiled_seedgen(comms[r], 2, 1, T.shard(cloud, plans[r]["points_box"]), root=0)
    ts = [threading.Thread(target=again, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(180)
    assert out[0] is not None and out[0]["root"] and out[1] is not None
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("tiles", [(2, 1), (3, 2)])
def test_rccl_ranks_as_processes(tiles, tmp_path):
    """The library's RCCL communicator between real ranks: `world` processes on the box's one GPU, each with its
    own NCCL_HOSTID so that RCCL accepts them (it refuses two ranks on one device of one host) and links them
    over its socket transport on loopback. Every frame's collectives are the production path's: ncclAllGather
    of the piece tables, grouped ncclSend / ncclRecv of the halo strips between neighbouring tiles only (3 x 2:
    corner tiles have 3 neighbours, the middle column 5), ncclAllReduce(max) of the thinning flags, the
    send-to-root of the final tiles and the grouped ncclSend / ncclRecv of the cluster exchange (also in 4 KB
    rounds), all enqueued on the frame's stream. Roots rotate; each root's frame, grids and GvdGraph equal the single-GPU frame
    (tests/rccl_rank_child.py)."""
    import subprocess
    import sys
    world = tiles[0] * tiles[1]
    here = os.path.dirname(os.path.abspath(__file__))
    uid = str(tmp_path / "uid.bin")
    procs = []
    for r in range(world):
        env = dict(os.environ, NCCL_HOSTID=f"aos-rank-{r}", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(here, "rccl_rank_child.py"), str(r), str(world),
                                       str(tiles[0]), str(tiles[1]), uid], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=150)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0 and "RCCL_RANK_OK" in o, f"rank {r} rc={p.returncode}:\n{o[-3000:]}"
    reports = [json.loads(o.split("RCCL_RANK_OK ", 1)[1].splitlines()[0]) for o in outs]
    print(json.dumps(reports))
    for rep in reports:
        assert len(rep["frames"]) == world + 1
    # a non-root rank receives no final tiles (they go to the root only), and its halo strips from its neighbours only
    for k in range(world + 1):
        root = reports[0]["frames"][k]["root"]
        recv = [rep["frames"][k]["recv_MB"] for rep in reports]
        assert all(recv[r] < recv[root] for r in range(world) if r != root), (k, recv)
