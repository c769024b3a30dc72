"""CPU coverage of the tiled multi-GPU frame (libaos_gpu tiled.hip):
- the tile plan the C-ABI computes (aos_tile_plan_compute needs no GPU);
- the communicator adapters (aos_tiles.TorchDistComm over gloo at world size 2, ThreadGroup), called
  through the same C function pointers libaos_gpu calls;
- the border union-find of the distributed cluster stage (aos_cluster_union, host code) over gloo ranks;
- a numpy emulation of tiled.hip's schedule (own-cell raster -> halo exchange -> inflate -> open ->
  Zhang-Suen in halo periods with max-reduced own-cell change flags) run by gloo ranks, whose gathered
  tiles must equal the oracle's whole-map grids and iteration count.
"""
import ctypes
import os
import socket
import threading

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import aos_gpu
import aos_tiles as T
import oracle_py as O
import orchard

KIT = 8   # kThinItersPerLaunch (aos_internal.h)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(target, world, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(out, key=lambda o: o[0])


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


# ---------------------------------------------------------------- plan
def test_plan_c3_is_2x4_tiles_of_4096_rows_by_2048_columns():
    cfg = orchard.CONFIGS["C3"]
    poly = orchard.polygon(cfg)
    p = aos_gpu.default_params(grid_resolution=cfg.res)
    plans = [T.tile_plan(p, poly, 4, 2, r) for r in range(8)]
    W, H = plans[0]["width"], plans[0]["height"]
    assert (W, H) == (8192, 8192)
    cover = np.zeros((H, W // 64), np.int32)
    for t in plans:
        assert (t["row1"] - t["row0"], t["word1"] - t["word0"]) == (4096, 32)
        assert (t["halo_rows"], t["halo_words"]) == (64, 1)
        cover[t["row0"]:t["row1"], t["word0"]:t["word1"]] += 1
        assert t["win_row0"] == max(0, t["row0"] - 64) and t["win_row1"] == min(H, t["row1"] + 64)
        assert t["win_word0"] == max(0, t["word0"] - 1) and t["win_word1"] == min(W // 64, t["word1"] + 1)
        ox, oy = t["origin"]
        res = t["resolution"]
        b = t["points_box"]   # the own cells' world box plus the ROR radius
        assert b[0] <= ox + 64 * t["word0"] * res - 0.2 and b[2] >= ox + min(W, 64 * t["word1"]) * res + 0.2
        assert b[1] <= oy + t["row0"] * res - 0.2 and b[3] >= oy + t["row1"] * res + 0.2
        assert t["exchange_bytes"] == 8 * max(2 * 64 * 32 + 2 * 4096, 2 * 4096 * 32)
    assert (cover == 1).all()


def test_plan_single_tile_and_too_small_tiles():
    cfg = orchard.CONFIGS["C0"]
    poly = orchard.polygon(cfg)
    p = aos_gpu.default_params(grid_resolution=cfg.res)
    t = T.tile_plan(p, poly, 1, 1, 0)
    assert (t["halo_rows"], t["halo_words"]) == (0, 0)
    assert (t["win_row0"], t["win_row1"], t["win_word0"], t["win_word1"]) == (0, 512, 0, 8)
    with pytest.raises(RuntimeError, match="smaller than its halo"):
        T.tile_plan(p, poly, 2, 16, 0)          # 32-row tiles, 64-row halo
    with pytest.raises(RuntimeError, match="rank outside"):
        T.tile_plan(p, poly, 2, 2, 4)


def test_tiling_for():
    assert [T.tiling_for(n) for n in (1, 2, 4, 6, 8)] == [(1, 1), (2, 1), (2, 2), (3, 2), (4, 2)]


def test_shard_keeps_the_points_box():
    cfg = orchard.CONFIGS["C0"]
    cloud = orchard.generate(cfg, n_points=20000)
    box = (10.0, 20.0, 30.5, 40.0)
    s = T.shard(cloud, box)
    xyz = orchard.xyz(cloud)
    inside = (xyz[:, 0] >= box[0]) & (xyz[:, 0] <= box[2]) & (xyz[:, 1] >= box[1]) & (xyz[:, 1] <= box[3])
    assert np.array_equal(s, cloud[inside])


# ---------------------------------------------------------------- communicators
def _comm_worker(rank, world, port, q):
    _init(rank, world, port)
    c = T.TorchDistComm(64, "cpu")
    c.send[:48] = torch.arange(48, dtype=torch.uint8) + 10 * rank
    rc = c.c.all_gather(None, 48)                      # as libaos_gpu calls it
    v = (ctypes.c_int32 * 3)(rank, 5 - rank, -rank)
    rc2 = c.c.all_reduce_max(None, v, 3)
    recv_ag = c.recv[: 48 * world].numpy().copy()
    # the personalised exchange (the cluster stage's cell routing): rank s sends A2A[s][d] bytes to rank d
    counts = (ctypes.c_uint64 * (world * world))(*[x for row in A2A for x in row])
    at = 0
    for d in range(world):
        c.send[at:at + A2A[rank][d]] = 100 + 10 * rank + d
        at += A2A[rank][d]
    rc3 = c.c.all_to_all(None, counts)
    nr = sum(A2A[s][rank] for s in range(world))
    q.put((rank, rc, rc2, recv_ag, list(v), rc3, c.recv[:nr].numpy().copy()))
    dist.destroy_process_group()


A2A = [[3, 5], [0, 7]]   # bytes rank s sends to rank d (an empty block included)


def _a2a_expected(rank, world):
    return np.concatenate([np.full(A2A[s][rank], 100 + 10 * s + rank, np.uint8) for s in range(world)])


def test_torch_dist_comm_gloo_world2():
    for rank, rc, rc2, recv, v, rc3, recv3 in _spawn(_comm_worker, 2):
        assert rc == 0 and rc2 == 0 and rc3 == 0
        assert np.array_equal(recv, np.concatenate([np.arange(48, dtype=np.uint8) + 10 * r for r in range(2)]))
        assert v == [1, 5, 0]
        assert np.array_equal(recv3, _a2a_expected(rank, 2))


# ---------------------------------------------------------------- distributed cluster labelling
def _pieces_of_tile(fg, y0, y1, x0, x1):
    """One rank's part of cluster_dist.hip step 1 on the CPU: 8-connected pieces of its own cells
    (scipy stands in for the GPU union-find), named by their first raster cell, the piece's n and
    integer sums, and its cells on the tile's edge."""
    from scipy import ndimage
    H, W = fg.shape
    sub = fg[y0:y1, x0:x1]
    lab, n = ndimage.label(sub, structure=np.ones((3, 3), bool))
    ys, xs = np.nonzero(lab)
    gid = (ys + y0) * W + (xs + x0)                  # raster order (np.nonzero is row-major)
    lv = lab[ys, xs] - 1
    root = np.full(n, np.iinfo(np.int32).max, np.int64)
    np.minimum.at(root, lv, gid)
    cnt = np.bincount(lv, minlength=n)
    sx = np.bincount(lv, weights=xs + x0, minlength=n).astype(np.int64)
    edge = (ys == 0) | (xs == 0) | (ys == sub.shape[0] - 1) | (xs == sub.shape[1] - 1)
    return root.astype(np.int32), cnt, sx, gid[edge].astype(np.int32), root[lv[edge]].astype(np.int32)


def _union_worker(rank, world, port, q, fg, tx, ty):
    _init(rank, world, port)
    H, W = fg.shape
    x_cut = [W * i // tx for i in range(tx + 1)]
    y_cut = [H * i // ty for i in range(ty + 1)]
    cx, cy = rank % tx, rank // tx
    mine = _pieces_of_tile(fg, y_cut[cy], y_cut[cy + 1], x_cut[cx], x_cut[cx + 1])
    tables = [None] * world
    dist.all_gather_object(tables, mine)             # the pieces / border all-gather
    root = np.concatenate([t[0] for t in tables])
    cnt = np.concatenate([t[1] for t in tables])
    sx = np.concatenate([t[2] for t in tables])
    bcell = np.concatenate([t[3] for t in tables])
    broot = np.concatenate([t[4] for t in tables])
    pc, ncl = aos_gpu.cluster_union(W, H, root, bcell, broot)
    q.put((rank, root, cnt, sx, pc, ncl))
    dist.destroy_process_group()


def _reference_clusters(fg):
    """Whole-map labelling in the reference's numbering (raster order of the first cell)."""
    from scipy import ndimage
    lab, n = ndimage.label(fg, structure=np.ones((3, 3), bool))
    ys, xs = np.nonzero(lab)
    first = np.full(n, np.iinfo(np.int64).max)
    np.minimum.at(first, lab[ys, xs] - 1, ys * fg.shape[1] + xs)
    order = np.argsort(first)
    cid = np.empty(n, np.int64)
    cid[order] = np.arange(n)
    return cid[lab - 1], lab > 0, first[order], n


@pytest.mark.parametrize("tiles", [(2, 1), (1, 2)])
def test_cluster_union_gloo_world2(tiles):
    """cluster_dist.hip's numbering: pieces labelled per tile, tables all-gathered over gloo, the
    library's aos_cluster_union on every rank -> the whole-map clusters in raster order of their first
    cell, with n and integer sums added over pieces (rows, blobs and diagonal contacts across the cut)."""
    rng = np.random.default_rng(7)
    H, W = 96, 160
    fg = rng.random((H, W)) < 0.12                   # noise: many small clusters, diagonal contacts
    fg[20, 5:150] = True                             # rows that cross the vertical cut
    fg[60, 10:140] = True
    fg[10:90, 80] = True                             # a column crossing the horizontal cut
    fg[47, 79], fg[48, 80] = True, True              # diagonal contact at the corner region
    tx, ty = tiles
    out = _spawn(_union_worker, 2, fg, tx, ty)
    cid_map, mask, first, n = _reference_clusters(fg)
    ys, xs = np.nonzero(mask)
    ref_n = np.bincount(cid_map[ys, xs], minlength=n)
    ref_sx = np.bincount(cid_map[ys, xs], weights=xs, minlength=n).astype(np.int64)
    for rank, root, cnt, sx, pc, ncl in out:
        assert ncl == n
        # every piece lies in its cluster, clusters numbered as the reference discovers them
        ry, rx = root // W, root % W
        assert np.array_equal(pc, cid_map[ry, rx])
        assert np.array_equal(np.bincount(pc, weights=cnt, minlength=n).astype(np.int64), ref_n)
        assert np.array_equal(np.bincount(pc, weights=sx, minlength=n).astype(np.int64), ref_sx)
        first_of = np.full(n, np.iinfo(np.int64).max)
        np.minimum.at(first_of, pc, root.astype(np.int64))
        assert np.array_equal(first_of, first)
    assert any((np.bincount(o[4]) > 1).any() for o in out)   # some clusters really cross the cut


def test_cluster_union_rejects_bad_tables():
    with pytest.raises(RuntimeError, match="unknown piece"):
        aos_gpu.cluster_union(8, 8, [0, 9], [3], [5])
    with pytest.raises(RuntimeError, match="duplicate"):
        aos_gpu.cluster_union(8, 8, [4, 4], [], [])
    pc, n = aos_gpu.cluster_union(8, 8, [], [], [])
    assert n == 0 and pc.size == 0


# ---------------------------------------------------------------- tiled streaming: scan routing
def _route_worker(rank, world, port, q, tx, ty):
    """One rank of a tiled streaming map: it receives every scan (broadcast, as every subscriber of
    /global_map does) and keeps the points of its tile's points box (aos_tiled_map_append's rule,
    grid_kernels.hip k_pack_xyz_box = aos_tiles.shard). Checks on the accumulated map: every point whose
    clamped cell the rank owns, and every point within the ROR radius of it, is in the rank's map; the
    owned counts all-reduced over the ranks cover every point once."""
    from scipy.spatial import cKDTree
    _init(rank, world, port)
    cfg = orchard.CONFIGS["C1"]
    poly = orchard.polygon(cfg)
    params = aos_gpu.default_params(grid_resolution=cfg.res)
    plan = T.tile_plan(params, poly, tx, ty, rank)
    scans = [orchard.generate_scan(cfg, k, n_points=40_000) for k in (0, 1300, 2500)]   # across both tiles
    whole = np.concatenate(scans)
    mine = np.concatenate([T.shard(s, plan["points_box"]) for s in scans])   # the rank's map after 3 appends
    pts = orchard.xyz(whole).astype(np.float64)
    ox, oy = plan["origin"]
    res = np.float64(np.float32(plan["resolution"]))
    W, H = plan["width"], plan["height"]
    cx = np.clip(np.trunc((pts[:, 0] - ox) / res), 0, W - 1).astype(np.int64)   # generateOccupancyGrid cell, clamped
    cy = np.clip(np.trunc((pts[:, 1] - oy) / res), 0, H - 1).astype(np.int64)
    # ROR candidates (PassThrough: inside the grid's clip box and z range) whose clamped cell is an own cell
    cand = ((pts[:, 0] >= ox) & (pts[:, 0] <= ox + W * res) & (pts[:, 1] >= oy) & (pts[:, 1] <= oy + H * res) &
            (pts[:, 2] >= params.clipping_minz) & (pts[:, 2] <= params.clipping_maxz))
    own = cand & (cx >= 64 * plan["word0"]) & (cx < min(W, 64 * plan["word1"])) & (cy >= plan["row0"]) & (cy < plan["row1"])
    in_map = {r.tobytes() for r in mine}
    tree = cKDTree(pts[:, :2])
    need = set(np.nonzero(own)[0].tolist())
    for nb in tree.query_ball_point(pts[own, :2], r=params.ror_radius):   # (2-D: a superset of the 3-D ball)
        need.update(nb)
    missing = sum(1 for i in need if whole[i].tobytes() not in in_map)
    cnt = torch.tensor([int(own.sum())], dtype=torch.int64)
    dist.all_reduce(cnt)
    q.put((rank, missing, len(need), mine.shape[0], int(cnt.item()), int(cand.sum()), whole.shape[0]))
    dist.destroy_process_group()


def test_tiled_stream_routing_gloo_world2():
    for rank, missing, needed, kept, owned_total, n_cand, n in _spawn(_route_worker, 2, 2, 1):
        assert missing == 0, (rank, missing, needed)
        assert needed > 1000 and kept < n          # each rank keeps a part of the broadcast scans
        assert owned_total == n_cand               # every candidate is owned by exactly one rank


def test_thread_group_comm():
    world = 3
    g = T.ThreadGroup(world, timeout=30)
    comms = [g.comm(r, 16, "cpu") for r in range(world)]
    res = [None] * world

    def work(r):
        c = comms[r]
        c.send[:8] = r + 1
        rc = c.c.all_gather(None, 8)
        v = (ctypes.c_int32 * 2)(r, -r)
        rc2 = c.c.all_reduce_max(None, v, 2)
        recv_ag = c.recv[:24].numpy().copy()
        m = [[(s + 2 * d) % 4 for d in range(world)] for s in range(world)]
        at = 0
        for d in range(world):
            c.send[at:at + m[r][d]] = 50 + 10 * r + d
            at += m[r][d]
        rc3 = c.c.all_to_all(None, (ctypes.c_uint64 * 9)(*[x for row in m for x in row]))
        want = np.concatenate([np.full(m[s][r], 50 + 10 * s + r, np.uint8) for s in range(world)])
        ok3 = np.array_equal(c.recv[:len(want)].numpy(), want)
        res[r] = (rc, rc2, recv_ag, list(v), rc3, ok3)

    ts = [threading.Thread(target=work, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    for rc, rc2, recv, v, rc3, ok3 in res:
        assert rc == 0 and rc2 == 0 and v == [2, 0] and rc3 == 0 and ok3
        assert np.array_equal(recv, np.repeat(np.arange(1, 4, dtype=np.uint8), 8))
    # a communicator without the optional callback exposes a NULL pointer (the library then uses all_gather)
    assert not comms[0].without_all_to_all().c.all_to_all


# ---------------------------------------------------------------- schedule emulation
def _zs_sub(img, it):
    """One ximgproc Zhang-Suen sub-iteration on a 0/1 image (border pixels untouched)."""
    P = np.pad(img, 1).astype(np.int32)
    p2, p3, p4, p5 = P[:-2, 1:-1], P[:-2, 2:], P[1:-1, 2:], P[2:, 2:]
    p6, p7, p8, p9 = P[2:, 1:-1], P[2:, :-2], P[1:-1, :-2], P[:-2, :-2]
    seq = [p2, p3, p4, p5, p6, p7, p8, p9, p2]
    A = sum(((seq[k] == 0) & (seq[k + 1] == 1)).astype(np.int32) for k in range(8))
    B = sum(seq[:8])
    m1, m2 = (p2 * p4 * p6, p4 * p6 * p8) if it == 0 else (p2 * p4 * p8, p2 * p6 * p8)
    d = (img == 1) & (A == 1) & (B >= 2) & (B <= 6) & (m1 == 0) & (m2 == 0)
    d[0, :] = d[-1, :] = d[:, 0] = d[:, -1] = False
    return np.where(d, 0, img).astype(np.uint8)


def _emu_worker(rank, world, port, q, tx, ty, res, poly, raster, R):
    _init(rank, world, port)
    p = aos_gpu.default_params(grid_resolution=res)
    plans = [T.tile_plan(p, poly, tx, ty, r) for r in range(world)]
    me = plans[rank]
    W = me["width"]

    def own(t):
        return t["row0"], t["row1"], 64 * t["word0"], min(W, 64 * t["word1"])

    wy0, wy1, wx0, wx1 = me["win_row0"], me["win_row1"], 64 * me["win_word0"], min(W, 64 * me["win_word1"])
    y0, y1, x0, x1 = own(me)
    mine = (slice(y0 - wy0, y1 - wy0), slice(x0 - wx0, x1 - wx0))

    def exchange(win):   # every rank publishes its own block; halo cells come from their owners
        blocks = [None] * world
        dist.all_gather_object(blocks, win[mine].copy())
        out = win.copy()
        for r, t in enumerate(plans):
            a0, a1, b0, b1 = own(t)
            ya, yb, xa, xb = max(a0, wy0), min(a1, wy1), max(b0, wx0), min(b1, wx1)
            if r != rank and ya < yb and xa < xb:
                out[ya - wy0:yb - wy0, xa - wx0:xb - wx0] = blocks[r][ya - a0:yb - a0, xa - b0:xb - b0]
        return out

    win = np.zeros((wy1 - wy0, wx1 - wx0), np.uint8)
    win[mine] = raster[y0:y1, x0:x1] != 0          # this tile's own kept candidates
    win = exchange(win)
    infl = (O.inflate(np.where(win == 1, 100, 0).astype(np.int8), R) == 100).astype(np.uint8)
    img = O.open_cross(infl)
    G = max(me["halo_rows"], 64 * me["halo_words"])
    halo = G > 0
    budget = G - R - 2 if halo else 1 << 30
    flags, nonempty, it, Tn, periods = [], 0, 0, 0, 0
    while True:
        nl = budget // (2 * KIT) if halo else (3 if it == 0 else 4)
        assert nl >= 1
        for _ in range(nl * KIT):
            chg = 0
            for sub in (0, 1):
                new = _zs_sub(img, sub)
                chg |= int((new[mine] != img[mine]).any())
                img = new
            if it == 0:
                nonempty = int(img[mine].any())
            flags.append(chg)
            it += 1
        budget -= nl * 2 * KIT
        periods += 1
        fl = torch.tensor([nonempty] + flags, dtype=torch.int32)
        dist.all_reduce(fl, op=dist.ReduceOp.MAX)
        fl = fl.numpy()
        Tn = 1 if not fl[0] else next((k + 1 for k in range(1, it) if not fl[1 + k]), 0)
        if Tn:
            break
        if halo:
            img = exchange(img)
            budget = G
    parts = [None] * world
    dist.all_gather_object(parts, (img[mine].copy(), infl[mine].copy()))
    if rank == 0:
        H = me["height"]
        sk, inf = np.zeros((H, W), np.uint8), np.zeros((H, W), np.uint8)
        for t, (a, b) in zip(plans, parts):
            a0, a1, b0, b1 = own(t)
            sk[a0:a1, b0:b1], inf[a0:a1, b0:b1] = a, b
        q.put((rank, Tn, periods, sk, inf))
    else:
        q.put((rank, Tn, periods, None, None))
    dist.destroy_process_group()


def _blob_scene():
    """C0 orchard plus a 12 m x 12 m filled square across the map centre: ~34 Zhang-Suen iterations,
    more than one halo period (the first period covers (64 - R - 2) / 2 = 29 sub-iteration pairs)."""
    cfg = orchard.CONFIGS["C0"]
    base = orchard.generate(cfg).view(np.float32).reshape(-1, 4)
    rng = np.random.default_rng(5)
    n = 40000
    blob = np.zeros((n, 4), np.float32)
    blob[:, 0] = rng.uniform(42.6, 54.6, n)
    blob[:, 1] = rng.uniform(42.6, 54.6, n)
    blob[:, 2] = rng.uniform(-0.3, 0.4, n)
    cloud = np.concatenate([base, blob]).view(np.uint8).reshape(-1, 16)
    return cfg, cloud, orchard.polygon(cfg)


@pytest.mark.parametrize("tiles", [(2, 2), (2, 1)])
def test_tiled_schedule_emulation_matches_oracle(tiles):
    cfg, cloud, poly = _blob_scene()
    ref = O.seedgen(cloud, poly, O.default_params(grid_resolution=cfg.res))
    assert ref["thin_iters"] > 29
    R = int(np.float32(0.8) / np.float32(cfg.res))
    tx, ty = tiles
    out = _spawn(_emu_worker, tx * ty, tx, ty, cfg.res, poly, ref["raster"], R)
    for _, Tn, periods, _, _ in out:
        assert Tn == ref["thin_iters"] and periods >= 2
    sk, inf = out[0][3], out[0][4]
    assert np.array_equal(inf, (ref["inflated"] != 0).astype(np.uint8))
    assert np.array_equal(sk, (ref["skeleton"] != 0).astype(np.uint8))
