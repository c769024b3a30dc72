"""One rank of a multi-process RCCL tiled frame on the ONE GPU of a test box (test_gpu_tiled.py::
test_rccl_ranks_as_processes starts `world` of these). Not a test module: a child process.

RCCL refuses two ranks on one device of one host ("Duplicate GPU detected"). Each rank here runs with its own
NCCL_HOSTID, so RCCL takes the ranks for separate hosts and connects them over its socket transport on the
loopback interface (NCCL_SOCKET_IFNAME=lo): the library's communicator (aos_rccl_*: ncclAllGather,
ncclAllReduce, grouped ncclSend / ncclRecv, all enqueued on the frame's stream) runs between real ranks; only
the wire differs from xGMI. Every rank runs the single-GPU frame of the whole cloud as its reference; the
frame's root compares its tiled outputs, grids and GvdGraph with it.

usage: rccl_rank_child.py RANK WORLD TILES_X TILES_Y UID_FILE
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tools"), os.path.join(ROOT, "active-orchard-slam_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import aos_gpu  # noqa: E402
import aos_tiles as T  # noqa: E402
import orchard  # noqa: E402
from parity_util import assert_seedgen_parity  # noqa: E402

GVD_KEYS = ("nodes", "edges", "edge_lengths", "edge_clearances", "node_labels", "node_cluster_indices",
            "node_label_counts", "node_label_clusters", "node_label_types")
GRIDS = ("inflated", "skeleton_frameless")


def main():
    rank, world, tx, ty = (int(a) for a in sys.argv[1:5])
    uid_file = sys.argv[5]
    cfg = orchard.CONFIGS["C1"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    params = aos_gpu.default_params(grid_resolution=cfg.res)

    ref = aos_gpu.Ctx(params, device=0)   # the single-GPU frame of the whole cloud
    ref.set_polygon(poly)
    g1 = ref.seedgen(cloud)
    grids1 = {w: ref.debug_grid(w, (g1["height"], g1["width"])) for w in GRIDS}
    gg1 = ref.gvd_from_seedgen()
    ref.close()

    if rank == 0:
        import ctypes
        uid = (ctypes.c_uint8 * 128)()
        aos_gpu._check(aos_gpu.lib().aos_rccl_unique_id(uid))
        with open(uid_file + ".tmp", "wb") as f:
            f.write(bytes(uid))
        os.replace(uid_file + ".tmp", uid_file)
    t0 = time.time()
    while not os.path.exists(uid_file):
        if time.time() - t0 > 120:
            raise RuntimeError("no unique id from rank 0")
        time.sleep(0.05)
    with open(uid_file, "rb") as f:
        uid = f.read()

    plan = T.tile_plan(params, poly, tx, ty, rank)
    part = T.shard(cloud, plan["points_box"])
    comm = T.RcclComm(plan["exchange_bytes"], device=0, rank=rank, world=world, unique_id=uid)
    ctx = aos_gpu.Ctx(params, device=0)
    ctx.set_polygon(poly)
    report = {"rank": rank, "frames": []}
    # frame k: root k mod world; the last frame's cluster exchange goes in 4 KB rounds
    frames = [(k % world, 0) for k in range(world)] + [(world - 1, 4096)]
    for k, (root, rounds) in enumerate(frames):
        aos_gpu.debug_faults(a2a_round_bytes=rounds)
        g = ctx.tiled_seedgen(comm, tx, ty, part, root=root)
        aos_gpu.debug_faults()
        st = ctx.tiled_stats()
        assert (g["thin_iters"], g["n_clipped"]) == (g1["thin_iters"], g1["n_clipped"]), k
        assert bool(g["root"]) == (rank == root), k
        if rank == root:
            assert_seedgen_parity(g, {**g1, "cluster_length": np.zeros(g1["n_clusters_all"])})
            assert g["n_bfs_replayed"] == g1["n_bfs_replayed"]
            for w in GRIDS:
                assert np.array_equal(ctx.debug_grid(w, (g["height"], g["width"])), grids1[w]), (k, w)
            gg = ctx.gvd_from_seedgen()
            assert gg["published"] == gg1["published"]
            for key in GVD_KEYS:
                assert np.array_equal(gg[key], gg1[key]), (k, key)
        report["frames"].append({"root": root, "rounds": rounds, "n_gather": st["n_gather"],
                                 "gather_MB": round(st["bytes_gather"] / 1e6, 3), "recv_MB": round(st["bytes_recv"] / 1e6, 3),
                                 "ms_frame": round(st["ms_frame"], 2),
                                 "ms_comm_gather": round(st["ms_comm_gather"], 2)})
    ctx.close()
    comm.close()
    print("RCCL_RANK_OK " + json.dumps(report), flush=True)


if __name__ == "__main__":
    main()
