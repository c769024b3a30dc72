"""Tiled multi-GPU frames (include/aos_gpu.h: aos_tile_plan_compute, aos_tiled_seedgen_process).

One map is split into tiles_x x tiles_y tiles, one rank per tile. This module holds the
host-side pieces a rank needs besides its aos_gpu.Ctx: the tile plan, the point shard of its tile, and
the communicators the library calls back into (aos_comm):
  - TorchDistComm: a torch.distributed process group; 'nccl' is RCCL, whose all-gather moves the
    device buffers over xGMI directly; gloo stages through host memory (CPU tests, rehearsals).
  - ThreadGroup: ranks as threads of one process (e.g. every tile of a map on the one GPU of a test box).
  - RcclComm: the library's own C++ communicator over RCCL (aos_rccl_*): one process per GPU, the
    collectives run without calling back into Python.
"""
from __future__ import annotations

import ctypes

import numpy as np

from aos_gpu import AllGatherFn, AllReduceMaxFn, AllToAllFn, Comm, Params, TilePlan, _check, lib


def tile_plan(params: Params, poly_xy, tiles_x: int, tiles_y: int, rank: int) -> dict:
    """aos_tile_plan_compute (host arithmetic, no GPU): the tile, halo window and point box of `rank`."""
    a = None if poly_xy is None else np.ascontiguousarray(poly_xy, dtype=np.float64).reshape(-1)
    t = TilePlan()
    _check(lib().aos_tile_plan_compute(ctypes.byref(params), None if a is None else a.ctypes.data,
                                       0 if a is None else a.size // 2, tiles_x, tiles_y, rank, ctypes.byref(t)))
    d = {k: getattr(t, k) for k, _ in TilePlan._fields_ if k not in ("points_box", "info")}
    d.update(points_box=tuple(t.points_box), width=t.info.width, height=t.info.height,
             origin=(t.info.origin_x, t.info.origin_y), resolution=t.info.resolution)
    return d


def tiling_for(world: int) -> tuple[int, int]:
    """(tiles_x, tiles_y) with tiles_x * tiles_y = world and tiles_x >= tiles_y; 8 ranks -> 4 x 2, the
    SURVEY §8e split of 8192^2 into tiles of 4096 rows x 2048 columns."""
    ty = int(np.sqrt(world))
    while world % ty:
        ty -= 1
    return world // ty, ty


def shard(cloud: np.ndarray, box, point_step=16, offs=(0, 4)) -> np.ndarray:
    """The records of a PointCloud2 byte array whose x/y lie inside a tile's points_box (inclusive)."""
    rec = np.ascontiguousarray(cloud).reshape(-1, point_step)
    x = rec[:, offs[0]:offs[0] + 4].copy().view(np.float32)[:, 0]
    y = rec[:, offs[1]:offs[1] + 4].copy().view(np.float32)[:, 0]
    m = (x >= box[0]) & (x <= box[2]) & (y >= box[1]) & (y <= box[3])
    return rec[m]


class _CommBase:
    """An aos_comm whose collectives are Python callables. send / recv are torch uint8 tensors on the
    rank's device (registered with the library once); `error` keeps the exception of a failed callback."""

    def __init__(self, rank: int, world: int, buf_bytes: int, device):
        import torch
        self.rank, self.world, self.device = rank, world, torch.device(device)
        self.buf_bytes = int(buf_bytes)
        self.send = torch.zeros(max(self.buf_bytes, 1), dtype=torch.uint8, device=self.device)
        self.recv = torch.zeros(max(world * self.buf_bytes, 1), dtype=torch.uint8, device=self.device)
        self.error = None
        self._ag = AllGatherFn(self._all_gather_cb)
        self._ar = AllReduceMaxFn(self._all_reduce_cb)
        self._a2a = AllToAllFn(self._all_to_all_cb)
        self.c = Comm(None, rank, world, self.send.data_ptr(), self.recv.data_ptr(), self.buf_bytes, self._ag,
                      self._ar, self._a2a)

    def without_all_to_all(self):
        """The same communicator without the optional all_to_all (the library then routes through all_gather)."""
        self.c.all_to_all = AllToAllFn()
        return self

    def _splits(self, counts):
        m = np.ctypeslib.as_array(counts, shape=(self.world * self.world,)).reshape(self.world, self.world)
        return [int(x) for x in m[self.rank, :]], [int(x) for x in m[:, self.rank]]

    def _sync(self):
        if self.device.type == "cuda":
            import torch
            torch.cuda.synchronize(self.device)

    def _all_gather_cb(self, user, nbytes):
        try:
            self.all_gather(int(nbytes))
            self._sync()
            return 0
        except BaseException as e:   # noqa: BLE001 — re-raised by Ctx.tiled_seedgen
            self.error = e
            self.abort()
            return -1

    def _all_to_all_cb(self, user, counts):
        try:
            send_split, recv_split = self._splits(counts)
            self.all_to_all(send_split, recv_split)
            self._sync()
            return 0
        except BaseException as e:   # noqa: BLE001
            self.error = e
            self.abort()
            return -1

    def _all_reduce_cb(self, user, ptr, n):
        try:
            a = np.ctypeslib.as_array(ptr, shape=(n,))
            a[:] = self.all_reduce_max(a.copy())
            return 0
        except BaseException as e:   # noqa: BLE001
            self.error = e
            self.abort()
            return -1

    def abort(self):
        pass


class TorchDistComm(_CommBase):
    """aos_comm over a torch.distributed process group (the default group unless `group` is given)."""

    def __init__(self, buf_bytes: int, device, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.nccl = dist.get_backend(group) == "nccl"
        super().__init__(dist.get_rank(group), dist.get_world_size(group), buf_bytes, device)

    def all_gather(self, n: int):
        import torch
        if self.nccl:
            self.dist.all_gather_into_tensor(self.recv[: n * self.world], self.send[:n], group=self.group)
            return
        s = self.send[:n].cpu()
        parts = [torch.empty_like(s) for _ in range(self.world)]
        self.dist.all_gather(parts, s, group=self.group)
        self.recv[: n * self.world].copy_(torch.cat(parts))

    def all_to_all(self, send_split, recv_split):
        import torch
        ns, nr = sum(send_split), sum(recv_split)
        if self.nccl:
            self.dist.all_to_all_single(self.recv[:nr], self.send[:ns], output_split_sizes=recv_split,
                                        input_split_sizes=send_split, group=self.group)
            return
        out = torch.empty(nr, dtype=torch.uint8)
        self.dist.all_to_all_single(out, self.send[:ns].cpu(), output_split_sizes=recv_split,
                                    input_split_sizes=send_split, group=self.group)
        self.recv[:nr].copy_(out)

    def all_reduce_max(self, a: np.ndarray) -> np.ndarray:
        import torch
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32))
        if self.nccl:
            t = t.to(self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return t.cpu().numpy()


class RcclComm:
    """aos_comm implemented in libaos_gpu.so over RCCL (aos_rccl_create): ncclAllGather of the library's
    HBM exchange buffers and ncclAllReduce(max) of the flags, no Python in the collectives. Rank 0 makes
    the unique id; a torch.distributed group (any backend) carries it to the other ranks, or pass
    `unique_id` (128 bytes) directly. Collective: every rank constructs it at the same time."""

    def __init__(self, buf_bytes: int, device: int, rank: int = 0, world: int = 1, group=None,
                 unique_id: bytes | None = None):
        self.rank, self.world, self.error = rank, world, None
        if unique_id is None:
            uid = (ctypes.c_uint8 * 128)()
            if rank == 0:
                _check(lib().aos_rccl_unique_id(uid))
            if world > 1:
                import torch.distributed as dist
                box = [bytes(uid)]
                dist.broadcast_object_list(box, src=0, group=group)
                uid = (ctypes.c_uint8 * 128).from_buffer_copy(box[0])
        else:
            uid = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(unique_id))
        self._h = ctypes.c_void_p()
        _check(lib().aos_rccl_create(uid, rank, world, int(device), int(buf_bytes), ctypes.byref(self._h)))
        self.c = Comm.from_buffer_copy(ctypes.string_at(lib().aos_rccl_comm(self._h), ctypes.sizeof(Comm)))

    def close(self):
        if self._h:
            lib().aos_rccl_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:   # noqa: BLE001 — interpreter shutdown
            pass


class ThreadGroup:
    """In-process communicator for `world` ranks driven by threads, one handle per thread. The barrier
    times out, so a failed rank cannot hang the others."""

    def __init__(self, world: int, timeout: float = 120.0):
        import threading
        self.world = world
        self.barrier = threading.Barrier(world, timeout=timeout)
        self.slots = [None] * world

    def comm(self, rank: int, buf_bytes: int, device) -> "_ThreadComm":
        return _ThreadComm(self, rank, buf_bytes, device)

    def abort(self):
        self.barrier.abort()


class _ThreadComm(_CommBase):
    def __init__(self, group: ThreadGroup, rank: int, buf_bytes: int, device):
        self.g = group
        super().__init__(rank, group.world, buf_bytes, device)

    def all_gather(self, n: int):
        g = self.g
        g.slots[self.rank] = self.send[:n]
        g.barrier.wait()
        for r in range(self.world):
            self.recv[r * n:(r + 1) * n].copy_(g.slots[r])
        self._sync()
        g.barrier.wait()   # every rank has read every send buffer before any is overwritten

    def all_to_all(self, send_split, recv_split):
        g = self.g
        g.slots[self.rank] = (self.send, send_split)
        g.barrier.wait()
        at = 0
        for r in range(self.world):
            buf, split = g.slots[r]
            off = sum(split[:self.rank])
            n = split[self.rank]
            assert n == recv_split[r]
            self.recv[at:at + n].copy_(buf[off:off + n])
            at += n
        self._sync()
        g.barrier.wait()

    def all_reduce_max(self, a: np.ndarray) -> np.ndarray:
        g = self.g
        g.slots[self.rank] = np.asarray(a, dtype=np.int32)
        g.barrier.wait()
        out = np.max(np.stack(g.slots), axis=0)
        g.barrier.wait()
        return out

    def abort(self):
        self.g.abort()
