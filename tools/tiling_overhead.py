"""The tiled frame's overhead on one GPU, without gloo (verdict r05 item 1): C3 (8192^2, 40 M points) through
aos_group (the library's own rank threads, in-process peer-copy communicator) at a given tiling, every rank on
cuda:0. Run it under rocprofv3 --kernel-trace; the summary then adds up every kernel of the timed frames (all
ranks: the GPU time the tiling costs in all) and compares it with the 1 x 1 run.

run:        python tools/tiling_overhead.py run TX TY FRAMES WARMUP      (prints one JSON line: host ms per frame)
summarize:  python tools/tiling_overhead.py summarize OUT.json DIR_1x1 DIR_2x1 ...   (rocprofv3 -d directories)

The timed frames are bracketed in the trace by two marker kernels launched through torch (at::native ...), so
the warm-up frames, allocations and graph captures stay outside the sum.
"""
import csv
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tools"), os.path.join(ROOT, "active-orchard-slam_amd")):
    sys.path.insert(0, p)


def run(tx, ty, frames, warmup):
    import torch

    import aos_gpu
    import aos_tiles as T
    import orchard
    cfg = orchard.CONFIGS["C3"]
    cloud, poly = orchard.generate(cfg), orchard.polygon(cfg)
    params = aos_gpu.default_params(grid_resolution=cfg.res)
    world = tx * ty
    grp = aos_gpu.Group(params, [0] * world, tx, ty)
    grp.set_polygon(poly)
    shards = [T.shard(cloud, grp.plan(r)["points_box"]) for r in range(world)]
    d_shards = [torch.from_numpy(s).cuda() for s in shards]
    del cloud
    ptrs = [d.data_ptr() for d in d_shards]
    npts = [int(s.shape[0]) for s in shards]

    def frame():
        return grp.process(ptrs, root=0, want_host=False, on_device=True, n_points=npts)

    for _ in range(warmup):
        g = frame()
    torch.cuda.synchronize()
    torch.ones(1, device="cuda").add_(1)   # marker: the timed frames start
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms = []
    for _ in range(frames):
        t1 = time.perf_counter()
        g = frame()
        ms.append((time.perf_counter() - t1) * 1e3)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    torch.ones(1, device="cuda").add_(1)   # marker: they end
    torch.cuda.synchronize()
    ms.sort()
    print(json.dumps({"tiles": [tx, ty], "frames": frames, "ms_per_frame": round(dt / frames * 1e3, 3),
                      "ms_p50": round(ms[len(ms) // 2], 3), "thin_iters": g["thin_iters"], "n_clipped": g["n_clipped"],
                      "shard_points": [int(s.shape[0]) for s in shards]}), flush=True)
    grp.close()


COMM_COPIES = ("copyBuffer",)   # the in-process communicator's peer copies (xGMI / RCCL between GPUs)


def kernel_sum(d):
    """(sum of kernel durations, their union (GPU busy time), the union without the communicator's copies, launches,
    per-kernel sums) over the timed frames."""
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = sorted(csv.DictReader(open(tr[0])), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "at::native" in r["Kernel_Name"]]
    a, b = marks[0], marks[-1]
    per = {}
    tot = 0
    iv = []
    for r in rows[a + 1:b]:
        if "at::native" in r["Kernel_Name"]:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:60]
        per[name] = per.get(name, 0) + (e - s)
        tot += e - s
        iv.append((s, e, name))

    def union(xs):
        u, cs, ce = 0, None, None
        for s, e in sorted(xs):
            if cs is None:
                cs, ce = s, e
            elif s <= ce:
                ce = max(ce, e)
            else:
                u, cs, ce = u + ce - cs, s, e
        return u + (ce - cs if cs is not None else 0)
    busy = union([(s, e) for s, e, _ in iv])
    busy_nc = union([(s, e) for s, e, n in iv if not any(c in n for c in COMM_COPIES)])
    comm = sum(e - s for s, e, n in iv if any(c in n for c in COMM_COPIES))
    return tot, busy, busy_nc, comm, len(iv), per


def summarize(out, dirs):
    res = []
    for d in dirs:
        info = json.load(open(os.path.join(d, "run.json")))
        tot, busy, busy_nc, comm, n, per = kernel_sum(d)
        f = info["frames"]
        res.append({**info, "kernel_ms_per_frame": round(tot / f / 1e6, 3), "busy_ms_per_frame": round(busy / f / 1e6, 3),
                    "comm_copy_ms_per_frame": round(comm / f / 1e6, 3),
                    "kernel_ms_without_comm_copies": round((tot - comm) / f / 1e6, 3),
                    "launches_per_frame": round(n / f, 1),
                    "top_kernels_ms_per_frame": {k: round(v / f / 1e6, 3)
                                                 for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:12]}})
    base = next((r for r in res if r["tiles"] == [1, 1]), None)
    for r in res:
        if base:
            r["kernel_ratio_vs_1x1"] = round(r["kernel_ms_per_frame"] / base["kernel_ms_per_frame"], 3)
            r["kernel_ratio_without_comm_copies"] = round(r["kernel_ms_without_comm_copies"] /
                                                          base["kernel_ms_without_comm_copies"], 3)
    doc = {"what": "C3 (8192^2, 40 M points) through aos_group on ONE GPU (every rank a thread on cuda:0, the library's "
                   "peer-copy communicator) with AOS_GROUP_SERIAL=1: one rank at a time has GPU work in flight, so no "
                   "two kernels overlap and the sum of the kernel durations over the timed frames (rocprofv3 "
                   "--kernel-trace) is the sum over ranks of each rank's GPU time as it would run alone: the GPU time "
                   "the tiling costs in all, vs the 1 x 1 frame. comm_copy: the communicator's device copies "
                   "(runtime blit kernels here; RCCL over xGMI between GPUs). ms_per_frame: host clock, ranks taking "
                   "turns on the one GPU",
           "serial": os.environ.get("AOS_GROUP_SERIAL") == "1",
           "runs": res}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for r in res:
        print(r["tiles"], r["kernel_ms_per_frame"], r.get("kernel_ratio_vs_1x1"), r["kernel_ms_without_comm_copies"],
              r.get("kernel_ratio_without_comm_copies"), r["busy_ms_per_frame"], r["ms_per_frame"])


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(*(int(x) for x in sys.argv[2:6]))
    else:
        summarize(sys.argv[2], sys.argv[3:])
