"""bench.py's multi-rank path on CPU (gloo, world_size 2): barrier-bracketed timed region, max over
ranks, whole-job throughput, and one independent tile (scene seed + rank) per rank."""
import os
import socket
import sys
import time

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import orchard  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def step():
        calls.append(1)
        time.sleep(0.02 * (rank + 1))   # rank 1 is the slow one
        return rank

    dt, res, per = bench.timed_region(step, steps=3, warmup=2, world=world, sync=lambda: None, dist=dist, device="cpu")
    q.put((rank, dt, len(calls), len(res), per))
    dist.destroy_process_group()


def test_timed_region_max_over_ranks_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    dts = {r: dt for r, dt, _, _, _ in out}
    pers = {r: per for r, _, _, _, per in out}
    # both ranks report the same (max) time, at least the slow rank's 3 x 40 ms
    assert abs(dts[0] - dts[1]) < 1e-12
    assert dts[0] >= 3 * 0.04
    # per-step times are max-reduced too (the median frame time is taken over them)
    assert pers[0] == pers[1] and len(pers[0]) == 3 and min(pers[0]) >= 0.04
    for _, _, ncalls, nres, _ in out:
        assert ncalls == 5 and nres == 3     # W untimed + exactly K timed steps


def test_throughput_is_whole_job():
    # 16.78 Mcells per step per rank, 2 ranks, 4 steps in 0.5 s
    assert abs(bench.throughput(16.777216, 2, 4, 0.5) - 268.435456) < 1e-9


def test_independent_tile_per_rank():
    cfg = orchard.CONFIGS["C0"]
    a = orchard.generate(cfg, seed=cfg.seed + 0, n_points=5000)
    b = orchard.generate(cfg, seed=cfg.seed + 1, n_points=5000)
    assert a.shape == b.shape and not np.array_equal(a, b)


def _hang_worker(q):
    """bench.tiled_extra with a tiled run that never returns (a collective that hangs): its watchdog must
    print rank 0's main result with the tiled error and end the process with a non-zero status, so the hang
    shows in the run's exit code (verdict r03)."""
    import argparse
    os.environ["AOS_BENCH_TILED_TIMEOUT"] = "1"
    bench.run = lambda *a, **k: time.sleep(3600)
    a = argparse.Namespace(steps=20, warmup=5, tiled=False, config="C2", no_cpu_baseline=False)
    bench.tiled_extra(a, {"rank": 0}, None, {"value": 1.0})


def test_tiled_extra_watchdog_and_error(capfd):
    import subprocess
    code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r); import test_bench_dist as t; "
            "t._hang_worker(None)" % (ROOT, os.path.join(ROOT, "tests")))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == bench.WATCHDOG_EXIT != 0
    assert "did not finish" in p.stderr
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
    import json
    d = json.loads(line)
    assert d["value"] == 1.0 and "did not finish" in d["tiled"]["error"]
    # a tiled run that raises is reported without losing the main result
    import argparse
    old = bench.run
    try:
        def boom(*a, **k):
            raise RuntimeError("rccl init failed")
        bench.run = boom
        a = argparse.Namespace(steps=20, warmup=5, tiled=False, config="C2", no_cpu_baseline=False)
        t = bench.tiled_extra(a, {"rank": 0}, None, {"value": 1.0})
        assert t == {"error": "RuntimeError: rccl init failed"}
    finally:
        bench.run = old


def test_tiled_stream_extra_configuration():
    """The --gpus N launch's second extra (tiled_stream, BASELINE configs[4] over the ranks): bench.run gets a
    tiled C4 configuration (C2 map + scans, sequential scans), and a failure is reported under its own key."""
    import argparse
    seen = {}
    old = bench.run
    try:
        def fake(b, E, dist, quiet=False):
            seen.update(tiled=b.tiled, stream=b.stream, config=b.config, steps=b.steps, warmup=b.warmup,
                        cpu=b.no_cpu_baseline)
            return {"value": 2.0, "stream": {"scan_latency_ms_p50": 1.0}, "extra": 1}
        bench.run = fake
        a = argparse.Namespace(steps=20, warmup=5, tiled=False, stream=False, config="C2", no_cpu_baseline=False)
        t = bench.tiled_extra(a, {"rank": 0}, None, {"value": 1.0}, stream=True)
        assert seen == {"tiled": True, "stream": True, "config": "C2", "steps": 16, "warmup": 2, "cpu": True}
        assert t == {"value": 2.0, "stream": {"scan_latency_ms_p50": 1.0}}
        assert bench.parse(["--tiled", "--stream"]).config == "C2" and bench.parse(["--tiled"]).config == "C3"
    finally:
        bench.run = old


def test_tiled_breakdown_keys():
    """--gpus N tiled lines: per rank, the frame split into time inside the all-gather / all-reduce callbacks
    and compute, and the root's serial part split into cluster stage (replays), rows + seeds and GVD prefix."""
    def st(root, frame, gather, reduce, cluster=0.0, replay=0.0, seeds=0.0, skipped=0):
        return {"ms_frame": frame, "ms_comm_gather": gather, "ms_comm_reduce": reduce, "n_gather": 5, "n_reduce": 3,
                "bytes_gather": 2_000_000, "ms_ror": 1.0, "ms_thin": 0.5, "ms_cluster": cluster, "ms_seeds": seeds,
                "ms_cluster_local": 0.2, "ms_cluster_global": 0.7, "ms_replay": replay, "n_replayed": 1,
                "ror_skipped": skipped, "is_root": int(root)}
    res = [({"root": True, "tiled_stats": st(True, 10.0, 2.0, 1.0, cluster=3.0, replay=1.5, seeds=1.0)}, None),
           ({"root": False, "tiled_stats": st(False, 8.0, 3.0, 1.0, skipped=1)}, None)]
    pend = {"gvd_start": {4: 0.004}}
    per_rank, split = bench.tiled_breakdown(res, pend, warmup=4, world=1, rank=0, dist=None)
    r0 = per_rank[0]
    assert r0["frames"] == 2 and r0["ms_frame"] == 9.0 and r0["ms_comm_gather"] == 2.5 and r0["ms_comm_reduce"] == 1.0
    assert r0["ms_compute"] == 5.5 and r0["collectives_per_frame"] == 8.0 and r0["ror_skipped_frames"] == 1
    assert split == {"cluster_stage": 3.0, "of_which_replays_on_root": 1.5, "rows_and_seeds": 1.0, "gvd_prefix": 4.0,
                     "root_frames": 1}


def test_pick_tiled_frames_rotating_roots():
    """bench --tiled at 4 ranks (rotating roots, pipelined GVD): rank 0's timed steps are mostly non-root
    results, and a step's graph is an older frame's. The report takes the last root frame and the last graph
    separately (round 4: pairing them made a 4-rank run look up rows in a non-root result)."""
    nonroot = {"root": False, "width": 8, "height": 8, "thin_iters": 3}
    root = {"root": True, "width": 8, "height": 8, "thin_iters": 3, "row_length": [1.0], "voronoi_seeds": [[0, 0]]}
    graph = {"nodes": [[0, 0]], "edges": []}
    res = [(nonroot, None), (root, None), (nonroot, graph), (nonroot, None)]
    g, gg = bench.pick_tiled_frames(res, res[-1][0], res[-1][1])
    assert g is root and gg is graph
    g, gg = bench.pick_tiled_frames([(nonroot, None)], nonroot, None)   # no root frame, no graph
    assert g is nonroot and gg is None


def _tiled_raise_worker():
    """bench.report for a --gpus 2 launch whose tiled sections raise (e.g. RCCL failing to load on the 8-GPU
    node): rank 0 prints the main line with the errors and the process exits non-zero (verdict r04 item 5)."""
    import argparse

    class FakeDist:
        def destroy_process_group(self):
            pass

    def boom(*a, **k):
        raise RuntimeError("ncclCommInitRank: unhandled system error")
    bench.run = boom
    a = argparse.Namespace(steps=20, warmup=5, tiled=False, stream=False, config="C2", no_cpu_baseline=False,
                           no_tiled_rate=False)
    E = {"world": 2, "rank": 0}
    sys.exit(bench.report(a, E, FakeDist(), {"value": 1.0}))


def test_tiled_error_exits_nonzero():
    import json
    import subprocess
    code = ("import sys; sys.path.insert(0, %r); sys.path.insert(0, %r); import test_bench_dist as t; "
            "t._tiled_raise_worker()" % (ROOT, os.path.join(ROOT, "tests")))
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert p.returncode == bench.TILED_ERROR_EXIT != 0, p.stderr
    d = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert d["value"] == 1.0
    assert "ncclCommInitRank" in d["tiled"]["error"] and "ncclCommInitRank" in d["tiled_stream"]["error"]
    assert "tiled section failed" in p.stderr
    # a clean run exits 0; a tiled section that returned a result is not an error
    assert bench.exit_status({"tiled": {"value": 3.0}, "tiled_stream": None}) == 0
    assert bench.exit_status(None) == 0


def test_ror_points_read_mean_over_timed_frames():
    """The roofline's bytes: the mean of n_ror_read over the timed frames; a skipped stage reads 0."""
    res = [({"n_ror_read": 100}, None), ({"n_ror_read": 0}, None), ({"n_ror_read": 200}, None)]
    assert bench.ror_points_read(res, 999) == 100.0
    assert bench.ror_points_read([({}, None)], 7) == 7.0


def test_cpu_baseline_child_process():
    """The CPU baseline in its own process pinned to one core (started before the GPU is touched, told to start
    after the main timed region); this process keeps the other cores."""
    import argparse
    allowed = os.sched_getaffinity(0)
    try:
        child = bench.spawn_cpu_baseline(argparse.Namespace(cpu_config="C0"))
        if child is None:   # a one-core CPU set: the baseline runs inline
            assert len(allowed) < 2
            return
        assert child.core not in os.sched_getaffinity(0)
        r = bench.finish_cpu_baseline(child)
    finally:
        os.sched_setaffinity(0, allowed)
    assert child.returncode == 0 and r["cores"] == 1 and r["kind"] == "port" and r["value"] > 0
    assert r["pinned_core"] == child.core and "child process" in r["sample"]
