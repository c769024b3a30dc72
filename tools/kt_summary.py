"""Per-frame summary of a rocprofv3 --kernel-trace --stats directory.

usage: python tools/kt_summary.py <rocprof out dir> <frames in the run>

Prints launches and GPU time per frame (all kernels, and grouped: rocprim/hipcub, copies, fills, ROR
stage, greedy / look-back kernels, the rest), then the kernels by total time. Copies and fills are the
runtime's blit kernels (__amd_rocclr_*); "host stores" are the library's kernels whose time is writing pinned
host memory across PCIe (k_copy_host, k_peek_host, k_gather_words). With the kernel trace present it also
prints the median frame from the trace itself (kernels between consecutive k_rt_touch launches: a frame's
first kernel), which leaves out the run's other work (warm-up allocations, the counted GVD frame).
"""
import csv
import glob
import os
import sys


def main():
    d, frames = sys.argv[1], int(sys.argv[2])
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not stats:
        print("no kernel_stats.csv under", d)
        return
    rows = list(csv.DictReader(open(stats[0])))
    groups = {"rocprim": ("rocprim", "hipcub"), "copies": ("copyBuffer", "copyImage"), "fills": ("fillBuffer",),
              "host stores": ("k_copy_host", "k_peek_host", "k_gather_words"),
              "ror": ("k_rt_",), "dedup/scan": ("k_lfmis", "k_dedup_small", "k_scan_1p", "k_ci_")}
    tot_n = tot_t = 0.0
    g_n = {k: 0.0 for k in groups}
    g_t = {k: 0.0 for k in groups}
    for r in rows:
        n, t = float(r["Calls"]), float(r["TotalDurationNs"])
        tot_n += n
        tot_t += t
        for k, pats in groups.items():
            if any(p in r["Name"] for p in pats):
                g_n[k] += n
                g_t[k] += t
                break
    print(f"per frame ({frames} frames): {tot_n / frames:.1f} launches, {tot_t / frames / 1e3:.1f} us GPU time")
    for k in groups:
        print(f"  {k:12s} {g_n[k] / frames:7.1f} launches {g_t[k] / frames / 1e3:9.1f} us")
    frame_from_trace(d)
    print("kernels by total time (per frame: calls, us; average us):")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        print(f"  {float(r['Calls']) / frames:6.1f} {float(r['TotalDurationNs']) / frames / 1e3:9.1f} "
              f"{float(r['AverageNs']) / 1e3:9.2f}  {r['Name'][:110]}")


def frame_from_trace(d):
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not tr:
        return
    rows = sorted(csv.DictReader(open(tr[0])), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "k_rt_touch" in r["Kernel_Name"]]
    per = []
    for a, b in zip(starts, starts[1:]):
        n = b - a
        t = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b])
        copy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b]
                   if "copyBuffer" in r["Kernel_Name"] or "k_copy_host" in r["Kernel_Name"] or
                   "k_peek_host" in r["Kernel_Name"] or "k_gather_words" in r["Kernel_Name"])
        per.append((n, t / 1e3, copy / 1e3))
    if not per:
        return
    per.sort()
    n_med = per[len(per) // 2][0]
    t_med = sorted(p[1] for p in per)[len(per) // 2]
    nc_med = sorted(p[1] - p[2] for p in per)[len(per) // 2]
    print(f"trace frames ({len(per)}): median {n_med} launches, {t_med:.1f} us kernel time, {nc_med:.1f} us without "
          f"copies and host stores (min / max launches {per[0][0]} / {per[-1][0]})")


if __name__ == "__main__":
    main()
