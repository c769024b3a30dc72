"""Per-frame summary of a rocprofv3 --kernel-trace --stats directory.

usage: python tools/kt_summary.py <rocprof out dir> <frames in the run>

Prints launches and GPU time per frame (all kernels, and grouped: rocprim/hipcub, copies, fills, ROR
stage, greedy / look-back kernels, the rest), then the kernels by total time. Copies and fills are the
runtime's blit kernels (__amd_rocclr_*).
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
    print("kernels by total time (per frame: calls, us; average us):")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        print(f"  {float(r['Calls']) / frames:6.1f} {float(r['TotalDurationNs']) / frames / 1e3:9.1f} "
              f"{float(r['AverageNs']) / 1e3:9.2f}  {r['Name'][:110]}")


if __name__ == "__main__":
    main()
