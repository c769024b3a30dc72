"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes per kernel.

MI355X_MICROARCH.md 'HBM': FETCH_SIZE and WRITE_SIZE are reported in KiB and come from separate
passes on gfx950 (TCC slots); FETCH_SIZE reports half the bytes of 16 B/lane streaming reads, so it
is doubled here; WRITE_SIZE is taken as is.

usage: python tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv OUT.json
"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("aos::", "").replace("void ", "").strip()
        acc[name].append(float(r["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes ({sys.argv[1]}, {sys.argv[2]})",
           "correction": "FETCH_SIZE x2 (gfx950, 16 B/lane streaming reads); KiB -> bytes", "kernels": {}}
    for k in sorted(set(fetch) & set(write)):
        f, nf = fetch[k]
        w, nw = write[k]
        out["kernels"][k] = {"fetch_bytes_raw": f, "fetch_bytes": 2.0 * f, "write_bytes": w,
                             "bytes_per_launch": 2.0 * f + w, "launches": [nf, nw]}
    # the ROR stage a1-a4 (one launch of each per frame): count + column scan (k_rt_colscan; round 3:
    # k_rt_colsum / colpre / colfix) + scatter + the big-tile kernels (k_rt_big*) + the per-tile neighbour
    # counts (k_rt_ror<...>) + the staged array's read-ahead during the upload (k_rt_touch, round 4)
    parts = [k for k in out["kernels"] if k.startswith(("k_rt_part", "k_rt_col", "k_rt_big", "k_rt_ror", "k_rt_touch"))]
    # the timed frames read the host upload's packed cloud (layout 2); a device-resident frame of the same run (the
    # bench's counted GVD frame) launches the layout-1 partition passes, which are not this stage's
    if any(k.startswith("k_rt_part<") and ", 2," in k for k in parts):
        parts = [k for k in parts if not (k.startswith("k_rt_part<") and ", 2," not in k)]
    if parts:
        out["kernels"]["ror_stage"] = {"bytes_per_launch": sum(out["kernels"][k]["bytes_per_launch"] for k in parts),
                                       "kernels": sorted(parts)}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    top = sorted(out["kernels"].items(), key=lambda kv: -kv[1]["bytes_per_launch"])[:8]
    for k, v in top:
        print(f"{k:40s} {v['bytes_per_launch'] / 1e6:10.2f} MB/launch")


if __name__ == "__main__":
    main()
