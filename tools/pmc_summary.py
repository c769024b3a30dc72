"""Per-kernel averages of rocprofv3 --pmc counter_collection CSVs (one or more pass directories).

usage: python tools/pmc_summary.py DIR [DIR ...] [--match SUBSTR]
Prints, per kernel, each counter's mean over its launches; SQ wave-cycle counters as a share of
SQ_WAVE_CYCLES where that counter is present.
"""
import collections
import csv
import glob
import os
import sys


def load(dirs):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("aos::", "").strip()
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = None
    if "--match" in sys.argv:
        match = sys.argv[sys.argv.index("--match") + 1]
        args = [a for a in args if a != match]
    acc = load(args)
    for k in sorted(acc):
        if match and match not in k:
            continue
        c = {n: sum(v) / len(v) for n, v in acc[k].items()}
        wc = c.get("SQ_WAVE_CYCLES")
        parts = []
        for n in sorted(c):
            s = f"{n}={c[n]:.4g}"
            if wc and n.startswith(("SQ_WAIT", "SQ_ACTIVE")):
                s += f" ({100 * c[n] / wc:.0f}%)"
            parts.append(s)
        print(f"{k[:60]:60s} " + " ".join(parts))


if __name__ == "__main__":
    main()
