"""Per frame of a rocprofv3 kernel trace: which kernels ran while a given kernel ran (the cluster stage's k_fg beside
the runtime's copy kernels). usage: python tools/kt_overlap.py kt_kernel_trace.csv [kernel-prefix]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    key = sys.argv[2] if len(sys.argv) > 2 else "aos::k_fg("
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:48], r["Stream_Id"])
          for r in rows]
    ev.sort()
    for s, e, name, st in ev:
        if not name.startswith(key.split("(")[0]):
            continue
        beside = [(max(s, s2), min(e, e2), n2, st2) for s2, e2, n2, st2 in ev
                  if n2 != name and s2 < e and e2 > s]
        desc = ", ".join(f"{n2} {1e-3 * (b - a):.1f} us" for a, b, n2, _ in beside) or "-"
        print(f"{name} {1e-3 * (e - s):7.1f} us  beside: {desc}")


if __name__ == "__main__":
    main()
