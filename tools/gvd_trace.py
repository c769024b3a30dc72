"""Host timeline of the GVD calls on one C2 frame (AOS_TRACE=1 marks on stderr) plus the median of each
phase's duration over --reps calls (diagnostics: where the replay-bound GVD call spends its host time)."""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys
sys.path[:0] = [{tools!r}, {pkg!r}]
import aos_gpu, orchard
cfg = orchard.CONFIGS["C2"]
c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res, gvd_markers=0))
c.set_polygon(orchard.polygon(cfg))
c.seedgen(orchard.generate(cfg), want_host=False)
for r in range({reps}):
    c.gvd_from_seedgen()
c.close()
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    code = CHILD.format(tools=os.path.join(ROOT, "tools"), pkg=os.path.join(ROOT, "active-orchard-slam_amd"), reps=a.reps + 2)
    env = dict(os.environ, AOS_TRACE="1")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    if p.returncode:
        sys.stderr.write(p.stderr[-3000:])
        sys.exit(p.returncode)
    rows = [ln for ln in p.stderr.splitlines() if ln.startswith("[aos trace gvd]")][2:]
    phases = {}
    for ln in rows:
        marks = re.findall(r" (\w+) ([0-9.]+)", ln.split(":", 1)[1])
        prev = 0.0
        for name, t in marks:
            phases.setdefault(name, []).append(float(t) - prev)
            prev = float(t)
    print(rows[-1])
    for k, v in phases.items():
        v.sort()
        print(f"{k:14s} p50 {v[len(v) // 2]:8.3f} ms  min {v[0]:8.3f}")


if __name__ == "__main__":
    main()
