import sys
sys.path[:0] = ["tools", "active-orchard-slam_amd", "tests"]
import numpy as np, torch
import aos_gpu, orchard
cfg = orchard.CONFIGS["C2"]
poly = orchard.polygon(cfg)
base = orchard.generate(cfg)
variant = sys.argv[1]
ref = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res)); ref.set_polygon(poly)
full = torch.from_numpy(base).to("cuda:0")
if "sync0" in variant: torch.cuda.synchronize()
r = ref.seedgen(full.data_ptr(), n_points=full.shape[0], on_device=True)
Ts = [r["thin_iters"]]
for k in range(2):
    scan = orchard.generate_scan(cfg, 40 * k)
    full = torch.cat([full, torch.from_numpy(scan).to("cuda:0")])
    torch.cuda.synchronize()
    if "host" in variant:
        r = ref.seedgen(full.cpu().numpy())
    else:
        r = ref.seedgen(full.data_ptr(), n_points=full.shape[0], on_device=True)
    Ts.append(r["thin_iters"])
    if "fresh" in variant:
        c2 = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res)); c2.set_polygon(poly)
        Ts.append(("fresh", c2.seedgen(full.cpu().numpy())["thin_iters"]))
        c2.close()
print(variant, Ts, flush=True)
