import sys, time, os
sys.path.insert(0, "tools"); sys.path.insert(0, "active-orchard-slam_amd")
import torch, numpy as np
import aos_gpu, orchard
cfg = orchard.CONFIGS["C2"]
cloud = orchard.generate(cfg)
d = torch.from_numpy(cloud).to("cuda:0")
c = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res)); c.set_polygon(orchard.polygon(cfg))
def t(f, k=5):
    f(); torch.cuda.synchronize()
    ts = []
    for _ in range(k):
        t0 = time.perf_counter(); f(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    return 1e3 * min(ts)
print("device in, device out  %.2f ms" % t(lambda: c.seedgen(d.data_ptr(), n_points=cloud.shape[0], on_device=True, want_host=False)))
print("host in,   device out  %.2f ms" % t(lambda: c.seedgen(cloud, want_host=False)))
print("device in, host out    %.2f ms" % t(lambda: c.seedgen(d.data_ptr(), n_points=cloud.shape[0], on_device=True, want_host=True)))
print("host in,   host out    %.2f ms" % t(lambda: c.seedgen(cloud, want_host=True)))
x = np.empty(16_777_216, np.int8)
print("numpy copy of one grid %.2f ms" % t(lambda: x.copy()))
import ctypes
L = aos_gpu.lib()
v, keep = aos_gpu.Ctx._view(d.data_ptr(), cloud.shape[0], 16, (0, 4, 8), True, True)
o = aos_gpu.SeedGenOut()
def call(wh):
    L.aos_seedgen_process(c.h, ctypes.byref(v), wh, ctypes.byref(o))
print("C call, device out     %.2f ms" % t(lambda: call(0)))
print("C call, host out       %.2f ms" % t(lambda: call(1)))
n = o.info.width * o.info.height
print("numpy copy from pinned %.2f ms" % t(lambda: np.ctypeslib.as_array(o.occupancy, shape=(n,)).astype(np.int8, copy=True)))
