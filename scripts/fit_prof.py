"""Fit timing probe: compute_mll / invert_k at one N, wall vs device (HIP events), for rocprofv3."""
import sys, time
import numpy as np
import torch
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo
import bench

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C3"]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
x, y, pm, pv, ls, betas, _, _ = bench.make_config_problem(cfg, 1)
n, n_obj = x.shape[0], len(pm)
dev = torch.device("cuda", 0)
xd, yd = torch.tensor(x, device=dev), torch.tensor(y, device=dev)
km = torch.zeros((n_obj, n, n), dtype=torch.float64, device=dev)
f = lambda: bo.kernels.compute_mll(xd, yd, km, pm, pv, ls, n)
g = lambda: bo.kernels.invert_k(n, km)
for fn, name in ((f, "mll"), (g, "inv")):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    e0.record()
    for _ in range(reps):
        t0 = time.perf_counter(); fn(); ts.append(time.perf_counter() - t0)
    e1.record(); torch.cuda.synchronize()
    print(f"{name} N={n}: wall median {np.median(ts)*1e3:.4f} ms, events {e0.elapsed_time(e1)/reps:.4f} ms per call", flush=True)

# diagnostic build: per-launch phase stamps (panel WG 0: 1 start, 2 MFMA done, 3 factor done;
# update WG 0: 8 start, 9 done) of one more MLL call
lib = bo._lib.load()
if hasattr(lib, "bo_debug_fit_timing"):
    import ctypes
    buf = (ctypes.c_longlong * 8192)()
    lib.bo_debug_fit_timing(buf, 4096)
    f(); torch.cuda.synchronize()
    cnt = lib.bo_debug_fit_timing(buf, 4096)
    ev = sorted((buf[2 * i + 1], buf[2 * i] >> 16, buf[2 * i] & 15) for i in range(cnt))
    t0 = ev[0][0]
    by_k = {}
    for t, k, tag in ev:
        by_k.setdefault(k, {})[tag] = (t - t0) * 0.01   # 100 MHz -> us
    for k in sorted(by_k):
        print("k", k, " ".join(f"{tag}:{v:.2f}" for tag, v in sorted(by_k[k].items())))
