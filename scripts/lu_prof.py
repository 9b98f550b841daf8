"""invert_k's LU fallback timing: C3's design at a fitted-like length scale (Cholesky fails,
numba_kernels.py:370-403 falls back to np.linalg.inv) -- wall vs HIP events, for rocprofv3."""
import sys, time
import numpy as np
import torch
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo
import bench

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C3"]
ls_fit = float(sys.argv[2]) if len(sys.argv) > 2 else 680.0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
x, y, pm, pv, ls, betas, _, _ = bench.make_config_problem(cfg, 1)
n, n_obj = x.shape[0], len(pm)
dev = torch.device("cuda", 0)
xd = torch.tensor(x, device=dev)
km = torch.zeros((n_obj, n, n), dtype=torch.float64, device=dev)
bo.kernels.update_k(km, xd, 0, n, pv, np.full(n_obj, ls_fit))
g = lambda: bo.kernels.invert_k(n, km)
before = bo._lib.fit_path_counts()
g(); torch.cuda.synchronize()
print("fit paths after one call:", {k: v - before.get(k, 0) for k, v in bo._lib.fit_path_counts().items()})
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
e0.record()
for _ in range(reps):
    t0 = time.perf_counter(); g(); ts.append(time.perf_counter() - t0)
e1.record(); torch.cuda.synchronize()
print(f"invert_k (LU fallback) N={n} ls={ls_fit}: wall median {np.median(ts)*1e3:.3f} ms, "
      f"events {e0.elapsed_time(e1)/reps:.3f} ms per call", flush=True)
