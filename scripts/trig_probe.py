"""Powell fit time at a config with numpy's tan/atan through the Python callback vs the C library's
(evaluation points may differ in the last bit): what the callback costs per fit."""
import sys, os, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo
import bench

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "C3"]
x, y, pm, pv, ls, _, _, _ = bench.make_config_problem(cfg, 1)
n, n_obj = x.shape[0], len(pm)
dev = torch.device("cuda", 0)
xd, yd = torch.tensor(x, device=dev), torch.tensor(y, device=dev)
km = torch.zeros((n_obj, n, n), dtype=torch.float64, device=dev)
calls = [0]
orig = bo._lib._numpy_trig
for rep in range(3):
    for nt in (True, False):
        l2, p2 = ls.copy(), pv.copy()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = bo.kernels.optimize_hyperparams_mll(xd, yd, km, pm, p2, l2, n, numpy_trig=nt)
        torch.cuda.synchronize()
        print(f"numpy_trig={nt}: {1e3 * (time.perf_counter() - t0):.3f} ms nfev {r.nfev} fun {r.fun!r}", flush=True)
