"""Is the fused predict's time data-dependent?  The C3 problem at N = 512 with the bench's state
and with the loop's (l = 680, K^-1 from the device LU path), back to back, interleaved.  Run with
BO_AMD_LIB pointing at an ablation build (BO_BUILD_VARIANT=NOTOPQ: no top-q) to split the cause."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
import bayesopt_smart_amd as bo  # noqa: E402

x, y, pm, pv, ls, betas, kinv, cand = bench.make_config_problem(bench.CONFIGS["C3"], 1)
n = x.shape[0]
dev = torch.device("cuda", 0)
cands = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])])
xd, yd, kd = (torch.tensor(a, device=dev) for a in (x, y, kinv))
km = torch.zeros((2, n, n), dtype=torch.float64, device=dev)
bo.kernels.update_k(km, xd, 0, n, pv, np.full(2, 680.0))
kd680 = bo.kernels.invert_k(n, km, lu_hint=[True, True]).contiguous()
calls = {"bench state": bo.predict_acquire(xd, yd, kd, cands, pm, pv, ls, betas, outputs=("acq",), topq=3,
                                           prepare=True),
         "l = 680, LU K^-1": bo.predict_acquire(xd, yd, kd680, cands, pm, pv, np.full(2, 680.0), betas,
                                                outputs=("acq",), topq=3, prepare=True),
         "l = 680, bench K^-1": bo.predict_acquire(xd, yd, kd, cands, pm, pv, np.full(2, 680.0), betas,
                                                   outputs=("acq",), topq=3, prepare=True)}
res = {k: [] for k in calls}
for rnd in range(8):
    for k, c in calls.items():
        c()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        c()
        c()
        b.record()
        torch.cuda.synchronize()
        if rnd:
            res[k].append(a.elapsed_time(b) / 2)
for k, v in res.items():
    print(f"{os.path.basename(bo._lib.LIB_PATH)} {k:20s} median {np.median(v):.3f} ms", flush=True)
