"""Does the fused predict slow down when it follows an idle or latency-bound phase (the drop-in
loop's order: Powell fit + LU inverse, then the predict)?  The C3 bench problem at N = 512:
HIP-event time of one predict call right after (a) another predict (back to back), (b) 5 ms of
host sleep, (c) a device Powell fit at the bench's N, (d) 20 ms of host sleep."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
import bayesopt_smart_amd as bo  # noqa: E402

cfg = bench.CONFIGS["C3"]
x, y, pm, pv, ls, betas, kinv, cand = bench.make_config_problem(cfg, 1)
n = x.shape[0]
dev = torch.device("cuda", 0)
cands = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])])
xd, yd, kd = (torch.tensor(a, device=dev) for a in (x, y, kinv))
call = bo.predict_acquire(xd, yd, kd, cands, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=3, prepare=True)
km = torch.zeros((2, n, n), dtype=torch.float64, device=dev)


def timed():
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    call()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b)


def fit():
    lsv, pvv = np.full(2, 680.0), pv.copy()
    bo.kernels.optimize_hyperparams_mll(xd, yd, km, pm, pvv, lsv, n)
    torch.cuda.synchronize()


# the loop's state: fitted-like length scales (680) and K^-1 from the device LU path
km2 = torch.zeros((2, n, n), dtype=torch.float64, device=dev)
bo.kernels.update_k(km2, xd, 0, n, pv, np.full(2, 680.0))
kd680 = bo.kernels.invert_k(n, km2, lu_hint=[True, True]).contiguous()
call680 = bo.predict_acquire(xd, yd, kd680, cands, pm, pv, np.full(2, 680.0), betas, outputs=("mu", "var", "acq"),
                             topq=3, prepare=True)


def timed680():
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    call680()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b)


res = {k: [] for k in ("back_to_back", "sleep5ms", "after_fit", "sleep20ms", "ls680_back_to_back",
                       "ls680_after_fit")}
call()
torch.cuda.synchronize()
for rnd in range(6):
    call()
    res["back_to_back"].append(timed())
    time.sleep(0.005)
    res["sleep5ms"].append(timed())
    fit()
    res["after_fit"].append(timed())
    time.sleep(0.02)
    res["sleep20ms"].append(timed())
    call680()
    res["ls680_back_to_back"].append(timed680())
    fit()
    res["ls680_after_fit"].append(timed680())
for k, v in res.items():
    print(f"{k:14s} median {np.median(v):.3f} ms  all {' '.join(f'{t:.2f}' for t in v)}", flush=True)
