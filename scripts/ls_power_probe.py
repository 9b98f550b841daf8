"""Is the fused predict's time data-dependent?  The C3 bench problem (N = 512, 1024^2 grid) at the
bench's length scale (l = 20: most K* entries underflow to 0) and at the drop-in loop's fitted
length scale (l ~ 680: every K* entry O(1), K^-1 entries large), same kernel instantiation and
outputs; median of HIP-event-timed direct calls, interleaved rounds."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
import bayesopt_smart_amd as bo  # noqa: E402

cfg = bench.CONFIGS["C3"]
x, y, pm, pv, ls, betas, _, cand = bench.make_config_problem(cfg, 1)
n = x.shape[0]
dev = torch.device("cuda", 0)
cands = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])])
xd, yd = torch.tensor(x, device=dev), torch.tensor(y, device=dev)
calls = {}
for tag, lsv, zero_kinv, outs in (("l20", 20.0, False, ("mu", "var", "acq")),
                                  ("l680", 680.0, False, ("mu", "var", "acq")),
                                  ("l20_out6", 20.0, False, ("mu", "var", "std_mu", "std_var", "ucb", "acq")),
                                  ("l680_out6", 680.0, False, ("mu", "var", "std_mu", "std_var", "ucb", "acq")),
                                  ("l680_out1", 680.0, False, ("acq",))):
    km = torch.zeros((2, n, n), dtype=torch.float64, device=dev)
    lsa = np.full(2, lsv)
    bo.kernels.update_k(km, xd, 0, n, pv, lsa)
    kinv = bo.kernels.invert_k(n, km)
    if zero_kinv:
        kinv.zero_()
    calls[tag] = bo.predict_acquire(xd, yd, kinv, cands, pm, pv, lsa, betas, outputs=outs, topq=3, prepare=True)
res = {k: [] for k in calls}
for rnd in range(3):
    for tag, c in calls.items():
        c()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in ev:
            a.record()
            c()
            b.record()
        torch.cuda.synchronize()
        res[tag] += [a.elapsed_time(b) for a, b in ev]
for tag, v in res.items():
    print(f"{tag:12s} predict step median {np.median(v):.3f} ms (min {np.min(v):.3f})", flush=True)
