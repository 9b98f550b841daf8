"""What the fused predict's output set costs at C3: the loop writes every array the reference's
state holds (mu, var, std_mu, std_var, ucb, acq: 11 doubles per candidate), the headline bench
mu, var, acq (5).  Event-timed prepared calls, interleaved, same box."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo  # noqa: E402
import bench  # noqa: E402

n_train = int(sys.argv[1]) if len(sys.argv) > 1 else 512
cfg = dict(bench.CONFIGS["C3"])
x, y, pm, pv, ls, betas, kinv, cand = bench.make_config_problem(cfg, 1)
if n_train > x.shape[0]:
    extra = np.random.default_rng(5).choice(1024 * 1024, size=n_train - x.shape[0], replace=False)
    x = np.concatenate([x, np.stack([extra // 1024, extra % 1024], 1).astype(np.float64)])
    y = bench.toy_function(x)
    kinv = bench._kinv(x, pv, ls)
dev = torch.device("cuda", 0)
cands = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])])
m, n_obj = cands.n, len(pm)
xd, yd, kd = (torch.tensor(a, device=dev) for a in (x, y, kinv))
full = {"mu": torch.empty((n_obj, m), dtype=torch.float64, device=dev),
        "var": torch.empty((n_obj, m), dtype=torch.float64, device=dev),
        "std_mu": torch.empty((n_obj, m), dtype=torch.float64, device=dev),
        "std_var": torch.empty((n_obj, m), dtype=torch.float64, device=dev),
        "ucb": torch.empty((n_obj, m), dtype=torch.float64, device=dev),
        "acq": torch.empty(m, dtype=torch.float64, device=dev)}
sets = {"all six (loop)": tuple(full), "mu,var,acq (bench)": ("mu", "var", "acq"), "acq only": ("acq",)}
rec = torch.empty(6, dtype=torch.float64, device=dev)
plans = {k: bo.predict_acquire(xd, yd, kd, cands, pm, pv, ls, betas, outputs=o, topq=3, offset=0, count=m,
                               out={n: full[n] for n in o}, device=dev, top_rec=rec, prepare=True)
         for k, o in sets.items()}
times = {k: [] for k in sets}
for rep in range(6):
    for k, run in plans.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            run()
        e1.record()
        torch.cuda.synchronize()
        if rep:
            times[k].append(e0.elapsed_time(e1) / 3)
for k, t in times.items():
    print(f"N={n_train} outputs {k:22s}: {np.median(t):.3f} ms per call (median of {len(t)})", flush=True)
