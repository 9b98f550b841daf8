"""C3 predict step cost by the per-candidate outputs written: none (top-q only), the bench's
(mu, var, acq) and the drop-in loop's six arrays (mu, var, std_mu, std_var, ucb, acq)."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo
import bench
from bayesopt_smart_amd.distributed import sharded_predict_acquire

cfg = bench.CONFIGS["C3"]
x, y, pm, pv, ls, betas, kinv, cand = bench.make_config_problem(cfg, 1)
if len(sys.argv) > 1:                      # another length scale (e.g. the fitted ~680): its K^-1
    ls = np.full_like(ls, float(sys.argv[1]))
    kinv = bench._kinv(x, pv, ls)
dev = torch.device("cuda", 0)
xd, yd, kd = (torch.tensor(a, device=dev) for a in (x, y, kinv))
cs = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])])
m = cs.n
outs = {k: torch.empty((2, m), dtype=torch.float64, device=dev) for k in ("mu", "var", "std_mu", "std_var", "ucb")}
outs["acq"] = torch.empty(m, dtype=torch.float64, device=dev)
for label, names in (("bench3", ("mu", "var", "acq")), ("all6", tuple(outs))):
    out = {k: outs[k] for k in names} or None
    for via in ("predict_acquire", "sharded"):
        def call():
            if via == "predict_acquire":
                r = bo.predict.predict_acquire(xd, yd, kd, cs, pm, pv, ls, betas, outputs=names, topq=3, out=out, device=dev)
                return r["top_idx"].cpu()
            return sharded_predict_acquire(xd, yd, kd, cs, pm, pv, ls, betas, 3, outputs=names, device=dev, out=out)
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            t0 = time.perf_counter(); call(); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
        print(f"{label:7s} {via:16s} median {np.median(ts) * 1e3:.3f} ms", flush=True)
