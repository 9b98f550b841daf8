"""Print a sha256 of the fused predict's outputs (mu, var, acq, the top-q record) at C3 with N
training rows (argv[1]), so two library builds can be compared bit for bit (BO_AMD_LIB selects
the build)."""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo  # noqa: E402
import bench  # noqa: E402

n_train = int(sys.argv[1])
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
out = {"mu": torch.empty((n_obj, m), dtype=torch.float64, device=dev),
       "var": torch.empty((n_obj, m), dtype=torch.float64, device=dev),
       "acq": torch.empty(m, dtype=torch.float64, device=dev)}
rec = torch.empty(6, dtype=torch.float64, device=dev)
bo.predict_acquire(xd, yd, kd, cands, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=3, offset=0,
                   count=m, out=out, device=dev, top_rec=rec)
torch.cuda.synchronize()
h = hashlib.sha256()
for k in ("mu", "var", "acq"):
    h.update(out[k].cpu().numpy().tobytes())
h.update(rec.cpu().numpy().tobytes())
print(f"N={n_train} outputs sha256 {h.hexdigest()[:16]}", flush=True)
