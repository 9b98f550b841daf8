"""A/B of the fp32 kernel's instantiations (cm32_predict_kernel<6, KQV>) on ONE problem: C5's
2^22 Sobol candidates at N = 2064 (16 rows in the last chunk: KQV = 1 is what the library picks;
KQV = 2, 3, 4 compute the padded k-quads as well and are still exact).  BO_C32_KQV forces the
instantiation; the outputs must be bit-identical, and the time should fall with KQV only by the
peeled chunk's skipped MFMAs (33 of 561 E-quad bodies x (4 - KQV) / 4).  Interleaved rounds;
a probe, not a bench line."""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo  # noqa: E402
import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2064
cfg = dict(bench.CONFIGS["C5"])
x0, _, _, _, ls, betas, _, cand = bench.make_config_problem(cfg, 1)
cs = cand[1]
dev = torch.device("cuda", 0)
extra = cs.points(np.random.default_rng(7).choice(cfg["m"], size=96, replace=False))
x = np.concatenate([x0, extra])[:n]
y = bench.toy_function_3d(x)
pm, pv = y.mean(0), y.var(0)
kinv = bench._kinv(x, pv, ls)
xd, yd, kd = (torch.tensor(a, device=dev) for a in (x, y, kinv))
calls, times = {}, {}
for k in (1, 2, 3, 4):
    os.environ["BO_C32_KQV"] = str(k)
    c = bo.predict_acquire(xd, yd, kd, cs, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=16,
                           device=dev, prepare=True, mode="fp32")
    res = c()
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for key in ("mu", "var", "acq", "top_val", "top_idx"):
        h.update(res[key].cpu().numpy().tobytes())
    calls[k], times[k] = (c, h.hexdigest()[:16]), []
for _ in range(3):
    for k in (1, 2, 3, 4):
        os.environ["BO_C32_KQV"] = str(k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        calls[k][0]()
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1))
os.environ.pop("BO_C32_KQV", None)
for k in (1, 2, 3, 4):
    print(f"N={n} forced KQV={k}: {np.median(times[k]):.1f} ms (median of 3; {times[k]}), sha {calls[k][1]}",
          flush=True)
