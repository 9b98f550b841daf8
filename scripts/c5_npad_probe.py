"""Fused predict time at C5's candidate set (2^22 unscrambled Sobol points, 3 objectives) for
training-set sizes around the fp32 kernel's 64-row chunks: N = 2048, 2049, 2064, 2096, 2111, 2112
(the drop-in loop's N grows by q = 16 per iteration), in fp32 (the config's stated precision).
Event-timed prepared calls; a record of how the padded rows scale, not a bench line."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo  # noqa: E402
import bench  # noqa: E402

cfg = dict(bench.CONFIGS["C5"])
x0, _, _, _, ls, betas, _, cand = bench.make_config_problem(cfg, 1)
cs = cand[1]
dev = torch.device("cuda", 0)
rng = np.random.default_rng(7)
extra = cs.points(rng.choice(cfg["m"], size=96, replace=False))
for n in (2048, 2049, 2064, 2096, 2111, 2112):
    x = np.unique(np.concatenate([x0, extra]), axis=0)[:n] if n > 2048 else x0
    y = bench.toy_function_3d(x)
    pm, pv = y.mean(0), y.var(0)
    kinv = bench._kinv(x, pv, ls)
    xd, yd, kd = (torch.tensor(a, device=dev) for a in (x, y, kinv))
    call = bo.predict_acquire(xd, yd, kd, cs, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=16,
                              device=dev, prepare=True, mode="fp32")
    call()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"N={x.shape[0]} fp32 fused predict: {np.median(ts):.1f} ms (median of 3), "
          f"scaled from N=2048 by (N/2048)^2: x{(x.shape[0] / 2048) ** 2:.3f}", flush=True)
