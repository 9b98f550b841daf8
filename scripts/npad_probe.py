"""Fused predict time at C3's grid for training-set sizes around a multiple of 32 (the drop-in
loop's N grows by the batch each iteration): N = 512, 515, 521, 530, 540, 544."""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench
import bayesopt_smart_amd as bo

cfg = bench.CONFIGS["C3"]
side = cfg["side"]
rng = np.random.default_rng(0)
dev = torch.device("cuda", 0)
cs = bo.CandidateSet.grid([(0, side), (0, side)])
res = []
for n in (512, 515, 521, 530, 540, 544):
    lin = rng.choice(side * side, size=n, replace=False)
    x = np.stack([lin // side, lin % side], axis=1).astype(np.float64)
    y = bench.toy_function(x)
    pm, pv = y.mean(0), y.var(0)
    ls = np.full(2, cfg["ls"]); betas = np.full(2, 2.0)
    kinv = bench._kinv(x, pv, ls)
    xd, yd, kd = (torch.tensor(a, device=dev) for a in (x, y, kinv))
    call = bo.predict_acquire(xd, yd, kd, cs, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=3,
                              device=dev, prepare=True)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        call()
    e1.record(); torch.cuda.synchronize()
    r = call()
    res.append((n, e0.elapsed_time(e1) / 10, r["top_idx"].cpu().numpy().tolist(), float(r["acq"].sum().item())))
for n, ms, idx, s in res:
    print(f"N={n}: {ms:.3f} ms per call, top {idx}, sum(acq) {s!r}", flush=True)
