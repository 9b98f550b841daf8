"""Fused predict time at C5's candidate set (2^22 unscrambled Sobol points, 3 objectives) for
training-set sizes around the fp32 kernel's 64-row chunks: N = 2048, 2049, 2064, 2080, 2096, 2111,
2112 (the drop-in loop's N grows by q = 16 per iteration), in fp32 (the config's stated precision).

Each N runs the shipped kernel (the PART peel: cm32_predict_kernel<DIM, KQV>, KQV live k-quads of
the last chunk) and the unpeeled one (BO_C32_NOPART=1), interleaved, and checks that their
outputs are bit-identical (sha256 of mu, var, acq and the top-16).  Event-timed prepared calls;
a record of how the padded rows scale, not a bench line."""
import hashlib
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
ns = [int(a) for a in sys.argv[1:]] or [2048, 2049, 2064, 2080, 2096, 2111, 2112]


def make_call(xd, yd, kd, pm, pv, nopart):
    if nopart:
        os.environ["BO_C32_NOPART"] = "1"
    try:
        call = bo.predict_acquire(xd, yd, kd, cs, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=16,
                                  device=dev, prepare=True, mode="fp32")
        res = call()
        torch.cuda.synchronize()
        h = hashlib.sha256()
        for k in ("mu", "var", "acq", "top_val", "top_idx"):
            h.update(res[k].cpu().numpy().tobytes())
        return call, h.hexdigest()[:16]
    finally:
        os.environ.pop("BO_C32_NOPART", None)


def timed(call, nopart):
    if nopart:
        os.environ["BO_C32_NOPART"] = "1"
    try:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)
    finally:
        os.environ.pop("BO_C32_NOPART", None)


base = None
for n in ns:
    x = np.concatenate([x0, extra])[:n]
    y = bench.toy_function_3d(x)
    pm, pv = y.mean(0), y.var(0)
    kinv = bench._kinv(x, pv, ls)
    xd, yd, kd = (torch.tensor(a, device=dev) for a in (x, y, kinv))
    cp, hp = make_call(xd, yd, kd, pm, pv, False)
    cu, hu = make_call(xd, yd, kd, pm, pv, True)
    tp, tu = [], []
    for _ in range(3):                       # interleaved: the peeled and the unpeeled kernel
        tp.append(timed(cp, False))
        tu.append(timed(cu, True))
    mp, mu = float(np.median(tp)), float(np.median(tu))
    if n == 2048:
        base = mp
    r_last = n % 64
    kqv = 4 if r_last == 0 or r_last > 48 else (r_last + 15) // 16
    scaled = f", N=2048 x (N/2048)^2 = {base * (n / 2048) ** 2:.1f} ms" if base else ""
    print(f"N={n} (last chunk {r_last or 64} rows, live k-quads {kqv}) fp32 fused predict: "
          f"peeled {mp:.1f} ms, unpeeled {mu:.1f} ms (medians of 3){scaled}; "
          f"outputs sha {hp} vs {hu}: {'bit-identical' if hp == hu else 'DIFFERENT'}", flush=True)
    del cp, cu
