"""C2's per-tile work: the fused kernel's event-timed duration with the outputs and the top-q varied
(the candidate work -- K*, the MFMA contractions -- is the same in every row), interleaved rounds.

    python scripts/c2_epilogue_probe.py [cfg=C2] [reps=30] [rounds=3]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bayesopt_smart_amd as bo  # noqa: E402
import bench  # noqa: E402

args = dict(a.split("=", 1) for a in sys.argv[1:] if "=" in a)
cfg_name = args.get("cfg", "C2")
reps, rounds = int(args.get("reps", 30)), int(args.get("rounds", 3))
cfg = bench.CONFIGS[cfg_name]
x, y, pm, pv, ls, betas, kinv, cand = bench.make_config_problem(cfg, 1)
c = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])]) if cand[0] == "grid" else cand[1]
dev = torch.device("cuda", 0)
xd, yd, kd = (torch.tensor(a, device=dev) for a in (x, y, kinv))
L = bo._lib.load()
variants = [
    ("bench: mu var ucb acq, q", ("mu", "var", "ucb", "acq"), cfg["q"]),
    ("acq only, q", ("acq",), cfg["q"]),
    ("mu var ucb acq, no top-q", ("mu", "var", "ucb", "acq"), 0),
    ("acq only, no top-q", ("acq",), 0),
    ("mu var ucb acq, q = 16", ("mu", "var", "ucb", "acq"), 16),
]
calls = [bo.predict_acquire(xd, yd, kd, c, pm, pv, ls, betas, outputs=o, topq=q, device=dev, prepare=True)
         for _, o, q in variants]
res = {v[0]: [] for v in variants}
for r in range(rounds):
    for (name, _, _), call in zip(variants, calls):
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        L.bo_profile_start(reps)
        for _ in range(reps):
            call()
        torch.cuda.synchronize()
        ms, k = ctypes.c_double(), ctypes.c_int()
        L.bo_profile_stop(ctypes.byref(ms), ctypes.byref(k))
        res[name].append(ms.value / max(k.value, 1))
base = np.median(res[variants[0][0]])
for name, v in res.items():
    med = np.median(v)
    print(f"{cfg_name} {name:28s} kernel {med * 1e3:8.2f} us ({(med / base - 1) * 100:+5.1f} %)  rounds {np.round(np.array(v) * 1e3, 1)}",
          flush=True)
