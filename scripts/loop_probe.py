"""The drop-in loop at C3 (optimize(), 4 iterations) run twice in one process: per-iteration
timings (the reference's keys) of a cold and a warm allocator / workspace state."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench
import bayesopt_smart_amd as bo
from bayesopt_smart_amd.bayesian_optimization import optimize

cfg = bench.CONFIGS["C3"]
x, y, pm, pv, ls, betas, _, cand = bench.make_config_problem(cfg, 1)
n, q = cfg["n_train"], cfg["q"]
cands = bo.CandidateSet.grid([(0, cand[1]), (0, cand[2])])
for run in range(2):
    total = n + 4 * q
    xv = np.zeros((total, 2)); yv = np.zeros((total, 2)); xv[:n] = x; yv[:n] = y
    recs = []
    optimize(xv, yv, None, None, None, None, None, None, None, None, cands, pm, pv.copy(), None, n, total, 2,
             lambda p: bench.toy_function(np.asarray(p, dtype=np.float64)[None])[0], betas, ls.copy(), q, None,
             callbacks=[lambda st: recs.append(dict(st["timings"]))])
    for r in recs:
        print(f"run {run}: " + " ".join(f"{k} {v * 1e3:.2f}" for k, v in r.items()), flush=True)
