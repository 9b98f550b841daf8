"""Diagnosis of the device MLL terms' bits: repeatability, one call over all objectives vs
single-objective calls, persistent vs launch-per-step schedule, and the Powell drivers."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bayesopt_smart_amd as bo  # noqa: E402
from oracle import oracle_np as O  # noqa: E402


def problem(n, dim, n_obj, ls, seed):
    from scipy.stats import qmc
    x = qmc.Sobol(dim, scramble=True, seed=seed).random(n) * 300.0
    y = np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20,
                  -((x[:, 2 % dim] - 5) ** 2) + 120][:n_obj], axis=1)
    return x, y, y.mean(0), y.var(0), np.full(n_obj, ls)


for (n, dim, n_obj) in [(96, 2, 2), (300, 6, 3), (512, 2, 2)]:
    x, y, pm, pv, ls = problem(n, dim, n_obj, 30.0, 7)
    xd, yd = torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda")
    km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
    rng = np.random.default_rng(1)
    bad_rep = bad_split = 0
    maxrel = 0.0
    for t in range(20):
        lsv = ls * np.exp(rng.uniform(-1, 3, size=n_obj))
        a = bo.kernels._mll_terms(xd, yd, km, pm, pv, lsv, n, list(range(n_obj)))
        b = bo.kernels._mll_terms(xd, yd, km, pm, pv, lsv, n, list(range(n_obj)))
        bad_rep += sum(a[o] != b[o] for o in range(n_obj))
        for o in range(n_obj):
            s = bo.kernels._mll_terms(xd, yd, km, pm, pv, lsv, n, [o])
            bad_split += s[o] != a[o]
        ref = O.compute_mll(x, y, np.zeros((n_obj, n, n)), pm, pv, lsv, n)
        maxrel = max(maxrel, abs(sum(a.values()) - ref) / abs(ref))
    print(f"N={n}: repeat mismatches {bad_rep}, single-vs-all mismatches {bad_split}, "
          f"max rel vs LAPACK {maxrel:.2e}, paths {bo._lib.fit_path_counts()}", flush=True)
    outs = {}
    for name, kw in [("native", {}), ("scipy", {"driver": "scipy"}), ("full", {"memo": False})]:
        lsv, pvv = ls.copy(), pv.copy()
        r = bo.kernels.optimize_hyperparams_mll(xd, yd, km, pm, pvv, lsv, n, **kw)
        outs[name] = (r.x.copy(), r.nfev)
        print(f"  {name}: nfev {r.nfev} x {r.x.tolist()}", flush=True)
    print(f"  native==scipy {np.array_equal(outs['native'][0], outs['scipy'][0])}, "
          f"scipy==full {np.array_equal(outs['scipy'][0], outs['full'][0])}", flush=True)
