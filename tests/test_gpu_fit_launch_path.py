"""The launch-per-step fit path (the default above N = 1536) at small and ragged N, odd and even
column-block counts: compute_mll and invert_k against the oracle (numba_kernels.py:152-235,
:370-403).  The path is chosen once per process, so the cases run in one child process with
BO_FIT_PATH=launches; the child reports the path counts, so a case that silently ran the
persistent kernel fails here."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/tests")
import bayesopt_smart_amd as bo
from oracle import oracle_np as O
from scipy.stats import qmc
import ctypes
lib = bo._lib.load()
out = []
for n, dim, n_obj, ls in ((40, 2, 2, 20.0), (100, 6, 3, 40.0), (333, 6, 3, 40.0), (512, 2, 2, 20.0),
                          (700, 6, 2, 40.0), (1090, 6, 3, 40.0)):
    x = qmc.Sobol(dim, scramble=True, seed=n).random(n) * 300.0
    y = np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20,
                  -((x[:, 2 % dim] - 5) ** 2) + 120][:n_obj], axis=1)
    pm, pv, lsv = y.mean(0), y.var(0), np.full(n_obj, ls)
    km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
    before = (ctypes.c_int64 * 3)()
    lib.bo_fit_path_counts(before)
    v = bo.kernels.compute_mll(torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda"), km, pm, pv, lsv, n)
    after = (ctypes.c_int64 * 3)()
    lib.bo_fit_path_counts(after)
    ref = O.compute_mll(x, y, np.zeros((n_obj, n, n)), pm, pv, lsv, n)
    k_h = km.cpu().numpy()
    got = bo.kernels.invert_k(n, km).cpu().numpy()
    inv_ref = O.invert_k(n, k_h)
    inv_rel = max(float(np.abs(got[o] - inv_ref[o]).max() /
                        (np.linalg.cond(k_h[o] + 1e-6 * np.eye(n)) * np.abs(inv_ref[o]).max()))
                  for o in range(n_obj))
    out.append(dict(n=n, mll=float(v), ref=float(ref), launches=after[1] - before[1],
                    persistent=after[0] - before[0], inv_rel=inv_rel))
print("RESULT " + json.dumps(out))
"""


def test_launch_path_mll_and_inverse_small_and_ragged_n():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    env = dict(os.environ, BO_FIT_PATH="launches")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = next(l for l in r.stdout.splitlines() if l.startswith("RESULT "))
    for c in json.loads(line[7:]):
        assert c["launches"] >= 1 and c["persistent"] == 0, c       # the path under test ran
        assert c["mll"] == pytest.approx(c["ref"], rel=1e-9), c
        assert c["inv_rel"] <= 1e-13, c
