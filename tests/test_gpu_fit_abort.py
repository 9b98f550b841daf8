"""The persistent factorisation's recovery path (bo_fit.hip: a bounded wait that gives up raises
the abort word, the remaining tasks are skipped, and the host reruns the call on the
launch-per-step path).  BO_FIT_TEST_ABORT=1 makes every persistent launch abort at once; the
results -- compute_mll's per-objective terms (numba_kernels.py:152-235, through the host's
completion-word poll) and invert_k's K^-1 (:370-403, status memset and extraction repeated) --
must be bit-identical to a BO_FIT_PATH=launches run, and the path counts must show the abort.
Each setting is read once per process, so each runs in its own child process."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
import bayesopt_smart_amd as bo
from scipy.stats import qmc
lib = bo._lib.load()
res = {}
for n, dim, n_obj, ls in ((96, 2, 2, 20.0), (512, 2, 2, 20.0), (300, 6, 3, 40.0)):
    x = qmc.Sobol(dim, scramble=True, seed=n).random(n) * 300.0
    y = np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20,
                  -((x[:, 2 % dim] - 5) ** 2) + 120][:n_obj], axis=1)
    pm, pv, lsv = y.mean(0), y.var(0), np.full(n_obj, ls)
    xd, yd = torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda")
    km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
    before = bo._lib.fit_path_counts()
    terms = bo.kernels._mll_terms(xd, yd, km, pm, pv, lsv, n, list(range(n_obj)))
    kinv = bo.kernels.invert_k(n, km).cpu().numpy()
    after = bo._lib.fit_path_counts()
    np.save(sys.argv[2] + f"/kinv_{n}.npy", kinv)
    res[n] = dict(terms=[terms[o].hex() for o in range(n_obj)],
                  counts={k: after[k] - before[k] for k in after})
print("RESULT " + json.dumps(res))
"""


def _child(env_extra, tmp):
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(tmp)], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = next(ln for ln in r.stdout.splitlines() if ln.startswith("RESULT "))
    return json.loads(line[7:])


def test_persistent_abort_rerun_equals_launch_path(tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    ab, ln = tmp_path / "abort", tmp_path / "launches"
    ab.mkdir()
    ln.mkdir()
    got = _child({"BO_FIT_TEST_ABORT": "1"}, ab)
    ref = _child({"BO_FIT_PATH": "launches"}, ln)
    for n in got:
        g, r = got[n], ref[n]
        # both calls (the MLL and the inverse) aborted and were rerun step by step
        assert g["counts"]["aborted"] == 2 and g["counts"]["launches"] == 2, g["counts"]
        assert g["counts"]["persistent"] == 0, g["counts"]
        assert r["counts"]["launches"] == 2 and r["counts"]["aborted"] == 0, r["counts"]
        assert g["terms"] == r["terms"], (n, g["terms"], r["terms"])
        np.testing.assert_array_equal(np.load(ab / f"kinv_{n}.npy"), np.load(ln / f"kinv_{n}.npy"))
