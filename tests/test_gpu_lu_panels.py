"""invert_k's LU path (numba_kernels.py:370-403: gesv) under every panel shape of bo_lu.hip:
the 8-wave panel, the 4-wave panel with 1 or 2 rows per lane, and the per-step choice of rows per
thread (N = 2048 runs 4, then 2, then 1).  The shapes differ only in which waves hold the rows:
the pivot choice (getrf's first largest |a|), the reciprocal and the FMAs are the same, so the
inverses must be identical (np.array_equal: +0 and -0 compare equal).  The shape is read once per
process (BO_LU_PANEL), so each runs in a child process; the default is also held to LAPACK."""

import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZES = (512, 700, 1040, 2048)

CHILD = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
import bayesopt_smart_amd as bo
out = {}
for n in map(int, sys.argv[3].split(",")):
    rng = np.random.default_rng(n)
    lin = rng.choice(1024 * 1024, size=n, replace=False)
    x = np.stack([lin // 1024, lin % 1024], 1).astype(np.float64)
    y = np.stack([np.sin(x[:, 0] / 90.0) * 40.0 + x[:, 1] / 10.0, np.cos(x[:, 1] / 70.0) * 30.0], 1)
    pv = y.var(0)
    xd = torch.tensor(x, device="cuda")
    km = torch.zeros((2, n, n), dtype=torch.float64, device="cuda")
    bo.kernels.update_k(km, xd, 0, n, pv, np.full(2, 680.0))         # fitted-like: cond > 1e16
    paths = []
    kinv = bo.kernels.invert_k(n, km, lu_hint=[True, True], paths=paths)
    assert all(p != 0 for p in paths), paths                          # the LU path ran
    out[f"kinv_{n}"] = kinv.cpu().numpy()
    out[f"k_{n}"] = km.cpu().numpy()
np.savez(sys.argv[2], **out)
"""


def _run(mode, path):
    env = dict(os.environ)
    env.pop("BO_LU_PANEL", None)
    if mode:
        env["BO_LU_PANEL"] = mode
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, path, ",".join(map(str, SIZES))], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (mode, r.stderr[-3000:])
    return np.load(path)


def test_lu_panel_shapes_give_identical_inverses():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    with tempfile.TemporaryDirectory() as d:
        res = {m: _run(m, os.path.join(d, f"{m or 'default'}.npz")) for m in (None, "wide", "small", "small256")}
    ref = res[None]
    for m in ("wide", "small", "small256"):
        for n in SIZES:
            np.testing.assert_array_equal(res[m][f"kinv_{n}"], ref[f"kinv_{n}"], err_msg=f"{m} N={n}")
    for n in SIZES:
        # the default's residual against LAPACK's gesv on the same matrix (test_gpu_api.py's bound)
        for o in range(2):
            a = ref[f"k_{n}"][o] + 1e-6 * np.eye(n)
            x = ref[f"kinv_{n}"][o]
            res_got = np.abs(a @ x - np.eye(n)).max()
            res_ref = np.abs(a @ np.linalg.inv(a) - np.eye(n)).max()
            assert res_got <= max(10 * res_ref, 1e-12), (n, o, res_got, res_ref)
