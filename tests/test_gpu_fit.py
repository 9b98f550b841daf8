"""The device hyper-parameter fit pinned to the reference's optimiser: optimize_hyperparams_mll
(numba_kernels.py:238-321) -- the native Powell driver around the device MLL, one library call --
against scipy.optimize.minimize(method="Powell") with the reference's options and bounds
(:305-315).

  * Over the SAME objective bits the native driver is scipy's Powell exactly: the same
    evaluation sequence, count and result, bit for bit (here over the device MLL terms;
    tests/test_powell.py does it over the CPU oracle's MLL).
  * Against scipy over LAPACK's MLL: the device MLL agrees with LAPACK to 1e-16 relative where
    the correlation matrix is well conditioned and to ~1e-8 once Powell drives the length scales
    up (cond ~1e8 at ls ~ 100-600 on these designs: scripts/fit_diag.py); Powell's comparisons
    amplify such last-bit differences into a different evaluation path (it does between LAPACK
    and the device exactly as between two LAPACK builds), so the pin is the optimiser's own
    tolerance: the fitted MLL within 1e-6 relative and the length scales within 1e-2 relative
    (ftol 1e-4, xtol 1e-3 of numba_kernels.py:305-315); the evaluation counts are printed."""
import numpy as np
import pytest
from scipy.optimize import minimize

from bayesopt_smart_amd.config import (HYPERPARAM_FTOL, HYPERPARAM_MAXITER, HYPERPARAM_MIN_BOUND,
                                       HYPERPARAM_XTOL)
from oracle import oracle_np as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bo():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    bo._lib.load()
    return bo


def _problem(n, dim, n_obj, seed):
    """2-D: distinct points of the 1024^2 grid, toy_function (the C3 family); 6-D: scrambled Sobol
    in [0, 300)^6, toy_function_3d (the C4/C5 family).  Length scales 20 / 40 to start."""
    rng = np.random.default_rng(seed)
    if dim == 2:
        lin = rng.choice(1024 * 1024, size=n, replace=False)
        x = np.stack([lin // 1024, lin % 1024], axis=1).astype(np.float64)
        ls = 20.0
    else:
        from scipy.stats import qmc
        x = qmc.Sobol(dim, scramble=True, seed=seed).random(n) * 300.0
        ls = 40.0
    y = np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20,
                  -((x[:, 2 % dim] - 5) ** 2) + 120][:n_obj], axis=1)
    return x, y, y.mean(0), y.var(0), np.full(n_obj, ls)


@pytest.mark.parametrize("n,dim,n_obj", [(96, 2, 2), (300, 6, 3), (512, 2, 2)])
def test_powell_fit_matches_scipy_over_lapack(bo, n, dim, n_obj):
    import torch
    x, y, pm, pv, ls = _problem(n, dim, n_obj, n)
    km_h = np.zeros((n_obj, n, n))
    ref = minimize(lambda p: -O.compute_mll(x, y, km_h, pm, p[n_obj:], p[:n_obj], n),
                   np.concatenate([ls, pv]), method="Powell",
                   bounds=[(HYPERPARAM_MIN_BOUND, None)] * (2 * n_obj),
                   options={"xtol": HYPERPARAM_XTOL, "ftol": HYPERPARAM_FTOL, "maxiter": HYPERPARAM_MAXITER})
    km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
    lsv, pvv = ls.copy(), pv.copy()
    got = bo.kernels.optimize_hyperparams_mll(torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda"),
                                              km, pm, pvv, lsv, n)
    print(f"N={n}: nfev {got.nfev} (scipy/LAPACK {ref.nfev}), device calls {got.device_calls}, "
          f"x {got.x.tolist()}")
    print(f"  scipy/LAPACK x {ref.x.tolist()} fun {ref.fun}; device fun {got.fun}")
    assert got.status == ref.status == 0
    assert abs(got.fun - ref.fun) <= 1e-6 * abs(ref.fun)
    np.testing.assert_allclose(got.x[:n_obj], ref.x[:n_obj], rtol=1e-2)
    np.testing.assert_array_equal(lsv, got.x[:n_obj])
    np.testing.assert_array_equal(pvv, got.x[n_obj:])
    # kernel_matrix: the Gram (pv e) of the last evaluated hyper-parameters, as compute_mll leaves it
    assert np.isfinite(km.cpu().numpy()).all()


@pytest.mark.parametrize("n,dim,n_obj", [(48, 2, 2), (96, 2, 2), (300, 6, 3), (512, 2, 2)])
def test_native_driver_equals_scipy_driver_on_device(bo, n, dim, n_obj):
    """The same device MLL terms under the native driver and under scipy's Powell: bit-identical
    result, evaluation count and final kernel_matrix (numpy's tan/atan in the line-search
    transform, as scipy uses)."""
    import torch
    x, y, pm, pv, ls = _problem(n, dim, n_obj, n + 1)
    xd, yd = torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda")
    out = []
    for driver in ("native", "scipy"):
        km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
        lsv, pvv = ls.copy(), pv.copy()
        r = bo.kernels.optimize_hyperparams_mll(xd, yd, km, pm, pvv, lsv, n, driver=driver)
        out.append((r.x.copy(), r.nfev, r.fun, r.device_calls, km.cpu().numpy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1:4] == out[1][1:4]
    np.testing.assert_array_equal(out[0][4], out[1][4])


def test_float32_branch_fit_uses_cobyla_and_its_jitter(bo):
    """float_type=np.float32 (config.py:54-61, numba_kernels.py:290-302): COBYLA over the MLL with
    CHOLESKY_JITTER 1e-4, against scipy's COBYLA over the oracle MLL with that jitter (pinned to
    the optimiser's tolerance, as the Powell fit above: the paths differ in the last bits)."""
    import torch
    n, n_obj = 64, 2
    x, y, pm, pv, ls = _problem(n, 2, n_obj, 5)
    km_h = np.zeros((n_obj, n, n))
    ref = minimize(lambda p: -O.compute_mll(x, y, km_h, pm, p[n_obj:], p[:n_obj], n, jitter=1e-4),
                   np.concatenate([ls, pv]), method="COBYLA", bounds=[(HYPERPARAM_MIN_BOUND, None)] * 4,
                   options={"maxiter": HYPERPARAM_MAXITER, "rhobeg": 1.0, "tol": HYPERPARAM_FTOL * 10})
    km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
    got = bo.kernels.optimize_hyperparams_mll(torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda"),
                                              km, pm, pv.copy(), ls.copy(), n, float_type=np.float32)
    print(f"COBYLA nfev {got.nfev} (scipy/LAPACK {ref.nfev}), fun {got.fun} ({ref.fun})")
    assert abs(got.fun - ref.fun) <= 1e-6 * abs(ref.fun)
    np.testing.assert_allclose(got.x[:n_obj], ref.x[:n_obj], rtol=1e-2)
    # and the float32 inverse's jitter: inv(K + 1e-3 I)
    km0 = np.zeros((n_obj, n, n))
    O.update_k(km0, x, 0, n, pv, ls)
    inv = bo.kernels.invert_k(n, km0, float_type=np.float32)
    for o in range(n_obj):
        np.testing.assert_allclose(inv[o], np.linalg.inv(km0[o] + 1e-3 * np.eye(n)),
                                   rtol=0, atol=1e-9 * np.abs(inv[o]).max())
