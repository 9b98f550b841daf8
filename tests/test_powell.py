"""The native Powell driver (bo_powell_minimize, csrc/bo_powell.hip) against scipy's Powell --
the optimiser optimize_hyperparams_mll calls in the reference (numba_kernels.py:305-315) -- on the
same objectives, with the reference's options and bounds.  Host code only (no GPU): the driver's
objective is a Python callback here, the oracle's MLL (oracle_np.compute_mll) among them.

The restatement is operation for operation; tan/atan come from the C library, whose last bit
differs from numpy's SIMD tan for ~0.5 % of arguments, so an evaluation point can move by an ulp:
the evaluation count must be equal and x within 1e-9 relative."""
import numpy as np
import pytest
from scipy.optimize import minimize

from bayesopt_smart_amd.config import (HYPERPARAM_FTOL, HYPERPARAM_MAXITER, HYPERPARAM_MIN_BOUND,
                                       HYPERPARAM_XTOL)
from bayesopt_smart_amd.kernels import powell_minimize
from oracle import oracle_np as O

OPTS = {"xtol": HYPERPARAM_XTOL, "ftol": HYPERPARAM_FTOL, "maxiter": HYPERPARAM_MAXITER}


def _both(fun, x0, bounds, **opts):
    o = dict(OPTS, **opts)
    ref = minimize(fun, x0, method="Powell", bounds=bounds, options=o)
    got = powell_minimize(fun, x0, bounds, xtol=o["xtol"], ftol=o["ftol"], maxiter=o["maxiter"])
    return ref, got


def _mll_problem(n, seed, dim=2, n_obj=2, side=300):
    rng = np.random.default_rng(seed)
    x = rng.integers(0, side, size=(n, dim)).astype(np.float64)
    y = np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1 % dim] - 150) ** 2) + 20][:n_obj], axis=1)
    return x, y, y.mean(0), y.var(0)


@pytest.mark.parametrize("n,seed", [(6, 0), (12, 1), (24, 2), (40, 3)])
def test_native_powell_equals_scipy_on_the_oracle_mll(n, seed):
    """optimize_hyperparams_mll's problem at demo sizes: -compute_mll over [ls, ls, pv, pv]."""
    x, y, pm, pv = _mll_problem(n, seed)
    km = np.zeros((2, n, n))
    fun = lambda p: -O.compute_mll(x, y, km, pm, p[2:], p[:2], n)  # noqa: E731
    x0 = np.concatenate([[1.0, 1.0], pv])
    bounds = [(HYPERPARAM_MIN_BOUND, None)] * 4
    ref, got = _both(fun, x0, bounds)
    assert got.nfev == ref.nfev and got.nit == ref.nit and got.status == ref.status
    np.testing.assert_allclose(got.x, ref.x, rtol=1e-9, atol=0)
    assert abs(got.fun - ref.fun) <= 1e-12 * max(1.0, abs(ref.fun))


def test_native_powell_equals_scipy_on_bounded_functions():
    def rosen(p):
        return float(np.sum(100.0 * (p[1:] - p[:-1] ** 2) ** 2 + (1 - p[:-1]) ** 2))

    def sep(p):
        return float(np.sum((np.log(p) - np.log([3.0, 700.0, 0.5])) ** 2))
    for fun, x0, bounds in [
            (rosen, np.array([1.3, 0.7, 0.8, 1.9]), [(HYPERPARAM_MIN_BOUND, None)] * 4),
            (rosen, np.array([-1.2, 1.0]), [(-2.0, 2.0), (-1.0, 3.0)]),
            (sep, np.array([1.0, 1.0, 1.0]), [(HYPERPARAM_MIN_BOUND, None)] * 3),
            (sep, np.array([5.0, 5.0, 5.0]), [(1e-3, 10.0), (1e-3, None), (None, 2.0)])]:
        ref, got = _both(fun, x0, bounds, xtol=1e-6, ftol=1e-8)
        assert got.nfev == ref.nfev and got.nit == ref.nit, (fun.__name__, got.nfev, ref.nfev)
        np.testing.assert_allclose(got.x, ref.x, rtol=1e-9, atol=1e-12)


def test_native_powell_maxiter_and_exception():
    def slow(p):
        return float(np.sum((p - 3.0) ** 2) + np.sin(5 * p).sum())
    ref, got = _both(slow, np.zeros(3), [(-10.0, 10.0)] * 3, maxiter=2)
    assert got.nit == ref.nit == 2 and got.status == ref.status == 2 and got.nfev == ref.nfev

    class Boom(Exception):
        pass

    def bad(p):
        if p[0] > 0.5:
            raise Boom()
        return float(p @ p)
    with pytest.raises(Boom):
        powell_minimize(bad, np.array([0.0, 1.0]), [(-1.0, 1.0)] * 2)
