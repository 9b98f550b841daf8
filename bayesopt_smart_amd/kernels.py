"""Drop-in mirror of bayesopt/numba_kernels.py on the MI355X.

Same names, argument meaning, in-place conventions and error behaviour as the reference
functions; the arithmetic runs in libbo_amd.so kernels.  Arrays may be numpy arrays (as the
reference passes them: results are copied back in place) or HIP device tensors (no host
round trip).  The hyper-parameter optimiser driver (Powell, a sequential host algorithm) runs
natively in the library around the device MLL (bo_optimize_hyperparams_mll, a restatement of
scipy's Powell); the initial LHS design stays on the host, as SURVEY.md §2 scopes it.

``float_type`` (keyword; default config.NUMBA_FLOAT_TYPE at call time): np.float32 selects the
reference's float32 branch (config.py:57-66 jitters, COBYLA for the fit, numba_kernels.py:290-302);
the device arithmetic stays binary64.
"""

from __future__ import annotations

import ctypes as C

import numpy as np
import torch
from scipy.optimize import minimize

from . import _lib
from scipy.optimize import OptimizeResult

from .config import (HYPERPARAM_FTOL, HYPERPARAM_MAXITER, HYPERPARAM_METHOD,
                     HYPERPARAM_MIN_BOUND, HYPERPARAM_XTOL, NUMBA_FLOAT_TYPE, precision_constants,
                     resolve_float_type)
from .device import F64, Workspace, require_device, stream_handle


# ------------------------------------------------------------------------ helpers
class _Arg:
    """A caller array on the device; numpy inputs are staged and (if written) copied back."""

    def __init__(self, arr, dev, dtype=F64, write=False):
        self.src = arr
        self.write = write
        if isinstance(arr, torch.Tensor):
            if arr.device.type != "cuda" or arr.dtype != dtype or not arr.is_contiguous():
                raise ValueError("device arrays must be contiguous HIP tensors of the right dtype")
            self.t = arr
            self.host = False
        else:
            a = np.asarray(arr)
            self.t = torch.as_tensor(np.ascontiguousarray(a, dtype=torch_to_np(dtype)), device=dev)
            self.host = True

    @property
    def ptr(self):
        return self.t.data_ptr()

    def finish(self):
        if self.write and self.host:
            torch.cuda.current_stream(self.t.device).synchronize()
            self.src[...] = self.t.cpu().numpy().reshape(np.shape(self.src))


def torch_to_np(dtype):
    return {torch.float64: np.float64, torch.int64: np.int64, torch.uint8: np.uint8}[dtype]


def _host_vec(v, n):
    a = np.asarray(v.cpu().numpy() if isinstance(v, torch.Tensor) else v, dtype=np.float64).ravel()
    if a.size < n:
        raise ValueError("per-objective parameter array too short")
    return (C.c_double * max(n, 1))(*[float(x) for x in a[:n]])


def _dev_of(*arrs):
    for a in arrs:
        if isinstance(a, torch.Tensor) and a.device.type == "cuda":
            return a.device
    return require_device()


# ----------------------------------------------------------------------- init/prior
def initialize_lhs_integer(x_vector, y_vector, bounds, function, n_samples=8):
    """numba_kernels.py:50-95 — integer Latin hypercube (numpy global RNG, same draw order
    as the reference's debug mode); evaluates `function` on the host."""
    bounds = np.asarray(bounds)
    dim = len(bounds)
    samples = np.empty((n_samples, dim), dtype=NUMBA_FLOAT_TYPE)
    for d in range(dim):
        perm = np.random.permutation(n_samples)
        lo, hi = bounds[d, 0], bounds[d, 1]
        step = (hi - lo) / n_samples
        for i in range(n_samples):
            low = lo + perm[i] * step
            high = lo + (perm[i] + 1) * step
            samples[i, d] = min(int(np.random.uniform(low, high)), hi - 1)
    for i in range(n_samples):
        x_vector[i] = samples[i]
        y_vector[i] = function(x_vector[i])
    return n_samples


def compute_prior_mean(y_vector, n_evaluations, n_objectives):
    """numba_kernels.py:103-122 (O(N) host statistic of the initial design)."""
    y = y_vector.cpu().numpy() if isinstance(y_vector, torch.Tensor) else np.asarray(y_vector)
    return np.array([np.mean(y[:n_evaluations, o]) for o in range(n_objectives)], dtype=np.float64)


def compute_prior_variance(y_vector, n_evaluations, n_objectives):
    """numba_kernels.py:125-144 (population variance)."""
    y = y_vector.cpu().numpy() if isinstance(y_vector, torch.Tensor) else np.asarray(y_vector)
    return np.array([np.var(y[:n_evaluations, o]) for o in range(n_objectives)], dtype=np.float64)


# --------------------------------------------------------------------------- GP fit
def update_k(kernel_matrix, x_vector, last_eval, current_eval, prior_variance, length_scales):
    """numba_kernels.py:329-367 — RBF Gram rows [last_eval, current_eval) (+ mirror)."""
    dev = _dev_of(kernel_matrix, x_vector)
    km = _Arg(kernel_matrix, dev, write=True)
    x = _Arg(x_vector, dev)
    n_obj, ld = km.t.shape[0], km.t.shape[-1]
    lib = _lib.load()
    _lib.check(lib.bo_update_k(km.ptr, ld, n_obj, x.ptr, x.t.shape[1], int(last_eval), int(current_eval),
                               _host_vec(prior_variance, n_obj), _host_vec(length_scales, n_obj),
                               stream_handle(dev)), "bo_update_k")
    km.finish()


def invert_k(current_eval, kernel_matrix, *, float_type=None, lu_hint=None, paths=None):
    """numba_kernels.py:370-403 — inv(K[:N,:N] + KERNEL_JITTER I) per objective (1e-6; 1e-3 in the
    float32 branch): Cholesky plus one Newton step, or the blocked LU with partial pivoting when it
    fails.

    Returns a new array of the caller's kind (numpy in, numpy out; tensor in, tensor out).
    Raises numpy.linalg.LinAlgError on an exactly singular pivot.
    `lu_hint` (per-objective booleans, optional): when all are true the Cholesky attempt is
    skipped and every objective takes the LU path (a loop whose previous iteration's Cholesky
    failed for them).  `paths` (a list, optional) receives the per-objective path taken:
    0 Cholesky, 1 blocked LU, 2 Gauss-Jordan.
    """
    dev = _dev_of(kernel_matrix)
    km = _Arg(kernel_matrix, dev)
    n_obj, ld = km.t.shape[0], km.t.shape[-1]
    n = int(current_eval)
    out = torch.empty((n_obj, n, n), dtype=F64, device=dev)
    lib = _lib.load()
    ws = Workspace.get(lib.bo_invert_k_workspace_size(n_obj, n), dev)
    jitter = precision_constants(float_type)[0]
    hint = None
    if lu_hint is not None:
        hint = (C.c_int32 * n_obj)(*[1 if lu_hint[o] else 0 for o in range(n_obj)])
    taken = (C.c_int32 * n_obj)()
    _lib.check(lib.bo_invert_k_ex(out.data_ptr(), km.ptr, ld, n_obj, n, jitter, hint, taken, ws.data_ptr(),
                                  ws.numel(), stream_handle(dev)), "bo_invert_k")
    if paths is not None:
        paths[:] = [int(taken[o]) for o in range(n_obj)]
    return out if isinstance(kernel_matrix, torch.Tensor) else out.cpu().numpy()


def compute_mll(x_vector, y_vector, kernel_matrix, prior_mean, prior_variance, length_scales,
                current_eval, *, float_type=None):
    """numba_kernels.py:152-235 — summed marginal log likelihood (Gram rebuilt in place).

    Raises numpy.linalg.LinAlgError when K/pv + CHOLESKY_JITTER I is not positive definite (:214).
    """
    dev = _dev_of(kernel_matrix, x_vector, y_vector)
    km = _Arg(kernel_matrix, dev, write=True)
    x = _Arg(x_vector, dev)
    y = _Arg(y_vector, dev)
    n_obj, ld = km.t.shape[0], km.t.shape[-1]
    n = int(current_eval)
    lib = _lib.load()
    ws = Workspace.get(lib.bo_compute_mll_workspace_size(n_obj, n), dev)
    out = (C.c_double * n_obj)()
    st = lib.bo_compute_mll_each_jitter(out, x.ptr, x.t.shape[1], y.ptr, y.t.stride(0), km.ptr, ld, n_obj,
                                        _host_vec(prior_mean, n_obj), _host_vec(prior_variance, n_obj),
                                        _host_vec(length_scales, n_obj), n, precision_constants(float_type)[1],
                                        ws.data_ptr(), ws.numel(), stream_handle(dev))
    km.finish()
    _lib.check(st, "bo_compute_mll")
    tot = 0.0
    for o in range(n_obj):                      # np.sum over the objectives (:235): sequential, < 8 terms
        tot += out[o]
    return tot


def _mll_terms(xd, yd, km, prior_mean, prior_variance, length_scales, n, objs, jitter=1e-8):
    """Per-objective MLL terms (bo_compute_mll_each) of the objectives `objs` (device arrays;
    one call over all objectives, or one single-objective call for one of them)."""
    lib = _lib.load()
    n_obj_all, ld = km.shape[0], km.shape[-1]
    dev = km.device
    if len(objs) == n_obj_all:
        o0, cnt = 0, n_obj_all
    else:
        assert len(objs) == 1
        o0, cnt = objs[0], 1
    out = (C.c_double * cnt)()
    ws = Workspace.get(lib.bo_compute_mll_workspace_size(cnt, n), dev)
    sel = lambda v: _host_vec(np.asarray(v, dtype=np.float64)[o0:o0 + cnt], cnt)  # noqa: E731
    st = lib.bo_compute_mll_each_jitter(out, xd.data_ptr(), xd.shape[1], yd.data_ptr() + 8 * o0, yd.stride(0),
                                        km.data_ptr() + 8 * o0 * ld * ld, ld, cnt, sel(prior_mean),
                                        sel(prior_variance), sel(length_scales), n, jitter, ws.data_ptr(),
                                        ws.numel(), stream_handle(dev))
    _lib.check(st, "bo_compute_mll_each")
    return {o0 + i: out[i] for i in range(cnt)}


_POWELL_MESSAGES = {0: "Optimization terminated successfully.",
                    1: "Maximum number of function evaluations has been exceeded.",
                    2: "Maximum number of iterations has been exceeded.",
                    3: "NaN result encountered.",
                    4: "The result is outside of the provided bounds."}


def _powell_result(x, r, direc):
    return OptimizeResult(fun=float(r.fun), direc=direc, nit=int(r.nit), nfev=int(r.nfev),
                          status=int(r.warnflag), success=r.warnflag == 0,
                          message=_POWELL_MESSAGES.get(int(r.warnflag), ""), x=x)


def powell_minimize(fun, x0, bounds, xtol=1e-4, ftol=1e-4, maxiter=None, maxfev=None, numpy_trig=True):
    """``scipy.optimize.minimize(fun, x0, method="Powell", bounds=bounds, options=...)`` on the
    library's native driver (bo_powell_minimize: scipy 1.15's algorithm restated in C++).
    `numpy_trig`: the one-sided line searches' tan/atan are numpy's (scipy's evaluation points
    bit for bit), else the C library's.  `bounds`: sequence of (lo, hi) pairs, None = unbounded.
    Returns an OptimizeResult like scipy's; an exception raised by `fun` propagates."""
    x = np.array(x0, dtype=np.float64).ravel()
    n = x.size
    lb = np.array([-np.inf if b[0] is None else b[0] for b in bounds], dtype=np.float64)
    ub = np.array([np.inf if b[1] is None else b[1] for b in bounds], dtype=np.float64)
    err = []

    def cb(xp, nn, fp, _user):
        try:
            fp[0] = float(fun(np.ctypeslib.as_array(xp, shape=(nn,)).copy()))
            return 0
        except BaseException as exc:   # re-raised below; the driver stops at the non-zero status
            err.append(exc)
            return 100
    cfun = _lib.OBJECTIVE_FN(cb)
    res = _lib.PowellResult()
    direc = np.zeros((n, n))
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    st = _lib.load().bo_powell_minimize(cfun, None, dp(x), n, dp(lb), dp(ub), float(xtol), float(ftol),
                                        -1 if maxiter is None else int(maxiter),
                                        -1 if maxfev is None else int(maxfev),
                                        _lib.NUMPY_TRIG if numpy_trig else _lib.TRIG_FN(), dp(direc), C.byref(res))
    if err:
        raise err[0]
    _lib.check(st, "bo_powell_minimize")
    return _powell_result(x, res, direc)


def optimize_hyperparams_mll(x_vector, y_vector, kernel_matrix, prior_mean, prior_variance,
                             length_scales, current_eval, memo=True, *, float_type=None, driver="native",
                             numpy_trig=True):
    """numba_kernels.py:238-321 — maximise the device MLL over [ls..., var...] (bounds >= 1e-5);
    updates length_scales and prior_variance in place, returns the OptimizeResult.  The training
    arrays are staged on the device once for all ~100-300 MLL evaluations.

    float64 (the reference's default branch): Powell (:305-315).  driver "native" (default) runs
    the whole fit as ONE library call, bo_optimize_hyperparams_mll: the Powell driver in C++ around
    the device MLL, no Python per evaluation except numpy's tan/atan for the one-sided line
    searches (`numpy_trig`, so that the evaluation points are scipy's bit for bit; False: the C
    library's, no Python at all); driver "scipy" runs scipy's Powell over the same device terms
    (the pre-round-4 path, kept for comparison).  float32 (:290-302): scipy's COBYLA
    with rhobeg 1.0 and tol 10 ftol over the MLL with the float32 jitter.

    `memo`: the MLL is a sum of per-objective terms, each a function of (x, y, pm, ls_o) only --
    the correlation matrix K / pv does not depend on pv (:195-198; the device builds it pv-free) --
    and Powell moves mostly one coordinate at a time: each term is computed once per distinct
    ls_o (bo_compute_mll_each over the objectives whose ls changed) and summed in objective order
    like np.sum (:235).  The returned values are bit-identical to recomputing every term (the same
    device arithmetic), so Powell's path is unchanged; evaluations that move only pv need no
    device call (about half of them).  kernel_matrix ends as the reference leaves it: the Gram of
    the last evaluated hyper-parameters."""
    ft = resolve_float_type(float_type)
    _, chol_jitter, _ = precision_constants(ft)
    dev = _dev_of(kernel_matrix, x_vector, y_vector)
    n_obj = np.asarray(length_scales).shape[0] if not isinstance(length_scales, torch.Tensor) \
        else length_scales.shape[0]
    xd = _Arg(x_vector, dev).t
    yd = _Arg(y_vector, dev).t
    km = _Arg(kernel_matrix, dev, write=True)
    ls0 = length_scales.cpu().numpy() if isinstance(length_scales, torch.Tensor) else np.asarray(length_scales)
    pv0 = prior_variance.cpu().numpy() if isinstance(prior_variance, torch.Tensor) else np.asarray(prior_variance)
    pm = np.asarray(prior_mean.cpu().numpy() if isinstance(prior_mean, torch.Tensor) else prior_mean,
                    dtype=np.float64)
    n = int(current_eval)
    lib = _lib.load()
    if ft == np.float64 and driver == "native" and memo and HYPERPARAM_METHOD == "Powell":
        ls_io = np.array(ls0, dtype=np.float64)
        pv_io = np.array(pv0, dtype=np.float64)
        pm_c = np.ascontiguousarray(pm[:n_obj])
        ws = Workspace.get(lib.bo_compute_mll_workspace_size(n_obj, n), dev)
        res = _lib.PowellResult()
        direc = np.zeros((2 * n_obj, 2 * n_obj))
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        st = lib.bo_optimize_hyperparams_mll(
            xd.data_ptr(), xd.shape[1], yd.data_ptr(), yd.stride(0), km.ptr, km.t.shape[-1], n_obj, dp(pm_c),
            dp(pv_io), dp(ls_io), n, chol_jitter, HYPERPARAM_XTOL, HYPERPARAM_FTOL, HYPERPARAM_MAXITER,
            HYPERPARAM_MIN_BOUND, _lib.NUMPY_TRIG if numpy_trig else _lib.TRIG_FN(), ws.data_ptr(), ws.numel(),
            stream_handle(dev), C.byref(res), dp(direc))
        if st != _lib.ERR_UNSUPPORTED:
            km.finish()
            _lib.check(st, "bo_optimize_hyperparams_mll")
            out = _powell_result(np.concatenate([ls_io, pv_io]), res, direc)
            out.device_calls = int(res.device_calls)
            _assign(length_scales, ls_io)
            _assign(prior_variance, pv_io)
            return out
        # a line search unbounded in both directions (not produced by these bounds): scipy's driver
    initial_guess = np.concatenate([ls0, pv0]).astype(np.float64)
    bounds = [(HYPERPARAM_MIN_BOUND, None)] * (2 * n_obj)
    cache = [dict() for _ in range(n_obj)]
    last = [None]
    calls = [0]

    def objective(params):
        ls, pv = params[:n_obj], params[n_obj:]
        last[0] = params.copy()
        if not memo:
            calls[0] += 1
            return -compute_mll(xd, yd, km.t, pm, pv, ls, current_eval, float_type=ft)
        todo = [o for o in range(n_obj) if float(ls[o]) not in cache[o]]
        if todo:
            objs = todo if len(todo) == 1 else list(range(n_obj))
            calls[0] += 1
            for o, v in _mll_terms(xd, yd, km.t, pm, pv, ls, current_eval, objs, chol_jitter).items():
                cache[o][float(ls[o])] = v
        tot = 0.0
        for o in range(n_obj):                  # np.sum over < 8 terms: sequential (:235)
            tot += cache[o][float(ls[o])]
        return -tot

    if ft == np.float32:                        # numba_kernels.py:290-302
        res = minimize(objective, initial_guess, method="COBYLA", bounds=bounds,
                       options={"maxiter": HYPERPARAM_MAXITER, "rhobeg": 1.0, "tol": HYPERPARAM_FTOL * 10})
    else:
        res = minimize(objective, initial_guess, method=HYPERPARAM_METHOD, bounds=bounds,
                       options={"xtol": HYPERPARAM_XTOL, "ftol": HYPERPARAM_FTOL,
                                "maxiter": HYPERPARAM_MAXITER})
    res.device_calls = calls[0]
    if memo and last[0] is not None:            # the reference's compute_mll side effect
        update_k(km.t, xd, 0, current_eval, last[0][n_obj:], last[0][:n_obj])
    km.finish()
    _assign(length_scales, res.x[:n_obj])
    _assign(prior_variance, res.x[n_obj:])
    return res


def _assign(dst, values):
    if isinstance(dst, torch.Tensor):
        dst.copy_(torch.as_tensor(values, dtype=dst.dtype))
    else:
        dst[:] = values


# ----------------------------------------------------------------------- GP predict
def _cand_kind(t):
    return _lib.CAND_I64 if t.dtype == torch.int64 else _lib.CAND_F64


def update_k_star(k_star, x_vector, input_space, last_eval, current_eval, prior_variance,
                  length_scales):
    """numba_kernels.py:406-442 — materialised k_star[o, e, i] rows [last_eval, current_eval).
    (The fused path, predict.predict_acquire, never materialises it.)"""
    dev = _dev_of(k_star, x_vector, input_space)
    ks = _Arg(k_star, dev, write=True)
    x = _Arg(x_vector, dev)
    is_int = (not input_space.is_floating_point()) if isinstance(input_space, torch.Tensor) \
        else np.issubdtype(np.asarray(input_space).dtype, np.integer)
    cand = _Arg(input_space, dev, dtype=torch.int64 if is_int else F64)
    n_obj, ld_rows, m = ks.t.shape
    lib = _lib.load()
    _lib.check(lib.bo_update_k_star(ks.ptr, ld_rows, n_obj, x.ptr, x.t.shape[1], _cand_kind(cand.t),
                                    cand.ptr, m, int(last_eval), int(current_eval),
                                    _host_vec(prior_variance, n_obj), _host_vec(length_scales, n_obj),
                                    stream_handle(dev)), "bo_update_k_star")
    ks.finish()


def _mean_variance(mu_objectives, variance_objectives, k_star, kinv, y_vector, prior_mean,
                   prior_variance, current_eval):
    dev = _dev_of(k_star, kinv, mu_objectives, variance_objectives)
    ks = _Arg(k_star, dev)
    ki = _Arg(kinv, dev)
    n_obj, ld_rows, m = ks.t.shape
    n = int(current_eval)
    mu = _Arg(mu_objectives, dev, write=True) if mu_objectives is not None else None
    var = _Arg(variance_objectives, dev, write=True) if variance_objectives is not None else None
    if y_vector is None:
        y = torch.zeros((n, n_obj), dtype=F64, device=dev)
    else:
        y = _Arg(y_vector, dev).t
    pm = prior_mean if prior_mean is not None else np.zeros(n_obj)
    pv = prior_variance if prior_variance is not None else np.ones(n_obj)
    lib = _lib.load()
    ws = Workspace.get(lib.bo_update_mean_variance_workspace_size(n_obj, n), dev)
    _lib.check(lib.bo_update_mean_variance(mu.ptr if mu else None, var.ptr if var else None, ks.ptr,
                                           ld_rows, n_obj, m, ki.ptr, ki.t.shape[-1], y.data_ptr(),
                                           y.stride(0), n, _host_vec(pm, n_obj), _host_vec(pv, n_obj),
                                           ws.data_ptr(), ws.numel(), stream_handle(dev)),
               "bo_update_mean_variance")
    for a in (mu, var):
        if a is not None:
            a.finish()


def update_mean(mu_objectives, k_star, inverted_kernel_matrix, y_vector, prior_mean, current_eval):
    """numba_kernels.py:450-488 — mu = pm + K*^T (Kinv (y - pm))."""
    _mean_variance(mu_objectives, None, k_star, inverted_kernel_matrix, y_vector, prior_mean, None,
                   current_eval)


def update_variance(variance_objectives, k_star, inverted_kernel_matrix, prior_variance, current_eval):
    """numba_kernels.py:491-535 — var = max(pv - sum_e K* (Kinv K*), 1e-10)."""
    _mean_variance(None, variance_objectives, k_star, inverted_kernel_matrix, None, None,
                   prior_variance, current_eval)


def standardize_objectives(std_mu_objectives, std_variance_objectives, mu_objectives,
                           variance_objectives, prior_mean, prior_variance):
    """numba_kernels.py:538-570."""
    dev = _dev_of(std_mu_objectives, mu_objectives)
    smu = _Arg(std_mu_objectives, dev, write=True)
    svar = _Arg(std_variance_objectives, dev, write=True)
    mu = _Arg(mu_objectives, dev)
    var = _Arg(variance_objectives, dev)
    n_obj, m = mu.t.shape
    lib = _lib.load()
    zeros = _host_vec(np.zeros(n_obj), n_obj)
    _lib.check(lib.bo_standardize_ucb_hvi(smu.ptr, svar.ptr, None, None, mu.ptr, var.ptr, n_obj, m,
                                          _host_vec(prior_mean, n_obj), _host_vec(prior_variance, n_obj),
                                          zeros, stream_handle(dev)), "bo_standardize_ucb_hvi")
    smu.finish()
    svar.finish()
