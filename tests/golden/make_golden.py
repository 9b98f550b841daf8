"""Generate the golden fixtures under tests/golden/ from the reference itself.

Runs ONLY in the build container, where the reference is mounted read-only at
/root/reference.  It imports the reference package in its own debug mode
(BAYESIAN_DEBUG=True turns numba.njit/prange into identity/range,
bayesopt/config.py:16, bayesopt/numba_kernels.py:24-39) because numba is not
installed, calls the reference functions on seeded inputs and stores inputs
and outputs as small .npz files.  Nothing here is copied from the reference;
the fixtures are data.  Never run on the GPU box (the reference is not there);
the tests only read the .npz files.

    BAYESIAN_DEBUG=True python tests/golden/make_golden.py [names...]

Fixture list: SURVEY.md §8c (G1-G7).
"""

from __future__ import annotations

import hashlib
import os
import sys
import time

import numpy as np

REF = os.environ.get("BO_REFERENCE_PATH", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    os.environ["BAYESIAN_DEBUG"] = "True"
    sys.path.insert(0, REF)
    import bayesopt  # noqa: F401
    from bayesopt import numba_kernels as nk, acquisition as acq, pareto
    from bayesopt import bayesian_optimization as bo
    from examples import benchmark_functions as bf
    return nk, acq, pareto, bo, bf


def _eval(fn, x):
    return np.array([fn(row) for row in x], dtype=np.float64)


def _predict_fixture(nk, acq, x, y, cand, ls, betas, store_kstar=0, qs=(3, 16)):
    """Run the reference chain bayesian_optimization.py:129-207 on (x, y, cand)."""
    n, n_obj = y.shape
    pm = nk.compute_prior_mean(y, n, n_obj)
    pv = nk.compute_prior_variance(y, n, n_obj)
    km = np.zeros((n_obj, n, n))
    nk.update_k(km, x, 0, n, pv, ls)
    kinv = nk.invert_k(n, km)
    m = cand.shape[0]
    ks = np.zeros((n_obj, n, m))
    t0 = time.time()
    nk.update_k_star(ks, x, cand, 0, n, pv, ls)
    print(f"    update_k_star {time.time() - t0:.1f}s", flush=True)
    mu = np.zeros((n_obj, m))
    var = np.zeros((n_obj, m))
    nk.update_mean(mu, ks, kinv, y, pm, n)
    t0 = time.time()
    nk.update_variance(var, ks, kinv, pv, n)
    print(f"    update_variance {time.time() - t0:.1f}s", flush=True)
    smu = np.zeros_like(mu)
    svar = np.zeros_like(var)
    nk.standardize_objectives(smu, svar, mu, var, pm, pv)
    ucb = np.zeros_like(mu)
    acq.update_ucb(ucb, smu, svar, betas)
    a = np.zeros(m)
    acq.update_hypervolume_improvement(a, ucb)
    d = dict(x=x, y=y, cand=cand, ls=ls, betas=betas, pm=pm, pv=pv,
             mu=mu, var=var, std_mu=smu, std_var=svar, ucb=ucb, acq=a)
    if n <= 128:
        d["K"], d["Kinv"] = km, kinv
    else:
        # large N: keep the fixture small; pin K and K^-1 bit-for-bit by digest
        d["K_sha256"] = np.frombuffer(hashlib.sha256(np.ascontiguousarray(km).tobytes()).digest(), np.uint8)
        d["Kinv_sha256"] = np.frombuffer(hashlib.sha256(np.ascontiguousarray(kinv).tobytes()).digest(), np.uint8)
    for q in qs:
        d[f"select_q{q}"] = acq.select_next_batch(cand, a, x, batch_size=q)
    if store_kstar:
        d["kstar_head"] = ks[:, :, :store_kstar].copy()
    return d


def _grid_sample(rng, side, m, n_train, extra_train_in_cand=8):
    """m distinct candidates from the side x side int64 grid; training points partly inside."""
    lin = rng.choice(side * side, size=m + n_train, replace=False)
    cand_lin = np.sort(lin[:m])
    train_lin = lin[m:]
    # put a few training points inside the candidate set so the exclusion walk is exercised
    train_lin[:extra_train_in_cand] = rng.choice(cand_lin, size=extra_train_in_cand, replace=False)
    cand = np.stack([cand_lin // side, cand_lin % side], axis=1).astype(np.int64)
    x = np.stack([train_lin // side, train_lin % side], axis=1).astype(np.float64)
    return cand, x


def g1(nk, acq, pareto, bo, bf):
    rng = np.random.default_rng(101)
    cand, x = _grid_sample(rng, 1024, 4096, 64)
    y = _eval(bf.toy_function, x)
    return _predict_fixture(nk, acq, x, y, cand, np.array([20.0, 25.0]), np.array([2.0, 1.5]),
                            store_kstar=1024)


def g1_grid(nk, acq, pareto, bo, bf):
    """Implicit-grid case: the full 64x96 'ij' grid as the class builds it (:338-340)."""
    rng = np.random.default_rng(102)
    side0, side1 = 64, 96
    ranges = [np.arange(0, side0), np.arange(0, side1)]
    mesh = np.meshgrid(*ranges, indexing="ij")
    cand = np.stack([m_.ravel() for m_ in mesh], axis=-1)
    lin = rng.choice(side0 * side1, size=40, replace=False)
    x = cand[lin].astype(np.float64)
    y = _eval(bf.toy_function, x)
    d = _predict_fixture(nk, acq, x, y, cand, np.array([6.0, 9.0]), np.array([2.0, 2.0]))
    d["grid_lo"] = np.array([0, 0])
    d["grid_shape"] = np.array([side0, side1])
    return d


def g2(nk, acq, pareto, bo, bf):
    rng = np.random.default_rng(202)
    cand, x = _grid_sample(rng, 1024, 16384, 512, extra_train_in_cand=32)
    y = _eval(bf.toy_function, x)
    return _predict_fixture(nk, acq, x, y, cand, np.array([20.0, 20.0]), np.array([2.0, 2.0]))


def g3(nk, acq, pareto, bo, bf):
    from scipy.stats import qmc
    rng = np.random.default_rng(303)
    sob = qmc.Sobol(6, scramble=False).random_base2(13) * 300.0       # 8192 x 6, f64
    cand = sob
    idx = rng.choice(cand.shape[0], size=256, replace=False)
    x = cand[idx].copy()
    y = _eval(bf.toy_function_3d, x)
    return _predict_fixture(nk, acq, x, y, cand, np.array([40.0, 40.0, 40.0]),
                            np.array([2.0, 2.0, 2.0]))


def g4(nk, acq, pareto, bo, bf):
    rng = np.random.default_rng(404)
    d = {}
    for n in (64, 256):
        lin = rng.choice(300 * 300, size=n, replace=False)
        x = np.stack([lin // 300, lin % 300], axis=1).astype(np.float64)
        y = _eval(bf.toy_function, x)
        pm = nk.compute_prior_mean(y, n, 2)
        pv = nk.compute_prior_variance(y, n, 2)
        grid = []
        vals = []
        for l0 in (5.0, 20.0, 60.0):
            for l1 in (10.0, 40.0):
                for s in (1.0, 1e3, pv[0]):
                    ls = np.array([l0, l1])
                    var = np.array([s, pv[1]])
                    km = np.zeros((2, n, n))
                    try:
                        v = nk.compute_mll(x, y, km, pm, var, ls, n)
                    except np.linalg.LinAlgError:
                        v = np.nan
                    grid.append([l0, l1, s, pv[1]])
                    vals.append(v)
        d[f"x_{n}"] = x
        d[f"y_{n}"] = y
        d[f"pm_{n}"] = pm
        d[f"params_{n}"] = np.array(grid)
        d[f"mll_{n}"] = np.array(vals)
    return d


def g5(nk, acq, pareto, bo, bf):
    rng = np.random.default_rng(505)
    d = {}
    for n in (50, 500, 2048):
        for n_obj in (2, 3):
            y = rng.integers(0, 12, size=(n, n_obj)).astype(np.float64)
            y[rng.choice(n, size=max(1, n // 25), replace=False)] = y[0]        # duplicates
            nan_rows = rng.choice(n, size=max(1, n // 50), replace=False)
            y[nan_rows, rng.integers(0, n_obj, size=nan_rows.size)] = np.nan     # NaNs
            t0 = time.time()
            mask = pareto.is_pareto_efficient(y)
            print(f"    pareto n={n} nobj={n_obj} {time.time() - t0:.1f}s", flush=True)
            d[f"y_{n}_{n_obj}"] = y
            d[f"mask_{n}_{n_obj}"] = mask
    # continuous objectives (no ties) too
    y = rng.normal(size=(1000, 2))
    d["y_cont"] = y
    d["mask_cont"] = pareto.is_pareto_efficient(y)
    return d


def g6(nk, acq, pareto, bo, bf):
    """Headless demo configuration (examples/demo_2d.py:125-178) for 3 iterations."""
    states = []

    def cb(state):
        states.append(dict(iteration=state["iteration"], x_next=np.array(state["x_next"]),
                           hyperparams=np.array(state["hyperparams"]),
                           acq=np.array(state["acquisition_values"])))

    np.random.seed(42)
    opt = bo.BayesianOptimization(bf.toy_function, [(0, 300), (0, 300)], n_objectives=2,
                                  initial_samples=6, n_iterations=3, batch_size=3,
                                  betas=np.array([2.0, 2.0]), callbacks=[cb])
    x0 = opt.x_vector.copy()
    y0 = opt.y_vector.copy()
    pm0 = opt.prior_mean.copy()
    pv0 = opt.prior_variance.copy()
    opt.optimize()
    d = dict(x0=x0, y0=y0, pm0=pm0, pv0=pv0, x_final=opt.x_vector, y_final=opt.y_vector,
             n_evaluations=np.array(opt.n_evaluations))
    for s in states:
        it = s["iteration"]
        d[f"x_next_{it}"] = s["x_next"]
        d[f"hyper_{it}"] = s["hyperparams"]
        top = np.argsort(s["acq"])[::-1][:64]
        d[f"acq_top_idx_{it}"] = top
        d[f"acq_top_val_{it}"] = s["acq"][top]
    return d


def g7(nk, acq, pareto, bo, bf):
    """Ill-conditioned regime: Powell-fitted hyper-parameters (documented non-parity)."""
    rng = np.random.default_rng(707)
    lin = rng.choice(300 * 300, size=48, replace=False)
    x = np.stack([lin // 300, lin % 300], axis=1).astype(np.float64)
    y = _eval(bf.toy_function, x)
    n = 48
    pm = nk.compute_prior_mean(y, n, 2)
    pv = nk.compute_prior_variance(y, n, 2)
    ls = np.array([1.0, 1.0])
    km = np.zeros((2, n, n))
    res = nk.optimize_hyperparams_mll(x, y, km, pm, pv, ls, n)
    cand_lin = rng.choice(300 * 300, size=2048, replace=False)
    cand = np.stack([cand_lin // 300, cand_lin % 300], axis=1).astype(np.int64)
    d = _predict_fixture(nk, acq, x, y, cand, ls.copy(), np.array([2.0, 2.0]))
    d["powell_x"] = np.array(res.x)
    d["cond"] = np.array([np.linalg.cond(d["K"][o] + 1e-6 * np.eye(n)) for o in range(2)])
    return d


FIXTURES = {"g1_predict_2d": g1, "g1_grid": g1_grid, "g2_predict_512": g2,
            "g3_predict_6d3o": g3, "g4_mll": g4, "g5_pareto": g5, "g6_trajectory": g6,
            "g7_illcond": g7}


def main(names):
    mods = _import_reference()
    for name in names or FIXTURES:
        t0 = time.time()
        print(f"[{name}]", flush=True)
        d = FIXTURES[name](*mods)
        path = os.path.join(OUT, f"{name}.npz")
        np.savez_compressed(path, **d)
        print(f"  -> {path} ({os.path.getsize(path) / 1e6:.2f} MB, {time.time() - t0:.1f}s)",
              flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
