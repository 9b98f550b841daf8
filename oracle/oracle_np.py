"""CPU oracle: numpy restatement of the reference's GP-predict + acquisition path.

TEST INFRASTRUCTURE ONLY.  Nothing in ``bayesopt_smart_amd`` imports this module;
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg use it, and only as the checker / the timed CPU baseline, never as the
product path.

Every function restates one reference function (paths relative to the
reference repository alebal123bal/BayesOpt_smart) with the same argument
meaning and the same in-place conventions.  Where the reference's arithmetic
order is reproducible in numpy (everything except LAPACK internals and
transcendental ulps) the restatement reproduces it, and
``tests/test_oracle_golden.py`` pins it bit-for-bit (or to 1 ulp where noted)
against golden vectors produced by the reference itself
(``tests/golden/make_golden.py``).
"""

from __future__ import annotations

import numpy as np

# Constants mirrored from bayesopt/config.py:57-66 (fp64 branch, NUMBA_FLOAT_TYPE=f64).
KERNEL_JITTER = 1e-6
CHOLESKY_JITTER = 1e-8
MIN_VARIANCE = 1e-10


# --------------------------------------------------------------------------- GP fit
def update_k(kernel_matrix, x_vector, last_eval, current_eval, prior_variance, length_scales):
    """bayesopt/numba_kernels.py:329-367 — RBF Gram, upper triangle then mirror.

    k[o,i,j] = pv[o] * exp(-0.5 * ||x_i - x_j||^2 / ls[o]**2) for last<=i<=j<cur,
    then the lower triangle of rows last..cur is mirrored from the upper one.
    """
    n_obj = kernel_matrix.shape[0]
    lo, hi = int(last_eval), int(current_eval)
    if hi <= lo:
        return
    xi = x_vector[lo:hi]
    xa = x_vector[:hi]
    for r, i in enumerate(range(lo, hi)):
        diff = xi[r][None, :] - xa[i:hi]                    # x_i - x_j, j >= i  (:354)
        sq = np.einsum("jd,jd->j", diff, diff)              # np.dot(diff, diff) (:355)
        for o in range(n_obj):
            kernel_matrix[o, i, i:hi] = prior_variance[o] * np.exp(
                -0.5 * sq / (length_scales[o] ** 2))        # (:358-361)
    for o in range(n_obj):                                   # mirror (:364-367)
        for i in range(lo, hi):
            kernel_matrix[o, i + 1:hi, i] = kernel_matrix[o, i, i + 1:hi]


def invert_k(current_eval, kernel_matrix):
    """bayesopt/numba_kernels.py:370-403 — inv(K + KERNEL_JITTER*I) per objective (LAPACK gesv)."""
    n_obj = kernel_matrix.shape[0]
    n = int(current_eval)
    out = np.zeros((n_obj, n, n), dtype=np.float64)
    for o in range(n_obj):
        k = np.array(kernel_matrix[o, :n, :n], dtype=np.float64, copy=True)
        k[np.diag_indices(n)] += KERNEL_JITTER                # (:397-398)
        out[o] = np.linalg.inv(k)                              # (:401)
    return out


def compute_prior_mean(y_vector, n_evaluations, n_objectives):
    """bayesopt/numba_kernels.py:103-122."""
    return np.array([np.mean(y_vector[:n_evaluations, o]) for o in range(n_objectives)],
                    dtype=np.float64)


def compute_prior_variance(y_vector, n_evaluations, n_objectives):
    """bayesopt/numba_kernels.py:125-144 (population variance)."""
    return np.array([np.var(y_vector[:n_evaluations, o]) for o in range(n_objectives)],
                    dtype=np.float64)


def compute_mll(x_vector, y_vector, kernel_matrix, prior_mean, prior_variance,
                length_scales, current_eval, jitter=CHOLESKY_JITTER):
    """bayesopt/numba_kernels.py:152-235 — sum over objectives of the GP marginal log likelihood.

    Raises numpy.linalg.LinAlgError when K/pv + 1e-8 I is not positive definite (:214).
    `jitter`: CHOLESKY_JITTER of the branch (config.py:57-66; 1e-4 in the float32 branch).
    """
    update_k(kernel_matrix, x_vector, 0, current_eval, prior_variance, length_scales)
    n_obj = y_vector.shape[1]
    n = int(current_eval)
    vals = np.empty(n_obj, dtype=np.float64)
    for o in range(n_obj):
        k = np.ascontiguousarray(kernel_matrix[o, :n, :n] / prior_variance[o])   # (:195-198)
        yc = np.ascontiguousarray(y_vector[:n, o] - prior_mean[o])             # (:201-204)
        std = np.std(yc)
        if std > 0.0:
            yc /= std                                                          # (:206-208)
        l = np.linalg.cholesky(k + jitter * np.eye(n))                        # (:211-214)
        inter = np.linalg.solve(l, yc)                                         # (:216)
        alpha = np.linalg.solve(l.T, inter)                                    # (:219)
        data_fit = -0.5 * np.dot(yc, alpha)
        logdet = 2.0 * np.sum(np.log(np.diag(l)))
        vals[o] = data_fit + (-0.5 * logdet) + (-0.5 * n * np.log(2.0 * np.pi))
    return np.sum(vals)


# ----------------------------------------------------------------------- GP predict
def update_k_star(k_star, x_vector, input_space, last_eval, current_eval,
                  prior_variance, length_scales, chunk=1 << 16):
    """bayesopt/numba_kernels.py:406-442 — k_star[o,e,i] = pv[o]*exp(-0.5*||x_e - c_i||^2/ls[o]^2).

    Rows e in [last_eval, current_eval) are written; other rows are untouched.
    The candidate axis is processed in chunks to bound host memory.
    """
    n_obj = k_star.shape[0]
    m = input_space.shape[0]
    for e in range(int(last_eval), int(current_eval)):
        xe = x_vector[e]
        for c0 in range(0, m, chunk):
            c1 = min(m, c0 + chunk)
            diff = xe[None, :] - input_space[c0:c1]          # int64 -> f64 promotion (:436)
            sq = np.einsum("id,id->i", diff, diff)           # (:437)
            for o in range(n_obj):
                k_star[o, e, c0:c1] = prior_variance[o] * np.exp(
                    -0.5 * sq / (length_scales[o] ** 2))


def update_mean(mu_objectives, k_star, inverted_kernel_matrix, y_vector, prior_mean, current_eval):
    """bayesopt/numba_kernels.py:450-488 — mu = pm + K*^T (Kinv (y - pm))."""
    n = int(current_eval)
    for o in range(mu_objectives.shape[0]):
        kinv = np.ascontiguousarray(inverted_kernel_matrix[o, :n, :n])
        dy = np.ascontiguousarray(y_vector[:n, o] - prior_mean[o])
        ks = np.ascontiguousarray(k_star[o, :n, :])
        partial = kinv @ dy                                   # (:483)
        mu_objectives[o, :] = prior_mean[o] + np.ascontiguousarray(ks.T) @ partial   # (:486-488)


def update_variance(variance_objectives, k_star, inverted_kernel_matrix, prior_variance, current_eval):
    """bayesopt/numba_kernels.py:491-535 — var = max(pv - sum_e K*[e]*(Kinv K*)[e], MIN_VARIANCE).

    The reference's serial quadratic-form loop (:525-529) sums e in increasing order per
    candidate; ``(ks * z).sum(0)`` on a C-contiguous (n, m) array reduces row by row in the
    same order, so the result is bit-identical.
    """
    n = int(current_eval)
    for o in range(variance_objectives.shape[0]):
        kinv = np.ascontiguousarray(inverted_kernel_matrix[o, :n, :n])
        ks = np.ascontiguousarray(k_star[o, :n, :])
        z = kinv @ ks                                         # (:521)
        q = (ks * z).sum(0)                                   # (:525-529)
        variance_objectives[o, :] = np.maximum(prior_variance[o] - q, MIN_VARIANCE)


def standardize_objectives(std_mu_objectives, std_variance_objectives, mu_objectives,
                           variance_objectives, prior_mean, prior_variance):
    """bayesopt/numba_kernels.py:538-570."""
    for o in range(mu_objectives.shape[0]):
        std_mu_objectives[o] = (mu_objectives[o] - prior_mean[o]) / np.sqrt(prior_variance[o])
        std_variance_objectives[o] = variance_objectives[o] / prior_variance[o]


def upper_confidence_bound(mu, variance, beta):
    """bayesopt/acquisition.py:33-52."""
    return mu + beta * np.sqrt(np.abs(variance))


def update_ucb(ucb, mu_objectives, variance_objectives, betas):
    """bayesopt/acquisition.py:55-81."""
    for o in range(mu_objectives.shape[0]):
        ucb[o] = upper_confidence_bound(mu_objectives[o], variance_objectives[o], betas[o])


def update_hypervolume_improvement(acquisition_values, ucb):
    """bayesopt/acquisition.py:89-108 — acq[i] = sum_o ucb[o, i] (o ascending)."""
    acc = ucb[0].copy()
    for o in range(1, ucb.shape[0]):
        acc = acc + ucb[o]
    acquisition_values[:] = acc


def select_next_batch(input_space, acquisition_values, evaluated_points, batch_size=3):
    """bayesopt/acquisition.py:116-144 — descending argsort walk, skipping evaluated points."""
    order = np.argsort(acquisition_values)[::-1]
    ev = np.asarray(evaluated_points)
    batch = []
    for idx in order:
        cand = input_space[idx]
        if ev.shape[0] == 0 or not np.any(np.all(cand == ev, axis=1)):
            batch.append(cand)
            if len(batch) == batch_size:
                break
    return np.array(batch)


def select_next_batch_indices(acquisition_values, excluded_mask, batch_size):
    """Deterministic restatement of select_next_batch's order used for tie-free parity.

    Order: NaN first (np.argsort puts NaN last ascending, the reference reverses it),
    then descending value, ties by ascending index; excluded candidates skipped.
    """
    a = np.asarray(acquisition_values, dtype=np.float64)
    idx = np.arange(a.shape[0])
    nan = np.isnan(a)
    key_val = np.where(nan, 0.0, a)
    order = np.lexsort((idx, -key_val, ~nan))
    order = order[~np.asarray(excluded_mask, dtype=bool)[order]]
    return order[:batch_size]


# --------------------------------------------------------------------------- Pareto
def is_pareto_efficient(y_vector):
    """bayesopt/pareto.py:12-45 — weak-dominance non-dominated mask under maximisation.

    Vectorised over the inner j-loop with the reference's break semantics: for a still
    efficient i, the first j>i dominating i stops the scan; every j before it that i
    dominates is marked inefficient.
    """
    yn = -np.asarray(y_vector, dtype=np.float64)
    n = yn.shape[0]
    eff = np.ones(n, dtype=bool)
    for i in range(n):
        if not eff[i]:
            continue
        rest = yn[i + 1:]
        j_dom_i = np.all(rest <= yn[i], axis=1) & np.any(rest < yn[i], axis=1)
        i_dom_j = np.all(yn[i] <= rest, axis=1) & np.any(yn[i] < rest, axis=1)
        hit = np.flatnonzero(j_dom_i)
        stop = hit[0] if hit.size else rest.shape[0]
        eff[i + 1:i + 1 + stop][i_dom_j[:stop]] = False
        if hit.size:
            eff[i] = False
    return eff


def compute_pareto_front(x_vector, y_vector):
    """bayesopt/pareto.py:48-64."""
    m = is_pareto_efficient(y_vector)
    return x_vector[m], y_vector[m]


# ---------------------------------------------------------------- fused convenience
def predict_acquire(x_train, y_train, input_space, prior_mean, prior_variance, length_scales,
                    betas, kinv=None, chunk=1 << 15):
    """The reference chain bayesian_optimization.py:129-199 on host, chunked over candidates.

    Returns dict(mu, var, std_mu, std_var, ucb, acq, kinv).  Used as the parity
    checker for the fused device kernel and as the timed CPU baseline.
    """
    x_train = np.ascontiguousarray(x_train, dtype=np.float64)
    n = x_train.shape[0]
    n_obj = len(prior_mean)
    if kinv is None:
        km = np.zeros((n_obj, n, n))
        update_k(km, x_train, 0, n, prior_variance, length_scales)
        kinv = invert_k(n, km)
    m = input_space.shape[0]
    out = {k: np.empty((n_obj, m)) for k in ("mu", "var", "std_mu", "std_var", "ucb")}
    out["acq"] = np.empty(m)
    for c0 in range(0, m, chunk):
        c1 = min(m, c0 + chunk)
        ks = np.empty((n_obj, n, c1 - c0))
        update_k_star(ks, x_train, input_space[c0:c1], 0, n, prior_variance, length_scales)
        sl = slice(c0, c1)
        mu, var = out["mu"][:, sl], out["var"][:, sl]
        tmp_mu = np.empty((n_obj, c1 - c0))
        tmp_var = np.empty((n_obj, c1 - c0))
        update_mean(tmp_mu, ks, kinv, y_train, prior_mean, n)
        update_variance(tmp_var, ks, kinv, prior_variance, n)
        mu[:] = tmp_mu
        var[:] = tmp_var
        smu = np.empty_like(tmp_mu)
        svar = np.empty_like(tmp_var)
        standardize_objectives(smu, svar, tmp_mu, tmp_var, prior_mean, prior_variance)
        out["std_mu"][:, sl] = smu
        out["std_var"][:, sl] = svar
        u = np.empty_like(smu)
        update_ucb(u, smu, svar, betas)
        out["ucb"][:, sl] = u
        a = np.empty(c1 - c0)
        update_hypervolume_improvement(a, u)
        out["acq"][sl] = a
    out["kinv"] = kinv
    return out


def grid_points(bounds):
    """bayesopt/bayesian_optimization.py:338-340 — int64 'ij' meshgrid candidates."""
    ranges = [np.arange(b[0], b[1]) for b in bounds]
    mesh = np.meshgrid(*ranges, indexing="ij")
    return np.stack([m.ravel() for m in mesh], axis=-1)


# ------------------------------------------------------- exact hypervolume improvement
# The reference names a hypervolume-improvement acquisition with a reference point
# (bayesian_optimization.py:65, :425; acquisition.py:89-108) but computes the sum of UCBs, so
# nothing in the reference pins the exact HVI: PARITY UNPINNED by the reference.  These two
# functions are an independent brute-force statement (recursive slicing over the last
# objective, no box decomposition) that the library's box decomposition and device kernel
# are checked against on small fronts.
def hypervolume(points, ref_point):
    """Volume of the union of boxes [ref, p] over rows p (maximisation).  Rows with NaN or not
    strictly above ref on every axis add nothing.  O(P^m): small fronts only."""
    p = np.asarray(points, dtype=np.float64).reshape(-1, len(ref_point))
    r = np.asarray(ref_point, dtype=np.float64)
    keep = np.all(np.isfinite(p), axis=1) & np.all(p > r, axis=1)
    p = p[keep]
    if p.shape[0] == 0:
        return 0.0
    m = p.shape[1]
    if m == 1:
        return float(p[:, 0].max() - r[0])
    # slabs of the last objective between consecutive distinct values, top down: the slab
    # (z_next, z] is covered by the (m-1)-dim union of the rows with last >= z
    z = np.unique(p[:, -1])[::-1]
    vol = 0.0
    for t, zt in enumerate(z):
        lower = z[t + 1] if t + 1 < len(z) else r[-1]
        vol += (zt - lower) * hypervolume(p[p[:, -1] >= zt, :-1], r[:-1])
    return float(vol)


def hypervolume_improvement_exact(points, front, ref_point):
    """HV(front u {p}) - HV(front) per row p of `points`; NaN rows give NaN."""
    pts = np.asarray(points, dtype=np.float64)
    f = np.asarray(front, dtype=np.float64).reshape(-1, len(ref_point))
    base = hypervolume(f, ref_point)
    out = np.empty(pts.shape[0])
    for i, q in enumerate(pts):
        out[i] = np.nan if np.isnan(q).any() else hypervolume(np.vstack([f, q[None]]), ref_point) - base
    return out
