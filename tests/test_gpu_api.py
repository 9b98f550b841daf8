"""GPU parity of the drop-in API mirrors (kernels / acquisition / pareto / orchestrator)
against the reference's own outputs (tests/golden) and the CPU oracle."""

import numpy as np
import pytest

from oracle import oracle_np as O
from conftest import load_golden, predict_fixture
from parity import check_predict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bo():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    bo._lib.load()
    return bo


def test_update_k_matches_reference(bo):
    d = predict_fixture("g1_predict_2d")
    n = d["x"].shape[0]
    km = np.zeros((2, n, n))
    bo.kernels.update_k(km, d["x"], 0, n, d["pv"], d["ls"])
    np.testing.assert_allclose(km, d["K"], rtol=1e-14, atol=0)
    # incremental rows (last_eval > 0) leave earlier rows untouched, like the reference
    km2 = np.full((2, n, n), 7.0)
    bo.kernels.update_k(km2, d["x"], 40, n, d["pv"], d["ls"])
    assert np.all(km2[:, :40, :40] == 7.0)
    np.testing.assert_allclose(km2[:, 40:, 40:], d["K"][:, 40:, 40:], rtol=1e-14)


@pytest.mark.parametrize("n", [64, 300])
def test_invert_k_matches_lapack(bo, n):
    d = predict_fixture("g1_predict_2d")
    rng = np.random.default_rng(n)
    x = np.unique(rng.integers(0, 1024, size=(2 * n, 2)), axis=0)[:n].astype(np.float64)
    km = np.zeros((2, n, n))
    O.update_k(km, x, 0, n, d["pv"], d["ls"])
    ref = O.invert_k(n, km)
    got = bo.kernels.invert_k(n, km)
    cond = max(np.linalg.cond(km[o] + 1e-6 * np.eye(n)) for o in range(2))
    scale = np.abs(ref).max()
    assert np.abs(got - ref).max() <= 1e-13 * cond * scale


def _sobol_problem(n, dim, n_obj, ls, seed):
    from scipy.stats import qmc
    x = qmc.Sobol(dim, scramble=True, seed=seed).random(n) * 300.0
    y = np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20,
                  -((x[:, 2 % dim] - 5) ** 2) + 120][:n_obj], axis=1)
    return x, y, y.mean(0), y.var(0), np.full(n_obj, ls)


@pytest.mark.parametrize("n,dim,n_obj,ls", [(512, 2, 2, 20.0), (1024, 6, 3, 40.0), (2048, 6, 3, 40.0),
                                            (3000, 6, 2, 40.0)])
def test_invert_k_large_n_matches_lapack(bo, n, dim, n_obj, ls):
    """The blocked-Cholesky inverse at the configs' N (C3 512, C4 1024, C5 2048) and beyond the
    round-1 cap, against LAPACK's inv (numba_kernels.py:370-403)."""
    import torch
    x, y, pm, pv, lsv = _sobol_problem(n, dim, n_obj, ls, n)
    km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
    bo.kernels.update_k(km, torch.tensor(x, device="cuda"), 0, n, pv, lsv)
    got = bo.kernels.invert_k(n, km).cpu().numpy()
    k_h = km.cpu().numpy()
    ref = O.invert_k(n, k_h)
    for o in range(n_obj):
        a = k_h[o] + 1e-6 * np.eye(n)
        cond = np.linalg.cond(a) if n <= 2048 else 1e6
        scale = np.abs(ref[o]).max()
        assert np.abs(got[o] - ref[o]).max() <= 1e-13 * cond * scale, (o, cond)
        res_got = np.abs(a @ got[o] - np.eye(n)).max()
        res_ref = np.abs(a @ ref[o] - np.eye(n)).max()
        assert res_got <= max(10.0 * res_ref, 1e-12), (o, res_got, res_ref)


@pytest.mark.parametrize("n,dim,n_obj,ls", [(512, 2, 2, 20.0), (1024, 6, 3, 40.0), (2048, 6, 3, 40.0)])
def test_compute_mll_large_n_matches_reference_algorithm(bo, n, dim, n_obj, ls):
    """compute_mll at the configs' N against the oracle (LAPACK cholesky + solves,
    numba_kernels.py:152-235), and the caller's kernel_matrix rebuilt as the reference does."""
    import torch
    x, y, pm, pv, lsv = _sobol_problem(n, dim, n_obj, ls, n + 1)
    km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
    v = bo.kernels.compute_mll(torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda"), km, pm, pv,
                               lsv, n)
    km_h = np.zeros((n_obj, n, n))
    ref = O.compute_mll(x, y, km_h, pm, pv, lsv, n)
    assert v == pytest.approx(ref, rel=1e-9)
    # the Gram as update_k writes it (exp of large negative arguments: ulp-level, relative to pv)
    np.testing.assert_allclose(km.cpu().numpy(), km_h, rtol=1e-14, atol=1e-15 * pv.max())


def test_invert_k_pivoting_and_singular(bo):
    # a matrix that needs row interchanges (zero leading pivot after the jitter is tiny)
    a = np.array([[[0.0, 2.0, 1.0], [3.0, 1.0, 0.0], [1.0, 0.0, 4.0]]])
    got = bo.kernels.invert_k(3, a)
    np.testing.assert_allclose(got[0], np.linalg.inv(a[0] + 1e-6 * np.eye(3)), rtol=1e-12)
    sing = np.array([[[-1e-6, 0.0], [0.0, 1.0]]])      # + 1e-6 jitter -> exactly singular
    with pytest.raises(np.linalg.LinAlgError):
        bo.kernels.invert_k(2, sing)


def test_compute_mll_matches_reference(bo):
    d = load_golden("g4_mll")
    for n in (64, 256):
        x, y, pm = d[f"x_{n}"], d[f"y_{n}"], d[f"pm_{n}"]
        for p, ref in zip(d[f"params_{n}"], d[f"mll_{n}"]):
            km = np.zeros((2, n, n))
            try:
                v = bo.kernels.compute_mll(x, y, km, pm, p[2:4], p[0:2], n)
            except np.linalg.LinAlgError:
                v = np.nan
            if np.isnan(ref):
                assert np.isnan(v), (n, p)
            else:
                assert v == pytest.approx(ref, rel=1e-7, abs=1e-6), (n, p)


def test_unfused_chain_matches_reference(bo):
    d = predict_fixture("g1_predict_2d")
    n, m = d["x"].shape[0], d["cand"].shape[0]
    ks = np.zeros((2, n, m))
    bo.kernels.update_k_star(ks, d["x"], d["cand"], 0, n, d["pv"], d["ls"])
    np.testing.assert_allclose(ks[:, :, : d["kstar_head"].shape[2]], d["kstar_head"], rtol=1e-14, atol=1e-300)
    mu = np.zeros((2, m))
    var = np.zeros((2, m))
    bo.kernels.update_mean(mu, ks, d["Kinv"], d["y"], d["pm"], n)
    bo.kernels.update_variance(var, ks, d["Kinv"], d["pv"], n)
    smu, svar, ucb, acq = (np.zeros((2, m)), np.zeros((2, m)), np.zeros((2, m)), np.zeros(m))
    bo.kernels.standardize_objectives(smu, svar, mu, var, d["pm"], d["pv"])
    bo.acquisition.update_ucb(ucb, smu, svar, d["betas"])
    bo.acquisition.update_hypervolume_improvement(acq, ucb)
    check_predict(dict(mu=mu, var=var, std_mu=smu, std_var=svar, ucb=ucb, acq=acq), d, d["pv"])
    u0 = bo.acquisition.upper_confidence_bound(smu[0], svar[0], d["betas"][0])
    np.testing.assert_array_equal(u0, ucb[0])
    for q in (3, 16):
        sel = bo.acquisition.select_next_batch(d["cand"], acq, d["x"], q)
        np.testing.assert_array_equal(sel, d[f"select_q{q}"])


def test_select_next_batch_large_batch_and_exhaustion(bo):
    rng = np.random.default_rng(3)
    cand = np.stack(np.meshgrid(np.arange(20), np.arange(10), indexing="ij"), -1).reshape(-1, 2)
    acq = rng.permutation(cand.shape[0]).astype(np.float64)
    ev = cand[rng.choice(cand.shape[0], 30, replace=False)].astype(np.float64)
    ref = O.select_next_batch(cand, acq, ev, 100)           # > BO_MAX_TOPQ: rounds
    got = bo.acquisition.select_next_batch(cand, acq, ev, 100)
    np.testing.assert_array_equal(got, ref)
    got = bo.acquisition.select_next_batch(cand, acq, ev, 500)   # fewer available than asked
    np.testing.assert_array_equal(got, O.select_next_batch(cand, acq, ev, 500))


@pytest.mark.parametrize("kind", ["grid", "f64"])
@pytest.mark.parametrize("q", [3, 8, 16, 33, 48])
def test_select_exclusion_at_the_top(bo, kind, q):
    """bo_select_topq's streaming kernel tests the exclusion only for elements that beat their
    wave's running q-th entry: here the best candidates of the whole set are evaluated points
    (128 of them, every 2^14-th element, more than any q, so that many waves meet
    several of them), plus evaluated points scattered over the top of the order.  Exact
    selection order against numpy, every q up to BO_MAX_TOPQ."""
    import torch
    side0, side1 = 2048, 1024
    m = side0 * side1
    stride = 1 << 14
    rng = np.random.default_rng(q)
    acq = rng.standard_normal(m)
    hot = 7 + stride * np.arange(m // stride)
    acq[hot] = 100.0 + np.arange(hot.size)                  # the best of all, evaluated below
    lin = np.arange(m)
    cand_pts = np.stack([lin // side1, lin % side1], axis=1)
    top = np.argsort(-acq, kind="stable")[:200]
    scatter = top[hot.size::3][:20]                         # more evaluated points near the top
    ev = cand_pts[np.concatenate([hot, scatter])].astype(np.float64)
    if kind == "grid":
        cands = bo.predict.CandidateSet.grid([(0, side0), (0, side1)])
    else:
        cands = bo.predict.CandidateSet.explicit(cand_pts.astype(np.float64))
    got = bo.acquisition.select_indices(torch.tensor(acq, device="cuda"), cands, ev, q)
    excl = np.zeros(m, dtype=bool)
    excl[hot] = True
    excl[scatter] = True
    order = np.lexsort((lin, -np.where(excl, -np.inf, acq)))
    np.testing.assert_array_equal(got, order[:q])


def test_pareto_mask_bit_exact(bo):
    d = load_golden("g5_pareto")
    for key in d.files:
        if key.startswith("y_"):
            np.testing.assert_array_equal(bo.pareto.is_pareto_efficient(d[key]), d["mask_" + key[2:]], err_msg=key)
    px, py = bo.pareto.compute_pareto_front(np.arange(1000)[:, None], d["y_cont"])
    np.testing.assert_array_equal(px[:, 0], np.flatnonzero(d["mask_cont"]))


def test_demo_trajectory_against_reference(bo):
    """Headless demo configuration (examples/demo_2d.py:125-178): the LHS design is the
    reference's exactly; hyper-parameters (Powell on the device MLL) and the chosen batches
    follow the reference's trajectory."""
    d = load_golden("g6_trajectory")
    from bayesopt_smart_amd.bayesian_optimization import BayesianOptimization

    def toy(x):
        return np.array([-((x[0] - 150) ** 2) + 100, -((x[1] - 150) ** 2) + 20], dtype=np.float64)

    states = []

    class Recorder:
        def __call__(self, state):
            # the access pattern of the reference's callbacks (callbacks.py:73-145, :203-245)
            assert state["x_vector"].shape[1] == 2
            _ = state["timings"]["total"], state.get("x_next"), state["mu_objectives"].shape
            states.append({"it": state["iteration"], "x_next": np.array(state["x_next"]),
                           "hyper": np.array(state["hyperparams"])})

    np.random.seed(42)
    opt = BayesianOptimization(toy, [(0, 300), (0, 300)], n_objectives=2, initial_samples=6,
                               n_iterations=3, batch_size=3, betas=np.array([2.0, 2.0]),
                               callbacks=[Recorder()])
    np.testing.assert_array_equal(opt.x_vector[:6], d["x0"][:6])
    np.testing.assert_array_equal(opt.prior_mean, d["pm0"])
    np.testing.assert_array_equal(opt.prior_variance, d["pv0"])
    opt.optimize()
    assert opt.n_evaluations == int(d["n_evaluations"])
    first = states[0]
    np.testing.assert_allclose(first["hyper"], d["hyper_6"], rtol=2e-2)
    np.testing.assert_array_equal(first["x_next"], d["x_next_6"])
    front = opt.pareto_analysis()
    assert front.shape[1] == 2 and front.shape[0] >= 1


def test_illcond_no_crash(bo):
    """Powell-fitted hyper-parameters (cond ~1e10): outside the parity regime; the device path
    must not crash and must stay finite."""
    d = load_golden("g7_illcond")
    kinv = bo.kernels.invert_k(d["x"].shape[0], np.array(d["K"]))
    cands = bo.predict.CandidateSet.explicit(d["cand"])
    r = bo.predict.predict_acquire(d["x"], d["y"], kinv, cands, d["pm"], d["pv"], d["ls"], d["betas"],
                                   outputs=("mu", "var", "acq"), topq=3)
    import torch
    torch.cuda.synchronize()
    for k in ("mu", "var", "acq"):
        assert np.isfinite(r[k].cpu().numpy()).all()
    assert (r["top_idx"].cpu().numpy() >= 0).all()


def test_orchestrator_exact_hvi_acquisition(bo):
    """acquisition="hvi" (extension; parity unpinned by the reference, see tests/test_hvi.py):
    the loop's acquisition array is the exact HVI of the UCB vectors it also stores, over the
    Pareto front of the evaluated points, and x_next is the oracle's selection on that array."""
    from bayesopt_smart_amd.bayesian_optimization import BayesianOptimization
    from bayesopt_smart_amd.acquisition import hypervolume_boxes

    def toy(x):
        return np.array([-((x[0] - 150) ** 2) + 100, -((x[1] - 150) ** 2) + 20], dtype=np.float64)

    seen = []
    np.random.seed(42)
    opt = BayesianOptimization(toy, [(0, 300), (0, 300)], n_objectives=2, initial_samples=6,
                               n_iterations=1, batch_size=3, betas=np.array([2.0, 2.0]),
                               acquisition="hvi", reference_point=[-3e4, -3e4],
                               callbacks=[lambda s: seen.append(np.array(s["x_next"]))])
    opt.optimize()
    x, y = opt.x_vector[:6], opt.y_vector[:6]
    u = opt.ucb
    pts = (opt.prior_mean[:, None] + np.sqrt(opt.prior_variance)[:, None] * u).T
    front = y[O.is_pareto_efficient(y)]
    boxes = hypervolume_boxes(front, opt.reference_point)
    lo, hi = boxes[:, :2], boxes[:, 2:]
    ref = np.zeros(pts.shape[0])
    for b in range(boxes.shape[0]):   # box-sum restated in numpy (pinned in tests/test_hvi.py)
        ref += np.prod(np.maximum(np.minimum(pts, hi[b]) - lo[b], 0.0), axis=1)
    acq = opt.acquisition_values
    assert np.all(np.abs(acq - ref) <= 1e-9 * np.maximum(1.0, np.abs(ref)))
    sub = np.random.default_rng(0).choice(pts.shape[0], 30, replace=False)
    brute = O.hypervolume_improvement_exact(pts[sub], front, opt.reference_point)
    assert np.all(np.abs(acq[sub] - brute) <= 1e-7 * np.maximum(1.0, np.abs(brute)))
    grid = O.grid_points([(0, 300), (0, 300)])
    np.testing.assert_array_equal(seen[0], O.select_next_batch(grid, ref, x, 3))


def test_orchestrator_exact_hvi_loop_extends_the_exclusion_mask(bo):
    """The exact-HVI loop keeps one exclusion mask per shard (acquisition.ExclusionMask) and
    extends it by each iteration's batch: over 4 iterations every batch equals the oracle's
    select_next_batch (acquisition.py:116-144) over that iteration's acquisition array with the
    points evaluated before it excluded."""
    from bayesopt_smart_amd.bayesian_optimization import BayesianOptimization

    def toy(x):
        return np.array([-((x[0] - 60) ** 2) + 100, -((x[1] - 50) ** 2) + 20], dtype=np.float64)

    states = []
    np.random.seed(7)
    opt = BayesianOptimization(toy, [(0, 120), (0, 120)], n_objectives=2, initial_samples=6,
                               n_iterations=4, batch_size=3, betas=np.array([2.0, 2.0]),
                               acquisition="hvi", reference_point=[-3e4, -3e4],
                               callbacks=[lambda s: states.append((s["iteration"], np.array(s["x_vector"]),
                                                                   np.array(s["acquisition_values"]),
                                                                   np.array(s["x_next"])))])
    opt.optimize()
    grid = O.grid_points([(0, 120), (0, 120)])
    assert len(states) == 4
    for it, xv, acq, xn in states:
        np.testing.assert_array_equal(xn, O.select_next_batch(grid, acq, xv[:it], 3))


@pytest.mark.parametrize("it", [6, 9, 12])
def test_demo_trajectory_replay_each_iteration(bo, it):
    """Every recorded iteration of the reference's headless demo run (G6), replayed on the
    device from the reference's own state at that iteration -- evaluated points x[:it], y[:it],
    the Powell-fitted length scales and prior variances it used (numba_kernels.py:318-321
    updates them in place), the initial prior mean: the acquisition values of the reference's
    top-64 candidates within 1e-5 max(1, |v|), and the selected batch equal to the reference's
    (tie-aware: the reference's argsort order is unspecified within 10x the tolerance)."""
    import torch
    d = load_golden("g6_trajectory")
    x, y = d["x_final"][:it], d["y_final"][:it]
    hyp = d[f"hyper_{it}"]
    ls, pv, pm = hyp[:2].copy(), hyp[2:].copy(), d["pm0"]
    km = np.zeros((2, it, it))
    bo.kernels.update_k(km, x, 0, it, pv, ls)
    kinv = bo.kernels.invert_k(it, km)
    cands = bo.CandidateSet.grid([(0, 300), (0, 300)])
    r = bo.predict_acquire(x, y, kinv, cands, pm, pv, ls, np.array([2.0, 2.0]), outputs=("acq",), topq=3)
    torch.cuda.synchronize()
    acq = r["acq"].cpu().numpy()
    top_idx, top_val = d[f"acq_top_idx_{it}"], d[f"acq_top_val_{it}"]
    tol = 1e-5 * np.maximum(1.0, np.abs(top_val))
    assert np.all(np.abs(acq[top_idx] - top_val) <= tol)
    # the reference's order over non-evaluated candidates (select_next_batch, acquisition.py:134-142)
    grid = O.grid_points([(0, 300), (0, 300)])
    ev = {tuple(p) for p in x.astype(np.int64)}
    keep = [t for t in range(top_idx.size) if tuple(grid[top_idx[t]]) not in ev]
    ridx, rval = top_idx[keep], top_val[keep]
    sel = r["top_idx"].cpu().numpy()
    np.testing.assert_array_equal(grid[ridx[:3]], d[f"x_next_{it}"])     # the fixture's own batch
    for t in range(3):
        tt = 1e-5 * max(1.0, abs(rval[t]))
        gap = rval[t] - rval[t + 1] > 10 * tt and (t == 0 or rval[t - 1] - rval[t] > 10 * tt)
        if gap:
            assert sel[t] == ridx[t], (it, t, sel[t], ridx[t])
        else:
            assert abs(acq[sel[t]] - rval[t]) <= 2 * tt, (it, t)


@pytest.mark.parametrize("n", [512, 518, 1000, 2048])
def test_invert_k_lu_path_matches_lapack(bo, n):
    """invert_k's blocked LU path (bo_lu.hip: getrf partial pivoting + getrs with the identity,
    numba_kernels.py:401) at the C3 and C5 N: objective 0's K is made non-symmetric (the Cholesky
    is then not taken), objective 1 stays symmetric (Cholesky); both against LAPACK's inv."""
    import torch
    rng = np.random.default_rng(n)
    x = rng.uniform(0, 300, size=(n, 2))
    pv, ls = np.array([3e3, 5e2]), np.array([25.0, 40.0])
    km = np.zeros((2, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    km[0] += np.triu(rng.uniform(-1e-3, 1e-3, size=(n, n)) * pv[0], 1)   # not symmetric
    before = bo._lib.invert_k_path_counts()
    got = bo.kernels.invert_k(n, torch.tensor(km, device="cuda")).cpu().numpy()
    after = bo._lib.invert_k_path_counts()
    assert after["lu"] - before["lu"] == 1 and after["cholesky"] - before["cholesky"] == 1
    ref = O.invert_k(n, km)
    for o in range(2):
        a = km[o] + 1e-6 * np.eye(n)
        cond = np.linalg.cond(a)
        scale = np.abs(ref[o]).max()
        assert np.abs(got[o] - ref[o]).max() <= 1e-13 * cond * scale, (o, cond)
        # the residual directly (the cond-scaled bound is loose at N = 2048), both paths against
        # LAPACK's own gesv residual (the reference's np.linalg.inv): the LU path is gesv's
        # algorithm; the Cholesky path (objective 1) reaches it through its Newton step
        # (inv_refine_kernel)
        res_got = np.abs(a @ got[o] - np.eye(n)).max()
        res_ref = np.abs(a @ ref[o] - np.eye(n)).max()
        print(f"objective {o}: cond {cond:.2e}, residual {res_got:.2e} (LAPACK {res_ref:.2e})")
        assert res_got <= max(10.0 * res_ref, 1e-12), (o, res_got, res_ref)


@pytest.mark.parametrize("n", [700, 2048])
def test_invert_k_lu_batched_objectives(bo, n):
    """Every objective whose Cholesky fails goes through ONE batched LU launch sequence (grid y =
    the objective): a dense random matrix (a row swap at nearly every column), a row-permuted
    diagonally dominant matrix (each step's 16 pivots undo a permutation: swap chains through rows
    moved earlier in the same step), a non-symmetric kernel matrix, and one symmetric kernel
    matrix that takes the Cholesky; each against LAPACK's inv (numba_kernels.py:401)."""
    import torch
    rng = np.random.default_rng(n + 1)
    x = rng.uniform(0, 300, size=(n, 2))
    km = np.zeros((4, n, n))
    O.update_k(km[2:], x, 0, n, np.array([3e3, 5e2]), np.array([25.0, 40.0]))
    km[0] = rng.standard_normal((n, n))
    perm = rng.permutation(n)
    km[1] = (np.diag(rng.uniform(5.0, 9.0, n)) + rng.uniform(-0.1, 0.1, size=(n, n)) / np.sqrt(n))[perm]
    km[2] += np.triu(rng.uniform(-1e-3, 1e-3, size=(n, n)) * 3e3, 1)
    before = bo._lib.invert_k_path_counts()
    got = bo.kernels.invert_k(n, torch.tensor(km, device="cuda")).cpu().numpy()
    after = bo._lib.invert_k_path_counts()
    assert after["lu"] - before["lu"] == 3 and after["cholesky"] - before["cholesky"] == 1
    ref = O.invert_k(n, km)
    for o in range(4):
        cond = np.linalg.cond(km[o] + 1e-6 * np.eye(n))
        scale = np.abs(ref[o]).max()
        err = np.abs(got[o] - ref[o]).max()
        a = km[o] + 1e-6 * np.eye(n)
        res_got = np.abs(a @ got[o] - np.eye(n)).max()
        res_ref = np.abs(a @ ref[o] - np.eye(n)).max()
        print(f"objective {o}: cond {cond:.2e}, max |d| / max |ref| {err / scale:.2e}, "
              f"residual {res_got:.2e} (LAPACK {res_ref:.2e})")
        assert err <= 1e-13 * cond * scale, (o, cond)
        # every objective against LAPACK's gesv residual (the Cholesky one, 3, after its Newton step)
        assert res_got <= max(10.0 * res_ref, 1e-12), (o, res_got, res_ref)


def test_invert_k_lu_path_ill_conditioned(bo):
    """The regime that makes the Cholesky fail (Powell-fitted length scales drive
    cond(K + 1e-6 I) to 1e14..1e18; the reference's inv still returns): the LU path returns a
    finite inverse whose residual |(K + 1e-6 I) X - I| is at LAPACK's level for that condition."""
    rng = np.random.default_rng(4)
    n = 300
    x = rng.uniform(0, 300, size=(n, 2))
    pv, ls = np.array([2e9]), np.array([400.0])
    km = np.zeros((1, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    a = km[0] + 1e-6 * np.eye(n)
    before = bo._lib.invert_k_path_counts()
    got = bo.kernels.invert_k(n, km)[0]
    after = bo._lib.invert_k_path_counts()
    ref = np.linalg.inv(a)
    assert np.isfinite(got).all()
    res_got = np.abs(a @ got - np.eye(n)).max()
    res_ref = np.abs(a @ ref - np.eye(n)).max()
    print(f"cond {np.linalg.cond(a):.2e}, residual device {res_got:.3e}, LAPACK {res_ref:.3e}, paths {after}")
    assert res_got <= max(100.0 * res_ref, 1e-6)
    # LAPACK's Cholesky of this matrix fails; so does the device's: the LU path ran, once
    assert after["lu"] - before["lu"] == 1 and after["cholesky"] == before["cholesky"]


@pytest.mark.parametrize("n,dim,n_obj", [(96, 2, 2), (300, 6, 3)])
def test_powell_memo_equals_full_evaluations(bo, n, dim, n_obj):
    """optimize_hyperparams_mll's memoised per-objective terms (bo_compute_mll_each) return the
    same MLL bits as recomputing every term: the same Powell path, result and evaluation count;
    kernel_matrix ends as the Gram of the last evaluated hyper-parameters, as in the reference."""
    import torch
    x, y, pm, pv, ls = _sobol_problem(n, dim, n_obj, 30.0, 7)
    xd, yd = torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda")
    out = []
    for memo in (False, True):
        km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
        lsv, pvv = ls.copy(), pv.copy()
        r = bo.kernels.optimize_hyperparams_mll(xd, yd, km, pm, pvv, lsv, n, memo=memo)
        out.append((r.x.copy(), r.nfev, r.fun, km.cpu().numpy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    assert out[0][1] == out[1][1] and out[0][2] == out[1][2]
    np.testing.assert_array_equal(out[0][3], out[1][3])
    # each term only depends on ls_o: the sum of the terms is compute_mll
    km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
    terms = bo.kernels._mll_terms(xd, yd, km, pm, pv, ls, n, list(range(n_obj)))
    assert sum(terms[o] for o in range(n_obj)) == bo.kernels.compute_mll(xd, yd, km, pm, pv, ls, n)
    one = bo.kernels._mll_terms(xd, yd, km, pm, pv * 3.0, ls, n, [n_obj - 1])
    assert one[n_obj - 1] == terms[n_obj - 1]          # pv-free: bit-identical
