"""End-to-end parity of the drop-in chain at the configs' N, on the DEVICE's own inverse.

The reference iteration (bayesian_optimization.py:129-207) is
    update_k (numba_kernels.py:329-367) -> invert_k (:370-403, LAPACK gesv)
    -> update_k_star ... select_next_batch (:406-570, acquisition.py:33-144).
Here the device runs the whole chain -- bo_update_k, bo_invert_k (Cholesky + Newton step, or the
blocked LU) and the fused predict/acquire/top-q -- and is compared, on EVERY candidate, with the
oracle chain: oracle_np.update_k -> oracle_np.invert_k (numpy's inv = LAPACK gesv, the
reference's call) -> oracle/cpu_ref.c.  No K^-1 is shared between the two sides (the other
config-size tests feed LAPACK's K^-1 to both).  Tolerances: SURVEY.md §8c (tests/parity.py);
the top-q is judged tie-aware on the CPU acquisition array.

Two inverse paths, each at every config: "cholesky" (what the device picks at these well-conditioned
inputs) and "lu" (`lu_hint` forces every objective onto the blocked LU + getrs, bo_invert_k_ex --
the path the drop-in loop actually takes at fitted length scales, DeviceBackend._lu_hint).  The
oracle side is the same LAPACK gesv either way, so the two parametrisations share one CPU array.

Configs (SURVEY.md §8d inputs): C3 (N = 512, the full 1024^2 'ij' grid, q = 3), C4 (N = 1024,
the 2^21 unscrambled Sobol set, q = 3) and C5's shard 0 of 8 (N = 2048, 2^19 Sobol candidates,
f64, q = 16).  The CPU arrays of C3 and C4 share tests/fullref.py's cache with
test_gpu_predict.py / test_gpu_configs.py (same problem, same oracle K^-1)."""

import numpy as np
import pytest

from oracle import oracle_np as O
from parity import check_predict, check_topq
from fullref import cpu_full, grid_points_2d

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bo():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    bo._lib.load()
    return bo


def _toy(x):
    return np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20], axis=1)


def _toy3(x):
    return np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20,
                     -((x[:, 2] - 5) ** 2) + 120], axis=1)


def _problem(bo, cfg):
    """(x, y, pm, pv, ls, betas, q, device candidate set, offset, count, host points, cache key,
    excluded mask)."""
    if cfg == "C3":
        side, n = 1024, 512
        lin = np.random.default_rng(0).choice(side * side, size=n, replace=False)
        x = np.stack([lin // side, lin % side], axis=1).astype(np.float64)
        y = _toy(x)
        cands = bo.CandidateSet.grid([(0, side), (0, side)])
        excl = np.zeros(side * side, dtype=bool)
        excl[lin] = True
        return x, y, 20.0, 3, cands, 0, side * side, lambda: grid_points_2d(side, side), "C3", excl
    if cfg == "C4":
        from scipy.stats import qmc
        m, n = 1 << 21, 1024
        pts = qmc.Sobol(6, scramble=False).random(m) * 300.0
        x = pts[np.random.default_rng(1).choice(m, size=n, replace=False)]
        cands = bo.CandidateSet.sobol_set(6, m, scale=300.0)     # bit-identical to scipy's set
        xs = {tuple(p) for p in x}
        excl = np.array([tuple(p) in xs for p in pts])
        return x, _toy3(x), 40.0, 3, cands, 0, m, lambda: pts, ("C45", n, m), excl
    # C5, shard 0 of 8 (bench.py's problem and partition)
    import bench
    from bayesopt_smart_amd.distributed import shard_range
    x, y, _, _, _, _, _, cand = bench.make_config_problem(bench.CONFIGS["C5"], 1)
    cands = cand[1]
    off, cnt = shard_range(cands.n, 0, 8)
    pts = cands.points(np.arange(off, off + cnt))
    xs = {tuple(p) for p in x}
    excl = np.array([tuple(p) in xs for p in pts])
    return x, y, 40.0, 16, cands, off, cnt, lambda: pts, ("C5chain", 0), excl


@pytest.mark.parametrize("path", ["cholesky", "lu"])
@pytest.mark.parametrize("cfg", ["C3", "C4", "C5shard0"])
def test_device_chain_matches_oracle_chain(bo, cfg, path):
    import torch
    x, y, ls_v, q, cands, off, cnt, host_pts, key, excl = _problem(bo, cfg)
    n, n_obj = x.shape[0], y.shape[1]
    pm, pv = y.mean(0), y.var(0)                       # compute_prior_mean / _variance
    ls, betas = np.full(n_obj, ls_v), np.full(n_obj, 2.0)
    # device chain: update_k -> invert_k -> fused predict / acquisition / top-q
    xd, yd = torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda")
    km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
    bo.kernels.update_k(km, xd, 0, n, pv, ls)
    before = bo._lib.invert_k_path_counts()
    taken = []
    kinv_dev = bo.kernels.invert_k(n, km, lu_hint=[path == "lu"] * n_obj, paths=taken)
    after = bo._lib.invert_k_path_counts()
    # well-conditioned: Cholesky + Newton step unless the hint sends every objective to the LU
    assert after[path] - before[path] == n_obj, (before, after)
    assert taken == [0 if path == "cholesky" else 1] * n_obj, taken
    r = bo.predict_acquire(xd, yd, kinv_dev, cands, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=q,
                           offset=off, count=cnt)
    torch.cuda.synchronize()
    got = {k: r[k].cpu().numpy() for k in ("mu", "var", "acq", "top_idx")}
    # oracle chain: the reference's update_k and LAPACK's inv, then the reference algorithm on the host
    km_h = np.zeros((n_obj, n, n))
    O.update_k(km_h, x, 0, n, pv, ls)
    kinv_ref = O.invert_k(n, km_h)
    np.testing.assert_allclose(km.cpu().numpy(), km_h, rtol=1e-14, atol=1e-15 * pv.max())
    ref = cpu_full(key, x, y, host_pts(), kinv_ref, pm, pv, ls, betas)
    check_predict({k: got[k] for k in ("mu", "var", "acq")}, ref, pv)
    check_topq(got["top_idx"] - off, ref["acq"], excl, q)
    # the device inverse itself, at gesv's residual (the reference's np.linalg.inv)
    kd = kinv_dev.cpu().numpy()
    for o in range(n_obj):
        a = km_h[o] + 1e-6 * np.eye(n)
        res_got = np.abs(a @ kd[o] - np.eye(n)).max()
        res_ref = np.abs(a @ kinv_ref[o] - np.eye(n)).max()
        print(f"{cfg} {path} objective {o}: residual {res_got:.2e} (LAPACK {res_ref:.2e})")
        assert res_got <= max(10.0 * res_ref, 1e-12), (o, res_got, res_ref)
