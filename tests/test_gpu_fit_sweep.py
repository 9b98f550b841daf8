"""A seeded sweep over the fit kernels' shapes: invert_k on both of its paths and compute_mll,
against LAPACK and the oracle, at every N class the schedules distinguish.

  * invert_k (numba_kernels.py:370-403; bo_invert_k_ex): the augmented blocked Cholesky + the
    Newton step (split-k tiles up to N = 1024, full-k above) and, with lu_hint on every objective,
    the blocked LU (getrf partial pivoting + getrs; the 8-wave panel up to N_p = 512, the small
    panel above, 1, 2 and 4 rows per thread).  Held to LAPACK gesv's own residual:
    |(K + 1e-6 I) X - I|_max <= max(10 res_LAPACK, 1e-12), the bound of tests/test_gpu_api.py, with
    the path counts checked;
  * compute_mll (numba_kernels.py:152-235; the persistent single-launch factorisation up to 48
    column blocks, N = 1536, one launch per step above) against the oracle at 1e-9 relative (the
    bound of tests/test_gpu_api.py), NaN where the oracle's is NaN, and the caller's kernel_matrix
    as update_k writes it.
N: 1, 2, 15 .. 33 (one 32-column block and its edges), 100, 255 .. 257, 513, 777, 1025, 1537, 1600;
objectives 1, 3 and 8 (BO_MAX_OBJ); 1-, 2- and 5-D inputs.  Well-conditioned problems (the same
length-scale rule as tests/test_gpu_sweep.py), where LAPACK's inverse and the MLL are defined to
the tolerance."""
import numpy as np
import pytest

from oracle import oracle_np as O

pytestmark = pytest.mark.gpu

CASES = [(n, n_obj, dim) for n, n_obj, dim in [
    (1, 1, 2), (2, 3, 1), (15, 8, 2), (16, 1, 5), (17, 3, 2), (31, 8, 1), (32, 3, 2), (33, 1, 5),
    (100, 8, 2), (255, 3, 5), (256, 1, 2), (257, 8, 2), (513, 3, 2), (777, 1, 5), (777, 8, 2),
    (1025, 3, 5), (1537, 1, 2), (1600, 3, 2)]]


def _problem(n, n_obj, dim):
    rng = np.random.default_rng(7 * n + n_obj + 100 * dim)
    x = np.unique(rng.uniform(0, 300, size=(n + 8, dim)), axis=0)[:n]
    x = x[rng.permutation(n)]
    y = np.stack([-((x[:, o % dim] - 40.0 * o) ** 2) / 50.0 + rng.normal(size=n) * 5 for o in range(n_obj)], 1)
    pm = y.mean(0)
    pv = y.var(0) if n > 1 else np.full(n_obj, 10.0)
    spacing = 300.0 / max(1.0, n ** (1.0 / dim))
    ls0 = max(0.5, 0.8 * spacing)
    for _ in range(20):
        ls = ls0 * rng.uniform(0.8, 1.2, size=n_obj)
        km = np.zeros((n_obj, n, n))
        O.update_k(km, x, 0, n, pv, ls)
        ev = [np.abs(np.linalg.eigvalsh(km[o] / pv[o] + 1e-6 * np.eye(n))) for o in range(n_obj)]
        cond = max(e.max() / e.min() for e in ev)
        if cond < 1e6:
            return x, y, pm, pv, ls, km, cond
        ls0 *= 0.7
    raise AssertionError("no well-conditioned length scale")


@pytest.fixture(scope="module")
def bo():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    bo._lib.load()
    return bo


@pytest.mark.parametrize("path", ["cholesky", "lu"])
@pytest.mark.parametrize("n,n_obj,dim", CASES, ids=[f"n{n}-obj{o}-d{d}" for n, o, d in CASES])
def test_invert_k_paths_vs_lapack(bo, n, n_obj, dim, path):
    import torch
    x, y, pm, pv, ls, km, cond = _problem(n, n_obj, dim)
    before = bo._lib.invert_k_path_counts()
    taken = []
    got = bo.kernels.invert_k(n, torch.tensor(km, device="cuda"), lu_hint=[path == "lu"] * n_obj,
                              paths=taken).cpu().numpy()
    after = bo._lib.invert_k_path_counts()
    assert after[path] - before[path] == n_obj, (before, after)
    assert taken == [{"cholesky": 0, "lu": 1}[path]] * n_obj, taken
    ref = O.invert_k(n, km)
    worst = 0.0
    for o in range(n_obj):
        a = km[o] + 1e-6 * np.eye(n)
        res_got = np.abs(a @ got[o] - np.eye(n)).max()
        res_ref = np.abs(a @ ref[o] - np.eye(n)).max()
        worst = max(worst, res_got / max(res_ref, 1e-300))
        assert res_got <= max(10.0 * res_ref, 1e-12), (o, res_got, res_ref)
    print(f"N {n} obj {n_obj} d {dim} {path}: cond {cond:.1e}, worst residual / LAPACK's {worst:.2f}")


@pytest.mark.parametrize("n,n_obj,dim", CASES, ids=[f"n{n}-obj{o}-d{d}" for n, o, d in CASES])
def test_compute_mll_vs_oracle(bo, n, n_obj, dim):
    import torch
    x, y, pm, pv, ls, _, cond = _problem(n, n_obj, dim)
    km = torch.zeros((n_obj, n, n), dtype=torch.float64, device="cuda")
    before = bo._lib.fit_path_counts()
    try:
        v = bo.kernels.compute_mll(torch.tensor(x, device="cuda"), torch.tensor(y, device="cuda"), km, pm, pv,
                                   ls, n)
    except np.linalg.LinAlgError:
        v = np.nan
    after = bo._lib.fit_path_counts()
    sched = "persistent" if -(-n // 32) <= 48 else "launches"       # BO_FIT_PERSIST_MAX_NBT
    other = "launches" if sched == "persistent" else "persistent"
    assert after[sched] > before[sched] and after[other] == before[other], (before, after)
    assert after["aborted"] == before["aborted"]
    km_h = np.zeros((n_obj, n, n))
    with np.errstate(all="ignore"):
        ref = O.compute_mll(x, y, km_h, pm, pv, ls, n)
    print(f"N {n} obj {n_obj} d {dim}: cond {cond:.1e}, mll {v!r} (oracle {ref!r})")
    if np.isnan(ref):
        assert np.isnan(v)
        return
    assert v == pytest.approx(ref, rel=1e-9)
    np.testing.assert_allclose(km.cpu().numpy(), km_h, rtol=1e-14, atol=1e-15 * pv.max())
