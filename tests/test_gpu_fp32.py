"""BO_PREDICT_FP32 (BASELINE config C5: "fp32 with fp64 reference check"): the f32 matrix-core
variant of the fused predict + acquisition kernel against the f64 oracle.

Tolerances (written here, SURVEY.md §8c "fp32 (C5)"): variance |d| <= 1e-3 pv; mean
|d| <= 1e-3 sqrt(pv); the acquisition inherits sqrt(|std var|), whose error near evaluated
points (std var -> 0) is up to sqrt(1e-3) per objective, so |d acq| <= sum_o (1e-3 + beta_o
sqrt(1e-3)) pointwise and a median error below 1e-4; selected candidates must be within that
bound of the reference's best acquisition values."""
import numpy as np
import pytest

from oracle import oracle_np as O
from fullref import cpu_full

pytestmark = pytest.mark.gpu

VAR_TOL = 1e-3


@pytest.fixture(scope="module")
def bo():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    bo._lib.load()
    return bo


def test_mfma_f32_layout(bo):
    import torch
    rng = np.random.default_rng(0)
    a = rng.normal(size=(16, 4)).astype(np.float32)
    b = rng.normal(size=(4, 16)).astype(np.float32)
    ta, tb = torch.as_tensor(a, device="cuda"), torch.as_tensor(b, device="cuda")
    td = torch.empty((16, 16), dtype=torch.float32, device="cuda")
    bo._lib.check(bo._lib.load().bo_selftest_mfma_f32(ta.data_ptr(), tb.data_ptr(), td.data_ptr(), None),
                  "selftest")
    torch.cuda.synchronize()
    np.testing.assert_allclose(td.cpu().numpy(), a.astype(np.float64) @ b, rtol=1e-5, atol=1e-5)


def _problem(rng, n, dim, n_obj, cand, ls):
    x = cand[rng.choice(cand.shape[0], n, replace=False)].astype(np.float64)
    y = rng.normal(size=(n, n_obj)) * 40 + 7
    pm, pv = y.mean(0), y.var(0)
    lsv = np.full(n_obj, ls)
    betas = rng.uniform(0.5, 2.5, size=n_obj)
    km = np.zeros((n_obj, n, n))
    O.update_k(km, x, 0, n, pv, lsv)
    kinv = O.invert_k(n, km)
    return x, y, pm, pv, lsv, betas, kinv


@pytest.mark.parametrize("n,dim,n_obj,m,ls", [(300, 6, 3, 20000, 40.0), (2048, 6, 3, 65536, 40.0),
                                              (100, 2, 2, 0, 6.0)])
def test_fp32_vs_f64_oracle(bo, n, dim, n_obj, m, ls):
    import torch
    rng = np.random.default_rng(n)
    if m:
        from scipy.stats import qmc
        cand = qmc.Sobol(dim, scramble=False).random(m) * 300.0
        cands = bo.CandidateSet.explicit(cand)
    else:
        cands = bo.CandidateSet.grid([(0, 128), (0, 96)])
        cand = O.grid_points([(0, 128), (0, 96)]).astype(np.float64)
        m = cand.shape[0]
    x, y, pm, pv, lsv, betas, kinv = _problem(rng, n, dim, n_obj, cand, ls)
    res = bo.predict_acquire(x, y, kinv, cands, pm, pv, lsv, betas, outputs=("mu", "var", "acq"),
                             topq=16, mode="fp32")
    torch.cuda.synchronize()
    got = {k: res[k].cpu().numpy() for k in ("mu", "var", "acq", "top_idx")}
    # every candidate against the f64 CPU reference (oracle/cpu_ref.c)
    ref = cpu_full(("fp32", n, dim, m), x, y, cand, kinv, pm, pv, lsv, betas)
    sq = np.sqrt(pv)[:, None]
    dv = np.abs(got["var"] - ref["var"]) / pv[:, None]
    dm = np.abs(got["mu"] - ref["mu"]) / sq
    assert dv.max() <= VAR_TOL, dv.max()
    assert dm.max() <= VAR_TOL, dm.max()
    acq_tol = float(np.sum(1e-3 + betas * np.sqrt(VAR_TOL)))
    da = np.abs(got["acq"] - ref["acq"])
    assert da.max() <= acq_tol * max(1.0, np.abs(ref["acq"]).max()), da.max()
    assert np.median(da) <= 1e-4, np.median(da)
    # selection: 16 distinct, non-evaluated candidates whose reference acquisition is within the
    # bound of the reference's own best non-evaluated values
    top = got["top_idx"]
    assert np.unique(top).size == 16 and (top >= 0).all()
    xs = {tuple(r) for r in x}
    assert not any(tuple(cand[i]) in xs for i in top)
    ref_top = ref["acq"][top]
    full_ref_best = np.sort(ref["acq"][[tuple(c) not in xs for c in cand]])[::-1][:16]
    assert ref_top.min() >= full_ref_best[-1] - 2 * acq_tol
