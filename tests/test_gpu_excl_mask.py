"""The persistent exclusion mask (bo_excl_mask_update) and the masked selections
(bo_select_topq_masked, bo_hvi_select_topq_masked) against the reference's exclusion rule,
acquisition.py:137-139: a candidate is skipped iff it equals an evaluated point in every
coordinate (numeric ==, so -0.0 == 0.0 and an int64 grid coordinate equals the same float).

Every mask is compared bit for bit with numpy's membership test over the whole candidate set;
every masked selection with numpy's order (NaN first, descending value, ascending index) and
with the unmasked call."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bo():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    return bo


def _rows_in(pts, x):
    """Rows of pts equal (numeric ==, every coordinate) to some row of x."""
    if x.shape[0] == 0:
        return np.zeros(pts.shape[0], dtype=bool)
    z = lambda a: np.where(a == 0.0, 0.0, a)                # -0.0 == 0.0  # noqa: E731
    v = lambda a: np.ascontiguousarray(z(np.asarray(a, dtype=np.float64))).view(  # noqa: E731
        np.dtype((np.void, 8 * a.shape[1]))).ravel()
    ok = ~np.isnan(x).any(axis=1)
    return np.isin(v(pts), v(x[ok]))


def _grid_points(rng, cands, n_on):
    """n_on grid points (some duplicated) plus points that match no candidate: off the grid,
    non-integer, NaN, one coordinate out of range; and -0.0 for a zero coordinate."""
    idx = rng.choice(cands.n, n_on, replace=False)
    on = cands.points(idx).astype(np.float64)
    on[on == 0.0] = -0.0
    off = on[: 8].copy()
    off[:, 0] += 0.5                                           # non-integer
    far = on[8:12].copy()
    far[:, -1] = cands.lo[-1] + cands.shape[-1]                 # one past the last axis
    neg = on[12:14].copy()
    neg[:, 0] = cands.lo[0] - 1
    nan = on[14:15].copy()
    nan[0, 0] = np.nan
    return np.concatenate([on, on[:5], off, far, neg, nan])


@pytest.mark.parametrize("offset,count", [(0, None), (300_017, 200_000)])
def test_grid_mask_matches_membership(bo, offset, count):
    from bayesopt_smart_amd.acquisition import ExclusionMask
    cands = bo.predict.CandidateSet.grid([(-3, 509), (0, 1000)])
    count = cands.n - offset if count is None else count
    rng = np.random.default_rng(offset + 1)
    ev = _grid_points(rng, cands, 400)
    # some points inside this shard for sure
    ev = np.concatenate([ev, cands.points(offset + rng.choice(count, 50, replace=False)).astype(np.float64)])
    m = ExclusionMask(cands, offset, count, "cuda")
    m.update(ev[:100])
    m.update(ev)                                   # the extension adds the new rows only
    pts = cands.points(offset + np.arange(count)).astype(np.float64)
    want = _rows_in(pts, ev)
    assert want.sum() >= 50
    np.testing.assert_array_equal(m.excluded(), want)
    full = ExclusionMask(cands, offset, count, "cuda").update(ev)
    np.testing.assert_array_equal(full.bits.cpu().numpy(), m.bits.cpu().numpy())
    # a changed prefix rebuilds (the mask then holds exactly the new set)
    m.update(ev[50:])
    np.testing.assert_array_equal(m.excluded(), _rows_in(pts, ev[50:]))


@pytest.mark.parametrize("kind", ["sobol", "f64", "i64"])
def test_scan_mask_matches_membership(bo, kind):
    from bayesopt_smart_amd.acquisition import ExclusionMask
    rng = np.random.default_rng(7)
    if kind == "sobol":
        cands = bo.predict.CandidateSet.sobol_set(5, 200_000, lo=-2.0, scale=40.0)
    elif kind == "f64":
        cands = bo.predict.CandidateSet.explicit(rng.uniform(-5, 5, size=(150_000, 4)))
    else:
        cands = bo.predict.CandidateSet.explicit(rng.integers(-50, 50, size=(150_000, 3)))
    offset, count = 10_000, cands.n - 20_000
    ev = cands.points(rng.choice(cands.n, 300, replace=False)).astype(np.float64)
    ev = np.concatenate([ev, ev[:7] + 1e-9, ev[:3]])           # near misses and duplicates
    m = ExclusionMask(cands, offset, count, "cuda").update(ev[:200]).update(ev)
    pts = cands.points(offset + np.arange(count)).astype(np.float64)
    np.testing.assert_array_equal(m.excluded(), _rows_in(pts, ev))


@pytest.mark.parametrize("q", [1, 3, 4, 5, 16, 48])
@pytest.mark.parametrize("kind", ["grid", "sobol"])
def test_masked_select_equals_unmasked_and_numpy(bo, q, kind):
    """The best candidates are evaluated points (more of them than any q): the masked selection
    must skip them exactly as the per-call exclusion does."""
    import torch
    from bayesopt_smart_amd.acquisition import ExclusionMask
    if kind == "grid":
        cands = bo.predict.CandidateSet.grid([(0, 1024), (0, 1024)])
    else:
        cands = bo.predict.CandidateSet.sobol_set(3, 1 << 20, scale=10.0)
    n = cands.n
    rng = np.random.default_rng(q)
    acq = rng.standard_normal(n)
    hot = rng.choice(n, 512, replace=False)
    acq[hot[:128]] = 50.0 + np.arange(128)                  # the top of the order: excluded
    acq[rng.choice(n, 3)] = 50.5                             # ties with excluded values
    acq[11] = np.nan                                        # NaN is selected first
    ev = cands.points(hot).astype(np.float64)
    acq_d = torch.tensor(acq, device="cuda")
    m = ExclusionMask(cands, 0, n, "cuda").update(ev)
    got = bo.acquisition.select_indices(acq_d, cands, ev, q, mask=m)
    ref = bo.acquisition.select_indices(acq_d, cands, ev, q)
    excl = np.zeros(n, dtype=bool)
    excl[hot] = True
    order = np.lexsort((np.arange(n), -np.where(excl, -np.inf, np.nan_to_num(acq, nan=np.inf))))
    np.testing.assert_array_equal(got, order[:q])
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("q", [3, 16])
def test_masked_select_on_a_shard(bo, q):
    """A rank's shard [offset, offset + count): the mask covers the shard (local bit j = global
    candidate offset + j) and the masked selection returns global indices, equal to the
    per-call exclusion over the same shard and to numpy's order on it."""
    import ctypes
    import torch
    from bayesopt_smart_amd import _lib
    from bayesopt_smart_amd.acquisition import ExclusionMask, _grid_args
    cands = bo.predict.CandidateSet.grid([(0, 1024), (0, 1024)])
    offset, count = 3 * (1 << 18) + 77, (1 << 18) - 300          # shard 3 of 4, ragged
    rng = np.random.default_rng(q + 100)
    acq = rng.standard_normal(count)
    hot_local = rng.choice(count, 200, replace=False)
    acq[hot_local[:40]] = 30.0 + np.arange(40)                 # the shard's top: evaluated
    out_of_shard = rng.choice(offset, 100, replace=False)      # evaluated points elsewhere
    ev = cands.points(np.concatenate([offset + hot_local, out_of_shard])).astype(np.float64)
    m = ExclusionMask(cands, offset, count, "cuda").update(ev)
    lib = _lib.load()
    acq_d = torch.tensor(acq, device="cuda")
    ws = torch.empty(lib.bo_select_topq_workspace_size(count, q), dtype=torch.uint8, device="cuda")
    res = {}
    for masked in (True, False):
        tv = torch.empty(q, dtype=torch.float64, device="cuda")
        ti = torch.empty(q, dtype=torch.int64, device="cuda")
        if masked:
            st = lib.bo_select_topq_masked(acq_d.data_ptr(), count, offset, m.ptr, q, tv.data_ptr(), ti.data_ptr(),
                                           ws.data_ptr(), ws.numel(), None)
        else:
            ex = torch.tensor(ev, device="cuda")
            lo, sh = _grid_args(cands)
            st = lib.bo_select_topq(acq_d.data_ptr(), count, cands.kind_code, None, lo, sh, 2, offset,
                                    ex.data_ptr(), ex.shape[0], q, tv.data_ptr(), ti.data_ptr(), ws.data_ptr(),
                                    ws.numel(), None)
        _lib.check(st, "select")
        torch.cuda.synchronize()
        res[masked] = ti.cpu().numpy()
    excl = np.zeros(count, dtype=bool)
    excl[hot_local] = True
    order = np.lexsort((np.arange(count), -np.where(excl, -np.inf, acq)))
    np.testing.assert_array_equal(res[True], offset + order[:q])
    np.testing.assert_array_equal(res[True], res[False])
    del ctypes


def test_masked_select_everything_excluded(bo):
    """A shard whose candidates are all evaluated yields an empty batch (index -1 entries)."""
    import torch
    from bayesopt_smart_amd.acquisition import ExclusionMask
    cands = bo.predict.CandidateSet.grid([(0, 40), (0, 50)])
    ev = cands.points(np.arange(cands.n)).astype(np.float64)
    m = ExclusionMask(cands, 0, cands.n, "cuda").update(ev)
    assert m.excluded().all()
    got = bo.acquisition.select_indices(torch.zeros(cands.n, dtype=torch.float64, device="cuda"), cands, ev, 3,
                                        mask=m)
    assert got.size == 0
