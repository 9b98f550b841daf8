"""A seeded sweep over the standalone batch selection (select_next_batch, acquisition.py:116-144;
bo_select_topq and bo_select_topq_masked) against its exact order on the host.

The reference walks np.argsort(acquisition_values)[::-1] and skips every candidate equal to an
evaluated point (acquisition.py:134-142), so the order is: NaN first, then descending value, and
-- the reference's argsort tie order being unspecified -- exact ties by ascending index (the order
every path of this build uses).  The selection is integer work: it must equal that
order exactly.

Sizes: M = 1 .. 2^20 + 3 (below, at and above one wave, one workgroup and the small/large kernels'
split); q = 1 .. 48 (BO_MAX_TOPQ) and 64 (taken in rounds); value sets: normal, rounded to one
decimal (many exact ties), all equal, NaNs (including at the top), +-inf, signed zeros and
subnormals; exclusion by the per-call evaluated points and by the persistent mask (ExclusionMask)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 63, 64, 65, 1000, 4097, 65537, (1 << 20) + 3]
QS = [1, 3, 4, 5, 16, 48, 64]
DISTS = ["normal", "ties", "equal", "nan", "inf", "zeros", "subnormal"]


def _values(dist, m, rng):
    if dist == "normal":
        return rng.normal(size=m)
    if dist == "ties":
        return np.round(rng.normal(size=m), 1)
    if dist == "equal":
        return np.full(m, 0.25)
    if dist == "nan":
        a = rng.normal(size=m)
        a[rng.choice(m, max(1, m // 50), replace=False)] = np.nan
        a[0] = np.nan
        return a
    if dist == "inf":
        a = rng.normal(size=m)
        k = max(1, m // 40)
        a[rng.choice(m, k, replace=False)] = np.inf
        a[rng.choice(m, k, replace=False)] = -np.inf
        return a
    if dist == "zeros":
        return np.where(rng.random(m) < 0.5, 0.0, -0.0) * np.where(rng.random(m) < 0.9, 1.0, 0.0) + \
            np.where(rng.random(m) < 0.05, rng.normal(size=m), 0.0)
    if dist == "subnormal":
        return rng.integers(-40, 40, size=m) * 5e-324
    raise ValueError(dist)


def _want(acq, excl, q):
    """The reference's order over the non-excluded candidates, first q."""
    nan = np.isnan(acq)
    key = np.where(nan, 0.0, acq)
    order = np.lexsort((np.arange(acq.size), -key, ~nan))
    order = order[~excl[order]]
    return order[:q]


CASES = [(m, q, d) for m in SIZES for q in QS for d in DISTS
         if not (m > 70000 and d not in ("normal", "ties", "nan")) and not (m > 5000 and q in (4, 5))]


@pytest.fixture(scope="module")
def bo():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    bo._lib.load()
    return bo


@pytest.mark.parametrize("m,q,dist", CASES, ids=[f"m{m}-q{q}-{d}" for m, q, d in CASES])
def test_select_matches_reference_order(bo, m, q, dist):
    import torch
    rng = np.random.default_rng(m * 1000 + q * 10 + DISTS.index(dist))
    acq = _values(dist, m, rng)
    rows = 1 << max(0, (m - 1).bit_length() // 2)
    cols = -(-m // rows)
    cands_all = bo.CandidateSet.grid([(0, rows), (0, cols)])
    # the first m candidates of a rows x cols grid: an explicit int64 copy (the reference's
    # input_space) so the per-call path compares coordinates
    pts = cands_all.points(np.arange(m))
    cands = bo.CandidateSet.explicit(pts)
    n_ev = min(m - 1, max(1, m // 30)) if m > 1 else 0
    ev_idx = rng.choice(m, n_ev, replace=False) if n_ev else np.zeros(0, dtype=np.int64)
    # an evaluated point at the very top of the order where there is one
    top = _want(acq, np.zeros(m, dtype=bool), 1)
    if n_ev and top.size:
        ev_idx[0] = top[0]
    ev = pts[ev_idx].astype(np.float64)
    excl = np.zeros(m, dtype=bool)
    excl[ev_idx] = True
    want = _want(acq, excl, q)
    acq_d = torch.tensor(acq, device="cuda")
    got = bo.acquisition.select_indices(acq_d, cands, ev, q)
    np.testing.assert_array_equal(got, want)
    if q <= 48:
        mask = bo.acquisition.ExclusionMask(cands, 0, m, "cuda").update(ev)
        np.testing.assert_array_equal(mask.excluded(), excl)
        got_m = bo.acquisition.select_indices(acq_d, cands, ev, q, mask=mask)
        np.testing.assert_array_equal(got_m, want)
