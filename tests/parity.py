"""Tolerance rules shared by the parity tests.

  mu          |d| <= 1e-5 * max(|ref|, sqrt(pv))            (1e-5 relative, fp64)
  var         |d| <= 1e-5 * pv                              (variance cancellation near data)
  std_mu      |d| <= 1e-5 * max(1, |ref|)
  std_var     |d| <= 1e-5
  ucb, acq    |d| <= 1e-5 * max(1, |ref|)
  top-q       indices equal where the reference's gap to the next value exceeds 10x the
              acq tolerance; otherwise the reference acq values at the chosen indices must
              match the reference's own top values within the tolerance.
"""

import numpy as np

RTOL = 1e-5


def _fail(name, bad, got, ref):
    i = np.flatnonzero(bad.ravel())[:5]
    return f"{name}: {bad.sum()} / {bad.size} out of tolerance; e.g. idx {i} got {got.ravel()[i]} ref {ref.ravel()[i]}"


def check_predict(got, ref, pv):
    pv = np.asarray(pv, dtype=np.float64)[:, None]
    rules = {
        "mu": lambda r: RTOL * np.maximum(np.abs(r), np.sqrt(pv)),
        "var": lambda r: RTOL * pv * np.ones_like(r),
        "std_mu": lambda r: RTOL * np.maximum(1.0, np.abs(r)),
        "std_var": lambda r: RTOL * np.ones_like(r),
        "ucb": lambda r: RTOL * np.maximum(1.0, np.abs(r)),
        "acq": lambda r: RTOL * np.maximum(1.0, np.abs(r)),
    }
    for name, tol in rules.items():
        if name not in got:
            continue
        g = np.asarray(got[name], dtype=np.float64)
        r = np.asarray(ref[name], dtype=np.float64)
        assert g.shape == r.shape, (name, g.shape, r.shape)
        bad = ~(np.abs(g - r) <= tol(r))
        assert not bad.any(), _fail(name, bad, g, r)


def check_topq(got_idx, acq_ref, excluded, q, tol=None):
    """got_idx: selected global indices (in order); acq_ref: reference acq over all
    candidates; excluded: bool mask of evaluated candidates; tol: per-candidate acq tolerance
    (array over all candidates, or a scalar) replacing RTOL * max(1, |ref|) (the fp32 kernel)."""
    got_idx = np.asarray(got_idx, dtype=np.int64)
    got_idx = got_idx[got_idx >= 0]
    a = np.where(excluded, -np.inf, np.asarray(acq_ref, dtype=np.float64))
    n_avail = int((~excluded).sum())
    assert got_idx.size == min(q, n_avail)
    assert not excluded[got_idx].any(), "selected an evaluated point"
    order = np.argsort(-a, kind="stable")[: q + 1]
    ref_top = a[order]
    if tol is None:
        tol = RTOL * np.maximum(1.0, np.abs(ref_top))
    else:   # the larger of the two candidates' bounds: the chosen one and the rank's reference one
        tv = np.broadcast_to(np.asarray(tol, dtype=np.float64), a.shape)
        tol = np.maximum(tv[order], np.max(tv[got_idx]) if got_idx.size else 0.0)
    for t in range(got_idx.size):
        gap_ok = t + 1 < ref_top.size and (ref_top[t] - ref_top[t + 1]) > 10 * tol[t] and \
            (t == 0 or (ref_top[t - 1] - ref_top[t]) > 10 * tol[t])
        if gap_ok:
            assert got_idx[t] == order[t], f"rank {t}: got {got_idx[t]} ref {order[t]}"
        else:
            assert abs(a[got_idx[t]] - ref_top[t]) <= 2 * tol[t], (t, a[got_idx[t]], ref_top[t])
