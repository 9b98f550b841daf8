"""CPU model of the device fit's tile schedule (bayesopt_smart_amd/csrc/bo_fit.hip): the
right-looking blocked Cholesky of the AUGMENTED matrix [[K, .], [B, C]], with exactly the panel
row blocks and trailing-update tiles the kernels launch per step (including the skipped
structurally-zero tiles of the inverse), reproduces compute_mll (numba_kernels.py:152-235) and
invert_k (:370-403).  Runs in numpy with small tiles so that every branch of the schedule
(several steps, padding, ragged N) is exercised; the GPU tests check the kernels themselves."""

import numpy as np
import pytest

from oracle import oracle_np as O


def _tri(t):
    i = int((np.sqrt(8.0 * t + 1.0) - 1.0) * 0.5)
    while (i + 1) * (i + 2) // 2 <= t:
        i += 1
    while i * (i + 1) // 2 > t:
        i -= 1
    return i, t - i * (i + 1) // 2


def aug_factor(A, n, nb, ident):
    """bo_fit.hip aug_factor on one objective, tile size nb, in place (lower triangle)."""
    nbt = -(-n // nb)
    rb = nbt if ident else 1
    T = lambda p, q: (slice(p * nb, (p + 1) * nb), slice(q * nb, (q + 1) * nb))  # noqa: E731
    ok = True
    for k in range(nbt):
        ra = min(k + 1, rb) if ident else rb
        m = nbt - k - 1
        # chol_panel_kernel: diagonal tile, then the row blocks below (top + live bottom)
        d = A[T(k, k)]
        if np.any(~(np.linalg.eigvalsh(np.tril(d) + np.tril(d, -1).T) > 0)):
            ok = False
        L = np.linalg.cholesky(np.tril(d) + np.tril(d, -1).T)
        A[T(k, k)] = L
        rows = [k + 1 + i for i in range(m)] + [nbt + i for i in range(ra)]
        for p in rows:
            A[T(p, k)] = np.linalg.solve(L, A[T(p, k)].T).T           # X L^T = A_pk
        # chol_update_kernel: T1 top x top, T2 bottom x top, T3 bottom x bottom
        t1, t2 = m * (m + 1) // 2, ra * m
        for t in range(t1 + t2 + ra * (ra + 1) // 2):
            if t < t1:
                i, j = _tri(t)
                p, q = k + 1 + i, k + 1 + j
            elif t < t1 + t2:
                p, q = nbt + (t - t1) // m, k + 1 + (t - t1) % m
            else:
                i, j = _tri(t - t1 - t2)
                p, q = nbt + i, nbt + j
            A[T(p, q)] -= A[T(p, k)] @ A[T(q, k)].T
    return ok


def build(km, n, nb, ident, jitter, yc=None):
    nbt = -(-n // nb)
    rb = nbt if ident else 1
    na = (nbt + rb) * nb
    np_ = nbt * nb
    A = np.zeros((na, na))
    A[:np_, :np_] = np.eye(np_)
    A[:n, :n] = km + jitter * np.eye(n)
    if ident:
        A[np_:np_ + n, :n] = np.eye(n)
    else:
        A[np_, :n] = yc
    return A, np_


@pytest.mark.parametrize("n,nb", [(5, 4), (37, 8), (64, 16), (100, 32)])
def test_augmented_inverse_schedule(n, nb):
    rng = np.random.default_rng(n)
    x = rng.uniform(0, 30, size=(n, 2))
    km = np.zeros((1, n, n))
    O.update_k(km, x, 0, n, [3.0], [4.0])
    A, np_ = build(km[0], n, nb, True, 1e-6)
    assert aug_factor(A, n, nb, True)
    got = -np.tril(A[np_:np_ + n, np_:np_ + n])
    got = got + np.tril(got, -1).T
    ref = O.invert_k(n, km)[0]
    assert np.abs(got - ref).max() <= 1e-9 * np.abs(ref).max()


@pytest.mark.parametrize("n,nb", [(5, 4), (37, 8), (100, 32)])
def test_augmented_mll_schedule(n, nb):
    rng = np.random.default_rng(n + 1)
    x = rng.uniform(0, 30, size=(n, 2))
    y = rng.normal(size=(n, 2)) * 10
    pm, pv, ls = y.mean(0) + 1.0, y.var(0), np.array([4.0, 6.0])
    ref = O.compute_mll(x, y, np.zeros((2, n, n)), pm, pv, ls, n)
    km = np.zeros((2, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    tot = 0.0
    for o in range(2):
        yc = y[:, o] - pm[o]
        yc = yc / np.std(yc)
        A, np_ = build(km[o] / pv[o], n, nb, False, 1e-8, yc)
        assert aug_factor(A, n, nb, False)
        fit = -A[np_, np_]
        logdet = 2.0 * np.sum(np.log(np.diag(A)[:n]))
        tot += -0.5 * fit - 0.5 * logdet - 0.5 * n * np.log(2 * np.pi)
    assert tot == pytest.approx(ref, rel=1e-8)   # K/pv here has cond ~1e8: solve-order rounding
