"""CPU model of the device fit's launch schedule (bayesopt_smart_amd/csrc/bo_fit.hip): the
right-looking blocked Cholesky of the AUGMENTED matrix [[K, .], [B, C]] with one launch per
column step, each launch running the panel of step k (with step k-1's update of its own column
block, lookahead) beside step k-1's update of every other live tile -- exactly the panel slabs,
the update tiles (decoded from the linear task index as update_role decodes them) and the
structurally-zero tiles the kernels skip.  Reproduces compute_mll (numba_kernels.py:152-235) and
invert_k (:370-403).  Runs in numpy with small tiles so that every branch of the schedule (several
steps, padding, ragged N) is exercised; the GPU tests check the kernels themselves."""

import math

import numpy as np
import pytest

from oracle import oracle_np as O


def tri_row(t):
    u = int((math.sqrt(8.0 * t + 1.0) - 1.0) * 0.5)
    while (u + 1) * (u + 2) // 2 <= t:
        u += 1
    while u * (u + 1) // 2 > t:
        u -= 1
    return u


def lpart_S(u, base):
    return u * base + u * (u - 1) // 2


def decode(t, k, nbt, ident, TL, nb):
    """update_role's task decode: (row0, col0, first) of the tile of task t at launch k."""
    np_ = nbt * nb
    if t < TL:
        base = k + 1 if ident else 2
        bb = 2.0 * base - 1.0
        u = max(0, int((-bb + math.sqrt(bb * bb + 8.0 * t)) * 0.5))
        while lpart_S(u + 1, base) <= t:
            u += 1
        while lpart_S(u, base) > t:
            u -= 1
        c = nbt - 1 - u
        return (c + (t - lpart_S(u, base))) * nb, c * nb, False
    t -= TL
    u = tri_row(t)
    cp = k - 1 - u
    b = cp + (t - u * (u + 1) // 2)
    return np_ + b * nb, np_ + cp * nb, b == k - 1


def upd_kind(k, ident, defer):
    """fit_factor's update kind of launch k: 0 = step k-1 on every live tile; for the MLL,
    1 (odd k) = step k-1 on column block k+1 only, 2 (even k) = steps k-2 and k-1 (rank 64)."""
    return 0 if (ident or not defer) else (1 if k & 1 else 2)


def step_counts(k, nbt, ident, defer=False):
    """fit_factor's per-launch counts: panel workgroups, L-part and C-part update tiles."""
    n_panel = (nbt if ident else nbt - k) if k < nbt else 0
    TL = TC = 0
    if k >= 1:
        m = nbt - 1 - k
        base = k + 1 if ident else 2
        TL = m * base + m * (m - 1) // 2 if m > 0 else 0
        TC = k * (k + 1) // 2 if ident else 0
        if upd_kind(k, ident, defer) == 1:
            TL = nbt - k if k + 1 < nbt else 0
    return n_panel, TL, TC


def fit_schedule(A, n, nb, ident, defer=False):
    """bo_fit.hip fit_factor on one objective (tile nb), in place; returns False on a bad pivot.
    defer: the MLL's schedule (update_role<1> on odd launches, update_role<2> on even ones)."""
    nbt = -(-n // nb)
    np_ = nbt * nb
    ok = True
    steps = nbt + 1 if ident else nbt
    for k in range(steps):
        n_panel, TL, TC = step_counts(k, nbt, ident, defer)
        kind = upd_kind(k, ident, defer)
        old = A.copy()                          # every role of launch k reads the launch's input
        cK, cP = k * nb, (k - 1) * nb
        for w in range(n_panel):                # panel role: diagonal tile + slab block sb
            sb = k + 1 + w
            rows = list(range(cK, cK + nb)) + list(range(sb * nb, sb * nb + nb))
            C = old[rows, cK:cK + nb].copy()
            if k > 0:
                Lr = old[rows, cP:cP + nb].copy()
                if ident and sb == nbt + k:     # bottom block k: structurally zero in column k-1
                    Lr[nb:] = 0.0
                C -= Lr @ old[cK:cK + nb, cP:cP + nb].T
            D = np.tril(C[:nb])
            D = D + np.tril(D, -1).T
            if np.any(~(np.linalg.eigvalsh(D) > 0)):
                ok = False
                continue
            L = np.linalg.cholesky(D)
            if w == 0:
                A[cK:cK + nb, cK:cK + nb] = np.tril(L) + np.triu(old[cK:cK + nb, cK:cK + nb], 1)
            A[sb * nb:sb * nb + nb, cK:cK + nb] = np.linalg.solve(L, C[nb:].T).T
        tiles = set()
        R = 2 if kind == 2 else 1               # steps applied by this launch's update role
        cS = (k - R) * nb
        for t in range(TL + TC):                # update role
            if kind == 1:
                r0, c0, first = (k + 1 + t) * nb, (k + 1) * nb, False
            else:
                r0, c0, first = decode(t, k, nbt, ident, TL, nb)
            assert (r0, c0) not in tiles
            tiles.add((r0, c0))
            upd = old[r0:r0 + nb, cS:cS + R * nb] @ old[c0:c0 + nb, cS:cS + R * nb].T
            A[r0:r0 + nb, c0:c0 + nb] = (0.0 if first else old[r0:r0 + nb, c0:c0 + nb]) - upd
        if kind == 1 and k >= 1:
            assert tiles == {(r * nb, (k + 1) * nb) for r in range(k + 1, nbt + 1)} if k + 1 < nbt else not tiles
        # the live set the decode enumerates: L part (columns > k, rows from the diagonal to the
        # live bottom) and, for the inverse, C's lower tiles of the live bottom blocks
        elif k >= 1:
            rb_hi = nbt + (k if ident else 1)
            want = {(r * nb, c * nb) for c in range(k + 1, nbt) for r in range(c, rb_hi)}
            if ident:
                want |= {(np_ + b * nb, np_ + cp * nb) for cp in range(k) for b in range(cp, k)}
            assert tiles == want
    return ok


def build(km, n, nb, ident, jitter, yc=None):
    """fit_init_kernel: K + jitter (padding identity), B = I or the one row yc, C unset (NaN:
    the schedule must never read it before its first contribution)."""
    nbt = -(-n // nb)
    np_ = nbt * nb
    na = 2 * np_ if ident else np_ + nb
    A = np.full((na, na if ident else np_), np.nan)
    A[:np_, :np_] = np.eye(np_)
    A[:n, :n] = km + jitter * np.eye(n)
    if ident:                                    # only the tiles b <= j are written (B = I)
        for b in range(nbt):
            A[np_ + b * nb:np_ + (b + 1) * nb, b * nb:np_] = 0.0
        A[np_:np_ + n, :n] = np.eye(n)
    else:
        A[np_:, :] = 0.0
        A[np_, :n] = yc
    A[np.triu_indices(A.shape[0], 1, A.shape[1])] = np.nan   # never written by the init kernel
    return A, np_


@pytest.mark.parametrize("n,nb", [(5, 4), (37, 8), (64, 16), (100, 32), (70, 8)])
def test_augmented_inverse_schedule(n, nb):
    rng = np.random.default_rng(n)
    x = rng.uniform(0, 30, size=(n, 2))
    km = np.zeros((1, n, n))
    O.update_k(km, x, 0, n, [3.0], [4.0])
    A, np_ = build(km[0], n, nb, True, 1e-6)
    assert fit_schedule(A, n, nb, True)
    got = -np.tril(A[np_:np_ + n, np_:np_ + n])
    got = got + np.tril(got, -1).T
    ref = O.invert_k(n, km)[0]
    assert np.abs(got - ref).max() <= 1e-9 * np.abs(ref).max()


@pytest.mark.parametrize("defer", [False, True])
@pytest.mark.parametrize("n,nb", [(5, 4), (37, 8), (100, 32), (70, 8), (60, 4), (64, 4)])
def test_augmented_mll_schedule(n, nb, defer):
    rng = np.random.default_rng(n + 1)
    x = rng.uniform(0, 30, size=(n, 2))
    y = rng.normal(size=(n, 2)) * 10
    pm, pv, ls = y.mean(0) + 1.0, y.var(0), np.array([4.0, 6.0])
    ref = O.compute_mll(x, y, np.zeros((2, n, n)), pm, pv, ls, n)
    km = np.zeros((2, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    tot = 0.0
    nbt = -(-n // nb)
    for o in range(2):
        yc = y[:, o] - pm[o]                    # unscaled: |z|^2 / var(yc) is the data fit
        A, np_ = build(km[o] / pv[o], n, nb, False, 1e-8, yc)
        assert fit_schedule(A, n, nb, False, defer)
        z = A[np_, :np_]
        fit = float(np.sum(z * z)) / np.var(yc)
        logdet = 2.0 * np.sum(np.log(np.diag(A)[:n]))
        tot += -0.5 * fit - 0.5 * logdet - 0.5 * n * np.log(2 * np.pi)
        assert nbt >= 1
    assert tot == pytest.approx(ref, rel=1e-8)   # K/pv here has cond ~1e8: solve-order rounding


def test_not_pd_is_flagged():
    n, nb = 20, 4
    km = -np.eye(n)
    A, _ = build(km, n, nb, False, 1e-8, np.zeros(n))
    assert not fit_schedule(A, n, nb, False)
