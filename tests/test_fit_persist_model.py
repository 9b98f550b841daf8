"""CPU model of the device fit's PERSISTENT schedule (bayesopt_smart_amd/csrc/bo_fit.hip:
fit_factor_persist + fit_persist_kernel): the task queue of the augmented blocked Cholesky --
per block k the tiles of step k-1's update that column block k+1 needs (A_{k-1}[k+1]), the panels
P(k, w), the rest of step k-1's update (A_{k-1}[rest], and the inverse's C tiles) -- with the
kernel's task decode, its dependency flags (panel done, tile versions) and its rule that a
workgroup takes the next task in queue order only after finishing the current one.

The tasks run in a RANDOM interleaving of W workers, each operating on the matrix's current
contents as the device does (no launch-wide snapshot), so a missing or wrong dependency shows as
a wrong factorisation; every run must finish (no deadlock) and reproduce compute_mll
(numba_kernels.py:152-235) and invert_k (:370-403).  Test infrastructure only."""

import math

import numpy as np
import pytest

from oracle import oracle_np as O
from test_fit_blocking_model import build, lpart_S, tri_row


def plan(nbt, ident, n_obj):
    """fit_factor_persist's block offsets (tasks per block)."""
    steps = nbt + 1 if ident else nbt
    blk, tot = [], 0
    for k in range(steps):
        blk.append(tot)
        n1 = (nbt - 1 if ident else nbt - k) if (k >= 1 and k + 1 < nbt) else 0
        npn = (nbt if ident else nbt - k) if k < nbt else 0
        tl2, tc = n2(nbt, ident, k)
        tot += -(-n_obj * n1 // 4) + n_obj * npn + -(-n_obj * (tl2 + tc) // 4)
    blk.append(tot)
    return steps, blk


def n2(nbt, ident, k):
    if k < 1:
        return 0, 0
    m2, base = nbt - k - 2, (k + 1 if ident else 2)
    return (m2 * base + m2 * (m2 - 1) // 2 if m2 > 0 else 0), (k * (k + 1) // 2 if ident else 0)


def s0(nbt, ident, rb):
    return rb - nbt if (ident and rb >= nbt) else 0


def decode(t, nbt, ident, n_obj, steps, blk):
    """fit_persist_kernel's decode of task t: ('P', k, o, w) or ('A', s, [tiles]) with tiles
    (o, rb, cb, cpart, first), one per wave."""
    k = max(i for i in range(steps) if blk[i] <= t)
    r = t - blk[k]
    n1 = (nbt - 1 if ident else nbt - k) if (k >= 1 and k + 1 < nbt) else 0
    T1 = -(-n_obj * n1 // 4)
    npn = (nbt if ident else nbt - k) if k < nbt else 0
    nP = n_obj * npn
    if T1 <= r < T1 + nP:
        return ("P", k, (r - T1) // npn, (r - T1) % npn)
    tiles = []
    for wave in range(4):
        if r < T1:
            u = 4 * r + wave
            if u >= n_obj * n1:
                continue
            o, i = divmod(u, n1)
            rb = k + 1 + i if not ident else (k + 1 + i if i < nbt - k - 1 else nbt + (i - (nbt - k - 1)))
            tiles.append((o, rb, k + 1, False, False))
        else:
            tl2, tc = n2(nbt, ident, k)
            per = tl2 + tc
            u = 4 * (r - T1 - nP) + wave
            if per == 0 or u >= n_obj * per:
                continue
            o, tt = divmod(u, per)
            if tt < tl2:
                base = k + 1 if ident else 2
                bb = 2.0 * base - 1.0
                uu = max(0, int((-bb + math.sqrt(bb * bb + 8.0 * tt)) * 0.5))
                while lpart_S(uu + 1, base) <= tt:
                    uu += 1
                while lpart_S(uu, base) > tt:
                    uu -= 1
                c = nbt - 1 - uu
                tiles.append((o, c + (tt - lpart_S(uu, base)), c, False, False))
            else:
                tt -= tl2
                uu = tri_row(tt)
                cp = k - 1 - uu
                b = cp + (tt - uu * (uu + 1) // 2)
                tiles.append((o, b, cp, True, b == k - 1))
    return ("A", k - 1, tiles)


def deps(task, nbt, ident):
    """[(flag key, wanted value)] the kernel waits on; flags: ('p', o, k, w) panel done,
    ('v', o, rb, cb) / ('c', o, b, cp) tile versions (steps applied)."""
    if task[0] == "P":
        _, k, o, w = task
        sb = k + 1 + w
        if k == 0:
            return []
        d = [(("p", o, k - 1, 0), 1), (("v", o, k, k), k - 1),
             (("v", o, sb, k), max(k - 1 - s0(nbt, ident, sb), 0))]
        if not (ident and sb == nbt + k):
            d.append((("p", o, k - 1, sb - k), 1))
        return d
    _, s, tiles = task
    d = []
    for (o, rb, cb, cpart, first) in tiles:
        sr, sc = (nbt + rb, nbt + cb) if cpart else (rb, cb)
        d += [(("p", o, s, sr - s - 1), 1), (("p", o, s, sc - s - 1), 1)]
        if not first:
            d.append(((("c" if cpart else "v"), o, rb, cb), s - rb if cpart else s - s0(nbt, ident, rb)))
    return d


def run(As, nbt, nb, ident, n_obj, workers, rng):
    """Random interleaving of `workers` persistent workgroups over the task queue; the matrices
    As[o] are updated in place.  Returns the per-objective log-det and |z|^2 partial sums."""
    steps, blk = plan(nbt, ident, n_obj)
    total = blk[-1]
    np_ = nbt * nb
    flags = {}
    logdet = [0.0] * n_obj
    zz = [0.0] * n_obj
    nxt = 0
    held = [None] * workers
    done = 0
    while done < total:
        for i in range(workers):                      # idle workgroups dequeue in order
            if held[i] is None and nxt < total:
                held[i] = (nxt, decode(nxt, nbt, ident, n_obj, steps, blk))
                nxt += 1
        ready = [i for i in range(workers) if held[i] is not None and
                 all(flags.get(key, 0) >= want for key, want in deps(held[i][1], nbt, ident))]
        assert ready, f"deadlock at task {nxt}"
        i = ready[rng.integers(len(ready))]
        t, task = held[i]
        held[i] = None
        done += 1
        if task[0] == "P":
            _, k, o, w = task
            A = As[o]
            sb = k + 1 + w
            cK, cP = k * nb, (k - 1) * nb
            rows = list(range(cK, cK + nb)) + list(range(sb * nb, sb * nb + nb))
            C = A[rows, cK:cK + nb].copy()
            if k > 0:
                Lr = A[rows, cP:cP + nb].copy()
                if ident and sb == nbt + k:
                    Lr[nb:] = 0.0
                C -= Lr @ A[cK:cK + nb, cP:cP + nb].T
            D = np.tril(C[:nb])
            D = D + np.tril(D, -1).T
            L = np.linalg.cholesky(D)
            # only the slab rows are stored (the diagonal tile's input stays for the other panels)
            A[sb * nb:sb * nb + nb, cK:cK + nb] = np.linalg.solve(L, C[nb:].T).T
            if w == 0:
                d = np.diag(L)[: max(0, min(nb, n_valid[o] - cK))]
                logdet[o] += float(np.sum(np.log(d)))
            if not ident and sb == nbt:
                zz[o] += float(np.sum(A[np_, cK:cK + nb] ** 2))
            flags[("p", o, k, w)] = 1
        else:
            _, s, tiles = task
            for (o, rb, cb, cpart, first) in tiles:
                A = As[o]
                r0, c0 = ((np_ + rb * nb, np_ + cb * nb) if cpart else (rb * nb, cb * nb))
                Lp = A[:, s * nb:(s + 1) * nb]
                upd = Lp[r0:r0 + nb] @ Lp[c0:c0 + nb].T
                A[r0:r0 + nb, c0:c0 + nb] = (0.0 if first else A[r0:r0 + nb, c0:c0 + nb]) - upd
            for (o, rb, cb, cpart, first) in tiles:
                key = ("c" if cpart else "v", o, rb, cb)
                flags[key] = (s - rb + 1) if cpart else (s - s0(nbt, ident, rb) + 1)
    assert nxt == total and all(h is None for h in held)
    return logdet, zz


n_valid = {}


@pytest.mark.parametrize("n,nb,workers,seed", [(5, 4, 1, 0), (37, 8, 3, 1), (64, 8, 16, 2), (100, 16, 7, 3),
                                               (70, 8, 64, 4), (61, 4, 5, 5)])
def test_persistent_inverse_schedule(n, nb, workers, seed):
    rng = np.random.default_rng(seed)
    x = rng.uniform(0, 100, size=(n, 2))
    km = np.zeros((2, n, n))
    O.update_k(km, x, 0, n, [3.0, 5.0], [4.0, 6.0])
    As = []
    for o in range(2):
        A, np_ = build(km[o], n, nb, True, 1e-6)
        As.append(A)
        n_valid[o] = n
    nbt = -(-n // nb)
    run(As, nbt, nb, True, 2, workers, rng)
    ref = O.invert_k(n, km)
    for o in range(2):
        got = -np.tril(As[o][np_:np_ + n, np_:np_ + n])
        got = got + np.tril(got, -1).T
        cond = np.linalg.cond(km[o] + 1e-6 * np.eye(n))
        assert np.abs(got - ref[o]).max() <= 1e-15 * cond * np.abs(ref[o]).max(), cond


@pytest.mark.parametrize("n,nb,workers,seed", [(5, 4, 2, 0), (37, 8, 4, 1), (100, 32, 2, 2), (70, 8, 9, 3),
                                               (96, 8, 40, 4)])
def test_persistent_mll_schedule(n, nb, workers, seed):
    rng = np.random.default_rng(seed + 10)
    x = rng.uniform(0, 100, size=(n, 2))
    y = rng.normal(size=(n, 2)) * 10
    pm, pv, ls = y.mean(0) + 1.0, y.var(0), np.array([4.0, 6.0])
    ref = O.compute_mll(x, y, np.zeros((2, n, n)), pm, pv, ls, n)
    km = np.zeros((2, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    As = []
    for o in range(2):
        A, np_ = build(km[o] / pv[o], n, nb, False, 1e-8, y[:, o] - pm[o])
        As.append(A)
        n_valid[o] = n
    nbt = -(-n // nb)
    logdet, zz = run(As, nbt, nb, False, 2, workers, rng)
    tot = 0.0
    for o in range(2):
        fit = zz[o] / np.var(y[:, o] - pm[o])
        tot += -0.5 * fit - 0.5 * 2.0 * logdet[o] - 0.5 * n * np.log(2 * np.pi)
    assert tot == pytest.approx(ref, rel=1e-8)


def test_every_dependency_points_backwards():
    """Each task's flags are set only by tasks earlier in the queue (deadlock freedom for any
    number of resident workgroups: the queue order is a topological order)."""
    for nbt, ident, n_obj in [(1, False, 1), (3, False, 2), (9, False, 3), (2, True, 1), (7, True, 2)]:
        steps, blk = plan(nbt, ident, n_obj)
        setter = {}
        for t in range(blk[-1]):
            task = decode(t, nbt, ident, n_obj, steps, blk)
            for key, want in deps(task, nbt, ident):
                if want > 0:
                    assert (key, want) in setter and setter[(key, want)] < t, (nbt, ident, t, key, want)
            if task[0] == "P":
                setter[(("p", task[2], task[1], task[3]), 1)] = t
            else:
                s = task[1]
                for (o, rb, cb, cpart, first) in task[2]:
                    v = (s - rb + 1) if cpart else (s - s0(nbt, ident, rb) + 1)
                    setter[((("c" if cpart else "v"), o, rb, cb), v)] = t
