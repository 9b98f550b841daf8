"""CPU model of the LU path's permutation records (bayesopt_smart_amd/csrc/bo_lu.hip: build_perm,
put_perm/apply_perm): a step's 16 row swaps (rows 16 s + j <-> piv[j], in order, as LAPACK's
laswp applies getrf's ipiv) composed by wave 0 into <= 32 (pos <- src) pairs -- lane u holds slot
u: its row and the row whose data ends there; a row not yet in a slot is appended at slot m --
then applied through the row -> slot maps.  The model follows round 4's slot algorithm and the
kernel's data-parallel one (round 5: each lane follows its row's data) and
compares it with the swaps applied one by one.  Test infrastructure only; no GPU."""
import numpy as np
import pytest

LB = 16


def build_perm(s, piv):
    """build_perm: returns the record's (pos, src) pairs (slots whose row moved, in slot order)."""
    rows, srcs = [], []
    for j in range(LB):
        a, b = LB * s + j, int(piv[j])
        if a == b:
            continue
        if a in rows:
            ia = rows.index(a)
        else:
            rows.append(a); srcs.append(a); ia = len(rows) - 1
        if b in rows:
            ib = rows.index(b)
        else:
            rows.append(b); srcs.append(b); ib = len(rows) - 1
        srcs[ia], srcs[ib] = srcs[ib], srcs[ia]
    assert len(rows) <= 32                       # the record holds 32 slots
    return [(r, c) for r, c in zip(rows, srcs) if r != c]


def build_perm_parallel(s, piv):
    """build_perm as the kernel computes it since round 5: lane j < 16 takes row 16 s + j, lane
    16 + j row piv[j]; a row named twice keeps its first lane; each lane follows its row's data
    through the swaps to its final position v; the pairs (pos = v, src = row) of the moved rows,
    compacted in lane order."""
    rows = [LB * s + j for j in range(LB)] + [int(p) for p in piv]
    out = []
    for lane, r0 in enumerate(rows):
        if r0 in rows[:lane]:
            continue
        v = r0
        for j in range(LB):
            a, b = LB * s + j, int(piv[j])
            v = b if v == a else (a if v == b else v)
        if v != r0:
            out.append((v, r0))
    return out


def apply_record(x, rec):
    """apply_perm: rows named as sources are staged (buf[slot]), then written to their pos."""
    y = x.copy()
    buf = {slot: x[src].copy() for slot, (_, src) in enumerate(rec)}
    for slot, (pos, _) in enumerate(rec):
        y[pos] = buf[slot]
    return y


def apply_swaps(x, s, piv):
    y = x.copy()
    for j in range(LB):
        a, b = LB * s + j, int(piv[j])
        y[[a, b]] = y[[b, a]]
    return y


@pytest.mark.parametrize("seed", range(40))
def test_perm_record_equals_sequential_swaps(seed):
    rng = np.random.default_rng(seed)
    n = 64 + 16 * int(rng.integers(0, 8))
    s = int(rng.integers(0, n // LB))
    lo = LB * s
    kind = seed % 4
    if kind == 0:        # getrf pivots: each at or below its column's row
        piv = [int(rng.integers(lo + j, n)) for j in range(LB)]
    elif kind == 1:      # chains: pivots picked among rows already moved in this step
        piv = [int(rng.choice([lo + j, min(n - 1, lo + j + 1), lo + LB + int(rng.integers(0, 3))]))
               for j in range(LB)]
        piv = [min(max(p, lo + j), n - 1) for j, p in enumerate(piv)]
    elif kind == 2:      # no swaps
        piv = [lo + j for j in range(LB)]
    else:                # every pivot from below the block (32 distinct rows touched)
        s = min(s, n // LB - 2)
        lo = LB * s
        piv = [int(v) for v in rng.permutation(np.arange(lo + LB, n))[:LB]]
    x = rng.standard_normal((n, 3))
    for rec in (build_perm(s, piv), build_perm_parallel(s, piv)):
        np.testing.assert_array_equal(apply_record(x, rec), apply_swaps(x, s, piv))
        poss = [p for p, _ in rec]
        assert len(set(poss)) == len(poss) and sorted(poss) == sorted(c for _, c in rec)
    assert sorted(build_perm(s, piv)) == sorted(build_perm_parallel(s, piv))
