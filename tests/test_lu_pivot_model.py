"""A model of bo_lu.hip's pivot choice (panel_columns / col_search): getf2's pivot is the FIRST row
of largest |a| in the column, rows >= j (idamax; NaN never wins).  The device finds it in two
levels -- per wave, the maximum 64-bit key (bits(|a|) + 1; 0 for rows outside the column or NaN) as
two u32 maxima (high words, then the low words of the lanes holding the maximum high word), the
first register and then the first lane holding it by ballots; across waves, the maximum key, then
the lowest row among the waves holding it.  This checks the model against the definition on
columns full of exact ties, NaNs and signed zeros, for both row layouts the panels use:
the 8-wave layout (row = base + 64 w + lane + 512 r) and the 4-wave one (row = top + 64 RPL w +
64 r + lane)."""

import zlib

import numpy as np
import pytest


def piv_key(a, valid):
    f = np.abs(a)
    ok = valid & ~np.isnan(f)
    bits = f.view(np.uint64) + np.uint64(1)
    return np.where(ok, bits, np.uint64(0))


def u64_max_two_level(keys):
    hi = (keys >> np.uint64(32)).astype(np.uint32)
    h = hi.max()
    lo = np.where(hi == h, (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32), np.uint32(0))
    return (np.uint64(h) << np.uint64(32)) | np.uint64(lo.max())


def device_pivot(a, g0, n_p, nw, rpl, row_of):
    """a: the column's values by absolute row; row_of(w, r, lane) -> absolute row."""
    cands = []
    for w in range(nw):
        key = np.zeros((rpl, 64), dtype=np.uint64)
        rr = np.zeros((rpl, 64), dtype=np.int64)
        for r in range(rpl):
            for lane in range(64):
                row = row_of(w, r, lane)
                rr[r, lane] = row
                inside = 0 <= row < len(a)
                key[r, lane] = piv_key(np.array([a[row] if inside else 0.0]),
                                       np.array([inside and g0 <= row < n_p]))[0]
        mk = key.max(axis=0)                                  # per lane (its first largest)
        gk = u64_max_two_level(mk)
        wr = next(r for r in range(rpl) if (key[r] == gk).any())
        wl = int(np.flatnonzero(key[wr] == gk)[0])
        cands.append((gk, int(rr[wr, wl]) if gk != 0 else 0x7FFFFFFF))
    ks = np.array([c[0] for c in cands], dtype=np.uint64)
    G = u64_max_two_level(ks)
    p = min(c[1] for c in cands if c[0] == G)
    return None if G <= 1 else p                             # all zero / no candidate: singular


def reference_pivot(a, g0, n_p):
    col = a[g0:n_p]
    f = np.abs(col)
    ok = ~np.isnan(f)
    if not ok.any() or f[ok].max() == 0.0:
        return None
    m = f[ok].max()
    return g0 + int(np.flatnonzero(ok & (f == m))[0])


@pytest.mark.parametrize("layout", ["wide1", "wide2", "small1", "small2"])
@pytest.mark.parametrize("kind", ["ties", "random", "nan_zero"])
def test_pivot_model_matches_getf2(layout, kind):
    rng = np.random.default_rng(zlib.crc32(f"{layout}/{kind}".encode()))
    for trial in range(20):
        if layout.startswith("wide"):
            nw, rpl = 8, int(layout[-1])
            n_p = int(rng.integers(40, 512 * rpl + 1))
            base = int(rng.integers(0, 3)) * 16
            row_of = lambda w, r, lane, base=base: base + 64 * w + lane + 512 * r  # noqa: E731
            top = base + 16 if base > 0 else 0
            n_p = min(max(n_p, top + 1), base + 512 * rpl)     # the rows the layout holds
        else:
            nw, rpl = 4, int(layout[-1])
            top = int(rng.integers(0, 4)) * 16
            n_p = top + int(rng.integers(1, 256 * rpl + 1))
            row_of = lambda w, r, lane, top=top, rpl=rpl: top + 64 * rpl * w + 64 * r + lane  # noqa: E731
        j = int(rng.integers(0, 16))
        g0 = top + j
        if g0 >= n_p:
            continue
        size = max(n_p, 2048 + 64)
        if kind == "ties":
            a = rng.choice([-3.0, 3.0, 1.5, -1.5, 0.5], size=size)
        elif kind == "random":
            a = rng.standard_normal(size) * 10.0 ** rng.integers(-3, 3, size=size)
        else:
            a = rng.choice([0.0, -0.0, np.nan, 2.0, -2.0], size=size, p=[0.3, 0.3, 0.2, 0.1, 0.1])
            if trial % 5 == 0:
                a[:] = rng.choice([0.0, -0.0, np.nan], size=size)
        got = device_pivot(a, g0, n_p, nw, rpl, row_of)
        assert got == reference_pivot(a, g0, n_p), (layout, kind, trial, g0, n_p)
