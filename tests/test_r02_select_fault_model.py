"""The round-2 GPU fault ("unspecified launch failure" surfacing in
test_select_exclusion_at_the_top[48-grid] with the library of commit 2807c42): a CPU model of the
two kernels that test launched -- select_stream_kernel<0, 8> and bo_topq_merge_kernel as they were
at 2807c42 (`git show 2807c42:bayesopt_smart_amd/csrc/bo_select.hip`, `.../bo_common.h`) -- run on
the test's exact inputs (q = 48, the 2048 x 1024 grid, 128 "hot" + 20 scattered evaluated points,
numpy's default_rng(48) acquisition) and geometry (1024 workgroups of 4 waves: 4096 wave lists;
stride 1024 x 256; U = 8 elements per lane, one step per wave).

Every index the two kernels form is computed and checked against the extent of the buffer it
addresses: the acquisition loads, the per-wave LDS buffer (wbuf[wave][64]) in the compaction
and in wave_rank_insert, the readlane lane indices, the grid-coordinate decode and the LDS hash
set (probe slots, the stored row index into the evaluated points), the partial-list writes into
the workspace ([1024 * 4][q] entries), and the merge kernel's head registers, s_lists / s_buf
(capacity 1024, with the overflow fallbacks) and output slots.  The model also reproduces the
selection the kernels make, which the test compared with numpy.  Result: no
index leaves its buffer on this input -- the fault is not in these kernels' index arithmetic.
Test infrastructure only; no GPU."""

import numpy as np

Q = 48
SIDE0, SIDE1 = 2048, 1024
M = SIDE0 * SIDE1
BLOCKS, WAVES, U = 1024, 4, 8
STRIDE = BLOCKS * 256
CAP = 1024
LISTS = BLOCKS * WAVES


class Bounds:
    def __init__(self):
        self.checked = 0

    def __call__(self, idx, extent, what):
        idx = np.asarray(idx)
        self.checked += idx.size
        assert idx.size == 0 or (idx.min() >= 0 and idx.max() < extent), (what, int(idx.min()), int(idx.max()), extent)


def order_key(v, i):
    """bo_order_key: empty 0 < values (monotone, -0.0 == 0.0) < NaN; as Python ints."""
    v = np.asarray(v, dtype=np.float64) + 0.0
    b = v.view(np.uint64).astype(object)
    out = []
    for bb, vv, ii in zip(np.atleast_1d(b), np.atleast_1d(v), np.atleast_1d(i)):
        if ii < 0:
            out.append(0)
        elif vv != vv:
            out.append((1 << 64) - 1)
        else:
            out.append(((~int(bb)) & ((1 << 64) - 1)) if (int(bb) >> 63) else (int(bb) | (1 << 63)))
    return out


def sort_desc(keys, idxs):
    """Selection order: key descending, then index ascending (empty entries last)."""
    return sorted(zip(keys, idxs), key=lambda t: (-t[0], t[1]))


def test_round2_select_kernels_index_model():
    chk = Bounds()
    rng = np.random.default_rng(Q)
    acq = rng.standard_normal(M)
    stride14 = 1 << 14
    hot = 7 + stride14 * np.arange(M // stride14)
    acq[hot] = 100.0 + np.arange(hot.size)
    top = np.argsort(-acq, kind="stable")[:200]
    scatter = top[hot.size::3][:20]
    excl_lin = np.concatenate([hot, scatter])
    n_excl = excl_lin.size
    excl_set = set(int(v) for v in excl_lin)
    # LDS hash table: slots = bo_hash_slots(n_excl) (power of two >= 2 n, >= 64)
    slots = 64
    while slots < 2 * n_excl:
        slots <<= 1
    lds_bytes = slots * 12
    assert lds_bytes + 4 * 64 * 16 <= 160 * 1024               # dynamic + static wbuf fit the LDS
    chk(np.arange(n_excl), n_excl, "excl rows in the hash build")
    partial_v = np.full(LISTS * Q, -np.inf)
    partial_i = np.full(LISTS * Q, -1, dtype=np.int64)
    lane = np.arange(64)
    for blk in range(BLOCKS):
        for wave in range(WAVES):
            b_first = blk * 256 + wave * 64
            # one step: b0 = b_first (b_first + U * STRIDE >= M)
            assert b_first + U * STRIDE >= M
            j = b_first + np.arange(U)[:, None] * STRIDE + lane[None, :]      # [U][64]
            chk(j, M, "acq[j]")
            val = acq[j]
            gi = j.astype(np.int64)
            # event: every element beats the empty list
            keys = np.array(order_key(val.ravel(), gi.ravel()), dtype=object).reshape(U, 64)
            pend = np.ones((U, 64), dtype=bool)
            lst = []                                               # (key, idx) sorted, <= Q
            tkey, tidx = 0, -1                                     # the list's Q-th (empty)
            while True:
                cnt = int(pend.sum())
                if cnt == 0:
                    break
                bkey, bidx = 0, -1
                if cnt > 64:
                    # each lane's best pending element, sorted over the 64 lanes; the Q-th bounds
                    best = []
                    for ln in range(64):
                        c = [(keys[u, ln], gi[u, ln]) for u in range(U) if pend[u, ln]]
                        best.append(sort_desc(*zip(*c))[0] if c else (0, -1))
                    chk(Q - 1, 64, "readlane lane q-1")
                    bkey, bidx = sort_desc([b[0] for b in best], [b[1] for b in best])[Q - 1]
                take = np.zeros((U, 64), dtype=bool)
                for u in range(U):
                    for ln in range(64):
                        if pend[u, ln]:
                            k, i = keys[u, ln], gi[u, ln]
                            take[u, ln] = not ((bkey, -bidx) > (k, -i) and bidx >= 0)
                off = np.zeros((U, 64), dtype=np.int64)
                total = 0
                for u in range(U):
                    bits = take[u]
                    off[u] = total + np.cumsum(bits) - bits
                    total += int(bits.sum())
                for c0 in range(0, total, 64):
                    sel = take & (off >= c0) & (off < c0 + 64)
                    chk(off[sel] - c0, 64, "wbuf[wave][off - c0]")
                    chunk = sorted(zip(off[sel].tolist(), [keys[t] for t in zip(*np.nonzero(sel))],
                                       gi[sel].tolist()))
                    new = [(k, i) for _, k, i in chunk
                           if (tidx < 0 or (k, -i) > (tkey, -tidx))]
                    kept = []
                    for k, i in new:                               # cand_excluded: grid decode + hash
                        c1, c0_ = i % SIDE1, (i // SIDE1) % SIDE0
                        chk([c1], SIDE1, "grid coord 1")
                        chk([c0_], SIDE0, "grid coord 0")
                        if i not in excl_set:
                            kept.append((k, i))
                    if not kept:
                        continue
                    chk(len(kept) - 1, 64, "rank-insert lanes")
                    merged = sort_desc(*zip(*(lst + kept)))[:Q]
                    chk(len(merged) - 1, Q, "list slot (rank < q)")
                    lst = list(merged)
                    tkey, tidx = lst[Q - 1] if len(lst) >= Q else (0, -1)
                pend = pend & ~take
                for u in range(U):
                    for ln in range(64):
                        if pend[u, ln]:
                            k, i = keys[u, ln], gi[u, ln]
                            pend[u, ln] = tidx < 0 or (k, -i) > (tkey, -tidx)
            dst = (blk * WAVES + wave) * Q + np.arange(len(lst))
            chk(dst, LISTS * Q, "partial[(block * 4 + wave) * q + lane]")
            for t, (k, i) in enumerate(lst):
                partial_v[dst[t]] = acq[i]
                partial_i[dst[t]] = i
    # ---- bo_topq_merge_kernel (one workgroup of 256 threads; 16 heads per thread in registers)
    heads = np.arange(LISTS) * Q
    chk(heads, LISTS * Q, "merge heads L[l * q]")
    assert 16 * 256 >= LISTS
    hv, hi = partial_v[heads], partial_i[heads]
    tbest = []
    for w in range(4):                                             # each wave: 64 thread maxima
        th = []
        for t in range(w * 64, w * 64 + 64):
            ls = [(hv[l], hi[l]) for l in range(t, LISTS, 256) if hi[l] >= 0]
            th.append(max(ls, key=lambda e: (e[0], -e[1])) if ls else (-np.inf, -1))
        th.sort(key=lambda e: (-e[0], e[1]))
        tbest.append(th[Q - 1])
    T = max(tbest, key=lambda e: (e[0], -e[1]))
    nl = int(np.sum([(hi[l] >= 0) and not ((T[0], -T[1]) > (hv[l], -hi[l])) for l in range(LISTS)]))
    if nl <= CAP:
        lists = [l for l in range(LISTS) if hi[l] >= 0 and not ((T[0], -T[1]) > (hv[l], -hi[l]))]
        ent = np.array([l * Q + k for l in lists for k in range(Q)])
        chk(ent, LISTS * Q, "merge entries L[s_lists[k / q] * q + k % q]")
        s = [(partial_v[e], partial_i[e]) for e in ent
             if partial_i[e] >= 0 and not ((T[0], -T[1]) > (partial_v[e], -partial_i[e]))]
        if len(s) <= CAP:
            ranked = sorted(s, key=lambda e: (-e[0], e[1]))[:Q]
        else:
            ranked = None
    if nl > CAP or ranked is None:                                  # the fallback: q arg-best rounds
        chk(np.arange(LISTS * Q), LISTS * Q, "merge fallback L[k]")
        e = [(partial_v[k], partial_i[k]) for k in range(LISTS * Q) if partial_i[k] >= 0]
        ranked = sorted(e, key=lambda t: (-t[0], t[1]))[:Q]
    chk(len(ranked) - 1, Q, "out_v[rank]")
    got = np.array([i for _, i in ranked])
    # the selection the test expected (numpy): evaluated points excluded, descending, index order
    excl = np.zeros(M, dtype=bool)
    excl[excl_lin] = True
    order = np.lexsort((np.arange(M), -np.where(excl, -np.inf, acq)))
    np.testing.assert_array_equal(got, order[:Q])
    assert chk.checked > 2_000_000
