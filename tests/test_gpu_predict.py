"""GPU parity of the fused predict + acquisition kernel (bo_predict_acquire) against the
reference's own outputs (tests/golden/*.npz) and the CPU oracle (oracle/oracle_np.py)."""

import numpy as np
import pytest

from oracle import oracle_np as O
from parity import check_predict, check_topq
from conftest import predict_fixture
from fullref import cpu_full, grid_points_2d

pytestmark = pytest.mark.gpu

ALL = ("mu", "var", "std_mu", "std_var", "ucb", "acq")


@pytest.fixture(scope="module")
def bo():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    bo._lib.load()
    return bo


def _run(bo, d, cands, q=16, outputs=ALL, excl=None, mode="auto"):
    import torch
    res = bo.predict.predict_acquire(d["x"], d["y"], d["Kinv"], cands, d["pm"], d["pv"], d["ls"],
                                     d["betas"], outputs=outputs, topq=q, excl_points=excl, mode=mode)
    torch.cuda.synchronize()
    out = {k: v.cpu().numpy() for k, v in res.items() if not k.startswith("_")}
    return out


def _excluded(cand_pts, x):
    xs = {tuple(r) for r in np.asarray(x, dtype=np.float64)}
    return np.array([tuple(np.asarray(c, dtype=np.float64)) in xs for c in cand_pts])


def test_mfma_f64_layout(bo):
    import torch
    rng = np.random.default_rng(1)
    a = rng.integers(-8, 8, size=(16, 4)).astype(np.float64)
    b = rng.integers(-8, 8, size=(4, 16)).astype(np.float64)   # asymmetric
    ta, tb = torch.tensor(a, device="cuda"), torch.tensor(b, device="cuda")
    td = torch.empty((16, 16), dtype=torch.float64, device="cuda")
    bo._lib.check(bo._lib.load().bo_selftest_mfma_f64(ta.data_ptr(), tb.data_ptr(), td.data_ptr(), None), "selftest")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(td.cpu().numpy(), a @ b)


@pytest.mark.parametrize("mode", ["auto", "dense"])
@pytest.mark.parametrize("name", ["g1_predict_2d", "g2_predict_512", "g3_predict_6d3o"])
def test_predict_vs_reference_golden(bo, name, mode):
    d = predict_fixture(name)
    cands = bo.predict.CandidateSet.explicit(d["cand"])
    out = _run(bo, d, cands, mode=mode)
    check_predict(out, d, d["pv"])
    excl = _excluded(d["cand"], d["x"])
    check_topq(out["top_idx"], d["acq"], excl, 16)
    # the reference's own batch (acquisition.py:116-144) for q = 3 and q = 16
    for q in (3, 16):
        ref_sel = d[f"select_q{q}"]
        got = cands.points(out["top_idx"][:q])
        gaps = np.sort(d["acq"][~excl])[::-1]
        if np.all(np.abs(np.diff(gaps[: q + 1])) > 1e-4 * np.maximum(1.0, np.abs(gaps[:q]))):
            np.testing.assert_array_equal(got.astype(np.float64), ref_sel.astype(np.float64))


@pytest.mark.parametrize("mode", ["auto", "dense", "auto-exp", "dense-exp"])
def test_predict_implicit_grid(bo, mode):
    d = predict_fixture("g1_grid")
    cands = bo.predict.CandidateSet.grid([(0, int(d["grid_shape"][0])), (0, int(d["grid_shape"][1]))])
    out = _run(bo, d, cands, mode=mode)
    check_predict(out, d, d["pv"])
    check_topq(out["top_idx"], d["acq"], _excluded(d["cand"], d["x"]), 16)
    np.testing.assert_array_equal(cands.points(out["top_idx"][:3]), d["select_q3"])


@pytest.mark.parametrize("mode", ["auto", "dense"])
@pytest.mark.parametrize("n,dim,n_obj", [(7, 2, 2), (33, 3, 1), (130, 5, 4), (300, 2, 3), (600, 2, 2),
                                         (1100, 6, 3)])
def test_predict_shapes_vs_oracle(bo, n, dim, n_obj, mode):
    rng = np.random.default_rng(n)
    m = 3000
    side = 400 if dim == 2 else 60
    cand = np.unique(rng.integers(0, side, size=(m, dim)), axis=0).astype(np.int64)
    m = cand.shape[0]
    # distinct training points (parity is defined for well-conditioned K)
    x = np.unique(rng.integers(0, side, size=(3 * n, dim)), axis=0)
    x = x[rng.permutation(x.shape[0])[:n]].astype(np.float64)
    x[: n // 3] = cand[rng.choice(m, n // 3, replace=False)]          # some evaluated candidates
    x = np.unique(x, axis=0)
    n = x.shape[0]
    y = rng.normal(size=(n, n_obj)) * 50 + 10
    pm, pv = y.mean(0), y.var(0)
    ls = rng.uniform(3.0, 9.0, size=n_obj)
    betas = rng.uniform(0.5, 2.5, size=n_obj)
    km = np.zeros((n_obj, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    assert max(np.linalg.cond(km[o] + 1e-6 * np.eye(n)) for o in range(n_obj)) < 1e6
    kinv = O.invert_k(n, km)
    ref = O.predict_acquire(x, y, cand, pm, pv, ls, betas, kinv=kinv)
    d = dict(x=x, y=y, Kinv=kinv, pm=pm, pv=pv, ls=ls, betas=betas)
    out = _run(bo, d, bo.predict.CandidateSet.explicit(cand), q=8, mode=mode)
    check_predict(out, ref, pv)
    check_topq(out["top_idx"], ref["acq"], _excluded(cand, x), 8)


def test_sharded_calls_match_single_call(bo):
    """Candidate shards (the multi-GPU partition) reproduce the single-call result."""
    d = predict_fixture("g1_predict_2d")
    cands = bo.predict.CandidateSet.explicit(d["cand"])
    full = _run(bo, d, cands, q=16)
    vals, idxs, accs = [], [], []
    import torch
    m = cands.n
    for lo in range(0, m, 1000):
        cnt = min(1000, m - lo)
        r = bo.predict.predict_acquire(d["x"], d["y"], d["Kinv"], cands, d["pm"], d["pv"], d["ls"], d["betas"],
                                       outputs=("acq",), topq=16, offset=lo, count=cnt)
        torch.cuda.synchronize()
        vals.append(r["top_val"].cpu().numpy())
        idxs.append(r["top_idx"].cpu().numpy())
        accs.append(r["acq"].cpu().numpy())
    np.testing.assert_array_equal(np.concatenate(accs), full["acq"])
    v, i = bo.predict.merge_topq(np.concatenate(vals), np.concatenate(idxs), 16)
    np.testing.assert_array_equal(i, full["top_idx"])


def test_edge_cases(bo):
    import torch
    d = predict_fixture("g1_predict_2d")
    # empty candidate set
    cands = bo.predict.CandidateSet.explicit(d["cand"][:0].reshape(0, 2))
    r = bo.predict.predict_acquire(d["x"], d["y"], d["Kinv"], cands, d["pm"], d["pv"], d["ls"], d["betas"], topq=3)
    torch.cuda.synchronize()
    assert (r["top_idx"].cpu().numpy() == -1).all()
    # every candidate evaluated -> nothing selectable
    sub = d["cand"][:50]
    cands = bo.predict.CandidateSet.explicit(sub)
    r = bo.predict.predict_acquire(d["x"], d["y"], d["Kinv"], cands, d["pm"], d["pv"], d["ls"], d["betas"],
                                   topq=3, excl_points=sub.astype(np.float64))
    torch.cuda.synchronize()
    assert (r["top_idx"].cpu().numpy() == -1).all()
    # fewer selectable than q: only the non-excluded ones, in order
    r = bo.predict.predict_acquire(d["x"], d["y"], d["Kinv"], cands, d["pm"], d["pv"], d["ls"], d["betas"],
                                   topq=5, excl_points=sub[2:].astype(np.float64))
    torch.cuda.synchronize()
    got = r["top_idx"].cpu().numpy()
    assert sorted(got[:2].tolist()) == [0, 1] and (got[2:] == -1).all()


@pytest.mark.parametrize("m,q", [(300, 48), (None, 48), (None, 3), (70, 20)])
def test_topq_merge_exact_order(bo, m, q):
    """The final merge of the per-wave lists (bo_topq_merge_kernel): both its paths -- the
    threshold set sorted by rank, and the arg-best rounds when that set exceeds 64 entries (here:
    every wave holds fewer than q candidates) -- give exactly the selection order of the
    acquisition array the same call wrote (NaN first, descending, ties by index)."""
    import torch
    d = predict_fixture("g1_predict_2d")
    cand = d["cand"][:m]
    m = len(cand)
    cands = bo.predict.CandidateSet.explicit(cand)
    r = bo.predict.predict_acquire(d["x"], d["y"], d["Kinv"], cands, d["pm"], d["pv"], d["ls"], d["betas"],
                                   outputs=("acq",), topq=q)
    torch.cuda.synchronize()
    acq = r["acq"].cpu().numpy()
    excl = _excluded(cand, d["x"])
    a = np.where(excl, -np.inf, acq)
    order = np.lexsort((np.arange(m), -a))
    want = order[: min(q, int((~excl).sum()))]
    got = r["top_idx"].cpu().numpy()
    np.testing.assert_array_equal(got[: want.size], want)
    assert (got[want.size:] == -1).all()
    np.testing.assert_array_equal(r["top_val"].cpu().numpy()[: want.size], acq[want])


def test_full_size_c3_properties(bo):
    """C3 at full size (N=512, M=1024^2 implicit grid): every candidate against the CPU
    reference (oracle/cpu_ref.c), top-q judged on the CPU acquisition array, deterministic
    across runs and output sets, every mode within tolerance of the reference."""
    import torch
    rng = np.random.default_rng(0)
    side = 1024
    lin = rng.choice(side * side, size=512, replace=False)
    x = np.stack([lin // side, lin % side], axis=1).astype(np.float64)
    y = np.stack([-(x[:, 0] - 150) ** 2 + 100, -(x[:, 1] - 150) ** 2 + 20], axis=1)
    pm, pv = y.mean(0), y.var(0)
    ls, betas = np.array([20.0, 20.0]), np.array([2.0, 2.0])
    km = np.zeros((2, 512, 512))
    O.update_k(km, x, 0, 512, pv, ls)
    kinv = O.invert_k(512, km)
    d = dict(x=x, y=y, Kinv=kinv, pm=pm, pv=pv, ls=ls, betas=betas)
    cands = bo.predict.CandidateSet.grid([(0, side), (0, side)])
    out = _run(bo, d, cands, q=16, outputs=("mu", "var", "acq"))
    out2 = _run(bo, d, cands, q=16, outputs=("acq",))
    np.testing.assert_array_equal(out["acq"], out2["acq"])
    np.testing.assert_array_equal(out["top_idx"], out2["top_idx"])
    excl = np.zeros(side * side, dtype=bool)
    excl[lin] = True
    ref = cpu_full("C3", x, y, grid_points_2d(side, side), kinv, pm, pv, ls, betas)
    check_predict({k: out[k] for k in ("mu", "var", "acq")}, ref, pv)
    check_topq(out["top_idx"], ref["acq"], excl, 16)
    for mode in ("dense", "auto-exp", "dense-exp"):
        other = _run(bo, d, cands, q=16, outputs=("mu", "var", "acq"), mode=mode)
        check_predict({k: other[k] for k in ("mu", "var", "acq")}, ref, pv)
        check_topq(other["top_idx"], ref["acq"], excl, 16)


@pytest.mark.parametrize("shape,n,n_obj,offset", [
    ((4, 8, 64), 150, 2, 0),        # 3-D grid: rows keyed by the first two coordinates
    ((16, 1024), 480, 4, 0),        # 4 objectives: row factors rebuilt per objective (LDS)
    ((16, 1024), 300, 3, 3 * 1024 + 48),   # shard starting mid-row (offset % 16 == 0)
])
def test_predict_grid_row_factor_paths(bo, shape, n, n_obj, offset):
    """The integer-grid K* path (row factors per grid row, exp table over the last axis) in
    its cached and per-objective forms, on a 3-D grid and on a shard that starts mid-row,
    against the oracle on a candidate subsample."""
    import torch
    rng = np.random.default_rng(n)
    total = int(np.prod(shape))
    lin = rng.choice(total, size=n, replace=False)
    x = np.stack(np.unravel_index(lin, shape), axis=1).astype(np.float64)
    y = rng.normal(size=(n, n_obj)) * 30 + 5
    pm, pv = y.mean(0), y.var(0)
    ls = rng.uniform(1.5, 2.5, size=n_obj)
    betas = rng.uniform(0.5, 2.5, size=n_obj)
    km = np.zeros((n_obj, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    assert max(np.linalg.cond(km[o] + 1e-6 * np.eye(n)) for o in range(n_obj)) < 1e6
    kinv = O.invert_k(n, km)
    cands = bo.predict.CandidateSet.grid([(0, s) for s in shape])
    count = min(total - offset, 8192)
    res = bo.predict.predict_acquire(x, y, kinv, cands, pm, pv, ls, betas, outputs=("mu", "var", "acq"),
                                     topq=8, offset=offset, count=count)
    torch.cuda.synchronize()
    out = {k: res[k].cpu().numpy() for k in ("mu", "var", "acq", "top_idx")}
    sub = np.unique(np.r_[np.arange(0, min(count, 300)), rng.choice(count, 700, replace=False)])
    pts = np.stack(np.unravel_index(offset + sub, shape), axis=1).astype(np.int64)
    ref = O.predict_acquire(x, y, pts, pm, pv, ls, betas, kinv=kinv)
    check_predict({"mu": out["mu"][:, sub], "var": out["var"][:, sub], "acq": out["acq"][sub]},
                  {k: ref[k] for k in ("mu", "var", "acq")}, pv)
    # top-q over the shard against the shard's full acq array (checked above on the subsample)
    shard_pts = np.stack(np.unravel_index(offset + np.arange(count), shape), axis=1)
    excl = _excluded(shard_pts, x)
    check_topq(out["top_idx"] - offset, out["acq"], excl, 8)


@pytest.mark.parametrize("q", [1, 2, 3, 4, 5])
def test_grid_topq_exclusion_at_the_top(bo, q):
    """The fused kernel's top-q on the separable integer-grid path, where q <= 4 uses the lanes'
    own lists (cm_tiles LANEQ) and q = 5 the wave-shared list: with beta = 0 the acquisition is
    the standardised mean, which here peaks at the best training points, so the evaluated points
    (acquisition.py:137-139, excluded through the grid row's bitmap) lead the order.  The selection must be exactly the order of the call's own acquisition
    array over the non-evaluated candidates (descending, ties by index)."""
    import torch
    rng = np.random.default_rng(21 + q)
    side, n = 256, 40
    lin = rng.choice(side * side, size=n, replace=False)
    x = np.stack([lin // side, lin % side], axis=1).astype(np.float64)
    # a few high training points and short length scales: the mean peaks AT them
    y = np.zeros((n, 2))
    y[:6, 0] = [1000, 900, 800, 700, 600, 500]
    y[:6, 1] = [50, 40, 30, 20, 10, 5]
    y[6:] = rng.normal(size=(n - 6, 2))
    pm, pv = y.mean(0), y.var(0)
    ls, betas = np.array([3.0, 3.0]), np.zeros(2)
    km = np.zeros((2, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    kinv = O.invert_k(n, km)
    cands = bo.CandidateSet.grid([(0, side), (0, side)])
    r = bo.predict_acquire(x, y, kinv, cands, pm, pv, ls, betas, outputs=("acq",), topq=q)
    torch.cuda.synchronize()
    acq = r["acq"].cpu().numpy()
    excl = np.zeros(side * side, dtype=bool)
    excl[lin] = True
    order_all = np.lexsort((np.arange(side * side), -acq))
    assert excl[order_all[:q]].any(), "no evaluated point at the top: the case is not exercised"
    a = np.where(excl, -np.inf, acq)
    want = np.lexsort((np.arange(side * side), -a))[:q]
    np.testing.assert_array_equal(r["top_idx"].cpu().numpy(), want)
    np.testing.assert_array_equal(r["top_val"].cpu().numpy(), acq[want])


@pytest.mark.parametrize("n", [518, 530, 541])
def test_grid_part_lane_topq_vs_cpu(bo, n):
    """The drop-in loop's own kernel shape on the integer grid: N off a multiple of 32 (the PART
    instantiation, 1 / 3 / 3 live k-step pairs in the peeled chunk: N = 518 / 530 / 541) with
    q = 3 (the lane-local top-q lists), every candidate of a 512 x 1024 'ij' grid against the CPU
    reference (oracle/cpu_ref.c, SURVEY.md §8c tolerances) and the top-3 judged on the CPU
    acquisition array."""
    import torch
    rng = np.random.default_rng(n)
    rows, side = 512, 1024
    lin = rng.choice(rows * side, size=n, replace=False)
    x = np.stack([lin // side, lin % side], axis=1).astype(np.float64)
    y = np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20], axis=1)
    pm, pv = y.mean(0), y.var(0)
    ls, betas = np.array([20.0, 20.0]), np.array([2.0, 2.0])
    km = np.zeros((2, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    kinv = O.invert_k(n, km)
    cands = bo.CandidateSet.grid([(0, rows), (0, side)])
    r = bo.predict_acquire(x, y, kinv, cands, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=3)
    torch.cuda.synchronize()
    got = {k: r[k].cpu().numpy() for k in ("mu", "var", "acq", "top_idx")}
    ref = cpu_full(("grid_part", n), x, y, grid_points_2d(rows, side), kinv, pm, pv, ls, betas)
    check_predict({k: got[k] for k in ("mu", "var", "acq")}, ref, pv)
    excl = np.zeros(rows * side, dtype=bool)
    excl[lin] = True
    check_topq(got["top_idx"], ref["acq"], excl, 3)
