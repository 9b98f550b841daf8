"""A seeded sweep over the fused predict + acquisition kernel's instantiation space, every case
against the CPU reference (oracle/cpu_ref.c: update_k_star -> update_mean -> update_variance ->
standardize_objectives -> update_ucb -> update_hypervolume_improvement, numba_kernels.py:406-570,
acquisition.py:33-108) on every candidate of the call, and the top-q judged tie-aware on the CPU
acquisition array with the evaluated points excluded (acquisition.py:116-144).

The host plan (bo_predict.hip make_plan) picks the kernel from the call's shape; the cases are
chosen so that every branch of that choice runs at least once, off the BASELINE configs' own
shapes:
  * candidate kinds: the integer 'ij' grid (separable K*, SEP, when the last axis is a multiple of
    16 and the shard starts on one; otherwise the direct path), the device Sobol set, explicit f64
    and int64 arrays; 1-D, 2-D and 3-D grids, 1..8-D point sets;
  * N: 1, below, at and above the small kernel's 128 rows, residues 1..31 of the 32-row chunk (the
    PART peel, 1..3 live k-step pairs) and multiples of 32, up to the GROWS layout (rows and alpha
    in global memory, N = 1600 on the grid and 2100 on a 6-D set);
  * q = 1..4 (the lane-local top-q lists on the SEP path), 5, 7, 8 and 16 (the wave-shared list);
  * n_obj 1..8 (BO_MAX_OBJ); shards with a non-zero offset and a count that is not a multiple of the 64-
    candidate tile;
  * modes: auto (upper form), dense, auto-exp (no separable generation), and fp32 (the f32 kernel,
    cm32_predict_kernel<DIM, KQV>: every KQV -- last 64-row chunk with 1, 3 or 4 live k-quads).

Tolerances (tests/parity.py): f64 -- mu 1e-5 max(|ref|, sqrt(pv)), var 1e-5 pv,
acq 1e-5 max(1, |ref|); fp32 -- the first-order f32 bound of tests/test_gpu_fp32.py
(f32_model_eps, acq_bound), per candidate.  Training sets are distinct points with cond(K + 1e-6 I)
< 1e6, the bound of tests/test_gpu_predict.py (parity is defined for a well-
conditioned K); a length scale that breaks it is shrunk until it holds.  (At cond 1e7..5e7 two
CPU restatements -- oracle_np's numpy chain and cpu_ref.c's DGEMM order -- already differ by up to
1.7e-3 relative in acq, so a 1e-5 rule is not a parity check there.)"""
import numpy as np
import pytest

from oracle import oracle_np as O
from parity import check_predict, check_topq

# (id, kind, geometry, n, n_obj, q, mode, offset, count)
#   kind "grid": geometry = shape;  "sobol": geometry = dim (points lo 0, scale 300);
#   "f64" / "i64": geometry = (dim, m)  (random distinct points in [0, 300)^dim)
#   count None: a ragged count (the cpu budget, minus 37)
CASES = [
    ("grid-n1", "grid", (64, 128), 1, 1, 1, "auto", 0, None),
    ("grid-n17-q2", "grid", (64, 128), 17, 2, 2, "auto", 0, None),
    ("grid-n31-q3", "grid", (128, 256), 31, 3, 3, "auto", 0, None),
    ("grid-n96-small-q4", "grid", (128, 256), 96, 4, 4, "auto", 0, None),
    ("grid-n127-small-part-q5", "grid", (128, 256), 127, 2, 5, "auto", 0, None),
    ("grid-n129-part-q16", "grid", (128, 256), 129, 1, 16, "auto", 0, None),
    ("grid-n200-shard-q3", "grid", (256, 256), 200, 2, 3, "auto", 16 * 37, 30000),
    ("grid-n333-q4", "grid", (256, 512), 333, 3, 4, "auto", 0, None),
    ("grid-n512-shard-q3", "grid", (256, 512), 512, 2, 3, "auto", 64, 20000),
    ("grid-n545-q1", "grid", (512, 256), 545, 2, 1, "auto", 0, None),
    ("grid-n700-q8", "grid", (512, 256), 700, 4, 8, "auto", 4096, None),
    ("grid3d-n150-q3", "grid", (8, 16, 64), 150, 2, 3, "auto", 0, None),
    ("grid1d-n40-q2", "grid", (4096,), 40, 1, 2, "auto", 0, None),
    ("grid-nonsep-s130-q3", "grid", (100, 130), 150, 2, 3, "auto", 0, None),
    ("grid-nonsep-offset8-q3", "grid", (128, 256), 100, 2, 3, "auto", 8, None),
    ("grid-dense-n300-q3", "grid", (256, 256), 300, 2, 3, "dense", 0, None),
    ("grid-exp-n257-q4", "grid", (256, 256), 257, 3, 4, "auto-exp", 0, None),
    ("grid-n800-rw1-q4", "grid", (256, 256), 800, 4, 4, "auto", 0, None),
    ("grid-sepfallback-n1600-q3", "grid", (512, 256), 1600, 4, 3, "auto", 0, 4096 - 37),
    ("grid8d-grows-n1700-q3", "grid", (4, 4, 4, 4, 4, 4, 4, 16), 1700, 4, 3, "auto", 0, 2048 - 37),
    ("sobol3-n50-q1", "sobol", 3, 50, 1, 1, "auto", 0, None),
    ("sobol5-n65-small-q2", "sobol", 5, 65, 4, 2, "auto", 0, None),
    ("sobol4-n260-q7", "sobol", 4, 260, 2, 7, "auto", 0, None),
    ("sobol8-n777-q3", "sobol", 8, 777, 2, 3, "auto", 0, None),
    ("sobol6-n1024-shard-q16", "sobol", 6, 1024, 3, 16, "auto", 1000, 8192 - 37),
    ("sobol6-n2100-q5", "sobol", 6, 2100, 3, 5, "auto", 0, 3000 - 37),
    ("sobol8-grows-n1700-q5", "sobol", 8, 1700, 4, 5, "auto", 0, 2048 - 37),
    ("sobol6-dense-n450-q3", "sobol", 6, 450, 3, 3, "dense", 0, None),
    ("f64-d1-n33-q2", "f64", (1, 20000), 33, 1, 2, "auto", 0, None),
    ("f64-d2-n90-q3", "f64", (2, 20000), 90, 2, 3, "auto", 0, None),
    ("i64-d7-n410-q4", "i64", (7, 20000), 410, 3, 4, "auto", 0, None),
    ("fp32-sobol6-n100-q16", "sobol", 6, 100, 3, 16, "fp32", 0, None),
    ("fp32-sobol6-n513-kqv1-q3", "sobol", 6, 513, 3, 3, "fp32", 0, None),
    ("fp32-sobol6-n1090-kqv1-q8", "sobol", 6, 1090, 2, 8, "fp32", 0, None),
    ("fp32-sobol4-n700-kqv4-q4", "sobol", 4, 700, 3, 4, "fp32", 0, None),
    ("fp32-sobol8-n1200-kqv3-q2", "sobol", 8, 1200, 1, 2, "fp32", 0, None),
    ("fp32-grid-n150-q3", "grid", (128, 96), 150, 2, 3, "fp32", 0, None),
    # more objectives than the BASELINE configs (BO_MAX_OBJ = 8)
    ("grid-nobj8-n200-q3", "grid", (256, 256), 200, 8, 3, "auto", 0, None),
    ("grid-nobj5-n100-small-q2", "grid", (128, 256), 100, 5, 2, "auto", 0, None),
    ("sobol6-nobj6-n300-q5", "sobol", 6, 300, 6, 5, "auto", 0, None),
    ("fp32-sobol6-nobj5-n600-q4", "sobol", 6, 600, 5, 4, "fp32", 0, None),
]



def plan_path(case):
    """The branches of the host plan (bo_predict.hip make_plan, :487-550, and the launchers'
    template choice in bo_predict_impl.h) that one case takes -- a mirror of the plan's LDS
    arithmetic, used to show that the sweep reaches every branch."""
    cid, kind, geo, n, n_obj, q, mode, offset, count = case
    dim = len(geo) if kind == "grid" else (geo if kind == "sobol" else geo[0])
    dim_pad = 2 if dim <= 2 else 4 if dim <= 4 else 6 if dim <= 6 else 8
    lds_bytes, lds_doubles, waves, exp_tab = 160 * 1024, 160 * 1024 // 8, 4, 256
    if mode == "fp32":
        n_pad = -(-n // 64) * 64
        if (n_pad * dim_pad + n_obj * n_pad) * 4 <= lds_bytes:
            r = n % 64
            kqv = 4 if r == 0 else (r + 15) // 16
            return {"fp32", f"fp32-kqv{1 if kqv == 1 else 3 if kqv <= 3 else 4}"}
    n_pad = -(-n // 32) * 32
    base = n_pad * dim_pad + n_obj * n_pad
    plain = base + exp_tab
    lds, labels = plain, set()
    sep = False
    if kind == "grid" and mode not in ("auto-exp", "dense-exp"):
        s_last = geo[-1]
        tbl = n_obj * (2 * s_last - 1)
        rw_c = n_pad * (n_obj + 1) + (s_last + 63) // 64
        lds_c = base + tbl + waves * rw_c
        lds_1 = base + tbl + waves * n_pad * 2
        if s_last % 16 == 0 and s_last <= 32768 and offset % 16 == 0:
            if lds_1 <= lds_doubles:
                sep = True
                labels.add("sep-rwcache" if lds_c <= lds_doubles else "sep-rw1")
                lds = max(lds_c if lds_c <= lds_doubles else lds_1, plain)
            else:
                labels.add("sep-tables-too-large")
    grows = lds > lds_doubles
    if grows:
        sep, lds = False, exp_tab
        labels.discard("sep-rwcache")
        labels.discard("sep-rw1")
    labels.add("sep" if sep else ("direct-" + ("grid" if kind == "grid" else kind)))
    if grows:
        labels.add("grows")
    if not grows and n_pad <= 128 and lds * 8 <= lds_bytes // 2 - 1024:
        labels.add("small")
    if n % 32:
        labels.add("part")
    labels.add("dense" if mode.startswith("dense") else "upper")
    if q:
        labels.add("lane-topq" if sep and 1 <= q <= 4 else "wave-topq")
    return labels


REQUIRED = {"sep", "sep-rwcache", "sep-rw1", "sep-tables-too-large", "direct-grid", "direct-sobol",
            "direct-f64", "direct-i64", "grows", "small", "part", "upper", "dense", "lane-topq",
            "wave-topq", "fp32", "fp32-kqv1", "fp32-kqv3", "fp32-kqv4"}


def test_sweep_reaches_every_plan_branch():
    """Host logic (no GPU): the cases above reach every branch of the plan, and each branch
    combination a kernel instantiation stands for (SEP x small / PART / lane top-q, direct x
    grows / small / PART, fp32 x KQV)."""
    seen = [plan_path(c) for c in CASES]
    union = set().union(*seen)
    assert REQUIRED <= union, REQUIRED - union
    for combo in ({"sep", "small", "part"}, {"sep", "lane-topq", "part"}, {"sep", "wave-topq"},
                  {"direct-grid", "part"}, {"direct-sobol", "grows", "part"}, {"direct-grid", "grows"},
                  {"direct-sobol", "small", "part"}, {"sep", "dense"}, {"direct-sobol", "dense"}):
        assert any(combo <= s for s in seen), combo


CPU_BUDGET = 4e10          # candidates x N^2 x n_obj scored by the CPU reference per case


def _count(n, n_obj, avail):
    return int(min(avail, max(2048, CPU_BUDGET / (n * n * n_obj)))) - 37


def make_case(case, cand_points):
    """The problem of one case: training set, targets, K^-1 and the scored candidate rows.
    cand_points(idx) -> [k, d] f64 coordinates of global candidate indices (the CandidateSet's own
    points for the device kinds)."""
    cid, kind, geo, n, n_obj, q, mode, offset, count = case
    rng = np.random.default_rng(sum(map(ord, cid)))
    if kind == "grid":
        total = int(np.prod(geo))
    elif kind == "sobol":
        total = 1 << 16
    else:
        total = geo[1]
    if count is None:
        count = _count(n, n_obj, total - offset)
    count = min(count, total - offset)
    # a third of the training set from the scored shard (exercises the exclusion), the rest anywhere
    n_in = min(n // 3, count)
    lin_in = offset + rng.choice(count, n_in, replace=False)
    lin_out = rng.choice(total, min(total, 3 * n + 8), replace=False)
    lin = np.r_[lin_in, lin_out[~np.isin(lin_out, lin_in)]]
    pts = cand_points(lin)
    _, first = np.unique(pts, axis=0, return_index=True)
    x = pts[np.sort(first)][:n]
    assert x.shape[0] == n, (cid, x.shape)
    ext = np.ptp(cand_points(np.arange(0, total, max(1, total // 4096))), axis=0)
    spacing = float(np.mean(np.maximum(ext, 1.0))) / max(1.0, n ** (1.0 / x.shape[1]))
    ls0 = 40.0 if mode == "fp32" and kind == "sobol" else max(1.0, 0.8 * spacing)
    y = rng.normal(size=(n, n_obj)) * 30 + 5
    pm, pv = y.mean(0), (y.var(0) if n > 1 else np.full(n_obj, 900.0))
    betas = rng.uniform(0.5, 2.5, size=n_obj)
    for _ in range(12):
        ls = ls0 * rng.uniform(0.8, 1.2, size=n_obj)
        km = np.zeros((n_obj, n, n))
        O.update_k(km, x.astype(np.float64), 0, n, pv, ls)
        ev = [np.abs(np.linalg.eigvalsh(km[o] / pv[o] + 1e-6 * np.eye(n))) for o in range(n_obj)]
        cond = max(e.max() / e.min() for e in ev)                   # K is symmetric
        if cond < 1e6:
            break
        ls0 *= 0.7
    else:
        raise AssertionError(f"{cid}: no well-conditioned length scale")
    kinv = O.invert_k(n, km)
    return dict(x=x.astype(np.float64), y=y, pm=pm, pv=pv, ls=ls, betas=betas, kinv=kinv,
                offset=offset, count=count, q=q, mode=mode, cond=cond)


@pytest.fixture(scope="module")
def bo():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    bo._lib.load()
    return bo


def _cand_set(bo, kind, geo, rng_seed):
    if kind == "grid":
        return bo.CandidateSet.grid([(0, s) for s in geo])
    if kind == "sobol":
        return bo.CandidateSet.sobol_set(geo, 1 << 16, lo=0.0, scale=300.0)
    rng = np.random.default_rng(rng_seed)
    dim, m = geo
    pts = np.unique(rng.integers(0, 300, size=(m + m // 4, dim)), axis=0) if kind == "i64" else \
        np.unique(rng.uniform(0, 300, size=(m + m // 4, dim)), axis=0)
    pts = pts[rng.permutation(pts.shape[0])[:m]]
    return bo.CandidateSet.explicit(pts)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_kernel_variant_vs_cpu(bo, case):
    import torch
    from oracle import cpu_ref
    cid, kind, geo = case[:3]
    cs = _cand_set(bo, kind, geo, sum(map(ord, cid)))
    p = make_case(case, lambda idx: np.asarray(cs.points(idx), dtype=np.float64))
    off, cnt, q, mode = p["offset"], p["count"], p["q"], p["mode"]
    r = bo.predict_acquire(p["x"], p["y"], p["kinv"], cs, p["pm"], p["pv"], p["ls"], p["betas"],
                           outputs=("mu", "var", "acq"), topq=q, offset=off, count=cnt, mode=mode)
    torch.cuda.synchronize()
    got = {k: r[k].cpu().numpy() for k in ("mu", "var", "acq", "top_idx")}
    pts = np.asarray(cs.points(np.arange(off, off + cnt)), dtype=np.float64)
    ref = cpu_ref.predict_acquire(p["x"], p["y"], pts, p["kinv"], p["pm"], p["pv"], p["ls"], p["betas"])
    xs = {tuple(row) for row in p["x"]}
    excl = np.array([tuple(row) in xs for row in pts])
    assert excl.any() or cid == "grid-n1", f"{cid}: no evaluated point in the shard"
    print(f"{cid}: {sorted(plan_path(case))} N {p['x'].shape[0]} count {cnt} cond {p['cond']:.1e} "
          f"excluded {int(excl.sum())}")
    if mode != "fp32":
        check_predict({k: got[k] for k in ("mu", "var", "acq")}, ref, p["pv"])
        check_topq(got["top_idx"] - off, ref["acq"], excl, q)
        return
    from test_gpu_fp32 import acq_bound, f32_model_eps
    pm, pv = p["pm"], p["pv"]
    eps_mu, eps_var = f32_model_eps(p["x"], p["y"], pts, p["kinv"], pm, pv, p["ls"])
    if kind == "grid":                     # the 2-D grid design's floor (tests/test_gpu_fp32.py EPS_2D)
        eps_mu, eps_var = np.maximum(eps_mu, 1e-4), np.maximum(eps_var, 1e-4)
    dmu = np.abs(got["mu"] - ref["mu"]) / np.sqrt(pv)[:, None]
    dvar = np.abs(got["var"] - ref["var"]) / pv[:, None]
    assert (dmu <= eps_mu).all(), (cid, float(np.max(dmu / eps_mu)))
    assert (dvar <= eps_var).all(), (cid, float(np.max(dvar / eps_var)))
    tol = acq_bound(ref["var"], pv, p["betas"], eps_mu, eps_var)
    da = np.abs(got["acq"] - ref["acq"])
    assert (da <= tol).all(), (cid, int((da > tol).sum()), float(np.max(da / tol)))
    check_topq(got["top_idx"] - off, ref["acq"], excl, q, tol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("count", [0, 1, 15, 17, 63, 65])
@pytest.mark.parametrize("q", [1, 3, 5])
def test_tiny_grid_shards(bo, count, q):
    """Shards smaller than one wave's 16 candidates or one 64-candidate tile, on the separable grid
    path (lane-local top-q for q <= 4): every candidate against the CPU reference, the selection
    in the reference's order over the shard (evaluated points skipped), -1 past the shard's
    selectable candidates."""
    import torch
    from oracle import cpu_ref
    rng = np.random.default_rng(1000 + 10 * count + q)
    side, n = 256, 60
    off = 16 * 300
    lin = rng.choice(side * side - 1, size=n, replace=False)
    lin[lin >= off] += 1                               # distinct from off
    if count:
        lin[0] = off                                   # an evaluated point inside the shard
    x = np.stack([lin // side, lin % side], axis=1).astype(np.float64)
    y = rng.normal(size=(n, 2)) * 20
    pm, pv = y.mean(0), y.var(0)
    ls, betas = np.array([9.0, 11.0]), np.array([1.0, 2.0])
    km = np.zeros((2, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    kinv = O.invert_k(n, km)
    cs = bo.CandidateSet.grid([(0, side), (0, side)])
    r = bo.predict_acquire(x, y, kinv, cs, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=q,
                           offset=off, count=count)
    torch.cuda.synchronize()
    got = {k: r[k].cpu().numpy() for k in ("mu", "var", "acq", "top_idx", "top_val")}
    idx = np.arange(off, off + count)
    if count:
        pts = np.stack([idx // side, idx % side], axis=1).astype(np.float64)
        ref = cpu_ref.predict_acquire(x, y, pts, kinv, pm, pv, ls, betas)
        check_predict({k: got[k] for k in ("mu", "var", "acq")}, ref, pv)
    excl = np.isin(idx, lin)
    a = np.where(excl, -np.inf, got["acq"])
    want = idx[np.lexsort((idx, -a))][: min(q, int((~excl).sum()))]
    np.testing.assert_array_equal(got["top_idx"][: want.size], want)
    assert (got["top_idx"][want.size:] == -1).all()
