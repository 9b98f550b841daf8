"""GPU parity at the shapes of BASELINE.json configs C2, C4 and C5.

C1 is the CPU plumbing demo (tests/test_gpu_api.py covers its trajectory) and C3 is the bench
workload (tests/test_gpu_predict.py::test_full_size_c3_properties).  Inputs follow SURVEY.md
§8d: seeded designs, the reference's objectives (examples/benchmark_functions.py:33-73), prior
statistics from the samples, unscrambled Sobol candidates scaled to [0, 300)^6 for the 6-D
configs.  Parity is checked on EVERY candidate against oracle/cpu_ref.c (the reference
algorithm on the host cores, tests/fullref.py) with the SURVEY.md §8c tolerances, the top-q
selection is judged against the CPU acquisition array, and the shard merge must equal the
single call."""

import numpy as np
import pytest

from oracle import oracle_np as O
from parity import check_predict, check_topq
from fullref import cpu_full, grid_points_2d

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bo():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import bayesopt_smart_amd as bo
    bo._lib.load()
    return bo


def toy_function(x):
    """examples/benchmark_functions.py:33-50 (2 objectives from x[0], x[1])."""
    return np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20], axis=1)


def toy_function_3d(x):
    """examples/benchmark_functions.py:58-73 (3 objectives from x[0..2]; further dims inert)."""
    return np.stack([-((x[:, 0] - 150) ** 2) + 100, -((x[:, 1] - 150) ** 2) + 20,
                     -((x[:, 2] - 5) ** 2) + 120], axis=1)


def sobol(m, d):
    from scipy.stats import qmc
    return qmc.Sobol(d, scramble=False).random(m) * 300.0


def problem(x, y, ls, beta):
    n_obj = y.shape[1]
    n = x.shape[0]
    pm, pv = y.mean(0), y.var(0)
    km = np.zeros((n_obj, n, n))
    O.update_k(km, x, 0, n, pv, np.full(n_obj, ls))
    kinv = O.invert_k(n, km)
    return dict(x=x, y=y, Kinv=kinv, pm=pm, pv=pv, ls=np.full(n_obj, ls), betas=np.full(n_obj, beta))


def run(bo, d, cands, q, mode="auto", outputs=("mu", "var", "acq"), offset=0, count=None):
    import torch
    r = bo.predict.predict_acquire(d["x"], d["y"], d["Kinv"], cands, d["pm"], d["pv"], d["ls"],
                                   d["betas"], outputs=outputs, topq=q, mode=mode, offset=offset,
                                   count=count)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in r.items() if not k.startswith("_")}


def excluded_rows(cand, x):
    xs = {tuple(r) for r in np.asarray(x, dtype=np.float64)}
    return np.array([tuple(r) in xs for r in np.asarray(cand, dtype=np.float64)])


@pytest.mark.parametrize("mode", ["auto", "dense"])
def test_c2_grid_ucb(bo, mode):
    """C2: 2-D/2-obj, N=128, 512^2 'ij' grid; the per-objective UCB array is compared."""
    rng = np.random.default_rng(0)
    side = 512
    lin = rng.choice(side * side, size=128, replace=False)
    x = np.stack([lin // side, lin % side], axis=1).astype(np.float64)
    d = problem(x, toy_function(x), 20.0, 2.0)
    cands = bo.predict.CandidateSet.grid([(0, side), (0, side)])
    out = run(bo, d, cands, 3, mode, outputs=("mu", "var", "ucb", "acq"))
    ref = cpu_full("C2", x, d["y"], grid_points_2d(side, side), d["Kinv"], d["pm"], d["pv"], d["ls"],
                   d["betas"])
    check_predict({k: out[k] for k in ("mu", "var", "ucb", "acq")}, ref, d["pv"])
    excl = np.zeros(side * side, dtype=bool)
    excl[lin] = True
    check_topq(out["top_idx"], ref["acq"], excl, 3)


@pytest.mark.parametrize("mode", ["auto", "dense"])
@pytest.mark.parametrize("n,m_full,q", [(1024, 1 << 21, 3), (2048, 1 << 18, 16)])
def test_c4_c5_sobol_6d_3obj(bo, n, m_full, q, mode):
    """C4 (N=1024, 2^21 Sobol points, q=3) and C5's problem (N=2048, q=16) in f64 (C5's fp64
    reference check) on explicit f64 candidates.  C5's full 2^22 set is an 8-GPU workload; one
    GPU scores a 2^18 prefix of the sequence here."""
    rng = np.random.default_rng(1)
    cand = sobol(m_full, 6)
    x = cand[rng.choice(m_full, size=n, replace=False)]
    d = problem(x, toy_function_3d(x), 40.0, 2.0)
    cands = bo.predict.CandidateSet.explicit(cand)
    out = run(bo, d, cands, q, mode)
    ref = cpu_full(("C45", n, m_full), x, d["y"], cand, d["Kinv"], d["pm"], d["pv"], d["ls"], d["betas"])
    check_predict({k: out[k] for k in ("mu", "var", "acq")}, ref, d["pv"])
    # every training point is drawn from the candidate set: all of them are excluded
    check_topq(out["top_idx"], ref["acq"], excluded_rows(cand, x), q)
    if mode == "dense":
        return
    # the device Sobol generator (kind sobol: the kernel generates each point from its index)
    # reproduces the explicit scipy set bit for bit, outputs and selection included
    sob = bo.predict.CandidateSet.sobol_set(6, m_full, scale=300.0)
    o = run(bo, d, sob, q, mode)
    for k in ("mu", "var", "acq", "top_idx"):
        np.testing.assert_array_equal(o[k], out[k], err_msg=k)
    # the shard partition (distributed.shard_range over 4 ranks, each generating its own Sobol
    # index range) reproduces the single call
    from bayesopt_smart_amd.distributed import shard_range
    vals, idxs = [], []
    for r in range(4):
        off, cnt = shard_range(m_full, r, 4)
        o = run(bo, d, sob, q, outputs=("acq",), offset=off, count=cnt)
        np.testing.assert_array_equal(o["acq"], out["acq"][off:off + cnt])
        vals.append(o["top_val"])
        idxs.append(o["top_idx"])
    _, gi = bo.predict.merge_topq(np.concatenate(vals), np.concatenate(idxs), q)
    np.testing.assert_array_equal(gi, out["top_idx"])


def test_select_topq_nan_and_ties(bo):
    """select_next_batch's order on a stored acquisition array (acquisition.py:134-142): NaN
    first (np.argsort puts NaN last and the walk is reversed), then descending value, exact ties
    by ascending index; evaluated points skipped."""
    cand = np.stack(np.meshgrid(np.arange(40), np.arange(25), indexing="ij"), -1).reshape(-1, 2)
    acq = np.round(np.random.default_rng(5).normal(size=cand.shape[0]), 1)   # many exact ties
    acq[[17, 400, 901]] = np.nan
    ev = cand[[3, 17, 250]].astype(np.float64)
    got = bo.acquisition.select_next_batch(cand, acq, ev, 12)
    order = np.lexsort((np.arange(acq.size), -np.where(np.isnan(acq), 0.0, acq), ~np.isnan(acq)))
    skip = {3, 17, 250}
    ref = cand[[i for i in order if i not in skip][:12]]
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("kind", ["grid", "sobol"])
def test_graphed_prepared_call_equals_direct(bo, kind):
    """PreparedPredict.graphed() (bench.py's step: preparation, fused kernel and merge replayed
    as one HIP graph) writes exactly what the direct call writes, and a replay after the inputs
    are refilled in place sees the new inputs."""
    import torch
    rng = np.random.default_rng(11)
    if kind == "grid":
        side, n = 256, 128
        lin = rng.choice(side * side, size=n, replace=False)
        x = np.stack([lin // side, lin % side], axis=1).astype(np.float64)
        y = toy_function(x)
        cands = bo.CandidateSet.grid([(0, side), (0, side)])
    else:
        cands = bo.CandidateSet.sobol_set(6, 1 << 16, scale=300.0)
        x = cands.points(rng.choice(1 << 16, size=300, replace=False))
        y = toy_function_3d(x)
    n_obj = y.shape[1]
    pm, pv = y.mean(0), y.var(0)
    ls, betas = np.full(n_obj, 30.0), np.full(n_obj, 2.0)
    km = np.zeros((n_obj, x.shape[0], x.shape[0]))
    O.update_k(km, x, 0, x.shape[0], pv, ls)
    kinv = O.invert_k(x.shape[0], km)
    xd, yd, kd = (torch.tensor(a, device="cuda") for a in (x, y, kinv))
    direct = bo.predict_acquire(xd, yd, kd, cands, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=5)
    ref = {k: direct[k].cpu().numpy() for k in ("mu", "var", "acq", "top_idx")}
    prep = bo.predict_acquire(xd, yd, kd, cands, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=5,
                              prepare=True)
    run = prep.graphed()
    for k in ("mu", "var", "acq"):
        prep.res[k].fill_(0.0)
    res = run()
    torch.cuda.synchronize()
    for k in ("mu", "var", "acq", "top_idx"):
        np.testing.assert_array_equal(res[k].cpu().numpy(), ref[k], err_msg=k)
    # refill y in place: the replay reads the new values (same result as a direct call on them)
    yd.mul_(0.5)
    direct2 = bo.predict_acquire(xd, yd, kd, cands, pm, pv, ls, betas, outputs=("mu", "var", "acq"), topq=5)
    ref2 = {k: direct2[k].cpu().numpy() for k in ("mu", "acq", "top_idx")}
    res = run()
    torch.cuda.synchronize()
    for k in ("mu", "acq", "top_idx"):
        np.testing.assert_array_equal(res[k].cpu().numpy(), ref2[k], err_msg=k)
    assert not np.array_equal(ref2["mu"], ref["mu"])


def test_sharded_predict_acquire_device_path_single_rank(bo):
    """distributed.sharded_predict_acquire on the device (no scorer) with device='cuda' (an
    unindexed device string): one rank scores the whole set and selects what predict_acquire
    selects; its outputs land in the caller's `out` buffers."""
    import torch
    from bayesopt_smart_amd.distributed import sharded_predict_acquire
    rng = np.random.default_rng(21)
    side, n = 128, 64
    lin = rng.choice(side * side, size=n, replace=False)
    x = np.stack([lin // side, lin % side], axis=1).astype(np.float64)
    y = toy_function(x)
    pm, pv = y.mean(0), y.var(0)
    ls, betas = np.full(2, 9.0), np.full(2, 2.0)
    km = np.zeros((2, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    kinv = O.invert_k(n, km)
    cands = bo.CandidateSet.grid([(0, side), (0, side)])
    out = {"acq": torch.empty(side * side, dtype=torch.float64, device="cuda")}
    r, (gv, gi) = sharded_predict_acquire(x, y, kinv, cands, pm, pv, ls, betas, 5, outputs=("acq",),
                                          device="cuda", out=out)
    ref = bo.predict_acquire(x, y, kinv, cands, pm, pv, ls, betas, outputs=("acq",), topq=5)
    np.testing.assert_array_equal(gi, ref["top_idx"].cpu().numpy())
    np.testing.assert_array_equal(out["acq"].cpu().numpy(), ref["acq"].cpu().numpy())
    assert r["acq"].data_ptr() == out["acq"].data_ptr()


def test_replay_after_workspace_growth(bo):
    """The round-2 fault hypothesis: a prepared call or HIP graph that kept
    only the workspace POINTER, replayed after a larger call grew (re-allocated) the per-stream
    workspace and the old storage was handed out again, would write into freed memory.  Since
    round 3 the prepared call owns its workspace tensor.  Here: a graph and a prepared call are
    captured on a small problem; a call with q = 48 on a larger problem (the failing round-2
    test's q) grows the workspace; the freed storage is then refilled with garbage by fresh
    allocations; both replays must still reproduce the direct call bit for bit, and the
    workspace cache must now hold a different (larger) buffer."""
    import torch
    from bayesopt_smart_amd.device import Workspace
    rng = np.random.default_rng(5)
    side, n = 128, 64
    lin = rng.choice(side * side, size=n, replace=False)
    x = np.stack([lin // side, lin % side], axis=1).astype(np.float64)
    y = toy_function(x)
    pm, pv = y.mean(0), y.var(0)
    ls, betas = np.array([9.0, 13.0]), np.array([2.0, 2.0])
    km = np.zeros((2, n, n))
    O.update_k(km, x, 0, n, pv, ls)
    kinv = O.invert_k(n, km)
    xd, yd, kd = (torch.tensor(a, device="cuda") for a in (x, y, kinv))
    cands = bo.CandidateSet.grid([(0, side), (0, side)])
    args = (xd, yd, kd, cands, pm, pv, ls, betas)
    torch.cuda.synchronize()
    Workspace._cache.clear()          # start from a small workspace (earlier tests grew the shared one)
    ref = bo.predict_acquire(*args, outputs=("mu", "var", "acq"), topq=3)
    ref = {k: ref[k].cpu().numpy() for k in ("mu", "var", "acq", "top_idx")}
    prep = bo.predict_acquire(*args, outputs=("mu", "var", "acq"), topq=3, prepare=True)
    graph = bo.predict_acquire(*args, outputs=("mu", "var", "acq"), topq=3, prepare=True).graphed()
    torch.cuda.synchronize()
    ws_before = {k: v.data_ptr() for k, v in Workspace._cache.items()}
    # a much larger call on the same stream: N = 1024, the 1024^2 grid, q = 48
    side2, n2 = 1024, 1024
    lin2 = rng.choice(side2 * side2, size=n2, replace=False)
    x2 = np.stack([lin2 // side2, lin2 % side2], axis=1).astype(np.float64)
    y2 = toy_function(x2)
    pm2, pv2 = y2.mean(0), y2.var(0)
    km2 = np.zeros((2, n2, n2))
    O.update_k(km2, x2, 0, n2, pv2, ls * 4)
    kinv2 = O.invert_k(n2, km2)
    big = bo.predict_acquire(x2, y2, kinv2, bo.CandidateSet.grid([(0, side2), (0, side2)]), pm2, pv2, ls * 4,
                             betas, outputs=("acq",), topq=48)
    torch.cuda.synchronize()
    assert big["top_idx"].cpu().numpy().min() >= 0
    grown = [k for k, v in Workspace._cache.items() if k in ws_before and v.data_ptr() != ws_before[k]]
    assert grown, "the large call did not grow the workspace (the test would prove nothing)"
    # hand the freed storage out again and scribble over it
    junk = [torch.full((1 << 20,), float("nan"), dtype=torch.float64, device="cuda") for _ in range(64)]
    torch.cuda.synchronize()
    for run in (prep, graph):
        res = run()
        torch.cuda.synchronize()
        for k in ("mu", "var", "acq", "top_idx"):
            np.testing.assert_array_equal(res[k].cpu().numpy(), ref[k], err_msg=k)
    del junk
