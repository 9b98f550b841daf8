"""The multi-rank orchestrator loop (bayesopt_smart_amd/bayesian_optimization.py `optimize`, the
reference loop bayesian_optimization.py:108-247) on CPU ranks (gloo, world 2 and 3): the candidate
shards, the one-all_gather top-q exchange, rank 0's objective evaluations and hyper-parameters
broadcast to every rank, and the gathered state arrays for callbacks -- with the CPU oracle
standing in for the device kernels (OracleBackend: DeviceBackend's interface).  Every rank's
trajectory must equal the single-rank trajectory, and the callbacks' gathered acquisition array
the single-rank one."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SIDE, N_INIT, BATCH, T = 37, 8, 3, 8 + 3 * 3


def objective(x):
    x = np.asarray(x, dtype=np.float64)
    return np.array([-((x[0] - 15) ** 2) + 100.0, -((x[1] - 20) ** 2) + 20.0])


class OracleBackend:
    """DeviceBackend's interface on the CPU oracle: Powell over the oracle MLL (the options of
    kernels.optimize_hyperparams_mll), rank 0's hyper-parameters broadcast, the oracle K^-1, and
    the sharded select (distributed.sharded_predict_acquire with the oracle scorer)."""

    def __init__(self, cands, group=None):
        from bayesopt_smart_amd.bayesian_optimization import _world
        from bayesopt_smart_amd.distributed import shard_range
        self.cands, self.group = cands, group
        self.rank, self.world = _world(group)
        self.offset, self.count = shard_range(cands.n, self.rank, self.world)
        self.bufs = None
        self._acq = None

    def fit(self, x_vector, y_vector, n, prior_mean, prior_variance, length_scales):
        import time
        from scipy.optimize import minimize
        from bayesopt_smart_amd import config as C
        from bayesopt_smart_amd.bayesian_optimization import _broadcast_np
        from oracle import oracle_np as O
        x, y = x_vector[:n].astype(np.float64), y_vector[:n].astype(np.float64)
        n_obj = len(prior_mean)
        km = np.zeros((n_obj, n, n))
        res = minimize(lambda p: -O.compute_mll(x, y, km, prior_mean, p[n_obj:], p[:n_obj], n),
                       np.concatenate([length_scales, prior_variance]), method=C.HYPERPARAM_METHOD,
                       bounds=[(C.HYPERPARAM_MIN_BOUND, None)] * (2 * n_obj),
                       options={"xtol": C.HYPERPARAM_XTOL, "ftol": C.HYPERPARAM_FTOL,
                                "maxiter": C.HYPERPARAM_MAXITER})
        length_scales[:] = res.x[:n_obj]
        prior_variance[:] = res.x[n_obj:]
        _broadcast_np(length_scales, self.group)
        _broadcast_np(prior_variance, self.group)
        O.update_k(km, x, 0, n, prior_variance, length_scales)
        return res, (x, y, O.invert_k(n, km)), time.perf_counter()

    def select(self, fitted, prior_mean, prior_variance, length_scales, betas, batch_size, evaluated,
               acquisition="sum_ucb", y_evaluated=None, reference_point=None):
        from bayesopt_smart_amd.distributed import sharded_predict_acquire
        from test_distributed_gloo import _oracle_scorer
        x, y, kinv = fitted
        r, (_, gi) = sharded_predict_acquire(x, y, kinv, self.cands, prior_mean, prior_variance,
                                             length_scales, betas, batch_size, group=self.group,
                                             scorer=_oracle_scorer)
        self._acq = torch.as_tensor(r["acq"])
        return np.asarray(gi, dtype=np.int64)

    def state_arrays(self):
        acq = self._acq
        if self.world > 1:
            from bayesopt_smart_amd.distributed import gather_shards
            acq = gather_shards(acq, self.cands.n, self.group)
        z = torch.zeros((2, self.cands.n), dtype=torch.float64)
        return {"mu_objectives": z, "variance_objectives": z, "acquisition_values": acq}


def _run(group=None, cb_rank0_only=False):
    from bayesopt_smart_amd.bayesian_optimization import optimize
    from bayesopt_smart_amd.predict import CandidateSet
    rng = np.random.default_rng(5)
    lin = rng.choice(SIDE * SIDE, size=N_INIT, replace=False)
    x = np.zeros((T, 2))
    y = np.zeros((T, 2))
    x[:N_INIT] = np.stack([lin // SIDE, lin % SIDE], axis=1)
    y[:N_INIT] = np.stack([objective(p) for p in x[:N_INIT]])
    pm, pv = y[:N_INIT].mean(0), y[:N_INIT].var(0)
    ls, betas = np.array([5.0, 7.0]), np.array([2.0, 2.0])
    cands = CandidateSet.grid([(0, SIDE), (0, SIDE)])
    seen = []
    calls = []

    def fn(p):
        calls.append(tuple(p))
        return objective(p)

    backend = OracleBackend(cands, group)
    cb = [lambda st: seen.append(st["acquisition_values"].copy())]
    if cb_rank0_only and backend.rank != 0:
        cb = None      # a logging callback on rank 0 only: the gathers must still be collective
    x, y, last = optimize(x, y, None, None, None, None, None, None, None, None, cands, pm, pv,
                          np.zeros(2), N_INIT, T, 2, fn, betas, ls, BATCH, [(0, SIDE), (0, SIDE)],
                          callbacks=cb, backend=backend)
    return x, y, last, ls, seen, len(calls)


def _worker(rank, world, port, out, cb_rank0_only=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x, y, last, ls, seen, n_calls = _run(cb_rank0_only=cb_rank0_only)
        out[rank] = (x.tolist(), y.tolist(), last, ls.tolist(), [a.tolist() for a in seen], n_calls)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,cb_rank0_only", [(2, False), (3, False), (2, True)])
def test_gloo_orchestrator_reproduces_single_rank_trajectory(world, cb_rank0_only):
    x1, y1, last1, ls1, seen1, calls1 = _run()
    assert calls1 == T - N_INIT
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out, cb_rank0_only), nprocs=world, join=True)
    for r in range(world):
        x, y, last, ls, seen, n_calls = out[r]
        np.testing.assert_array_equal(np.array(x), x1)          # the same batches on every rank
        np.testing.assert_array_equal(np.array(y), y1)          # rank 0's evaluations, broadcast
        assert last == last1
        np.testing.assert_array_equal(np.array(ls), ls1)
        assert n_calls == (calls1 if r == 0 else 0)             # the objective runs on rank 0 only
        if cb_rank0_only and r != 0:
            assert seen == []
            continue
        assert len(seen) == len(seen1)
        for a, b in zip(seen, seen1):   # gathered shards == the whole array (the oracle's BLAS
            #                             rounds a shard's products at the ulp level differently)
            np.testing.assert_allclose(np.array(a), b, rtol=1e-12, atol=1e-12 * np.abs(b).max())
