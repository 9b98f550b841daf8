"""Multi-rank candidate sharding on the CPU (gloo, world_size 2): the shard partition covers
every candidate once, and the single all_gather exchange of per-rank top-q lists yields the
same global selection as one rank scoring everything (bayesopt/acquisition.py:116-144)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _local_topq(acq, excl, off, cnt, q):
    idx = np.arange(off, off + cnt)
    a = acq[off:off + cnt]
    keep = ~excl[off:off + cnt]
    idx, a = idx[keep], a[keep]
    nan = np.isnan(a)
    order = np.lexsort((idx, -np.where(nan, 0.0, a), ~nan))[:q]
    v = np.full(q, -np.inf)
    i = np.full(q, -1, dtype=np.int64)
    v[: order.size] = a[order]
    i[: order.size] = idx[order]
    return v, i


def _worker(rank, world, port, q, seed, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bayesopt_smart_amd.distributed import exchange_topq, shard_range
        rng = np.random.default_rng(seed)
        m = 1000
        acq = np.round(rng.normal(size=m), 2)          # many exact ties
        acq[rng.choice(m, 3, replace=False)] = np.nan    # NaN sorts first, as in the reference
        excl = np.zeros(m, dtype=bool)
        excl[rng.choice(m, 50, replace=False)] = True
        off, cnt = shard_range(m, rank, world)
        v, i = _local_topq(acq, excl, off, cnt, q)
        gv, gi = exchange_topq(torch.tensor(v), torch.tensor(i), q)
        out[rank] = (gv.tolist(), gi.tolist())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("q,seed", [(3, 0), (16, 1)])
def test_gloo_two_rank_topq_matches_single_rank(q, seed):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), q, seed, out), nprocs=world, join=True)
    rng = np.random.default_rng(seed)
    m = 1000
    acq = np.round(rng.normal(size=m), 2)
    acq[rng.choice(m, 3, replace=False)] = np.nan
    excl = np.zeros(m, dtype=bool)
    excl[rng.choice(m, 50, replace=False)] = True
    v, i = _local_topq(acq, excl, 0, m, q)
    for r in range(world):
        assert out[r][1] == i.tolist()


def test_shard_range_partitions():
    from bayesopt_smart_amd.distributed import shard_range
    for n in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0
            for (o, c), (o2, _) in zip(spans, spans[1:]):
                assert o + c == o2
            assert sum(c for _, c in spans) == n
