"""Candidate-shard parallelism over torch.distributed (RCCL on MI355X, gloo on CPU).

The candidate set partitions naturally: rank r scores the contiguous index range
``shard_range(M, r, P)`` with no data-path collective; the only exchange is the global
top-q (select_next_batch, bayesopt/acquisition.py:116-144): every rank contributes its
local top-q (value, global index) pairs to ONE all_gather and merges them in the
reference's selection order.  Payload P * q * 16 bytes -- latency-bound over xGMI.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .predict import merge_topq, predict_acquire


def shard_range(n, rank, world):
    """[offset, offset + count) of `n` candidates owned by `rank` (balanced, contiguous)."""
    base, rem = divmod(int(n), int(world))
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def exchange_topq(top_val, top_idx, q, group=None):
    """All-gather every rank's local top-q and merge (NaN first, descending, index ties).

    top_val/top_idx: tensors [q] on the collective's device (HIP for RCCL, CPU for gloo).
    Returns numpy (values, global indices) of length <= q, identical on every rank.
    """
    world = dist.get_world_size(group)
    gv = torch.empty(world * q, dtype=top_val.dtype, device=top_val.device)
    gi = torch.empty(world * q, dtype=top_idx.dtype, device=top_idx.device)
    dist.all_gather_into_tensor(gv, top_val.contiguous(), group=group)
    dist.all_gather_into_tensor(gi, top_idx.contiguous(), group=group)
    return merge_topq(gv.cpu().numpy(), gi.cpu().numpy(), q)


def sharded_predict_acquire(x_train, y_train, kinv, cands, prior_mean, prior_variance, length_scales,
                            betas, q, outputs=("acq",), group=None, device=None):
    """Score this rank's shard of `cands` and return (local results, global top-q)."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    off, cnt = shard_range(cands.n, rank, world)
    r = predict_acquire(x_train, y_train, kinv, cands, prior_mean, prior_variance, length_scales,
                        betas, outputs=outputs, topq=q, offset=off, count=cnt, device=device)
    if world == 1:
        sel = merge_topq(r["top_val"].cpu().numpy(), r["top_idx"].cpu().numpy(), q)
    else:
        sel = exchange_topq(r["top_val"], r["top_idx"], q, group)
    return r, sel
