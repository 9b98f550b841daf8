"""Candidate-shard parallelism over torch.distributed (RCCL on MI355X, gloo on CPU).

The candidate set partitions naturally: rank r scores the contiguous index range
``shard_range(M, r, P)`` with no data-path collective; the only exchange is the global
top-q (select_next_batch, bayesopt/acquisition.py:116-144): every rank contributes its
local top-q (value, global index) pairs to ONE all_gather and merges them in the
reference's selection order.  Payload P * q * 16 bytes -- latency-bound over xGMI.
"""

from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist

from .predict import merge_topq, predict_acquire


def collectives_on(group=None):
    """True when the exchange steps run as collectives: torch.distributed is initialised and the
    group has several ranks -- or BO_FORCE_COLLECTIVES=1, which runs every collective of the loop
    and the bench on a single rank too (tests/test_gpu_rccl_one_rank.py executes the RCCL path on
    one GPU that way)."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return dist.get_world_size(group) > 1 or os.environ.get("BO_FORCE_COLLECTIVES") == "1"


def shard_range(n, rank, world):
    """[offset, offset + count) of `n` candidates owned by `rank` (balanced, contiguous)."""
    base, rem = divmod(int(n), int(world))
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def exchange_topq_rec(rec, q, group=None, out=None):
    """ONE all_gather of every rank's top-q record block and the merge.

    rec: f64 tensor [2q] on the collective's device (HIP for RCCL, CPU for gloo): values in
    [:q], int64 global indices bit-cast into [q:] (predict_acquire(top_rec=...) writes it in
    place).  P * q * 16 bytes in total.  Returns numpy (values, global indices), length <= q,
    identical on every rank: NaN first, then descending value, ties by ascending index.
    """
    world = dist.get_world_size(group)
    if dist.get_backend(group) != "nccl" and rec.device.type != "cpu":
        rec = rec.cpu()                         # gloo ranks (CPU collectives) on one device
        out = None
    g = out if out is not None else torch.empty(world * 2 * q, dtype=rec.dtype, device=rec.device)
    dist.all_gather_into_tensor(g, rec.contiguous(), group=group)
    gh = g.cpu().numpy().reshape(world, 2 * q)      # one device-to-host copy of the whole block
    return merge_topq(gh[:, :q], gh[:, q:].view(np.int64), q)


def exchange_topq(top_val, top_idx, q, group=None):
    """exchange_topq_rec for separate value / index tensors [q] (packed into one record block)."""
    rec = torch.cat([top_val.to(torch.float64), top_idx.to(torch.int64).view(torch.float64)])
    return exchange_topq_rec(rec, q, group)


def front_hypervolume(front, reference_point, group=None, device=None, partial=None):
    """The hypervolume accumulator: HV of the Pareto front `front` (host [P, m], maximisation)
    above `reference_point`, with the box decomposition of the region the front does not
    dominate (bo_hvi_boxes) split across the ranks -- each rank sums its boxes' volume clipped
    to the front's bounding box (bo_box_volume_sum on the device) and ONE all_reduce(SUM)
    combines them: HV = prod_k (max_k f_k - r_k) - sum.  Identical on every rank.

    The reference names a reference point for its "hypervolume improvement"
    (bayesian_optimization.py:65, :425) but never computes a hypervolume: parity unpinned,
    checked against the oracle's recursive-slicing HV (tests).  `partial(boxes, upper)` replaces
    the device sum (CPU ranks in tests)."""
    from .acquisition import hypervolume_boxes
    r = np.asarray(reference_point, dtype=np.float64).ravel()
    f = np.asarray(front, dtype=np.float64).reshape(-1, r.size)
    keep = np.all(np.isfinite(f), axis=1) & np.all(f > r, axis=1)
    f = f[keep]
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if f.shape[0] == 0:
        return 0.0
    upper = f.max(axis=0)
    boxes = hypervolume_boxes(f, r)
    off, cnt = shard_range(boxes.shape[0], rank, world)
    mine = np.ascontiguousarray(boxes[off:off + cnt])
    if partial is not None:
        val = torch.tensor([float(partial(mine, upper))], dtype=torch.float64)
    else:
        import ctypes
        from . import _lib
        from .device import require_device, stream_handle
        dev = require_device(device)
        bd = torch.as_tensor(mine, device=dev)
        val = torch.zeros(1, dtype=torch.float64, device=dev)
        ub = (ctypes.c_double * r.size)(*upper.tolist())
        _lib.check(_lib.load().bo_box_volume_sum(bd.data_ptr() if bd.numel() else None, mine.shape[0], r.size,
                                                 ub, val.data_ptr(), stream_handle(dev)), "bo_box_volume_sum")
    if collectives_on(group):
        if dist.get_backend(group) != "nccl":
            val = val.cpu()
        dist.all_reduce(val, op=dist.ReduceOp.SUM, group=group)
    return float(np.prod(upper - r) - val.item())


def gather_shards(t, n, group=None):
    """The whole array from every rank's contiguous shard (shard_range(n, r, P) along the last
    axis): ONE all_gather of the shards padded to the largest, then trimmed.  A collective; on the
    backend's device (HIP for RCCL, host for gloo).  Returns a tensor [..., n]."""
    world = dist.get_world_size(group)
    dev = t.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    counts = [shard_range(n, r, world)[1] for r in range(world)]
    cmax = max(counts)
    lead = tuple(t.shape[:-1])
    pad = torch.zeros(lead + (cmax,), dtype=t.dtype, device=dev)
    pad[..., :t.shape[-1]] = t.to(dev)
    g = torch.empty(world * pad.numel(), dtype=t.dtype, device=dev)
    dist.all_gather_into_tensor(g, pad.reshape(-1), group=group)
    g = g.view((world,) + lead + (cmax,))
    return torch.cat([g[r, ..., :counts[r]] for r in range(world)], dim=-1)


def sharded_predict_acquire(x_train, y_train, kinv, cands, prior_mean, prior_variance, length_scales,
                            betas, q, outputs=("acq",), group=None, device=None, scorer=None, out=None,
                            mode="auto", float_type=None):
    """Score this rank's shard of `cands` and return (local results, global top-q).

    Rank r scores candidates shard_range(M, r, P) (its outputs, [n_obj, count] / [count], go to
    `out` when given); the global top-q (NaN first, descending value, ascending index, evaluated
    points excluded) comes from ONE all_gather of the ranks' 16-B record blocks.  `scorer`
    replaces predict_acquire with the same keyword interface (tests drive the partition and the
    exchange on CPU ranks with the oracle standing in for the device)."""
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    off, cnt = shard_range(cands.n, rank, world)
    score = scorer or predict_acquire
    if scorer is None:
        from .device import require_device
        dev = require_device(device)              # indexed: 'cuda' -> 'cuda:<current>'
        kw = {"device": dev}
    else:
        dev = torch.device("cpu")
        kw = {}
    if q > 0:
        kw["top_rec"] = torch.empty(2 * q, dtype=torch.float64, device=dev)
    if out is not None:
        kw["out"] = out
    if scorer is None:
        kw["mode"] = mode
        kw["float_type"] = float_type
    r = score(x_train, y_train, kinv, cands, prior_mean, prior_variance, length_scales, betas,
              outputs=outputs, topq=q, offset=off, count=cnt, **kw)
    if not collectives_on(group):
        sel = merge_topq(r["top_val"].cpu().numpy(), r["top_idx"].cpu().numpy(), q)
    else:
        sel = exchange_topq_rec(kw["top_rec"], q, group)
    return r, sel
