"""Device plumbing: HIP device checks, stream handles, cached workspaces.

PyTorch-ROCm is used only for device memory, streams and torch.distributed; every
computation on the hot path is a libbo_amd.so kernel.
"""

from __future__ import annotations

import torch

from . import _lib

F64 = torch.float64


def require_device(device=None):
    """Return a torch.device on a HIP GPU or raise (no CPU fallback on the product path)."""
    if not torch.cuda.is_available():
        raise RuntimeError("bayesopt_smart_amd needs a HIP device (torch.cuda.is_available() is False)")
    _lib.load()
    if device is None:
        return torch.device("cuda", torch.cuda.current_device())
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError(f"bayesopt_smart_amd tensors must live on a HIP device, got {dev}")
    # always an indexed device ('cuda' -> 'cuda:<current>'), so that device checks compare equal
    return dev if dev.index is not None else torch.device("cuda", torch.cuda.current_device())


def stream_handle(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()


def as_dev(x, device, dtype=F64):
    """Tensor on `device` with `dtype`, C-contiguous (copies only when needed)."""
    if isinstance(x, torch.Tensor):
        t = x.to(device=device, dtype=dtype)
    else:
        t = torch.as_tensor(x, dtype=dtype, device=device)
    return t.contiguous()


class Workspace:
    """Grow-only device scratch buffer, one per (device, stream): calls in flight on different
    streams never share scratch (their packed W, alpha and partial top-q lists would collide).
    A call on a stream reuses the buffer only after its previous calls on that same stream
    (stream order), so no extra synchronisation is needed.  A grown buffer's old storage is
    released through the caching allocator, which is stream-ordered as well."""

    _cache = {}

    @classmethod
    def get(cls, nbytes, device, stream=None):
        st = stream_handle(device) if stream is None else stream
        key = (device.type, device.index, int(st or 0))
        buf = cls._cache.get(key)
        if buf is None or buf.numel() < nbytes:
            # geometric growth (x1.5, 2 MiB granules): a loop whose N grows by a batch each
            # iteration re-allocates O(log N) times, not once per iteration
            grow = 0 if buf is None else buf.numel() + buf.numel() // 2
            size = max(int(nbytes), grow, 256)
            size = (size + (2 << 20) - 1) // (2 << 20) * (2 << 20) if size > (2 << 20) else size
            buf = torch.empty(size, dtype=torch.uint8, device=device)
            cls._cache[key] = buf
        return buf
