"""Scratch buffers kept across decompositions.

The solver's and the LR step's large work buffers (G's split halves, Y's halves, the
iterate blocks: ~220 MB per 4096^2 matrix) are pure scratch: never part of a result.
Allocating them afresh for every caldera() call makes PyTorch's caching allocator split and
re-split its large blocks until a request no longer fits, and every new hipMalloc of tens of
GB then stalls the host for about a second (measured: +0.6-1.0 s on some bench steps).
They are therefore cached here, keyed by (stream, name, shape, dtype, device): a later run
on the same stream reuses them (stream order makes that safe); runs interleaved on other
streams get their own.  `release()` drops everything.
"""
from __future__ import annotations

import torch

_CACHE: dict = {}


def get(name: str, shape, dtype, device) -> torch.Tensor:
    """A cached uninitialised tensor for `name` on the current stream of `device`."""
    dev = torch.device(device)
    sid = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0
    key = (sid, name, dev)
    shape = tuple(int(s) for s in shape)
    t = _CACHE.get(key)
    if t is None or t.shape != shape or t.dtype != dtype:
        _CACHE.pop(key, None)
        t = torch.empty(shape, dtype=dtype, device=dev)
        _CACHE[key] = t
    return t


def get_flat(name: str, numel: int, dtype, device) -> torch.Tensor:
    """A cached uninitialised 1-D tensor of at least `numel` elements (grown, never shrunk, so
    calls of varying sizes share one buffer); returns its first `numel` elements."""
    dev = torch.device(device)
    sid = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0
    key = (sid, name, dev)
    t = _CACHE.get(key)
    if t is None or t.numel() < numel or t.dtype != dtype:
        _CACHE.pop(key, None)
        t = torch.empty(max(int(numel), 1), dtype=dtype, device=dev)
        _CACHE[key] = t
    return t[:numel]


def release():
    """Free every cached scratch buffer (returned to PyTorch's caching allocator)."""
    _CACHE.clear()
