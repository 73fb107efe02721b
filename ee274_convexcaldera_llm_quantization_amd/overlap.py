"""Cooperative interleaving of independent matrix batches on separate HIP streams.

The hot path alternates device-wide GEMMs with one-workgroup-per-matrix p x p kernels
(Jacobi, whitening, fp64 Grams) that occupy only B of the 256 CUs, and it reads a few
scalars back to the host once per outer iteration (solver convergence, error history).
Splitting a batch into parts that run on their own streams lets one part's latency-bound
kernels and host round trips overlap another part's GEMMs.

The engine and solver are written as generators that `yield` right before every host
synchronisation; `run_interleaved` resumes each generator with its own stream made
current, so the work one part queues before its sync point is already on the GPU while
the host waits for the other part.  No threads: the GIL and the caching allocator see a
single host thread.
"""
from __future__ import annotations

import time

import torch


def run_to_end(gen):
    """Drive one generator to completion on the current stream; return its value."""
    try:
        while True:
            next(gen)
    except StopIteration as stop:
        return stop.value


def default_parts(batch: int) -> int:
    """How many interleaved parts a batch of `batch` same-shape matrices is split into by
    default: 2 from 16 matrices on, else 1.  With ready-first interleaving and no split-K under
    concurrency (round 5) two parts overlap one part's one-CU-per-matrix kernels (Jacobi,
    whitening: a launch of B/2 matrices holds B/2 CUs) and read-backs with the other's products.
    Config 2, one box: B = 256 302.5 -> 316.5 matrices/s (3 parts +0.6 %, 4 parts 298.2;
    `profiles/r05ab_*`, `r05ag_*`), B = 32 211.9 -> 241.9, B = 16 157.2 -> 178.3, but B = 8
    107.7 -> 105.5 and B = 4 67.3 -> 57.3 (`r05ah_*`: small batches rely on split-K, which
    interleaving turns off); config 3 186.3 -> 202.7, config 4's tall shape 180.1 -> 195.6,
    config 5 85.1 -> 89.0 (`r05ac_*`)."""
    return 2 if batch >= 16 else 1


_STREAMS: dict = {}


def _part_streams(device, n):
    """The same n streams of `device` on every call (the cached scratch of scratch.py is
    keyed by stream, so a fixed set keeps it bounded)."""
    dev = torch.device(device)
    lst = _STREAMS.setdefault(dev, [])
    while len(lst) < n:
        lst.append(torch.cuda.Stream(device=dev))
    return lst[:n]


def run_interleaved(gens, device, ready_first: bool = True, on_done=None):
    """Drive generators, each on its own stream of `device` (a fixed per-device set).
    Returns the list of their return values.  The caller's stream is joined before and after.
    on_done(i, value): called as generator i finishes, with its stream current (e.g. to start
    the gather of that batch's results while the others still run).

    ready_first (default): a generator that yielded (it is about to read results back) gets an
    event recorded behind the work it queued, and the host next resumes a generator whose
    event has completed -- in round-robin order among those -- so it never blocks on one
    stream while another stream's read-back is ready and its GPU queue runs dry.  Only when no
    event has completed does it wait (spinning on the events).  False: plain round-robin,
    each resume blocking on that generator's own stream."""
    if len(gens) == 1:
        v = run_to_end(gens[0])
        if on_done is not None:
            on_done(0, v)
        return [v]
    # concurrent batches fill the chip together: a small batch's split-fp16 products need no
    # split-K here (its partial sums and epilogue launches only add traffic: config-4 rank
    # share 0.159 -> 0.136 s, profiles/r05f_share*.log).  The policy is this thread's only
    # (_lib.split_k_policy), so a matrix's summation order depends on whether its batch is
    # split into parts (default_parts: from 16 matrices on), not on other threads' calls.
    from . import _lib
    with _lib.split_k_policy(False):
        return _run_interleaved(gens, device, ready_first, on_done)


def _run_interleaved(gens, device, ready_first, on_done=None):
    caller = torch.cuda.current_stream(device)
    streams = _part_streams(device, len(gens))
    for s in streams:
        s.wait_stream(caller)
    out = [None] * len(gens)
    live = list(range(len(gens)))
    try:
        if not ready_first:
            while live:
                for i in list(live):
                    torch.cuda.set_stream(streams[i])
                    try:
                        next(gens[i])
                    except StopIteration as stop:
                        out[i] = stop.value
                        live.remove(i)
                        if on_done is not None:
                            on_done(i, stop.value)
        else:
            events = [torch.cuda.Event() for _ in gens]
            pending = [False] * len(gens)  # yielded, event recorded, not yet resumed
            nxt = 0
            while live:
                # the first live generator at or after nxt (cyclically) that is ready: never
                # started / resumed since its work completed
                pick = None
                order = sorted(live, key=lambda j: (j - nxt) % len(gens))
                spins = 0
                while pick is None:
                    for j in order:
                        if not pending[j] or events[j].query():
                            pick = j
                            break
                    spins += 1
                    if pick is None and spins >= 64:
                        # every part is waiting on the GPU: poll at ~0.1 ms instead of keeping a
                        # host core at 100 % (other ranks share the host); still ready-first
                        time.sleep(1e-4)
                i = pick
                pending[i] = False
                torch.cuda.set_stream(streams[i])
                try:
                    next(gens[i])
                    events[i].record(streams[i])
                    pending[i] = True
                except StopIteration as stop:
                    out[i] = stop.value
                    live.remove(i)
                    if on_done is not None:
                        on_done(i, stop.value)
                nxt = (i + 1) % len(gens)
    finally:
        torch.cuda.set_stream(caller)
    for s in streams:
        caller.wait_stream(s)
    return out
