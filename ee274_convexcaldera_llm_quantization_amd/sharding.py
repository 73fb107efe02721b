"""Matrix-level data parallelism for whole-model decomposition (BASELINE configs[3]).

The reference decomposes a model's linear layers one after another in one process
(main.py:135-251, `apply_CALDERA_quantization`).  The units are independent (no state is
shared between `caldera()` calls), so here every rank (one process per GPU)
decomposes the matrices i with i % world == rank, batching same-shape matrices in lockstep
on its GPU, and the only collective is the final gather of the packed results to rank 0
(torch.distributed `gather`; backend "nccl" is RCCL over xGMI on MI355X, "gloo" on CPU).

Result payload (also the on-disk format, §8f item 2): one uint8 tensor per rank =
  [u64 little-endian meta length][meta JSON][blob]
with, per matrix, int2/int4 offset-binary packed Q codes (or int8/int16 codes for 8/16 bits),
fp32 L (m x r) and R (r x n), and in the JSON its name, shape, scales, global scale and
error history.  Packing first keeps the 224-matrix Llama-2-7B gather at ~2.9 GB instead of
~7.4 GB with the reference's unpacked int8 codes.
"""
from __future__ import annotations

import json
import struct
from dataclasses import dataclass, field

import numpy as np
import torch

LLAMA2_7B_PROJS = (("self_attn.q_proj", 4096, 4096), ("self_attn.k_proj", 4096, 4096),
                   ("self_attn.v_proj", 4096, 4096), ("self_attn.o_proj", 4096, 4096),
                   ("mlp.gate_proj", 11008, 4096), ("mlp.up_proj", 11008, 4096),
                   ("mlp.down_proj", 4096, 11008))


def llama2_7b_matrices(n_layers: int = 32):
    """Layer-major list of (name, m, n, seed) — 224 matrices for the full model; seed =
    layer * 7 + proj index."""
    out = []
    for layer in range(n_layers):
        for pi, (proj, m, n) in enumerate(LLAMA2_7B_PROJS):
            out.append((f"model.layers.{layer}.{proj}", m, n, layer * 7 + pi))
    return out


def shard_indices(n_items: int, world: int, rank: int):
    """Round-robin: item i -> rank i % world.  With 224 = 8 x 28 and the 7-projection
    pattern coprime with 8, every rank gets the same mix of shapes (balanced, no LPT)."""
    return list(range(rank, n_items, world))


@dataclass
class MatrixResult:
    name: str
    m: int
    n: int
    rank: int
    Q_bits: int
    codes: torch.Tensor          # packed uint8 (bits <= 4) or int8/int16 codes, flat
    Q_scale: float
    L: torch.Tensor              # (m, r) fp32
    R: torch.Tensor              # (r, n) fp32
    global_scale: float
    errors: dict = field(default_factory=dict)
    extra: dict = field(default_factory=dict)


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().contiguous().numpy()


def pack_results(results: list[MatrixResult]) -> torch.Tensor:
    """Serialise results into one uint8 tensor (CPU)."""
    metas, blobs, off = [], [], 0
    for r in results:
        entry = {"name": r.name, "m": r.m, "n": r.n, "rank": r.rank, "Q_bits": r.Q_bits,
                 "Q_scale": float(r.Q_scale), "global_scale": float(r.global_scale),
                 "errors": r.errors, "extra": r.extra, "arrays": {}}
        for key, t in (("codes", r.codes), ("L", r.L), ("R", r.R)):
            a = _np(t)
            b = a.tobytes()
            entry["arrays"][key] = {"offset": off, "nbytes": len(b), "dtype": str(a.dtype),
                                    "shape": list(a.shape)}
            blobs.append(b)
            off += len(b)
        metas.append(entry)
    meta = json.dumps(metas).encode()
    buf = struct.pack("<Q", len(meta)) + meta + b"".join(blobs)
    return torch.frombuffer(bytearray(buf), dtype=torch.uint8)


def unpack_results(buf: torch.Tensor) -> list[MatrixResult]:
    raw = bytes(buf.cpu().numpy().tobytes())
    (mlen,) = struct.unpack("<Q", raw[:8])
    metas = json.loads(raw[8:8 + mlen].decode())
    base = 8 + mlen
    out = []
    for e in metas:
        arrs = {}
        for key, d in e["arrays"].items():
            a = np.frombuffer(raw, dtype=np.dtype(d["dtype"]), count=int(np.prod(d["shape"])) if d["shape"] else 1,
                              offset=base + d["offset"]).reshape(d["shape"]).copy()
            arrs[key] = torch.from_numpy(a)
        out.append(MatrixResult(e["name"], e["m"], e["n"], e["rank"], e["Q_bits"], arrs["codes"],
                                e["Q_scale"], arrs["L"], arrs["R"], e["global_scale"], e["errors"],
                                e.get("extra", {})))
    return out


def save_results(path: str, results: list[MatrixResult]):
    with open(path, "wb") as f:
        f.write(bytes(pack_results(results).numpy().tobytes()))


def load_results(path: str) -> list[MatrixResult]:
    with open(path, "rb") as f:
        return unpack_results(torch.frombuffer(bytearray(f.read()), dtype=torch.uint8))


def gather_to_rank0(payload: torch.Tensor, group=None, device=None):
    """Gather every rank's uint8 payload to rank 0 (padded to the max size).  Returns the
    list of per-rank payloads on rank 0, None elsewhere.  device: where the collective
    runs (a HIP device for "nccl" = RCCL over xGMI, CPU for "gloo")."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = device if device is not None else payload.device
    n = torch.tensor([payload.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    mx = int(max(int(s.item()) for s in sizes))
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    buf[: payload.numel()] = payload.to(dev)
    gl = [torch.zeros(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gather_list=gl, dst=0, group=group)
    if rank != 0:
        return None
    return [g[: int(s.item())].cpu() for g, s in zip(gl, sizes)]


def decompose_sharded(items, decompose_batch, *, rank: int, world: int, max_batch: int = 16,
                      group=None, gather: bool = True, device=None):
    """items: list of (name, m, n, seed).  decompose_batch(list_of_items) -> list of
    MatrixResult (the GPU engine on MI355X; a stub in the CPU gloo tests).  Same-shape
    matrices of this rank's shard run together in batches of <= max_batch."""
    mine = [items[i] for i in shard_indices(len(items), world, rank)]
    by_shape: dict[tuple, list] = {}
    for it in mine:
        by_shape.setdefault((it[1], it[2]), []).append(it)
    batches = [group_items[s:s + max_batch] for group_items in by_shape.values()
               for s in range(0, len(group_items), max_batch)]
    results = []
    if hasattr(decompose_batch, "run_all"):  # all batches at once (interleaved on HIP streams)
        results = decompose_batch.run_all(batches)
    else:
        for b in batches:
            results.extend(decompose_batch(b))
    order = {it[0]: i for i, it in enumerate(items)}
    results.sort(key=lambda r: order[r.name])
    if not gather or world == 1:
        return results
    payloads = gather_to_rank0(pack_results(results), group=group, device=device)
    if payloads is None:
        return None
    allres = [r for pl in payloads for r in unpack_results(pl)]
    allres.sort(key=lambda r: order[r.name])
    return allres


def engine_decompose_batch(quant_params, device, H_of=None):
    """decompose_batch for the MI355X engine: synthetic fp16 weights randn*0.02 per seed
    (random-init model, no checkpoint access), H_of(name) -> diagonal or None."""
    from .engine import CalderaEngine, EngineParams
    from .overlap import run_interleaved

    def weights(batch_items):
        ws = []
        for name, m, n, seed in batch_items:
            torch.manual_seed(seed)
            ws.append((torch.randn(m, n) * 0.02).to(torch.float16))
        return torch.stack(ws).to(device)

    def results(batch_items, eng):
        return [MatrixResult(name, m, n, d["L"].shape[1], quant_params.Q_bits, d["codes"], d["Q_scale"], d["L"],
                             d["R"], d["global_scale"], d["errors"])
                for (name, m, n, seed), d in zip(batch_items, eng.last_packed)]

    def run_all(batches):
        """Every batch (one per shape class) on its own engine and HIP stream, interleaved at
        the host syncs: the one-CU-per-matrix p x p kernels of a small batch leave most of
        the 256 CUs to the other batches' GEMMs (config 4 share of one rank at 8 GPUs:
        0.43 s vs 0.78 s one batch after another, tools/bench_model.py)."""
        Ws = [weights(b) for b in batches]
        engines = [CalderaEngine(EngineParams.from_caldera_params(quant_params)) for _ in batches]
        run_interleaved([e.run_iter(W, H_of(b[0][0]) if H_of is not None else None)
                         for e, W, b in zip(engines, Ws, batches)], torch.device(device))
        return [r for b, e in zip(batches, engines) for r in results(b, e)]

    def run(batch_items):
        return run_all([batch_items])

    run.run_all = run_all
    return run
