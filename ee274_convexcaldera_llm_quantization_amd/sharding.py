"""Matrix-level data parallelism for whole-model decomposition (BASELINE configs[3]).

The reference decomposes a model's linear layers one after another in one process
(main.py:135-251, `apply_CALDERA_quantization`).  The units are independent (no state is
shared between `caldera()` calls), so here every rank (one process per GPU)
decomposes the matrices i with i % world == rank, batching same-shape matrices in lockstep on
its GPU (each with its own diagonal Hessian: per-matrix weights, ABI 5), and the only collective is the final gather of the packed results to
rank 0 (torch.distributed `gather`; backend "nccl" is RCCL over xGMI on MI355X, "gloo" on
CPU tests).

Result payload (also the on-disk format, §8f item 2): one uint8 tensor per rank =
  [magic "CQRS"][u32 format version][u64 little-endian meta length][meta JSON][pad to 16][blob]
with, per matrix, int2/int4 offset-binary packed Q codes (or int8/int16 codes for 8/16 bits),
fp32 L (m x r) and R (r x n), each 16-byte aligned, and in the JSON its name, shape, scales,
global scale, error history and array offsets.  The payload is assembled where the results
live: on the GPU the blob is concatenated in HBM (only the few-KB JSON crosses PCIe), the
RCCL gather moves it HBM -> HBM over xGMI, and rank 0 unpacks it into device views.
Packing keeps the 224-matrix Llama-2-7B gather at ~2.9 GB instead of ~7.4 GB with the
reference's unpacked int8 codes.

Resume (main.py:135-251 decomposes layer after layer; a crash loses everything): with
`resume_path`, names already in that results file are skipped and the file is rewritten
(atomically) with everything done so far after this rank's batches finish.
"""
from __future__ import annotations

import json
import os
import struct
from dataclasses import dataclass, field

import torch

LLAMA2_7B_PROJS = (("self_attn.q_proj", 4096, 4096), ("self_attn.k_proj", 4096, 4096),
                   ("self_attn.v_proj", 4096, 4096), ("self_attn.o_proj", 4096, 4096),
                   ("mlp.gate_proj", 11008, 4096), ("mlp.up_proj", 11008, 4096),
                   ("mlp.down_proj", 4096, 11008))
_ALIGN = 16
_MAGIC = b"CQRS"
_VERSION = 2   # 1 = round-2 payloads (no magic/version word): rejected, they parse differently
_HEAD = struct.Struct("<4sIQ")


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
    extra: dict = field(default_factory=dict)  # e.g. n_padded: codes on an (m, n_padded) grid


def _pad(nbytes: int) -> int:
    return (-nbytes) % _ALIGN


def _as_bytes(t: torch.Tensor, dev) -> torch.Tensor:
    return t.detach().contiguous().reshape(-1).view(torch.uint8).to(dev)


def pack_results(results: list[MatrixResult], device=None) -> torch.Tensor:
    """Serialise results into one uint8 tensor on `device` (default: the CPU).  On a HIP
    device the arrays never leave HBM: they are concatenated there, only the JSON is
    uploaded."""
    dev = torch.device("cpu") if device is None else torch.device(device)
    metas, parts, off = [], [], 0
    for r in results:
        entry = {"name": r.name, "m": r.m, "n": r.n, "rank": r.rank, "Q_bits": r.Q_bits,
                 "Q_scale": float(r.Q_scale), "global_scale": float(r.global_scale),
                 "errors": r.errors, "extra": r.extra, "arrays": {}}
        for key, t in (("codes", r.codes), ("L", r.L), ("R", r.R)):
            b = _as_bytes(t, dev)
            entry["arrays"][key] = {"offset": off, "nbytes": b.numel(), "dtype": str(t.dtype).split(".")[-1],
                                    "shape": list(t.shape)}
            parts.append(b)
            pad = _pad(b.numel())
            if pad:
                parts.append(torch.zeros(pad, dtype=torch.uint8, device=dev))
            off += b.numel() + pad
        metas.append(entry)
    meta = json.dumps(metas).encode()
    head = _HEAD.pack(_MAGIC, _VERSION, len(meta)) + meta
    head += b"\0" * _pad(len(head))
    head_t = torch.frombuffer(bytearray(head), dtype=torch.uint8).to(dev)
    return torch.cat([head_t] + parts)


def unpack_results(buf: torch.Tensor) -> list[MatrixResult]:
    """Inverse of pack_results; arrays are views of `buf` on its device.  Raises ValueError
    for a buffer without the payload magic or with an unknown format version."""
    h = _HEAD.size
    if buf.numel() < h:
        raise ValueError("unpack_results: buffer shorter than the payload header")
    magic, version, mlen = _HEAD.unpack(bytes(buf[:h].cpu().numpy().tobytes()))
    if magic != _MAGIC:
        raise ValueError("unpack_results: not a caldera result payload (bad magic)")
    if version != _VERSION:
        raise ValueError(f"unpack_results: unsupported payload format version {version} (expected {_VERSION})")
    metas = json.loads(bytes(buf[h:h + mlen].cpu().numpy().tobytes()).decode())
    base = h + mlen + _pad(h + mlen)
    out = []
    for e in metas:
        arrs = {}
        for key, d in e["arrays"].items():
            s = base + d["offset"]
            arrs[key] = buf[s:s + d["nbytes"]].view(getattr(torch, d["dtype"])).view(d["shape"])
        out.append(MatrixResult(e["name"], e["m"], e["n"], e["rank"], e["Q_bits"], arrs["codes"],
                                e["Q_scale"], arrs["L"], arrs["R"], e["global_scale"], e["errors"],
                                e.get("extra", {})))
    return out


def save_results(path: str, results: list[MatrixResult]):
    """Write the packed payload (host copy) atomically."""
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(pack_results(results).numpy().tobytes())
    os.replace(tmp, path)


def load_results(path: str) -> list[MatrixResult]:
    with open(path, "rb") as f:
        return unpack_results(torch.frombuffer(bytearray(f.read()), dtype=torch.uint8))


def gather_to_rank0(payload: torch.Tensor, group=None, device=None, to_host: bool = False):
    """Gather every rank's uint8 payload to rank 0 (padded to the max size).  Returns the
    list of per-rank payloads on rank 0 (on `device`, i.e. in HBM for "nccl"; host copies
    with to_host), None elsewhere.  device: where the collective runs (a HIP device for
    "nccl" = RCCL over xGMI, CPU for "gloo")."""
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
    out = [g[: int(s.item())] for g, s in zip(gl, sizes)]
    return [o.cpu() for o in out] if to_host else out


class PendingGather:
    """An issued gather_to_rank0_async: wait() -> rank 0's per-rank payloads (None elsewhere)."""

    def __init__(self, work, gl, sizes, buf):
        self.work, self.gl, self.sizes, self.buf = work, gl, sizes, buf

    def wait(self):
        self.work.wait()
        self.buf = None
        if self.gl is None:
            return None
        return [g[:n] for g, n in zip(self.gl, self.sizes)]


def gather_to_rank0_async(payload: torch.Tensor, group=None, device=None, sizes=None) -> PendingGather:
    """gather_to_rank0 issued asynchronously (the transfer runs on the collective's own stream
    while the caller's stream computes on; the payload is copied into a send buffer first, so
    the caller may free or reuse it).  sizes: every rank's payload size when the caller knows
    them (same-size batches), which skips the blocking size exchange."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = device if device is not None else payload.device
    if sizes is None:
        n = torch.tensor([payload.numel()], dtype=torch.int64, device=dev)
        st = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
        dist.all_gather(st, n, group=group)
        sizes = [int(x.item()) for x in st]
    sizes = [int(x) for x in sizes]
    assert len(sizes) == world and sizes[rank] == payload.numel(), "gather_to_rank0_async: sizes"
    mx = max(sizes)
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    buf[: payload.numel()] = payload.to(dev)
    gl = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
    work = dist.gather(buf, gather_list=gl, dst=0, group=group, async_op=True)
    return PendingGather(work, gl, sizes, buf)


def _plan(items, world: int, rank: int, max_batch: int, h_key=None, skip=()):
    """The batches rank `rank` decomposes: its round-robin shard grouped by shape (and h_key),
    in batches of <= max_batch.  Deterministic, so every rank can compute every rank's plan."""
    mine = [items[i] for i in shard_indices(len(items), world, rank) if items[i][0] not in skip]
    groups: dict[tuple, list] = {}
    for it in mine:
        groups.setdefault((it[1], it[2], None if h_key is None else h_key(it[0])), []).append(it)
    return [g[s:s + max_batch] for g in groups.values() for s in range(0, len(g), max_batch)]


def _blob(results, dev):
    """The arrays of `results` concatenated 16-byte aligned on `dev` (pack_results' blob without
    its header) and their metadata entries (offsets relative to this blob)."""
    metas, parts, off = [], [], 0
    for r in results:
        entry = {"name": r.name, "m": r.m, "n": r.n, "rank": r.rank, "Q_bits": r.Q_bits,
                 "Q_scale": float(r.Q_scale), "global_scale": float(r.global_scale),
                 "errors": r.errors, "extra": r.extra, "arrays": {}}
        for key, t in (("codes", r.codes), ("L", r.L), ("R", r.R)):
            b = _as_bytes(t, dev)
            entry["arrays"][key] = {"offset": off, "nbytes": b.numel(), "dtype": str(t.dtype).split(".")[-1],
                                    "shape": list(t.shape)}
            parts.append(b)
            pad = _pad(b.numel())
            if pad:
                parts.append(torch.zeros(pad, dtype=torch.uint8, device=dev))
            off += b.numel() + pad
        metas.append(entry)
    blob = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.uint8, device=dev)
    return blob, metas


# the last decompose_sharded call's gather (tests and bench.py read it)
LAST_GATHER: dict = {}


def _payload_device(results, world, gather, group, device):
    if device is not None:
        return torch.device(device)
    # where the payload is assembled and gathered: in HBM for RCCL ("nccl"), on the host
    # otherwise (gloo's gather takes CPU tensors), and for world 1 where the results live
    dev = torch.device("cpu")
    if world == 1 or not gather:
        return results[0].L.device if results else dev
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl" and results:
        return results[0].L.device
    return dev


def decompose_sharded(items, decompose_batch, *, rank: int, world: int, max_batch: int = 16,
                      group=None, gather: bool = True, device=None, h_key=None, resume_path=None,
                      on_batch_done=None):
    """items: list of (name, m, n, seed).  decompose_batch(list_of_items) -> list of
    MatrixResult (the GPU engine on MI355X; a stub in the CPU gloo tests).  Matrices of this
    rank's shard that share a shape run together in batches of <= max_batch, each with its
    own Hessian (h_key(name): an optional extra grouping key).  resume_path: per-rank results
    file; names in it are not decomposed again, and it is rewritten with this rank's results
    at the end.

    Overlapped gather (world > 1, no resume, decompose_batch.run_all taking on_batch_done and
    decompose_batch.blob_bound(m, n) -> an upper bound of one matrix's packed array bytes):
    batch j's arrays go to rank 0 by an asynchronous gather issued as soon as batch j (and every
    batch before it) has finished, so the transfers of earlier batches run under later batches'
    compute and only the tail is exposed.  Every rank computes every rank's plan (_plan), so all
    issue the same sequence of gathers, each padded to that batch's largest bound over the
    ranks; the metadata (names, scales, errors, offsets) follows in one small gather at the end.
    Otherwise everything is packed and gathered once, after the last batch.
    on_batch_done(j, results): called as this rank's batch j finishes (timing, tests)."""
    import time
    done = []
    skip = set()
    if resume_path is not None and os.path.exists(resume_path):
        names = {items[i][0] for i in shard_indices(len(items), world, rank)}
        done = [r for r in load_results(resume_path) if r.name in names]
        skip = {r.name for r in done}
    batches = _plan(items, world, rank, max_batch, h_key, skip)
    order = {it[0]: i for i, it in enumerate(items)}
    overlapped = (gather and world > 1 and not skip and resume_path is None
                  and hasattr(decompose_batch, "run_all") and hasattr(decompose_batch, "blob_bound"))
    LAST_GATHER.clear()
    LAST_GATHER.update(mode="overlapped" if overlapped else ("end" if gather and world > 1 else "none"))
    if overlapped:
        return _decompose_overlapped(items, decompose_batch, batches, rank, world, max_batch, group, device,
                                     h_key, order, on_batch_done)
    results = []
    if batches:
        if hasattr(decompose_batch, "run_all"):  # all batches at once (interleaved on HIP streams)
            if on_batch_done is not None:
                results = decompose_batch.run_all(batches, on_batch_done=on_batch_done)
            else:
                results = decompose_batch.run_all(batches)
        else:
            for j, b in enumerate(batches):
                rb = decompose_batch(b)
                if on_batch_done is not None:
                    on_batch_done(j, rb)
                results.extend(rb)
    dev = _payload_device(results, world, gather, group, device)
    if done:
        results.extend(MatrixResult(r.name, r.m, r.n, r.rank, r.Q_bits, r.codes.to(dev), r.Q_scale, r.L.to(dev),
                                    r.R.to(dev), r.global_scale, r.errors, r.extra) for r in done)
    results.sort(key=lambda r: order[r.name])
    if resume_path is not None and batches:
        save_results(resume_path, results)
    if not gather or world == 1:
        return results
    t0 = time.perf_counter()
    payloads = gather_to_rank0(pack_results(results, device=dev), group=group, device=dev)
    LAST_GATHER.update(exposed_s=time.perf_counter() - t0, rounds=1)
    if payloads is None:
        return None
    allres = [r for pl in payloads for r in unpack_results(pl)]
    allres.sort(key=lambda r: order[r.name])
    return allres


def _decompose_overlapped(items, decompose_batch, batches, rank, world, max_batch, group, device, h_key, order,
                          on_batch_done):
    import time
    import torch.distributed as dist
    plans = [batches if q == rank else _plan(items, world, q, max_batch, h_key) for q in range(world)]
    n_rounds = max(len(p) for p in plans)
    bound = decompose_batch.blob_bound
    caps = []
    for j in range(n_rounds):
        c = max((sum(bound(m, n) for _, m, n, _ in p[j]) if j < len(p) else 0) for p in plans)
        caps.append(c)
    backend = dist.get_backend(group)
    state = {"next": 0, "done": {}, "works": [], "recv": [], "metas": [], "lens": [], "dev": None,
             "t_issue": [], "bytes": 0}

    def issue(j, results):
        if state["dev"] is None:
            state["dev"] = (torch.device(device) if device is not None else
                            (results[0].L.device if backend == "nccl" and results else torch.device("cpu")))
        dev = state["dev"]
        blob, metas = _blob(results, dev)
        assert blob.numel() <= caps[j], ("blob_bound too small", j, blob.numel(), caps[j])
        buf = torch.zeros(caps[j], dtype=torch.uint8, device=dev)
        buf[:blob.numel()] = blob
        gl = [torch.empty(caps[j], dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
        state["works"].append(dist.gather(buf, gather_list=gl, dst=0, group=group, async_op=True))
        state["recv"].append((buf, gl))
        state["metas"].append(metas)
        state["lens"].append(blob.numel())
        state["t_issue"].append(time.perf_counter())
        state["bytes"] += caps[j]

    def batch_done(j, results):
        if on_batch_done is not None and j < len(batches):
            on_batch_done(j, results)
        state["done"][j] = results
        while state["next"] in state["done"]:
            k = state["next"]
            if caps[k] > 0:
                issue(k, state["done"][k])
            else:
                state["metas"].append([])
                state["lens"].append(0)
                state["recv"].append((None, None))
                state["works"].append(None)
            state["next"] += 1

    if batches:
        decompose_batch.run_all(batches, on_batch_done=batch_done)
    for j in range(len(batches), n_rounds):   # rounds this rank has no batch for: empty contributions
        batch_done(j, [])
    t_end = time.perf_counter()
    for w in state["works"]:
        if w is not None:
            w.wait()
    dev = state["dev"] if state["dev"] is not None else (torch.device(device) if device is not None
                                                          else torch.device("cpu"))
    # the metadata: one small gather of every rank's JSON (names, scales, errors, per-round offsets)
    meta = json.dumps({"metas": state["metas"], "lens": state["lens"]}).encode()
    meta_t = torch.frombuffer(bytearray(meta), dtype=torch.uint8).to(dev)
    metas_all = gather_to_rank0(meta_t, group=group, device=dev)
    if backend == "nccl":
        torch.cuda.synchronize(dev)
    LAST_GATHER.update(rounds=n_rounds, exposed_s=time.perf_counter() - t_end, issued_bytes=state["bytes"],
                       caps=caps)
    if metas_all is None:
        return None
    allres = []
    for q, mt in enumerate(metas_all):
        md = json.loads(bytes(mt.cpu().numpy().tobytes()).decode())
        for j, metas in enumerate(md["metas"]):
            if not metas:
                continue
            src = state["recv"][j][1][q]
            for e in metas:
                arrs = {}
                for key, d in e["arrays"].items():
                    s0 = d["offset"]
                    arrs[key] = src[s0:s0 + d["nbytes"]].view(getattr(torch, d["dtype"])).view(d["shape"])
                allres.append(MatrixResult(e["name"], e["m"], e["n"], e["rank"], e["Q_bits"], arrs["codes"],
                                           e["Q_scale"], arrs["L"], arrs["R"], e["global_scale"], e["errors"],
                                           e.get("extra", {})))
    allres.sort(key=lambda r: order[r.name])
    return allres


def engine_decompose_batch(quant_params, device, H_of=None):
    """decompose_batch for the MI355X engine: synthetic fp16 weights randn*0.02 per seed
    (random-init model, no checkpoint access), H_of(name) -> diagonal (n,) or None per matrix
    (distinct Hessians share a batch: api._Group groups them by code-path flags only)."""
    from .api import _Group
    from .overlap import run_interleaved

    def weights(batch_items):
        ws = []
        for name, m, n, seed in batch_items:
            torch.manual_seed(seed)
            ws.append((torch.randn(m, n) * 0.02).to(torch.float16))
        return torch.stack(ws).to(device)

    def h_of(batch_items):
        if H_of is None:
            return None
        hs = [H_of(it[0]) for it in batch_items]
        if all(h is hs[0] for h in hs):
            return None if hs[0] is None else hs[0].to(device)
        return [None if h is None else h.to(device) for h in hs]

    def results(batch_items, group):
        out = [None] * len(batch_items)
        for idx, eng, _ in group.parts:
            for b, d in zip(idx, eng.last_packed):
                name, m, n, seed = batch_items[b]
                extra = {"n_padded": d["n_padded"]} if "n_padded" in d else {}
                out[b] = MatrixResult(name, m, n, d["L"].shape[1], quant_params.Q_bits, d["codes"], d["Q_scale"],
                                      d["L"], d["R"], d["global_scale"], d["errors"], extra)
        return out

    def run_all(batches, on_batch_done=None):
        """Every batch (one per shape class) on its own engine and HIP stream, interleaved at
        the host syncs: the one-CU-per-matrix p x p kernels of a small batch leave most of
        the 256 CUs to the other batches' GEMMs (config 4 share of one rank at 8 GPUs:
        0.43 s vs 0.78 s one batch after another, tools/bench_model.py).  on_batch_done(j,
        results): as batch j's last engine part finishes."""
        dev = torch.device(device)
        groups = [_Group(quant_params, weights(b), h_of(b), dev, scale_W=True, use_tqdm=False, engine_kwargs=None,
                         streams=1, w_to_host=False) for b in batches]
        owner = [j for j, g in enumerate(groups) for _ in g.parts]
        left = [len(g.parts) for g in groups]

        def part_done(i, _):
            j = owner[i]
            left[j] -= 1
            if left[j] == 0 and on_batch_done is not None:
                on_batch_done(j, results(batches[j], groups[j]))

        run_interleaved([gen for g in groups for _, _, gen in g.parts], dev, on_done=part_done)
        return [r for b, g in zip(batches, groups) for r in results(b, g)]

    def run(batch_items):
        return run_all([batch_items])

    run.run_all = run_all
    run.blob_bound = lambda m, n: blob_bound(m, n, quant_params.Q_bits, quant_params.rank)
    return run


def blob_bound(m: int, n: int, q_bits: int, rank: int) -> int:
    """Upper bound of one m x n matrix's packed arrays (_blob): codes (offset-binary packed for
    2/4 bits on the (m, n padded to 4) grid, int8 / int16 codes otherwise), L (m x r fp32) and R
    (r x n fp32) with r <= rank, each padded to 16 bytes."""
    npad = n + (-n) % 4
    codes = m * npad * q_bits // 8 if q_bits <= 4 else m * npad * (1 if q_bits <= 8 else 2)
    return sum(b + (-b) % _ALIGN for b in (codes, 4 * m * rank, 4 * rank * n))
