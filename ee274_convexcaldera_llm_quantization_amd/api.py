"""Batched entry points behind the drop-in `caldera()` (src/caldera/decomposition/alg.py).

`caldera_batch` decomposes several same-shape weight matrices in lockstep on one HIP
device (the throughput path used by bench.py and the multi-GPU sharder) and returns one
CalderaDecomposition per matrix with the reference's field layout
(RCR/src/caldera/utils/dataclasses.py:87-106, populated as alg.py:71-112 does).
`caldera_groups` runs several such shape groups at once, all interleaved on HIP streams
(the layer-replacement caller's workload, main.py:146-196: every projection shape of the
selected layers, each layer with its own Hessian).
"""
from __future__ import annotations

import torch

from .engine import CalderaEngine, EngineParams, _Weights
from .overlap import default_parts, run_interleaved


def _diag_of(H: torch.Tensor, n: int) -> torch.Tensor:
    """diag(H) when H is a diagonal matrix (what main.py:163-165 passes: diag_embed of the
    per-channel Hessian) or already a 1-D diagonal; otherwise H itself (dense path)."""
    if H.dim() == 1:
        if H.shape[0] != n:
            raise ValueError(f"H diagonal has length {H.shape[0]}, expected {n}")
        return H
    if H.dim() != 2 or H.shape[0] != n or H.shape[1] != n:
        raise ValueError(f"H must be ({n}, {n}), got {tuple(H.shape)}")
    d = torch.diagonal(H)
    off = torch.count_nonzero(H) - torch.count_nonzero(d)
    if int(off.item()) != 0:
        return H.contiguous()
    return d.contiguous()


def _devices(device):
    dev_req = torch.device(device) if not isinstance(device, torch.device) else device
    comp = dev_req if dev_req.type == "cuda" else torch.device("cuda", torch.cuda.current_device())
    if comp.index is None:
        comp = torch.device("cuda", torch.cuda.current_device())
    return dev_req, comp


class _Group:
    """One same-shape batch: its stacked W on the compute device and its engine parts
    (indices into the batch, engine, generator)."""

    def __init__(self, quant_params, Ws, H, comp, *, scale_W, use_tqdm, engine_kwargs, streams, w_to_host=True):
        if isinstance(Ws, torch.Tensor) and Ws.dim() == 3:
            items = list(Ws.unbind(0))
            W = Ws
        else:
            items = list(Ws)
            W = None
        for w in items:
            if w.dim() != 2:
                raise ValueError("W must be a 2-D weight matrix")
        self.w_dev = items[0].device
        self.w_dtype = items[0].dtype
        if W is None:
            W = torch.stack([w.to(comp) for w in items])
        W = W.to(comp)
        if W.dtype not in (torch.float16, torch.float32):
            W = W.float()
        B, m, n = W.shape
        self.B, self.m, self.n = B, m, n
        params = EngineParams.from_caldera_params(quant_params)
        plan = []  # (indices, h) per engine part
        if isinstance(H, (list, tuple)):
            if len(H) != B:
                raise ValueError(f"{len(H)} per-matrix H for {B} matrices")
            hs = [None if x is None else _diag_of(x.to(comp).float(), n) for x in H]
            # groups: the same code-path flags for diagonals; each dense H alone
            kinds: dict = {}
            for b, x in enumerate(hs):
                key = ("dense", b) if (x is not None and x.dim() == 2) else _Weights.kind(x, n, params, comp)
                kinds.setdefault(key, []).append(b)
            for key, idx in kinds.items():
                if key[0] == "dense":
                    plan.append((idx, hs[idx[0]]))
                    continue
                if all(H[b] is None for b in idx):
                    hg = None            # H = I throughout: the shared (no-weights) form
                elif all(H[b] is H[idx[0]] for b in idx):
                    hg = hs[idx[0]]      # one Hessian object for the whole group: shared weights
                else:
                    hg = "per-matrix"
                k = max(1, min(int(streams if streams is not None else default_parts(len(idx))), len(idx)))
                bnd = [len(idx) * i // k for i in range(k + 1)]
                for i in range(k):
                    sub = idx[bnd[i]:bnd[i + 1]]
                    plan.append((sub, [hs[b] for b in sub] if hg == "per-matrix" else hg))
        else:
            h = None if H is None else _diag_of(H.to(comp).float(), n)  # (n,) diagonal or (n, n) dense
            k = max(1, min(int(streams if streams is not None else default_parts(B)), B))
            bnd = [B * i // k for i in range(k + 1)]
            plan = [(list(range(bnd[i], bnd[i + 1])), h) for i in range(k)]
        self.parts = []
        for i, (idx, hg) in enumerate(plan):
            if idx == list(range(idx[0], idx[0] + len(idx))):
                Wg = W[idx[0]:idx[0] + len(idx)]
            else:
                Wg = W.index_select(0, torch.tensor(idx, dtype=torch.long, device=comp))
            e = CalderaEngine(params, **(engine_kwargs or {}))
            self.parts.append((idx, e, e.run_iter(Wg, hg, scale_W, use_tqdm and i == 0, w_to_host=w_to_host)))

    def collect(self, part_results, dev_req, comp, decomposition_cls):
        res = [None] * self.B
        for (idx, _, _), part in zip(self.parts, part_results):
            for b, d in zip(idx, part):
                res[b] = d
        out = []
        lr_dev = dev_req if dev_req.type == "cpu" else comp
        w_dev, w_dtype, m, n = self.w_dev, self.w_dtype, self.m, self.n
        # alg.py:81 keeps W on the host: the engines copied it there while they ran (w_to_host)
        for d in res:
            dec = decomposition_cls(
                Q=d["Q"].to(w_dev),
                L=d["L"].to(lr_dev),
                R=d["R"].to(lr_dev),
            )
            dec.scaleWH = None
            dec.SU = torch.ones(n, dtype=w_dtype, device=w_dev)
            dec.SV = torch.ones(m, dtype=w_dtype, device=w_dev)
            dec.W = d["W"]
            for f in ("Q_idxs", "L_idxs", "R_idxs"):
                v = d[f]
                setattr(dec, f, v.to(lr_dev if f != "Q_idxs" else w_dev) if v is not None else None)
            for f in ("Q_scale", "L_scale", "R_scale"):
                v = d[f]
                setattr(dec, f, v.to(lr_dev if f != "Q_scale" else w_dev) if torch.is_tensor(v) else v)
            dec.errors = d["errors"]
            dec.global_scale = d["global_scale"]
            out.append(dec)
        return out


def _check_device():
    if not torch.cuda.is_available():
        raise RuntimeError("caldera-mi355x: no HIP device available (this engine has no CPU path)")


def caldera_batch(quant_params, Ws, H=None, *, device="cuda", use_tqdm=False, scale_W=True,
                  decomposition_cls=None, engine_kwargs=None, return_engine=False, streams=None):
    """Ws: list of (m, n) tensors or a (B, m, n) tensor.  H: None, (n,) diagonal, or (n, n), shared
    by the batch; or a list of B per-matrix H (each None, (n,) or (n, n)) -- the reference's
    own workload (main.py:163-196 calls caldera() per layer with that layer's Hall[name]).
    Per-matrix diagonals run in one lockstep batch (the kernels read each matrix's weights at
    a batch stride); matrices are grouped only by the flags that select code paths (H = I or
    not, unit error weights or not), a dense H runs as its own group, and the groups are
    interleaved on streams like the parts below.  A matrix's result is bit-identical to the
    same matrix in a batch of the same size whose H is shared.

    streams: number of parts the batch is split into, each decomposed by its own engine on
    its own HIP stream and interleaved at host-sync points (overlap.py).  Default
    `overlap.default_parts(B)`: 2 from 16 matrices on (one part's one-CU-per-matrix kernels and
    read-backs overlap the other's products: +5-14 % on configs 2-5), else 1.  Results do not
    depend on it beyond the solver tolerance (at large batches not at all: the parts take the
    same kernels as the whole batch).

    return_engine: also return the first part's engine; `eng.parts` lists every part's engine
    (each part's solver statistics cover its own matrices only)."""
    _check_device()
    if decomposition_cls is None:
        from .src.caldera.utils.dataclasses import CalderaDecomposition as decomposition_cls
    dev_req, comp = _devices(device)
    g = _Group(quant_params, Ws, H, comp, scale_W=scale_W, use_tqdm=use_tqdm, engine_kwargs=engine_kwargs,
               streams=streams)
    part_res = run_interleaved([gen for _, _, gen in g.parts], comp)
    out = g.collect(part_res, dev_req, comp, decomposition_cls)
    if return_engine:  # (a reference cycle: only when the caller asks for the engine)
        eng = g.parts[0][1]
        eng.parts = [e for _, e, _ in g.parts]
        return out, eng
    return out


def caldera_groups(quant_params, jobs, *, device="cuda", scale_W=True, decomposition_cls=None,
                   engine_kwargs=None, streams=None):
    """Several same-shape batches at once: jobs = [(Ws, H), ...] as caldera_batch takes them
    (H shared or per matrix).  Every group's engine parts run interleaved on their own HIP
    streams, so one shape's one-CU-per-matrix solves and read-backs overlap another shape's
    products.  Returns one list of CalderaDecomposition per job, in job order."""
    _check_device()
    if decomposition_cls is None:
        from .src.caldera.utils.dataclasses import CalderaDecomposition as decomposition_cls
    dev_req, comp = _devices(device)
    groups = [_Group(quant_params, Ws, H, comp, scale_W=scale_W, use_tqdm=False, engine_kwargs=engine_kwargs,
                     streams=streams) for Ws, H in jobs]
    gens = [gen for g in groups for _, _, gen in g.parts]
    res = run_interleaved(gens, comp)
    out, i = [], 0
    for g in groups:
        k = len(g.parts)
        out.append(g.collect(res[i:i + k], dev_req, comp, decomposition_cls))
        i += k
    return out
