"""Batched entry point behind the drop-in `caldera()` (src/caldera/decomposition/alg.py).

`caldera_batch` decomposes several same-shape weight matrices in lockstep on one HIP
device (the throughput path used by bench.py and the multi-GPU sharder) and returns one
CalderaDecomposition per matrix with the reference's field layout
(RCR/src/caldera/utils/dataclasses.py:87-106, populated as alg.py:71-112 does).
"""
from __future__ import annotations

import torch

from .engine import CalderaEngine, EngineParams
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


def caldera_batch(quant_params, Ws, H=None, *, device="cuda", use_tqdm=False, scale_W=True,
                  decomposition_cls=None, engine_kwargs=None, return_engine=False, streams=None):
    """Ws: list of (m, n) tensors or a (B, m, n) tensor.  H: None, (n,) diagonal, or (n, n).

    streams: number of parts the batch is split into, each decomposed by its own engine on
    its own HIP stream and interleaved at host-sync points (overlap.py).  Default
    `overlap.default_parts(B)`: 2 from 16 matrices on (one part's one-CU-per-matrix kernels and
    read-backs overlap the other's products: +5-14 % on configs 2-5), else 1.  Results do not
    depend on it beyond the solver tolerance (at large batches not at all: the parts take the
    same kernels as the whole batch)."""
    if not torch.cuda.is_available():
        raise RuntimeError("caldera-mi355x: no HIP device available (this engine has no CPU path)")
    if decomposition_cls is None:
        from .src.caldera.utils.dataclasses import CalderaDecomposition as decomposition_cls
    dev_req = torch.device(device) if not isinstance(device, torch.device) else device
    comp = dev_req if dev_req.type == "cuda" else torch.device("cuda", torch.cuda.current_device())
    if comp.index is None:
        comp = torch.device("cuda", torch.cuda.current_device())
    if isinstance(Ws, torch.Tensor) and Ws.dim() == 3:
        items = list(Ws.unbind(0))
        W = Ws
    else:
        items = list(Ws)
        W = None
    for w in items:
        if w.dim() != 2:
            raise ValueError("W must be a 2-D weight matrix")
    w_dev = items[0].device
    w_dtype = items[0].dtype
    if W is None:
        W = torch.stack([w.to(comp) for w in items])
    W = W.to(comp)
    if W.dtype not in (torch.float16, torch.float32):
        W = W.float()
    B, m, n = W.shape
    h = None if H is None else _diag_of(H.to(comp).float(), n)  # (n,) diagonal or (n, n) dense
    params = EngineParams.from_caldera_params(quant_params)
    if streams is None:
        streams = default_parts(B)
    streams = max(1, min(int(streams), B))
    bounds = [B * i // streams for i in range(streams + 1)]
    engines = [CalderaEngine(params, **(engine_kwargs or {})) for _ in range(streams)]
    gens = [e.run_iter(W[bounds[i]:bounds[i + 1]], h, scale_W, use_tqdm and i == 0, w_to_host=True)
            for i, e in enumerate(engines)]
    res = [d for part in run_interleaved(gens, comp) for d in part]
    eng = engines[0]
    if return_engine:  # (a reference cycle: only when the caller asks for the engine)
        eng.parts = engines
    out = []
    lr_dev = dev_req if dev_req.type == "cpu" else comp
    # alg.py:81 keeps W on the host: the engines copied it there while they ran (w_to_host)
    for b, d in enumerate(res):
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
    if return_engine:
        return out, eng
    return out
