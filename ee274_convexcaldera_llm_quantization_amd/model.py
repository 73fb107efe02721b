"""Layer-replacement caller: the reference's `apply_CALDERA_quantization`
(`main.py:135-251`) on the MI355X engine.

The reference walks `model.named_modules()`, and for each selected language-model
projection forms `H = diag_embed(Hall[name])` (main.py:163-165), runs `caldera()` with the
driver's parameters (main.py:167-182, `scale_W=False`), writes `out = Q + L @ R` back into
the module (main.py:199-202), and undoes the write when the relative Frobenius error
`||W - out|| / ||W||` exceeds `error_threshold` (main.py:212-220).  Everything else with a
weight is counted as unquantised language or vision parameters (main.py:242-251), and the
bit accounting of main.py:321-329 is reported.

Here the selection and accounting are the reference's (including its substring layer match,
`any(f'layers.{i}' in name ...)`, main.py:158), the Hessian diagonal is passed as a vector
(no n x n diag_embed), `Q + L R` is one fused HIP GEMM epilogue, and the Hadamard branch
(main.py:224-240, `H1 W H2` with normalised Sylvester matrices padded to powers of two) runs
as HIP GEMMs on the device instead of numpy on the host.  Layers that share a shape are
decomposed in one lockstep batch, each with its own Hessian diagonal (the engine reads
per-matrix weights at a batch stride; api.caldera_batch groups by code-path flags and
interleaves the groups on HIP streams), where the reference runs one caldera() per layer.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Sequence

import torch

from . import _lib as K

PROJ_KEYS = ("mlp.up_proj", "mlp.down_proj", "mlp.gate_proj", "q_proj", "k_proj", "v_proj", "o_proj")


@dataclass
class LayerSelection:
    """main.py:1-7, 147-160: which modules are decomposed."""
    scope: str = "language"                         # `'language' in name` (main.py:150)
    keys: Sequence[str] = PROJ_KEYS                 # main.py:155
    layers: Sequence[int] | None = tuple(range(17, 24))  # quantize_layer_start..end (main.py:2-4)
    min_dim: int = 500                              # both dims > 500 (main.py:157-158)
    limit: int = 10000                              # quantized_layer_limit (main.py:6)

    def in_scope(self, name: str, module) -> bool:
        return hasattr(module, "weight") and module.weight is not None and self.scope in name

    def selects(self, name: str, weight: torch.Tensor, counter: int) -> bool:
        return (any(k in name for k in self.keys)
                and weight.dim() == 2 and weight.size(0) > self.min_dim and weight.size(1) > self.min_dim
                and (self.layers is None or any(f"layers.{i}" in name for i in self.layers))
                and counter <= self.limit)


def driver_params(rank: int = 200):
    """The CalderaParams main.py:167-182 builds for every layer."""
    from .src.caldera.utils.dataclasses import CalderaParams
    from .src.caldera.utils.quantization import QuantizerFactory
    return CalderaParams(compute_quantized_component=True, compute_low_rank_factors=True, Q_bits=2,
                         L_bits=16, R_bits=16, rank=rank, iters=5, lplr_iters=5, activation_aware_LR=True,
                         update_order=["Q", "LR"],
                         quant_factory_Q=QuantizerFactory(method="uniform", block_size=64),
                         quant_factory_LR=QuantizerFactory(method="uniform", block_size=64),
                         rand_svd=False, sigma_reg=1e-8)


@dataclass
class LayerOutcome:
    name: str
    shape: tuple
    rel_error: float          # ||W - out||_F / ||W||_F (main.py:212)
    applied: bool             # False: error above the threshold, W restored (main.py:214-216)
    errors: dict = field(default_factory=dict)


@dataclass
class QuantizationReport:
    """Counters of main.py:140-143, 217-251 and the bit accounting of main.py:321-329."""
    quantized_param_count: int = 0
    unquantized_language_param_count: int = 0
    vision_param_count: int = 0
    layers: list = field(default_factory=list)
    skipped: list = field(default_factory=list)

    @property
    def total_bits(self) -> int:  # main.py:324 (2-bit quantised, 4-bit the rest)
        return self.quantized_param_count * 2 + self.unquantized_language_param_count * 4

    @property
    def prior_total_bits(self) -> int:  # main.py:326
        return self.quantized_param_count * 4 + self.unquantized_language_param_count * 4

    @property
    def bit_ratio(self) -> float | None:  # main.py:328-329
        d = self.prior_total_bits
        return self.total_bits / d if d else None

    @property
    def quantized_fraction(self) -> float | None:  # main.py:330
        d = self.quantized_param_count + self.unquantized_language_param_count
        return self.quantized_param_count / d if d else None


# ---------------------------------------------------------------------------- Hadamard
def normalized_hadamard(n: int, device, dtype=torch.float32) -> torch.Tensor:
    """Sylvester Hadamard / sqrt(n) (scipy.linalg.hadamard ordering, main.py:94-98)."""
    if n < 1 or n & (n - 1):
        raise ValueError("Hadamard order must be a power of two")
    Hm = torch.ones((1, 1), dtype=dtype, device=device)
    while Hm.shape[0] < n:
        Hm = torch.cat([torch.cat([Hm, Hm], 1), torch.cat([Hm, -Hm], 1)], 0)
    return Hm * (1.0 / math.sqrt(n))


def _next_pow2(n: int) -> int:
    return 1 << (n - 1).bit_length()


def hadamard_transform(W: torch.Tensor, inverse: bool = False, original_shape=None):
    """main.py:108-133 on the device: forward pads W to powers of two and returns
    (H1 W H2, (rows, cols)); inverse returns (H1 W H2)[:rows, :cols] (H symmetric and
    orthogonal).  Two fp32 HIP GEMMs."""
    rows, cols = (W.shape if not inverse else original_shape)
    pr, pc = _next_pow2(rows), _next_pow2(cols)
    dev = W.device
    H1, H2 = normalized_hadamard(pr, dev), normalized_hadamard(pc, dev)
    if inverse:
        Wp = W.float().contiguous()
    else:
        Wp = torch.zeros((pr, pc), dtype=torch.float32, device=dev)
        Wp[:rows, :cols] = W.float()
    T = K.gemm(H1, Wp, C=torch.empty((pr, pc), dtype=torch.float32, device=dev))
    out = K.gemm(T, H2, C=torch.empty((pr, pc), dtype=torch.float32, device=dev))
    if inverse:
        return out[:rows, :cols]
    return out, (rows, cols)


# ---------------------------------------------------------------------------- caller
def _reconstruct(dec, dev) -> torch.Tensor:
    """out = Q + L @ R (main.py:198) as one HIP GEMM with a D-epilogue, fp32."""
    Q = dec.Q.to(dev).float().contiguous()
    L = dec.L.to(dev).float().contiguous()
    R = dec.R.to(dev).float().contiguous()
    return K.gemm(L, R, C=torch.empty_like(Q), D=Q, gamma=1.0)


def _rel_error(W: torch.Tensor, out: torch.Tensor) -> float:
    """||W - out||_F / ||W||_F with fp64 sums (cq_weighted_sqsum)."""
    Wf = W.float().contiguous()
    num = K.weighted_sqsum((Wf - out).unsqueeze(0), None, Wf.shape[1])
    den = K.weighted_sqsum(Wf.unsqueeze(0), None, Wf.shape[1])
    return float(torch.sqrt(num / den).item())


def select_layers(model: torch.nn.Module, hessians=None, selection: LayerSelection | None = None,
                  log: Callable | None = None):
    """The module walk of main.py:146-251 without the decomposition: returns the jobs
    [(name, module, h)] in named_modules order and a report holding the unquantised-language
    and vision counters (quantised ones are added as jobs complete)."""
    sel = selection or LayerSelection()
    say = log or (lambda *a: None)
    rep = QuantizationReport()
    jobs = []
    counter = 1
    for name, module in model.named_modules():
        if sel.in_scope(name, module):
            w = module.weight
            if sel.selects(name, w, counter):
                h = None
                if hessians is not None:
                    h = hessians[name]  # main.py:163: KeyError for a layer without a Hessian
                counter += 1
                jobs.append((name, module, h))
            else:
                rep.unquantized_language_param_count += w.numel()
                rep.skipped.append(name)
                say(f"Skipped quantization for {name} with shape {tuple(w.size())}")
        elif hasattr(module, "weight") and module.weight is not None:
            rep.vision_param_count += module.weight.numel()
            say(f"Skipped quantization for {name} with shape {tuple(module.weight.size())}")
    return jobs, rep


def apply_caldera_quantization(model: torch.nn.Module, hessians=None, quant_params=None, *,
                               selection: LayerSelection | None = None, error_threshold: float = 0.99,
                               scale_W: bool = False, hadamard: bool = False, device="cuda",
                               max_batch: int = 64, keep_dtype: bool = True, decompose: Callable | None = None,
                               log: Callable | None = None, hadamard_gate: bool = False) -> QuantizationReport:
    """main.py:135-251 on the MI355X engine.

    hessians: {module name: diagonal (n,) or dense (n, n)} — `Hall` (a missing name raises
      KeyError as `Hall[name]` does); None: H = I for every layer.
    quant_params: CalderaParams (default `driver_params()`, main.py:167-182).
    keep_dtype: write `out` back in the weight's dtype (the reference assigns the fp32 `out`,
      main.py:199, which only matters for a non-fp32 model).
    hadamard_gate: apply the 0.99 error gate and the bit accounting to the Hadamard branch
      too (off by default: main.py:221-240 writes the recovered weight unconditionally and
      counts nothing).
    decompose(quant_params, Ws, H) -> list of CalderaDecomposition: the engine unless given
      (tests pass a stand-in).  The engine runs every shape batch at once
      (`api.caldera_groups`: all batches interleaved on HIP streams).
    Returns the QuantizationReport (counters + per-layer outcomes)."""
    qp = quant_params if quant_params is not None else driver_params()
    say = log or (lambda *a: None)
    jobs, rep = select_layers(model, hessians, selection, say)
    # batches: same shape; every layer keeps its own Hessian (a list of per-matrix H, or one
    # shared H / None when the whole batch has the same object)
    groups: dict = {}
    for job in jobs:
        groups.setdefault(tuple(job[1].weight.shape), []).append(job)
    outcomes = {}
    batches = []  # (jobs, Ws, shapes, H)
    with torch.no_grad():
        for key, members in groups.items():
            for s in range(0, len(members), max_batch):
                part = members[s:s + max_batch]
                h = part[0][2] if all(j[2] is part[0][2] for j in part) else [j[2] for j in part]
                Ws, shapes = [], []
                for name, module, hj in part:
                    W = module.weight.data
                    if hadamard:  # main.py:224-232: transform, decompose the fp32 transform
                        if hj is not None and _next_pow2(W.shape[1]) != W.shape[1]:
                            raise ValueError(f"{name}: Hadamard padding changes n ({W.shape[1]}) but H is n x n")
                        Wt, shp = hadamard_transform(W.to(device))
                        Ws.append(Wt)
                        shapes.append(shp)
                    else:
                        Ws.append(W)
                batches.append((part, Ws, shapes, h))
        if decompose is None:
            from .api import caldera_groups
            all_decs = caldera_groups(qp, [(Ws, h) for _, Ws, _, h in batches], device=device, scale_W=scale_W)
        else:
            all_decs = [decompose(qp, Ws, h) for _, Ws, _, h in batches]
    for (part, Ws, shapes, h), decs in zip(batches, all_decs):
        with torch.no_grad():
            for (name, module, _), dec, i in zip(part, decs, range(len(part))):
                W = module.weight.data
                dev = W.device if W.device.type == "cuda" else torch.device(device)
                out = _reconstruct(dec, dev)
                if hadamard:
                    out = hadamard_transform(out, inverse=True, original_shape=shapes[i]).contiguous()
                err = _rel_error(W.to(dev), out)
                if hadamard and not hadamard_gate:
                    # main.py:221-240: the Hadamard branch always writes the recovered
                    # weight back, with no error gate and no parameter counting
                    module.weight.data = out.to(W.dtype).to(W.device)
                    say(f"Applied CALDERA (Hadamard) to {name}.weight, shape: {tuple(W.shape)}")
                    outcomes[name] = LayerOutcome(name, tuple(W.shape), err, True, dict(dec.errors))
                    continue
                ok = err <= error_threshold
                if ok:
                    module.weight.data = (out.to(W.dtype) if keep_dtype else out).to(W.device)
                    rep.quantized_param_count += W.numel()
                    say(f"Applied CALDERA to {name}.weight, shape: {tuple(W.shape)}")
                else:
                    rep.unquantized_language_param_count += W.numel()
                    say(f"Error of the decomposition is greater than threshold for {name}. Skipping quantization")
                outcomes[name] = LayerOutcome(name, tuple(W.shape), err, ok, dict(dec.errors))
    rep.layers = [outcomes[j[0]] for j in jobs]
    return rep
