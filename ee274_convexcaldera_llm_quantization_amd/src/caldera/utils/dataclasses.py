"""Drop-in for RCR/src/caldera/utils/dataclasses.py:1-113.

The three dataclasses callers construct and read — `CalderaParams` (:11-84),
`CalderaDecomposition` (:87-106) and `QuantInfo` (:109-113) — are generated here from field
tables: same field names, order, types and defaults (so the same constructor signatures and
`dataclasses.fields()`), built with `dataclasses.make_dataclass`.
"""
from dataclasses import dataclass, field, make_dataclass  # noqa: F401  (star-exported like the reference's)

import torch

from .quantization import (
    QuantizerFactory,
    AbstractQuantizer,
    LowMemoryQuantizer,
)


def _spec(name, typ, default=None, factory=None, doc=None):
    meta = {"help": doc} if doc else {}
    f = field(default_factory=factory, metadata=meta) if factory is not None else field(default=default, metadata=meta)
    return (name, typ, f)


_BITS = "quantisation bit width"

# dataclasses.py:11-84 — defaults as the reference's (update_order [] = no updates at all)
_PARAMS = [
    _spec("compute_quantized_component", bool, True, doc="include the quantised full-size component Q"),
    _spec("compute_low_rank_factors", bool, True, doc="include the low-rank factors L, R"),
    _spec("Q_bits", int, 2, doc=_BITS),
    _spec("L_bits", int, 2, doc=_BITS),
    _spec("R_bits", int, 2, doc=_BITS),
    _spec("rank", int, 64, doc="rank of L and R"),
    _spec("iters", int, 20),
    _spec("lplr_iters", int, 5),
    _spec("activation_aware_LR", bool, True, doc="activation-aware LPLR factors"),
    _spec("update_order", list[str], factory=list, doc='order of the "Q" / "LR" updates per iteration'),
    _spec("quant_factory_Q", QuantizerFactory, factory=QuantizerFactory, doc="quantiser factory for Q"),
    _spec("quant_factory_LR", QuantizerFactory, factory=QuantizerFactory, doc="quantiser factory for L and R"),
    _spec("rand_svd", bool, False, doc="randomised SVD (svd_lowrank) for the LR initialisation"),
    _spec("sigma_reg", float, 0, doc="eigenvalue floor that makes H positive definite"),
]

# dataclasses.py:87-106 — every field optional; scales 1 until a quantiser sets them
_DECOMP = [(n, torch.Tensor, None) for n in ("Q", "L", "R", "W", "Q_idxs", "L_idxs", "R_idxs")]
_DECOMP += [(n, float, 1) for n in ("Q_scale", "L_scale", "R_scale", "global_scale")]
_DECOMP += [(n, torch.Tensor, None) for n in ("SU", "SV", "scaleWH")]

CalderaParams = make_dataclass("CalderaParams", _PARAMS, namespace={"__module__": __name__})
CalderaParams.__doc__ = "Parameters for the CALDERA decomposition (dataclasses.py:11-84)."

CalderaDecomposition = make_dataclass(
    "CalderaDecomposition",
    [(n, t, field(default=d)) for n, t, d in _DECOMP] + [("errors", dict[str, list[float]], field(default_factory=dict))],
    namespace={"__module__": __name__},
)
CalderaDecomposition.__doc__ = "Components and parameters of a CALDERA decomposition (dataclasses.py:87-106)."

QuantInfo = make_dataclass("QuantInfo", [("quant", AbstractQuantizer, field(default_factory=LowMemoryQuantizer))],
                           namespace={"__module__": __name__})
QuantInfo.__doc__ = "Quantisation-specific information (dataclasses.py:109-113)."
