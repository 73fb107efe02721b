"""Drop-in for RCR/src/caldera/decomposition/alg.py — `caldera()` on MI355X.

Importable exactly as the reference's callers do (main.py:20-23, caldera_playbook.ipynb):
    sys.path.append('<repo>/ee274_convexcaldera_llm_quantization_amd')
    from src.caldera.utils.dataclasses import CalderaParams
    from src.caldera.utils.quantization import QuantizerFactory
    from src.caldera.decomposition.alg import caldera
Like the reference (alg.py:8-9) this module star-exports the dataclasses and quantisers.
"""
import torch
from collections import namedtuple

from ..utils.dataclasses import *  # noqa: F401,F403  (alg.py:8)
from ..utils.quantization import *  # noqa: F401,F403  (alg.py:9)
from ..utils.dataclasses import CalderaParams, CalderaDecomposition, QuantInfo
from ..utils.quantization import QuantizerFactory
from ..utils._engine_import import api as _api


def caldera(
    quant_params: CalderaParams,
    W: torch.Tensor,
    H: torch.Tensor = None,
    device: str = "cuda",
    use_tqdm: bool = True,
    scale_W: bool = True,
):
    """Runs the CALDERA algorithm (alg.py:24-112), decomposing W into Q + LR.

    Computation always runs on the HIP device (device="cuda" on ROCm torch is the MI355X);
    output placement follows the reference: Q on W's device, L/R on `device`, W (scaled)
    on the CPU.  H may be None, diagonal (diag_embed(h), what main.py:163-165 passes: fused
    column weights) or dense (one device eigendecomposition, then GEMM transforms)."""
    return _api.caldera_batch(quant_params, [W], H, device=device, use_tqdm=use_tqdm,
                              scale_W=scale_W, decomposition_cls=CalderaDecomposition)[0]


def get_quant_info(quant_factory: QuantizerFactory, bits: int, device: str):
    """alg.py:238-242."""
    return QuantInfo(quant=quant_factory.get_quantizer(bits, device))


def quantize_matrix(A, quant_params, quant_info: QuantInfo = None):
    """alg.py:245-250: whole-matrix block, quantise + dequantise."""
    QuantReturn = namedtuple("QuantReturn", ["A_hat", "A_idxs", "scale"])
    quant_info.quant.block_size = A.shape[0] * A.shape[1]
    A_idxs, scales, shape = quant_info.quant.quantize_block(A)
    A_hat = quant_info.quant.dequantize_block(A_idxs, scales, shape)
    return QuantReturn(A_hat, A_idxs, scales)
