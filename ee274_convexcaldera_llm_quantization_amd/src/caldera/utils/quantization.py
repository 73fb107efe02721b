"""Drop-in for RCR/src/caldera/utils/quantization.py (QuantizerFactory / LowMemoryQuantizer).

Same names, constructor arguments, return layouts and exceptions as the reference
(quantization.py:7-319); the arithmetic runs in libcaldera_hip.so on the HIP device.  A CPU
tensor is quantised on the current HIP device and the results are returned on the CPU;
without a HIP device the call raises (there is no CPU fallback).
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import List

import torch

from ._engine_import import kernels as _K
from ._engine_import import qlog as _qlog

_BITWIDTHS = [2, 4, 8, 16]
_QUANTIZER_METHODS = ["uniform", "nf4", "nf2", "bbint4", "bbint2"]


class AbstractQuantizer(ABC):
    @abstractmethod
    def quantize_block(self, weight): ...

    @abstractmethod
    def dequantize_block(self, weight_quant, weight_params, weight_shape): ...


def _to_device(t: torch.Tensor):
    if t.is_cuda:
        return t, None
    if not torch.cuda.is_available():
        raise RuntimeError("caldera-mi355x: no HIP device available (this engine has no CPU path)")
    return t.to(torch.device("cuda", torch.cuda.current_device())), t.device


def bbint_bits(method: str) -> int:
    """Packing width of a bbint method (quantization.py:151 two codes per byte, :218-221 four)."""
    return 4 if method == "bbint4" else 2


class LowMemoryQuantizer(AbstractQuantizer):
    """quantization.py:18-307.  Every method (uniform, nf4, nf2, bbint4, bbint2) runs in
    libcaldera_hip.so on the HIP device; codes, scales and parameter tuples have the
    reference's shapes and dtypes."""

    def __init__(self, num_bits: int = 2, method: str = "uniform", block_size: int = 64):
        self.num_bits = num_bits
        assert self.num_bits in _BITWIDTHS, "Bit-width not supported!"
        self.method = method.lower()
        if self.method not in _QUANTIZER_METHODS:
            raise NotImplementedError(f"Quantization method '{self.method}' not supported yet.")
        self.block_size = block_size
        if self.method == "nf4" and self.num_bits != 4:
            raise ValueError("NF4 quantization supports only 4 bits.")
        if self.method == "nf2" and self.num_bits != 2:
            raise ValueError("NF2 quantization supports only 2 bits.")
        if self.method == "bbint4" and self.num_bits != 4:
            raise ValueError("bbint4 quantization supports only 4 bits.")

    def quantize_block(self, weight: torch.Tensor, epsilon: float = 1e-8):
        if len(weight.shape) != 2:
            raise ValueError(
                f"Support only for 2D matrix, but your input has {len(weight.shape)} dimensions."
            )
        total = weight.shape[0] * weight.shape[1]
        if total % self.block_size != 0:
            raise ValueError(
                f"Weight with shape {weight.shape[0]} x {weight.shape[1]} "
                f"is not divisible by block size {self.block_size}"
            )
        x, home = _to_device(weight)
        # reduced-precision inputs are promoted by the reference (maximum with an fp32 eps)
        x = x.detach().to(torch.float32).contiguous().view(1, total)
        bs = self.block_size

        def back(t):
            return t.to(home) if home is not None else t

        if self.method == "uniform":
            out = _K.quantize_uniform(x, bs, self.num_bits, epsilon, codes=True, deq=False)
            return back(out["codes"].view(-1, bs)), back(out["scale"].view(-1, 1)), weight.shape
        if self.method in ("nf4", "nf2"):
            out = _K.quantize_nf(x, bs, 4 if self.method == "nf4" else 2, epsilon, idx=True, deq=False)
            return back(out["idx"].view(-1, bs)), back(out["scale"].view(-1, 1)), weight.shape
        bits = bbint_bits(self.method)
        if bs % (8 // bits):
            raise RuntimeError(f"{self.method}: block size {bs} is not a multiple of {8 // bits} "
                               f"(the reference's strided packing fails on this shape)")
        out = _K.quantize_bbint(x, bs, bits, epsilon, packed=True, deq=False)
        _qlog.log_outliers(id(self), out["n_out"][0])
        params = (back(out["bmin"].view(-1, 1)), back(out["bscale"].view(-1, 1)), back(out["vals"]),
                  back(out["idx"]))
        return back(out["packed"].view(-1, bs * bits // 8)), params, weight.shape

    def dequantize_block(self, weight_quant: torch.Tensor, weight_params, weight_shape: List[int]):
        c, home = _to_device(weight_quant)
        c = c.contiguous()
        if self.method == "uniform":
            s, _ = _to_device(weight_params)
            out = _K.dequantize_uniform(c, s.contiguous().float(), self.num_bits)
        elif self.method in ("nf4", "nf2"):
            s, _ = _to_device(weight_params)
            out = _K.dequantize_nf(c.to(torch.uint8), s.contiguous().float(), 4 if self.method == "nf4" else 2)
        elif self.method in ("bbint4", "bbint2"):
            bits = bbint_bits(self.method)
            bmin, bscale, vals, idx = (_to_device(t)[0] for t in weight_params)
            nblk = bmin.numel()
            bs = c.numel() * 8 // bits // nblk
            out = _K.dequantize_bbint(c.to(torch.uint8), bits, bmin.contiguous().float(),
                                      bscale.contiguous().float(), vals.contiguous().float(),
                                      idx.contiguous(), bs)
        else:
            raise NotImplementedError(f"Dequantization method '{self.method}' not implemented.")
        out = out.view(-1).reshape(weight_shape)
        return out.to(home) if home is not None else out


class QuantizerFactory:
    def __init__(self, method="uniform", block_size=64):
        self.method = method
        self.block_size = block_size

    def get_quantizer(self, num_bits, device="cpu"):
        return LowMemoryQuantizer(num_bits=num_bits, method=self.method, block_size=self.block_size)

    def __str__(self):
        return f"QuantizerFactory(method={self.method}, block_size={self.block_size})"
