"""ctypes binding of libcaldera_hip.so (include/caldera_hip.h) + thin torch-tensor wrappers.

PyTorch is plumbing here: it owns device memory (caching allocator workspaces), the HIP
stream (`torch.cuda.current_stream().cuda_stream`) and RNG.  Every arithmetic step of the
hot path goes through one of the C-ABI entry points below; there is no torch or CPU
fallback — a missing library or a non-HIP tensor raises.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import threading

import torch

from . import scratch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libcaldera_hip.so")

CQ_F32, CQ_F16, CQ_BF16, CQ_F64 = 0, 1, 2, 3
EPI_LINEAR, EPI_RESID, EPI_WERR = 0, 1, 2
CQ_EINVAL, CQ_EHIP, CQ_EWORKSPACE = -1, -2, -3

c_i64, c_int, c_float, c_double, c_size, c_vp = (ctypes.c_int64, ctypes.c_int, ctypes.c_float,
                                                 ctypes.c_double, ctypes.c_size_t, ctypes.c_void_p)


class GemmArgs(ctypes.Structure):
    _fields_ = [
        ("M", c_i64), ("N", c_i64), ("K", c_i64), ("batch", c_i64),
        ("trans_a", c_int), ("trans_b", c_int),
        ("A", c_vp), ("lda", c_i64), ("stride_a", c_i64),
        ("B", c_vp), ("ldb", c_i64), ("stride_b", c_i64),
        ("C", c_vp), ("ldc", c_i64), ("stride_c", c_i64),
        ("D", c_vp), ("ldd", c_i64), ("stride_d", c_i64), ("d_f16", c_int),
        ("alpha", c_float), ("beta", c_float), ("gamma", c_float),
        ("alpha_v", c_vp), ("beta_v", c_vp), ("gamma_v", c_vp),
        ("epi", c_int),
        ("absmax_bits", c_vp),
        ("w", c_vp), ("stride_w", c_i64),
        ("err_out", c_vp),
        ("syrk", c_int),
        ("b_triu", c_int),
    ]


class X3Args(ctypes.Structure):
    _fields_ = [
        ("M", c_i64), ("N", c_i64), ("K", c_i64), ("batch", c_i64),
        ("Ah", c_vp), ("Al", c_vp), ("lda", c_i64), ("stride_a", c_i64),
        ("Bh", c_vp), ("Bl", c_vp), ("ldb", c_i64), ("stride_b", c_i64),
        ("inv_scale", c_vp),
        ("C", c_vp), ("ldc", c_i64), ("stride_c", c_i64),
        ("P", c_vp), ("ldp", c_i64), ("stride_p", c_i64),
        ("D", c_vp), ("ldd", c_i64), ("stride_d", c_i64),
        ("alpha_v", c_vp), ("beta_v", c_vp), ("gamma_v", c_vp),
        ("out_h", c_vp), ("out_l", c_vp), ("ldo", c_i64), ("stride_o", c_i64),
        ("out_scale", c_float),
        ("overflow", c_vp),
        ("tri", c_int),
        ("b_blocked", c_int),
        ("active", c_vp),
        ("a_blocked", c_int),
        ("o_blocked", c_int),
        ("sym_out", c_int),
        ("out_bound", c_vp),
        ("scale_out", c_vp),
        ("inv_out", c_vp),
        ("single", c_int),
        ("ksplit", c_int),
        ("split_ws", c_vp),
        ("b_exact", c_int),
        ("colw", c_vp),
        ("absmax_out", c_vp),
        ("Ct", c_vp),
        ("stride_ct", c_i64),
        ("stride_colw", c_i64),
    ]


_SIGS = {
    "cq_abi_version": (c_int, []),
    "cq_last_error": (ctypes.c_char_p, []),
    "cq_rms_scale_workspace": (c_size, [c_i64, c_i64]),
    "cq_rms_scale": (c_int, [c_int, c_vp, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_size, c_vp]),
    "cq_quantize_workspace": (c_size, [c_i64, c_i64, c_i64]),
    "cq_quantize_uniform": (c_int, [c_vp, c_i64, c_i64, c_i64, c_int, c_float, c_vp, c_vp, c_vp,
                                    c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_size, c_vp]),
    "cq_quantize_uniform_known_max": (c_int, [c_vp, c_i64, c_i64, c_int, c_float, c_vp, c_vp, c_vp,
                                              c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_size, c_vp]),
    "cq_unpack_codes": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp]),
    "cq_quantize_nf_workspace": (c_size, [c_i64, c_i64, c_i64]),
    "cq_quantize_nf": (c_int, [c_vp, c_i64, c_i64, c_i64, c_int, c_float, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                               c_vp, c_vp, c_size, c_vp]),
    "cq_dequant_nf": (c_int, [c_vp, c_vp, c_i64, c_i64, c_int, c_vp, c_vp]),
    "cq_bbint_workspace": (c_size, [c_i64, c_i64, c_i64]),
    "cq_bbint_stats": (c_int, [c_vp, c_i64, c_i64, c_i64, c_int, c_float, c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    "cq_bbint_emit": (c_int, [c_vp, c_i64, c_i64, c_i64, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                              c_i64, c_vp, c_vp, c_size, c_vp]),
    "cq_dequant_bbint": (c_int, [c_vp, c_int, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_i64, c_vp, c_vp]),
    "cq_dequant_uniform": (c_int, [c_vp, c_int, c_vp, c_i64, c_i64, c_int, c_vp, c_vp]),
    "cq_build_residual": (c_int, [c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp,
                                  c_vp, c_vp]),
    "cq_gemm_workspace": (c_size, [ctypes.POINTER(GemmArgs)]),
    "cq_gemm_f32": (c_int, [ctypes.POINTER(GemmArgs), c_vp, c_size, c_vp]),
    "cq_gram_f64_workspace": (c_size, [c_i64, c_i64, c_i64, c_i64]),
    "cq_gram_f64": (c_int, [c_i64, c_i64, c_i64, c_i64, c_vp, c_int, c_i64, c_i64, c_vp, c_int, c_i64,
                            c_i64, c_vp, c_vp, c_size, c_vp]),
    "cq_spd_whiten": (c_int, [c_vp, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp]),
    "cq_spd_whiten_rcond": (c_int, [c_vp, c_i64, c_i64, c_double, c_vp, c_vp, c_vp, c_vp]),
    "cq_jacobi_workspace": (c_size, [c_i64, c_i64]),
    "cq_jacobi_eigh": (c_int, [c_vp, c_i64, c_i64, c_int, c_double, c_vp, c_vp, c_vp, c_vp, c_vp,
                               c_size, c_vp]),
    "cq_jacobi_staged_workspace": (c_size, [c_i64, c_i64]),
    "cq_jacobi_eigh_staged": (c_int, [c_vp, c_i64, c_i64, c_int, c_int, c_double, c_int, c_vp, c_vp, c_vp, c_vp,
                                      c_vp, c_vp, c_size, c_vp]),
    "cq_extreme_eigs": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp]),
    "cq_ritz_workspace": (c_size, [c_i64, c_i64, c_i64]),
    "cq_ritz_residual": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_size,
                                 c_vp]),
    "cq_weighted_sqsum": (c_int, [c_int, c_vp, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_vp, c_size, c_vp]),
    "cq_scale_rc": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_i64, c_i64, c_i64, c_i64, c_i64, c_vp,
                            c_i64, c_vp, c_i64, c_vp]),
    "cq_sym_split_f16": (c_int, [c_vp, c_i64, c_i64, c_int, c_int, c_float, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "cq_transpose_split": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_float, c_vp, c_int, c_vp]),
    "cq_gemm_triu_split": (c_int, [c_vp, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_float, c_vp]),
    "cq_pow2_scale": (c_int, [c_vp, c_i64, c_i64, c_int, c_vp, c_vp]),
    "cq_split_f16": (c_int, [c_vp, c_i64, c_i64, c_vp, c_float, c_vp, c_vp, c_i64, c_vp]),
    "cq_gemm_x3": (c_int, [ctypes.POINTER(X3Args), c_vp]),
    "cq_q_update_workspace": (c_size, [c_i64, c_i64, c_i64, c_int]),
    "cq_q_update_list_geometry": (c_int, [c_i64, c_i64, c_i64, c_vp, c_vp, c_vp]),
    "cq_absmax": (c_int, [c_int, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "cq_residual_split_workspace": (c_size, [c_i64, c_i64, c_i64]),
    "cq_residual_split": (c_int, [c_int, c_vp, c_vp, c_vp, c_int, c_vp, c_float, c_vp, c_i64, c_i64, c_i64, c_vp, c_vp,
                                  c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_float, c_vp, c_i64, c_vp, c_vp, c_vp,
                                  c_size, c_vp]),
    "cq_sgram_count": (c_int, [c_vp, c_int, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp,
                               c_vp, c_i64, c_vp, c_vp, c_vp]),
    "cq_sgram_fill": (c_int, [c_vp, c_int, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp]),
    "cq_sgram_rows": (c_int, [c_i64]),
    "cq_pow2_from_absmax": (c_int, [c_vp, c_i64, c_int, c_vp]),
    "cq_sgram_split": (c_i64, [c_i64, c_i64]),
    "cq_sgram_spmm": (c_int, [c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_i64,
                              c_i64, c_vp, c_vp]),
    "cq_sgram_combine": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_vp, c_float, c_vp, c_vp, c_vp, c_vp, c_vp,
                                 c_vp]),
    "cq_codes_transpose": (c_int, [c_vp, c_int, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "cq_codes_matmul": (c_int, [c_vp, c_int, c_i64, c_i64, c_i64, c_vp, c_i64, c_i64, c_vp, c_i64, c_vp, c_i64, c_i64,
                                c_vp, c_i64, c_i64, c_int, c_vp]),
    "cq_codes_ysq_corr": (c_int, [c_vp, c_int, c_vp, c_int, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "cq_transpose_f16": (c_int, [c_vp, c_i64, c_i64, c_i64, c_vp, c_vp]),
    "cq_q_update_x3": (c_int, [c_int, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_int,
                               c_float, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_size, c_vp]),
    "cq_ritz_product_error": (c_int, [c_vp, c_vp, c_vp, c_i64, c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_size, c_vp]),
    "cq_batched_dot": (c_int, [c_int, c_vp, c_vp, c_i64, c_i64, c_vp, c_vp, c_size, c_vp]),
    "cq_act_sqsum_workspace": (c_size, [c_i64, c_i64]),
    "cq_act_sqsum_cols": (c_int, [c_int, c_vp, c_i64, c_i64, c_i64, c_vp, c_int, c_double, c_vp, c_size, c_vp]),
    "cq_act_sqsum_rows": (c_int, [c_int, c_vp, c_i64, c_i64, c_i64, c_vp, c_int, c_double, c_vp]),
}
EXPORTS = tuple(_SIGS)
ABI_VERSION = 5  # include/caldera_hip.h CQ_ABI_VERSION

_lib = None


def load(path: str = LIB_PATH):
    """Load libcaldera_hip.so and declare every export (no device calls)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; "
                           f"g.build()'` (hipcc --offload-arch=gfx950)")
    if path == LIB_PATH and not os.environ.get("CQ_ALLOW_STALE_LIB"):
        from . import build as _build
        if _build.needs_build():  # never run kernels older than the sources in the tree
            raise RuntimeError(f"{path} is stale (built from other sources than csrc/ now holds, or "
                               f"unstamped): rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path)
    # any build (also another one for an A/B timing, tools/probes/build_rev.sh) must speak this
    # ABI: the declarations below are this ABI's signatures, and calling an export of another
    # layout through them is undefined behaviour on the GPU rather than a clean error
    abi = getattr(lib, "cq_abi_version", None)
    if abi is None:
        raise RuntimeError(f"{path} does not export cq_abi_version")
    abi.restype, abi.argtypes = c_int, []
    if abi() != ABI_VERSION:
        raise RuntimeError(f"{path}: ABI version {abi()} != {ABI_VERSION} (include/caldera_hip.h); rebuild it "
                           f"from these sources")
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            raise RuntimeError(f"{path} does not export {name}")
        fn.restype, fn.argtypes = res, args
    _lib = lib
    return lib


class CalderaHipError(RuntimeError):
    pass


_SYNC_CHECK = bool(os.environ.get("CQ_SYNC_CHECK"))


def _check(st: int, what: str):
    if _SYNC_CHECK and st == 0:  # debugging: attribute an asynchronous fault to its launch
        import sys
        import traceback
        fr = traceback.extract_stack(limit=4)
        print(f"[cq] {what} <- {' <- '.join(f'{f.name}:{f.lineno}' for f in reversed(fr[:-1]))}",
              file=sys.stderr, flush=True)
        torch.cuda.synchronize()
    if st != 0:
        msg = load().cq_last_error().decode(errors="replace")
        if st == CQ_EINVAL:
            if "Bit-width not supported" in msg:
                raise AssertionError("Bit-width not supported!")
            raise ValueError(f"{what}: {msg}")
        raise CalderaHipError(f"{what}: status {st}: {msg}")


def _p(t: torch.Tensor | None):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(dev: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _require_hip(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("caldera-mi355x kernels need HIP device tensors (no CPU fallback)")


def _wst(w: torch.Tensor | None, B: int) -> int:
    """Batch stride of a column / error weight vector (ABI 5): (n,) is shared by the batch
    (stride 0); (B, n) holds one vector per matrix (distinct diagonal Hessians, stride n)."""
    if w is None or w.dim() == 1:
        return 0
    assert w.dim() == 2 and w.shape[0] == B and w.is_contiguous(), (tuple(w.shape), B)
    return w.shape[1] if B > 1 else 0


def workspace(nbytes: int, dev) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=dev)


# ---------------------------------------------------------------------------- wrappers
def rms_scale(W: torch.Tensor, do_scale: bool):
    """W (B, m, n) fp16/fp32 -> (gs (B,) fp32, Ws same dtype).  alg.py:38-42."""
    _require_hip(W)
    W = W.contiguous()
    dt = {torch.float16: CQ_F16, torch.float32: CQ_F32}[W.dtype]
    B = W.shape[0]
    numel = W[0].numel()
    gs = torch.empty(B, dtype=torch.float32, device=W.device)
    Ws = torch.empty_like(W)
    lib = load()
    ws = workspace(lib.cq_rms_scale_workspace(B, numel), W.device)
    _check(lib.cq_rms_scale(dt, _p(W), B, numel, int(bool(do_scale)), _p(gs), _p(Ws), _p(ws), ws.numel(),
                            _stream(W.device)), "cq_rms_scale")
    return gs, Ws


def weighted_sqsum(x: torch.Tensor, w: torch.Tensor | None, ncols: int) -> torch.Tensor:
    _require_hip(x, w)
    dt = {torch.float16: CQ_F16, torch.float32: CQ_F32}[x.dtype]
    B = x.shape[0]
    numel = x[0].numel()
    out = torch.empty(B, dtype=torch.float64, device=x.device)
    lib = load()
    ws = workspace(lib.cq_rms_scale_workspace(B, numel), x.device)
    _check(lib.cq_weighted_sqsum(dt, _p(x), B, numel, _p(w), ncols, _wst(w, B), _p(out), _p(ws), ws.numel(),
                                 _stream(x.device)), "cq_weighted_sqsum")
    return out


def batched_dot(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """out[b] = <x[b], y[b]> in fp64 (x, y (B, ...) fp32 or fp64, same shape, contiguous)."""
    _require_hip(x, y)
    assert x.shape == y.shape and x.dtype == y.dtype and x.is_contiguous() and y.is_contiguous()
    dt = {torch.float32: CQ_F32, torch.float64: CQ_F64}[x.dtype]
    B = x.shape[0]
    numel = x[0].numel()
    out = torch.empty(B, dtype=torch.float64, device=x.device)
    lib = load()
    ws = workspace(lib.cq_rms_scale_workspace(B, numel), x.device)
    _check(lib.cq_batched_dot(dt, _p(x), _p(y), B, numel, _p(out), _p(ws), ws.numel(), _stream(x.device)),
           "cq_batched_dot")
    return out


def code_dtype(bits: int):
    return torch.int8 if bits <= 8 else torch.int16


def quantize_uniform(x: torch.Tensor, block_size: int, bits: int, eps: float = 1e-8, *,
                     codes=True, packed=False, deq=True, err_w=None, err_ncols=1, want_err=False):
    """x (B, numel) fp32 contiguous.  quantization.py:244-269 / :290-307 (uniform)."""
    _require_hip(x, err_w)
    assert x.dtype == torch.float32 and x.is_contiguous()
    B, numel = x.shape
    dev = x.device
    out = {}
    out["codes"] = torch.empty((B, numel), dtype=code_dtype(bits), device=dev) if codes else None
    out["packed"] = (torch.empty((B, numel * bits // 8), dtype=torch.uint8, device=dev)
                     if packed and bits <= 4 else None)
    out["deq"] = torch.empty((B, numel), dtype=torch.float32, device=dev) if deq else None
    out["scale"] = torch.empty((B, numel // block_size), dtype=torch.float32, device=dev)
    out["err"] = torch.empty(B, dtype=torch.float64, device=dev) if (want_err or err_w is not None) else None
    lib = load()
    ws = workspace(lib.cq_quantize_workspace(B, numel, block_size), dev)
    _check(lib.cq_quantize_uniform(_p(x), B, numel, block_size, bits, eps, _p(out["codes"]),
                                   _p(out["packed"]), _p(out["deq"]), _p(out["scale"]), _p(err_w),
                                   err_ncols, _wst(err_w, B), _p(out["err"]), _p(ws), ws.numel(), _stream(dev)),
           "cq_quantize_uniform")
    return out


def quantize_known_max(x, absmax_bits, bits, eps=1e-8, *, codes=None, packed=None, deq=None,
                       scale=None, err_w=None, err_ncols=1, err_out=None):
    _require_hip(x)
    B = x.shape[0]
    numel = x[0].numel()
    lib = load()
    ws = workspace(lib.cq_quantize_workspace(B, numel, numel), x.device)
    _check(lib.cq_quantize_uniform_known_max(_p(x), B, numel, bits, eps, _p(absmax_bits), _p(codes),
                                             _p(packed), _p(deq), _p(scale), _p(err_w), err_ncols, _wst(err_w, B),
                                             _p(err_out), _p(ws), ws.numel(), _stream(x.device)),
           "cq_quantize_uniform_known_max")


def dequantize_uniform(codes: torch.Tensor, scale: torch.Tensor, bits: int, packed: bool = False,
                       numel: int | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """(float(c)/k) * scale per block; codes (..., ) int8/int16 or packed uint8; scale (nblocks,)."""
    _require_hip(codes, scale, out)
    total = numel if numel is not None else codes.numel()
    nb = scale.numel()
    if out is None:
        out = torch.empty(total, dtype=torch.float32, device=codes.device)
    assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() == total
    _check(load().cq_dequant_uniform(_p(codes), int(packed), _p(scale), total, total // nb, bits, _p(out),
                                     _stream(codes.device)), "cq_dequant_uniform")
    return out


def unpack_codes(packed: torch.Tensor, numel: int, bits: int, out: torch.Tensor | None = None) -> torch.Tensor:
    _require_hip(packed, out)
    B = packed.shape[0]
    codes = torch.empty((B, numel), dtype=torch.int8, device=packed.device) if out is None else out
    assert codes.shape == (B, numel) and codes.dtype == torch.int8 and codes.is_contiguous()
    _check(load().cq_unpack_codes(_p(packed), B, numel, bits, _p(codes), _stream(packed.device)),
           "cq_unpack_codes")
    return codes


def quantize_nf(x: torch.Tensor, block_size: int, bits: int, eps: float = 1e-8, *, idx=True, deq=True,
                err_w=None, err_ncols=1, err_out=None):
    """NF4 / NF2 (quantization.py:39-91, :270-279).  x (B, numel) fp32 contiguous ->
    dict(idx (B, numel) uint8, deq (B, numel) fp32, scale (B, numel // block_size) fp32)."""
    _require_hip(x, err_w, err_out)
    assert x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 2
    B, numel = x.shape
    dev = x.device
    out = {"idx": torch.empty((B, numel), dtype=torch.uint8, device=dev) if idx else None,
           "deq": torch.empty((B, numel), dtype=torch.float32, device=dev) if deq else None,
           "scale": torch.empty((B, numel // block_size), dtype=torch.float32, device=dev)}
    lib = load()
    ws = workspace(lib.cq_quantize_nf_workspace(B, numel, block_size), dev)
    _check(lib.cq_quantize_nf(_p(x), B, numel, block_size, bits, eps, _p(out["idx"]), _p(out["deq"]),
                              _p(out["scale"]), _p(err_w), err_ncols, _wst(err_w, B), _p(err_out), _p(ws), ws.numel(),
                              _stream(dev)), "cq_quantize_nf")
    return out


def dequantize_nf(idx: torch.Tensor, scale: torch.Tensor, bits: int) -> torch.Tensor:
    """level[idx] * scale[blk] (quantization.py:87-91); idx uint8, scale (nblocks,) fp32."""
    _require_hip(idx, scale)
    total = idx.numel()
    out = torch.empty(total, dtype=torch.float32, device=idx.device)
    _check(load().cq_dequant_nf(_p(idx), _p(scale), total, total // scale.numel(), bits, _p(out),
                                _stream(idx.device)), "cq_dequant_nf")
    return out


def quantize_bbint(x: torch.Tensor, block_size: int, bits: int, eps: float = 1e-8, *, packed=True, deq=True,
                   outliers=True, err_w=None, err_ncols=1, err_out=None):
    """bbint4 / bbint2 (quantization.py:107-243).  x (B, numel) fp32 contiguous -> dict(packed
    (B, numel*bits/8) uint8, deq (B, numel), bmin / bscale (B, nblk), n_out [B] (host ints),
    vals (sum n_out,) fp32, idx (sum n_out, 2) int64 — matrix b's rows follow matrix b-1's).
    One host synchronisation (the outlier count sizes the list)."""
    _require_hip(x, err_w, err_out)
    assert x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 2
    B, numel = x.shape
    dev = x.device
    nblk = numel // block_size
    lib = load()
    nws = lib.cq_bbint_workspace(B, numel, block_size)
    if nws == 0:
        raise ValueError(f"bbint: numel {numel} is not divisible by block size {block_size}")
    ws = workspace(nws, dev)
    bmin = torch.empty((B, nblk), dtype=torch.float32, device=dev)
    bscale = torch.empty((B, nblk), dtype=torch.float32, device=dev)
    n_out = torch.empty(B, dtype=torch.int64, device=dev)
    st = _stream(dev)
    _check(lib.cq_bbint_stats(_p(x), B, numel, block_size, bits, eps, _p(bmin), _p(bscale), _p(n_out), _p(ws),
                              ws.numel(), st), "cq_bbint_stats")
    counts = [int(v) for v in n_out.tolist()] if outliers else [0] * B
    tot = sum(counts)
    vals = torch.empty(tot, dtype=torch.float32, device=dev) if outliers else None
    oidx = torch.empty((tot, 2), dtype=torch.int64, device=dev) if outliers else None
    pk = torch.empty((B, numel * bits // 8), dtype=torch.uint8, device=dev) if packed else None
    dq = torch.empty((B, numel), dtype=torch.float32, device=dev) if deq else None
    _check(lib.cq_bbint_emit(_p(x), B, numel, block_size, bits, _p(bmin), _p(bscale), _p(pk), _p(dq),
                             _p(vals) if tot else None, _p(oidx) if tot else None, _p(err_w), err_ncols,
                             _wst(err_w, B), _p(err_out), _p(ws), ws.numel(), st), "cq_bbint_emit")
    return {"packed": pk, "deq": dq, "bmin": bmin, "bscale": bscale, "n_out": counts, "vals": vals, "idx": oidx}


def dequantize_bbint(packed: torch.Tensor, bits: int, bmin: torch.Tensor, bscale: torch.Tensor,
                     vals: torch.Tensor | None, idx: torch.Tensor | None, block_size: int) -> torch.Tensor:
    """u * scale + min per block, outliers scattered back (quantization.py:157-172, :224-243)."""
    _require_hip(packed, bmin, bscale, vals, idx)
    total = packed.numel() * 8 // bits
    out = torch.empty(total, dtype=torch.float32, device=packed.device)
    k = 0 if vals is None else vals.numel()
    _check(load().cq_dequant_bbint(_p(packed), bits, _p(bmin), _p(bscale), total, block_size,
                                   _p(vals) if k else None, _p(idx.contiguous()) if k else None, k, _p(out),
                                   _stream(packed.device)), "cq_dequant_bbint")
    return out


def build_residual(Ws, qcodes, qscale, bits, ycol, Y=None, res=None):
    """Y = (Ws - deq(Q)) * ycol[col];  res = Ws - deq(Q).  alg.py:124 + :211 (diagonal H)."""
    _require_hip(Ws, qcodes, qscale, ycol, Y, res)
    dt = {torch.float16: CQ_F16, torch.float32: CQ_F32}[Ws.dtype]
    B, m, n = Ws.shape
    _check(load().cq_build_residual(dt, _p(Ws), _p(qcodes), _p(qscale), bits, _p(ycol), _wst(ycol, B), B, m, n,
                                    _p(Y), _p(res), _stream(Ws.device)), "cq_build_residual")


def _mat(t: torch.Tensor):
    """(tensor (B, r, c) or (r, c) with unit column stride) -> (ptr, ld, batch_stride)."""
    if t.dim() == 2:
        assert t.stride(1) == 1
        return t, t.stride(0), 0
    assert t.dim() == 3 and t.stride(2) == 1, "matrices must have unit column stride"
    return t, t.stride(1), (t.stride(0) if t.shape[0] > 1 else 0)


def gemm(A, B, *, ta=False, tb=False, C=None, alpha=1.0, beta=0.0, D=None, gamma=0.0,
         epi=EPI_LINEAR, absmax=None, w=None, err_out=None, alpha_v=None, beta_v=None,
         gamma_v=None, batch=None, syrk=False, b_triu=False):
    """Batched C = alpha op(A) op(B) + beta C + gamma D (or RESID / WERR epilogues).
    b_triu: B (not transposed) is upper triangular -- its zero K slices are skipped."""
    _require_hip(A, B, C, D, w)
    A_, lda, sa = _mat(A)
    B_, ldb, sb = _mat(B)
    M = A.shape[-1] if ta else A.shape[-2]
    K = A.shape[-2] if ta else A.shape[-1]
    N = B.shape[-2] if tb else B.shape[-1]
    Kb = B.shape[-1] if tb else B.shape[-2]
    assert K == Kb, f"gemm: inner dims {K} vs {Kb}"
    if batch is None:
        batch = max(t.shape[0] if t is not None and t.dim() == 3 else 1 for t in (A, B, C, D))
    g = GemmArgs()
    g.M, g.N, g.K, g.batch = M, N, K, batch
    g.trans_a, g.trans_b = int(ta), int(tb)
    g.A, g.lda, g.stride_a = A_.data_ptr(), lda, sa
    g.B, g.ldb, g.stride_b = B_.data_ptr(), ldb, sb
    if C is not None:
        C_, ldc, sc = _mat(C)
        assert C.shape[-2] == M and C.shape[-1] == N
        g.C, g.ldc, g.stride_c = C_.data_ptr(), ldc, sc
    if D is not None:
        D_, ldd, sd = _mat(D)
        assert D.shape[-2] == M and D.shape[-1] == N, f"D shape {tuple(D.shape)} vs {(M, N)}"
        g.D, g.ldd, g.stride_d, g.d_f16 = D_.data_ptr(), ldd, sd, int(D.dtype == torch.float16)
        if D.dtype not in (torch.float16, torch.float32):
            raise TypeError("D must be fp16/fp32")
    g.alpha, g.beta, g.gamma = alpha, beta, gamma
    g.alpha_v = alpha_v.data_ptr() if alpha_v is not None else None
    g.beta_v = beta_v.data_ptr() if beta_v is not None else None
    g.gamma_v = gamma_v.data_ptr() if gamma_v is not None else None
    g.epi = epi
    g.absmax_bits = absmax.data_ptr() if absmax is not None else None
    if w is not None:
        g.w = w.data_ptr()
        g.stride_w = w.shape[-1] if (w.dim() == 2 and w.shape[0] > 1) else 0
    g.err_out = err_out.data_ptr() if err_out is not None else None
    g.syrk = int(bool(syrk))
    g.b_triu = int(bool(b_triu))
    lib = load()
    dev = A.device
    nws = lib.cq_gemm_workspace(ctypes.byref(g))
    ws = workspace(nws, dev) if nws else None
    _check(lib.cq_gemm_f32(ctypes.byref(g), _p(ws), 0 if ws is None else ws.numel(), _stream(dev)),
           "cq_gemm_f32")
    return C


def gram_f64(A, B, *, ta=False, tb=False, out=None):
    """C = op(A)^T op(B) style Gram: A is K x M (or M x K if ta), B is K x N (or N x K if tb)."""
    _require_hip(A, B)
    A_, lda, sa = _mat(A)
    B_, ldb, sb = _mat(B)
    K = A.shape[-1] if ta else A.shape[-2]
    M = A.shape[-2] if ta else A.shape[-1]
    N = B.shape[-2] if tb else B.shape[-1]
    batch = max(t.shape[0] if t.dim() == 3 else 1 for t in (A, B))
    if out is None:
        out = torch.empty((batch, M, N), dtype=torch.float64, device=A.device)
    lib = load()
    ws = workspace(lib.cq_gram_f64_workspace(M, N, K, batch), A.device)
    _check(lib.cq_gram_f64(M, N, K, batch, _p(A_), int(ta), lda, sa, _p(B_), int(tb), ldb, sb, _p(out),
                           _p(ws), ws.numel(), _stream(A.device)), "cq_gram_f64")
    return out


def spd_whiten(S: torch.Tensor, rcond2: float = 1e-30):
    """S (B, p, p) fp64 SPD (overwritten) -> (Wt32, Wt64, info) with Wt^T S Wt = I on the
    independent columns; pivots <= rcond2 * max diag are dropped (info = their count).
    Wt64 is S itself: the kernel leaves the fp64 Wt there (its Wt64 argument is scratch)."""
    _require_hip(S)
    B, p, _ = S.shape
    Wt32 = torch.empty((B, p, p), dtype=torch.float32, device=S.device)
    scr = torch.empty((B, p, p), dtype=torch.float64, device=S.device)
    info = torch.empty(B, dtype=torch.int32, device=S.device)
    _check(load().cq_spd_whiten_rcond(_p(S), p, B, float(rcond2), _p(Wt32), _p(scr), _p(info),
                                      _stream(S.device)), "cq_spd_whiten_rcond")
    return Wt32, S, info


def jacobi_eigh(A: torch.Tensor, max_sweeps: int = 30, tol: float = 1e-13, want64=False, want_vectors=True):
    """A (B, p, p) fp64 symmetric (overwritten) -> (evals desc (B,p) fp64, V32, V64, sweeps);
    want_vectors=False: eigenvalues only (V32 = V64 = None; the p <= 192 register kernel then
    skips its eigenvector rotations)."""
    _require_hip(A)
    B, p, _ = A.shape
    ev = torch.empty((B, p), dtype=torch.float64, device=A.device)
    V32 = torch.empty((B, p, p), dtype=torch.float32, device=A.device) if want_vectors else None
    want64 = want64 and want_vectors
    V64 = torch.empty((B, p, p), dtype=torch.float64, device=A.device) if want64 else None
    sw = torch.empty(B, dtype=torch.int32, device=A.device)
    lib = load()
    ws = workspace(lib.cq_jacobi_workspace(p, B), A.device)
    _check(lib.cq_jacobi_eigh(_p(A), p, B, max_sweeps, tol, _p(ev), _p(V32), _p(V64), _p(sw), _p(ws),
                              ws.numel(), _stream(A.device)), "cq_jacobi_eigh")
    return ev, V32, V64, sw


def extreme_eigs(T: torch.Tensor, steps: int = 40) -> torch.Tensor:
    """T (B, p, p) fp64 symmetric, p <= 512 (not overwritten) -> (B, 2) fp64 [largest,
    smallest eigenvalue] by Lanczos + bisection (cq_extreme_eigs): the filter bounds of the
    solver's cheap outer iterations without a values-only eigensolve."""
    _require_hip(T)
    B, p, _ = T.shape
    ends = torch.empty((B, 2), dtype=torch.float64, device=T.device)
    _check(load().cq_extreme_eigs(_p(T), p, B, int(steps), _p(ends), _stream(T.device)), "cq_extreme_eigs")
    return ends


class BlockJacobi:
    """cq_jacobi_eigh_staged (block Jacobi): begin + a first batch of sweeps, then further sweeps
    only while the device count of unconverged matrices (read back by the caller) is nonzero."""
    BEGIN, SWEEPS, END = 1, 2, 4

    def __init__(self, A: torch.Tensor, tol: float, want_vectors: bool = True):
        _require_hip(A)
        self.A, self.tol, self.want = A, tol, bool(want_vectors)
        self.B, self.p, _ = A.shape
        self.ws = workspace(load().cq_jacobi_staged_workspace(self.p, self.B), A.device)
        self.pending = torch.zeros(1, dtype=torch.int32, device=A.device)
        self.swept = 0

    def _call(self, phase, nsweeps=0, ev=None, V32=None, sw=None):
        _check(load().cq_jacobi_eigh_staged(_p(self.A), self.p, self.B, phase, nsweeps, self.tol, int(self.want),
                                            _p(ev), _p(V32), None, _p(sw), _p(self.pending), _p(self.ws),
                                            self.ws.numel(), _stream(self.A.device)), "cq_jacobi_eigh_staged")

    def launch(self, n: int, begin: bool = False):
        """n more sweeps (stream-ordered, no host sync)."""
        self._call((self.BEGIN if begin else 0) | self.SWEEPS, n)
        self.swept += n

    def pending_count(self) -> int:
        """Matrices still unconverged after the sweeps launched so far (host read-back)."""
        return int(self.pending.item())

    def sweeps(self, n: int, begin: bool = False) -> int:
        """n more sweeps; returns the number of matrices still unconverged (host read-back)."""
        self.launch(n, begin)
        return self.pending_count()

    def finish(self):
        dev = self.A.device
        ev = torch.empty((self.B, self.p), dtype=torch.float64, device=dev)
        V32 = torch.empty((self.B, self.p, self.p), dtype=torch.float32, device=dev) if self.want else None
        sw = torch.empty(self.B, dtype=torch.int32, device=dev)
        self._call(self.END, 0, ev, V32, sw)
        return ev, V32, None, sw


def ritz_residual(X, Z, theta, r):
    _require_hip(X, Z, theta)
    B, k, p = X.shape
    out = torch.empty(B, dtype=torch.float32, device=X.device)
    lib = load()
    ws = workspace(lib.cq_ritz_workspace(k, r, B), X.device)
    _check(lib.cq_ritz_residual(_p(X), _p(Z), _p(theta), k, p, r, B, _p(out), _p(ws), ws.numel(),
                                _stream(X.device)), "cq_ritz_residual")
    return out


def ritz_product_error(X, Z, theta, r, ysq):
    """Per-matrix estimate of the relative error of the rank-r projection (cq_ritz_product_error)."""
    _require_hip(X, Z, theta, ysq)
    B, k, p = X.shape
    out = torch.empty(B, dtype=torch.float32, device=X.device)
    lib = load()
    ws = workspace(lib.cq_ritz_workspace(k, r, B), X.device)
    _check(lib.cq_ritz_product_error(_p(X), _p(Z), _p(theta), k, p, r, B, _p(ysq), _p(out), _p(ws), ws.numel(),
                                     _stream(X.device)), "cq_ritz_product_error")
    return out


def scale_rc(X, *, trans=False, rowscale=None, colscale=None, out=None):
    """out[b] = op(X[b]) * rowscale[b][:,None] * colscale[b][None,:] (scales (B,len) or (len,))."""
    _require_hip(X, rowscale, colscale)
    X_, ldx, sx = _mat(X)
    B = X.shape[0] if X.dim() == 3 else 1
    rows, cols = (X.shape[-1], X.shape[-2]) if trans else (X.shape[-2], X.shape[-1])
    if out is None:
        out = torch.empty((B, rows, cols), dtype=torch.float32, device=X.device)
    Y_, ldy, sy = _mat(out)
    rss = rowscale.shape[-1] if rowscale is not None and rowscale.dim() == 2 and rowscale.shape[0] > 1 else 0
    css = colscale.shape[-1] if colscale is not None and colscale.dim() == 2 and colscale.shape[0] > 1 else 0
    if X.dim() == 3 and X.shape[0] > 1:
        sx = X.stride(0)
    if out.dim() == 3 and out.shape[0] > 1:
        sy = out.stride(0)
    _check(load().cq_scale_rc(_p(X_), ldx, sx, int(trans), _p(Y_), ldy, sy, rows, cols, B, _p(rowscale),
                              rss, _p(colscale), css, _stream(X.device)), "cq_scale_rc")
    return out


# ---------------------------------------------------------------------------- split-fp16 products
def sym_split_f16(G: torch.Tensor, x_scale: float, *, hi=None, lo=None, scale=None, inv_scale=None,
                  upper_only=False, blocked=False):
    """G (B, n, n) fp32 PSD -> (hi, lo fp16, scale (B,), inv_scale (B,) = 1/(scale*x_scale)).
    upper_only: only G's upper triangle is valid (x3 tri Gram); the split is mirrored."""
    _require_hip(G)
    assert G.dtype == torch.float32 and G.is_contiguous() and G.dim() == 3 and G.shape[1] == G.shape[2]
    B, n, _ = G.shape
    dev = G.device
    hi = torch.empty((B, n, n), dtype=torch.float16, device=dev) if hi is None else hi
    lo = torch.empty((B, n, n), dtype=torch.float16, device=dev) if lo is None else lo
    scale = torch.empty(B, dtype=torch.float32, device=dev) if scale is None else scale
    inv_scale = torch.empty(B, dtype=torch.float32, device=dev) if inv_scale is None else inv_scale
    _check(load().cq_sym_split_f16(_p(G), n, B, int(bool(upper_only)), int(bool(blocked)), float(x_scale), _p(hi),
                                   _p(lo), _p(scale),
                                   _p(inv_scale),
                                   _stream(dev)), "cq_sym_split_f16")
    return hi, lo, scale, inv_scale


def transpose_split(X: torch.Tensor, *, out=None, hi=None, lo=None, scale: float | torch.Tensor = 1.0,
                    blocked: bool = False):
    """X (B, r, c) fp32 contiguous -> X^T (B, c, r) fp32 (out) and/or its fp16 split (hi, lo)
    scaled by `scale` (a float, or a (B,) fp32 tensor of per-matrix scales)."""
    _require_hip(X)
    assert X.dtype == torch.float32 and X.is_contiguous() and X.dim() == 3
    B, r, c = X.shape
    sv = scale if torch.is_tensor(scale) else None
    sf = 1.0 if sv is not None else float(scale)
    _check(load().cq_transpose_split(_p(X), r, c, B, _p(out), _p(hi), _p(lo), sf, _p(sv), int(bool(blocked)),
                                     _stream(X.device)),
           "cq_transpose_split")
    return out, hi, lo


TRIU_SPLIT_MAX_P = 192


def triu_split_ok(M: int, p: int) -> bool:
    """Shapes cq_gemm_triu_split takes (p % 32 == 0, p <= 192, M % 32 == 0)."""
    return p % 32 == 0 and 0 < p <= TRIU_SPLIT_MAX_P and M % 32 == 0


def gemm_triu_split(X: torch.Tensor, Wt: torch.Tensor, C: torch.Tensor, hi: torch.Tensor, lo: torch.Tensor,
                    scale: float):
    """C = X Wt (Wt upper triangular) and hi/lo = the K-blocked split of C^T at `scale`: the
    same bits as gemm(X, Wt, b_triu=True) followed by transpose_split(C, blocked=True)."""
    _require_hip(X)
    B, M, p = X.shape
    assert X.dtype == Wt.dtype == C.dtype == torch.float32 and hi.dtype == lo.dtype == torch.float16
    assert X.is_contiguous() and Wt.is_contiguous() and C.is_contiguous() and hi.is_contiguous() and lo.is_contiguous()
    assert Wt.shape == (B, p, p) and C.shape == X.shape and hi.shape == (B, p, M) and lo.shape == hi.shape
    _check(load().cq_gemm_triu_split(_p(X), _p(Wt), M, p, B, _p(C), _p(hi), _p(lo), float(scale),
                                     _stream(X.device)), "cq_gemm_triu_split")
    return C


def pow2_scale(X: torch.Tensor, log2_target: int = 14, out=None):
    """(B,) fp32 power-of-two scales s[b] with max|X[b]| * s[b] < 2^log2_target."""
    _require_hip(X)
    assert X.dtype == torch.float32 and X.is_contiguous()
    B = X.shape[0]
    out = torch.empty(B, dtype=torch.float32, device=X.device) if out is None else out
    _check(load().cq_pow2_scale(_p(X), X.numel() // B, B, int(log2_target), _p(out), _stream(X.device)),
           "cq_pow2_scale")
    return out


def pow2_from_absmax(bits: torch.Tensor, log2_target: int = 14) -> torch.Tensor:
    """In place: (B,) bits of max|X[b]| (as written by gemm_x3 absmax_out, or a positive fp32
    bound such as a quantiser's scale) -> the fp32 power-of-two split scales pow2_scale would
    give for X (cq_pow2_from_absmax).  Returns the tensor viewed as fp32."""
    _require_hip(bits)
    assert bits.element_size() == 4 and bits.is_contiguous()
    out = bits.view(torch.float32)
    _check(load().cq_pow2_from_absmax(_p(out), bits.numel(), int(log2_target), _stream(bits.device)),
           "cq_pow2_from_absmax")
    return out


def split_f16(X: torch.Tensor, scale, *, hi=None, lo=None, blocked: bool = False):
    """fp16 halves of X * scale (scale: float or (B,) tensor), same shape as X; blocked: the
    K-blocked operand layout over X's last dimension (storage size unchanged)."""
    _require_hip(X)
    assert X.dtype == torch.float32 and X.is_contiguous()
    B = X.shape[0]
    hi = torch.empty(X.shape, dtype=torch.float16, device=X.device) if hi is None else hi
    lo = torch.empty(X.shape, dtype=torch.float16, device=X.device) if lo is None else lo
    sv = scale if torch.is_tensor(scale) else None
    sf = 1.0 if sv is not None else float(scale)
    _check(load().cq_split_f16(_p(X), X.numel() // B, B, _p(sv), sf, _p(hi), _p(lo),
                               X.shape[-1] if blocked else 0, _stream(X.device)),
           "cq_split_f16")
    return hi, lo


# automatic split-K of small-batch split-fp16 products (gemm_x3); False: every product in one
# pass, so results do not depend on the batch a matrix is decomposed in (slower at small B).
# The process default; split_k_policy() overrides it for the calling thread only.
AUTO_SPLIT_K = True
_POLICY = threading.local()


@contextlib.contextmanager
def split_k_policy(enabled: bool):
    """Within the block, this thread's gemm_x3 calls use automatic split-K iff `enabled`
    (overlap.run_interleaved turns it off while batches share the chip); other threads keep
    their own policy."""
    prev = getattr(_POLICY, "auto", None)
    _POLICY.auto = bool(enabled)
    try:
        yield
    finally:
        _POLICY.auto = prev


def auto_split_k() -> bool:
    v = getattr(_POLICY, "auto", None)
    return AUTO_SPLIT_K if v is None else v


def gemm_x3(Ah, Al, Bh, Bl, inv_scale, C, *, P=None, D=None, alpha_v=None, beta_v=None, gamma_v=None,
            out_h=None, out_l=None, out_scale=1.0, overflow=None, tri=False, b_blocked=False, active=None,
            a_blocked=False, o_blocked=False, sym_bound=None, scale_out=None, inv_out=None, lda=None, M=None,
            single=False, ksplit=None, b_exact=False, colw=None, absmax_out=None, Ct=None):
    """C (B, M, N) = alpha * A B^T * inv_scale + beta P + gamma D with A = Ah + Al (B, M, K) and
    B = Bh + Bl (B, N, K) fp16 halves (b_blocked: in the K-blocked layout of sym_split_f16,
    same storage size); optional fp16 split of C into out_h/out_l.
    sym_bound (B,) fp64: symmetric Gram mode (tri): the K-blocked split of C is written from
    its upper triangle with scale s[b] from the bound (scale_out, inv_out = 1/(s out_scale));
    C may then be None.  lda / M (a_blocked only): A holds lda >= M rows of which the first M
    are used (C has M rows).  b_exact: B is exactly fp16 (Bl = 0, e.g. W's halves written
    under a split scale >= 1); Bl is not read and may be None.  colw (N,) fp32: the product
    term of column j scaled by colw[j] (before beta P + gamma D; (B, N): per matrix).  absmax_out (B,) int32/uint32/fp32
    (plain products): zeroed here, receives the bits of max|C[b]| (pow2_from_absmax turns them
    into the next split's scale without a pass over C).  Ct (B, N, M) fp32: C^T as well (not
    with tri / sym_out; C required)."""
    assert Bl is not None or b_exact or single
    _require_hip(Ah, Al, Bh, Bl, C)
    Bt, MA, Kd = Ah.shape
    M = MA if M is None else M
    N = Bh.shape[1]
    assert lda is None or (a_blocked and lda == MA and M <= MA)
    assert Bh.shape[2] == Kd and (C is None or C.shape == (Bt, M, N))
    for t in (Ah, Al, Bh, Bl, C, P, D, out_h, out_l):
        assert t is None or t.is_contiguous()
    for t in (out_h, out_l):  # the split output is M x N per matrix (sym_out: M = N)
        assert t is None or t.numel() >= Bt * M * N, "gemm_x3: split output buffer too small"
    g = X3Args()
    g.M, g.N, g.K, g.batch = M, N, Kd, Bt
    g.Ah, g.Al, g.lda, g.stride_a = Ah.data_ptr(), Al.data_ptr(), (MA if a_blocked else Kd), MA * Kd
    g.Bh, g.Bl, g.ldb, g.stride_b = Bh.data_ptr(), (Bl.data_ptr() if Bl is not None else None), (
        N if b_blocked else Kd), N * Kd
    g.inv_scale = inv_scale.data_ptr()
    g.C, g.ldc, g.stride_c = (C.data_ptr() if C is not None else None), N, M * N
    if P is not None:
        g.P, g.ldp, g.stride_p = P.data_ptr(), N, M * N
    if D is not None:
        g.D, g.ldd, g.stride_d = D.data_ptr(), N, M * N
    g.alpha_v = alpha_v.data_ptr() if alpha_v is not None else None
    g.beta_v = beta_v.data_ptr() if beta_v is not None else None
    g.gamma_v = gamma_v.data_ptr() if gamma_v is not None else None
    if out_h is not None and sym_bound is None:
        g.out_h, g.out_l, g.ldo, g.stride_o = out_h.data_ptr(), out_l.data_ptr(), N, M * N
        g.out_scale = out_scale
        g.overflow = overflow.data_ptr()
    g.tri = int(bool(tri))
    g.b_blocked = int(b_blocked)  # 1: K-blocked by 32, 2: by 16 (4-stage kernel only)
    g.active = active.data_ptr() if active is not None else None
    g.a_blocked = int(a_blocked)
    g.o_blocked = int(bool(o_blocked))
    g.single = int(bool(single))
    g.b_exact = int(bool(b_exact))
    if colw is not None:
        assert colw.dtype == torch.float32 and colw.is_contiguous() and colw.shape[-1] == N
        g.colw, g.stride_colw = colw.data_ptr(), _wst(colw, Bt)
    if absmax_out is not None:
        assert absmax_out.numel() == Bt and absmax_out.element_size() == 4 and absmax_out.is_contiguous()
        absmax_out.zero_()
        g.absmax_out = absmax_out.data_ptr()
    if Ct is not None:
        _require_hip(Ct)
        assert C is not None and not tri and Ct.dtype == torch.float32 and Ct.is_contiguous() and Ct.shape == (Bt, N, M)
        g.Ct, g.stride_ct = Ct.data_ptr(), N * M
    # split-K where the batch has fewer output tiles than the chip has CUs (one caldera() call:
    # the filter's 192 x 4096 product is 11 tiles): chunks of >= 8 K steps, ~512 workgroups.
    # The chunked sum has another fp32 summation order than the one-pass product, so a matrix
    # decomposed alone (or in a small batch) and the same matrix inside a large batch agree to
    # the products' rounding, not bit for bit; AUTO_SPLIT_K = False pins one pass everywhere
    tiles = -(-N // 384) * -(-M // 192) * Bt
    splittable = not tri and sym_bound is None and C is not None and N % 4 == 0
    if ksplit is None and not auto_split_k():
        ksplit = 1
    if ksplit is None:  # automatic
        ks = min(Kd // 32 // 8, -(-512 // tiles)) if splittable and tiles < 256 and Kd >= 512 else 1
    else:
        ks = int(ksplit)
        assert ks == 1 or (splittable and ks <= Kd // 32), "gemm_x3: split-K not possible here"
    if ks > 1:
        g.ksplit = ks
        g.split_ws = scratch.get_flat("gemm_x3.split", ks * Bt * M * N, torch.float32, Ah.device).data_ptr()
    if sym_bound is not None:
        g.sym_out = 1
        g.out_bound, g.scale_out, g.inv_out = sym_bound.data_ptr(), scale_out.data_ptr(), inv_out.data_ptr()
        g.out_h, g.out_l, g.ldo, g.stride_o = out_h.data_ptr(), out_l.data_ptr(), N, M * N
        g.out_scale = out_scale
    _check(load().cq_gemm_x3(ctypes.byref(g), _stream(Ah.device)), "cq_gemm_x3")
    return C


def q_update_x3(W: torch.Tensor, L: torch.Tensor | None, R: torch.Tensor | None, bits: int, *, eps: float = 1e-8,
                codes=None, packed=None, scale=None, err_w=None, err_out=None, events=None, absmax_in=None,
                scale_hint=None, fallback_out=None):
    """Fused Q update: quantise res = W - L R (W alone if L is None) per matrix, never
    materialising res.  W (B, m, n) fp16/fp32, L (B, m, r), R (B, r, n) fp32 with r % 32 == 0.
    Fills packed (B, m*n*bits/8) uint8 and/or codes, scale (B,), err_out (B,) fp64.
    scale_hint (B,) fp32 (may be `scale` itself): the previous Q update's scales -- 2-bit
    packed codes are then produced with one recompute of L R (candidate lists, see
    include/caldera_hip.h); fallback_out (B,) int32 reports matrices that needed the second."""
    _require_hip(W, L, R, codes, packed, scale, err_w, err_out, scale_hint, fallback_out)
    assert W.is_contiguous()
    B, m, n = W.shape
    dt = {torch.float16: CQ_F16, torch.float32: CQ_F32}[W.dtype]
    dev = W.device
    r = 0 if L is None else L.shape[-1]
    halves = [None] * 4
    inv = None
    if r:
        sL = pow2_scale(L.contiguous(), 14)
        sR = pow2_scale(R.contiguous(), 14)
        Lh, Ll = split_f16(L.contiguous(), sL)
        Rth = torch.empty((B, n, r), dtype=torch.float16, device=dev)
        Rtl = torch.empty_like(Rth)
        transpose_split(R.contiguous(), hi=Rth, lo=Rtl, scale=sR)
        inv = 1.0 / (sL * sR)
        halves = [Lh, Ll, Rth, Rtl]
    lib = load()
    # the hint only matters to the 2-bit packed path on fp16 W (the C side ignores it
    # otherwise): only then is the list workspace (~0.22 B per element from 2^22 elements on:
    # single candidates 8 B each for 15.5 % of the 8-element groups, whole groups 36 B each for
    # 1.5 %; smaller matrices 50 % and 25 %) sized and cached (scratch.py)
    hint = (scale_hint is not None and r > 0 and bits == 2 and packed is not None and codes is None
            and W.dtype == torch.float16)
    if not hint:
        scale_hint = None
    ws = scratch.get("q_update.ws_list" if hint else "q_update.ws",
                     (max(int(lib.cq_q_update_workspace(m, n, B, int(hint))), 16),), torch.uint8, dev)
    if events is not None:  # HIP events around the quantise kernels only (bench roofline)
        events[0].record()
    _check(lib.cq_q_update_x3(dt, _p(W), m, n, r, B, *[_p(t) for t in halves], _p(inv), bits, float(eps), _p(codes),
                              _p(packed), _p(scale), _p(err_w), _wst(err_w, B), _p(err_out),
                              _p(absmax_in if r == 0 else None),
                              _p(scale_hint if r else None), _p(fallback_out), _p(ws), ws.numel(), _stream(dev)),
           "cq_q_update_x3")
    if events is not None:
        events[1].record()


def q_update_list_geometry(m: int, n: int, r: int, both: bool = False):
    """(rows of W per list region, capacity of its single-candidate list[, capacity of its
    list of groups with two or more candidates]) of the 2-bit single-recompute Q update
    (cq_q_update_list_geometry), or None where it does not apply."""
    rows, cap, capb = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
    if load().cq_q_update_list_geometry(m, n, r, ctypes.byref(rows), ctypes.byref(cap), ctypes.byref(capb)) != 0:
        return None
    return (int(rows.value), int(cap.value), int(capb.value)) if both else (int(rows.value), int(cap.value))


def absmax(X: torch.Tensor) -> torch.Tensor:
    """(B,) fp32 max |X[b]| of a (B, ...) fp16/fp32 tensor."""
    _require_hip(X)
    X = X.contiguous()
    B = X.shape[0]
    dt = {torch.float16: CQ_F16, torch.float32: CQ_F32}[X.dtype]
    out = torch.empty(B, dtype=torch.float32, device=X.device)
    _check(load().cq_absmax(dt, _p(X), X.numel() // B, B, _p(out), _stream(X.device)), "cq_absmax")
    return out


def sgram_split(k: int, L: int) -> int:
    """The l-split point of the sparse-code Gram's ELL for a k x L code matrix (L: no split)."""
    return int(load().cq_sgram_split(k, L))


def sgram_count(packed, k, L, row_nnz, perm, slice_off, total, W=None, qscale=None, wcol=None, corr_ws=None,
                corr_out=None, Lh=None, row_nnz1=None, slice_w1=None):
    """Sliced-ELL layout of the nonzero 2-bit codes per row (cq_sgram_count): packed (B, k*L/4).
    With W (B, k, L) fp16: corr_out (B,) fp64 = ||(W - s c) diag(ycol)||^2 - ||W diag(ycol)||^2
    (wcol = ycol^2), corr_ws (B * k,) fp64 scratch.  Lh < L (sgram_split): the l-split layout,
    row_nnz1 (B * k,) int32 scratch, slice_w1 (B * ceil(k / 64),) int32 out."""
    _require_hip(packed, row_nnz, perm, slice_off, total, W, qscale, wcol, corr_ws, corr_out, row_nnz1, slice_w1)
    B = total.numel()
    Lh = L if Lh is None else Lh
    ns = -(-k // 64)
    assert row_nnz.numel() >= B * k and perm.numel() >= B * k and slice_off.numel() >= B * (ns + 1)
    assert Lh >= L or (row_nnz1.numel() >= B * k and slice_w1.numel() >= B * ns and slice_w1.dtype == torch.int32)
    if W is not None:
        assert W.dtype == torch.float16 and W.is_contiguous() and W.shape == (B, k, L)
        assert corr_ws.numel() >= B * k and corr_ws.dtype == torch.float64 and corr_out.numel() == B
    _check(load().cq_sgram_count(_p(packed), 2, B, k, L, _p(row_nnz), _p(perm), _p(slice_off), _p(total), Lh,
                                 _p(row_nnz1), _p(slice_w1), _p(W), _p(qscale), _p(wcol), _wst(wcol, B), _p(corr_ws),
                                 _p(corr_out),
                                 _stream(packed.device)), "cq_sgram_count")


def sgram_fill(packed, k, L, row_nnz, perm, slice_off, ell, stride, Lh=None, slice_w1=None):
    _require_hip(packed, row_nnz, perm, slice_off, ell, slice_w1)
    B = slice_off.numel() // (-(-k // 64) + 1)
    assert ell.numel() >= B * stride
    Lh = L if Lh is None else Lh
    _check(load().cq_sgram_fill(_p(packed), 2, B, k, L, _p(row_nnz), _p(perm), _p(slice_off), _p(slice_w1), Lh,
                                stride, _p(ell), _stream(packed.device)), "cq_sgram_fill")


def codes_transpose(packed, rows, cols, out=None):
    """2-bit packed codes (B, rows*cols/4) -> the packed codes of the transposes (B, cols*rows/4)."""
    _require_hip(packed, out)
    B = packed.shape[0]
    assert packed.dtype == torch.uint8 and packed.is_contiguous() and packed.numel() == B * rows * cols // 4
    if out is None:
        out = torch.empty_like(packed)
    assert out.shape == packed.shape and out.is_contiguous() and out.data_ptr() != packed.data_ptr()
    _check(load().cq_codes_transpose(_p(packed), 2, B, rows, cols, _p(out), _stream(packed.device)),
           "cq_codes_transpose")
    return out


CODES_MATMUL_MAX_R = 256  # cq_codes_matmul's r limit (cq_sgram.hip: RV <= 4 columns per lane)


def codes_matmul(packed, rows, cols, X, r, out, *, colw=None, roww=None, trans=False):
    """out[b] = diag(roww) c[b] diag(colw) X[b][:, :r] (rows x r; trans: its transpose, r x rows) for
    2-bit packed codes c (B, rows, cols) and X (B, cols, ldx) fp32 (cq_codes_matmul)."""
    _require_hip(packed, X, colw, roww, out)
    B = packed.shape[0]
    assert roww is None or (roww.shape[-1] == rows and roww.dtype == torch.float32 and roww.is_contiguous())
    assert packed.numel() == B * rows * cols // 4 and X.shape[:2] == (B, cols) and X.stride(2) == 1
    assert X.dtype == torch.float32 and out.dtype == torch.float32 and out.is_contiguous()
    assert out.shape == ((B, r, rows) if trans else (B, rows, r))
    assert colw is None or (colw.shape[-1] == cols and colw.dtype == torch.float32 and colw.is_contiguous())
    _check(load().cq_codes_matmul(_p(packed), 2, B, rows, cols, _p(X), X.stride(1), X.stride(0), _p(colw), _wst(colw, B),
                                  _p(roww), _wst(roww, B), r, _p(out),
                                  out.shape[2], out.stride(0), int(bool(trans)), _stream(packed.device)),
           "cq_codes_matmul")
    return out


def codes_ysq_corr(packed, W, qscale, colw=None, out=None):
    """(B,) fp64: ||(W - s c) diag(ycol)||^2 - ||W diag(ycol)||^2 (colw = ycol^2) over the nonzero
    2-bit codes c of W (B, m, n) fp16 (cq_codes_ysq_corr)."""
    _require_hip(packed, W, qscale, colw, out)
    B, m, n = W.shape
    assert W.dtype == torch.float16 and W.is_contiguous() and packed.numel() == B * m * n // 4
    if out is None:
        out = torch.empty(B, dtype=torch.float64, device=W.device)
    _check(load().cq_codes_ysq_corr(_p(packed), 2, _p(W), CQ_F16, _p(qscale), _p(colw), _wst(colw, B), B, m, n, _p(out),
                                    _stream(W.device)), "cq_codes_ysq_corr")
    return out


def transpose_f16(X, out=None):
    """(B, rows, cols) fp16 -> (B, cols, rows) (cq_transpose_f16)."""
    _require_hip(X, out)
    B, rows, cols = X.shape
    assert X.dtype == torch.float16 and X.is_contiguous()
    if out is None:
        out = torch.empty((B, cols, rows), dtype=torch.float16, device=X.device)
    assert out.shape == (B, cols, rows) and out.is_contiguous()
    _check(load().cq_transpose_f16(_p(X), B, rows, cols, _p(out), _stream(X.device)), "cq_transpose_f16")
    return out


def sgram_rows(L: int) -> int:
    return int(load().cq_sgram_rows(L))


def sgram_spmm(W, packed, qscale, wcol, ell, perm, slice_off, stride, P, Lh=None, slice_w1=None):
    """P (B, k, k) = (W - (s/2) c) diag(wcol) c^T over the ELL codes (cq_sgram_spmm); wcol = the Gram's
    column weights w = ycol^2 (None: 1).  Lh / slice_w1: the l-split layout of sgram_count."""
    _require_hip(W, packed, qscale, wcol, ell, perm, slice_off, P, slice_w1)
    B, k, L = W.shape
    assert W.dtype == torch.float16 and W.is_contiguous() and P.shape == (B, k, k) and P.is_contiguous()
    assert wcol is None or (wcol.shape[-1] == L and wcol.dtype == torch.float32)
    Lh = L if Lh is None else Lh
    _check(load().cq_sgram_spmm(CQ_F16, _p(W), _p(packed), _p(qscale), _p(wcol), _wst(wcol, B), B, k, L, _p(ell), _p(perm),
                                _p(slice_off), _p(slice_w1), Lh, stride, _p(P), _stream(W.device)), "cq_sgram_spmm")


def sgram_combine(A, P, qscale, bound, out_scale, Gh, Gl, scale_out, inv_out, G32=None):
    """G = A - s (P + P^T) -> K-blocked split halves (cq_sgram_combine)."""
    _require_hip(A, P, qscale, bound, Gh, Gl, scale_out, inv_out, G32)
    B, k, _ = P.shape
    assert A.shape == P.shape and Gh.numel() >= B * k * k and Gl.numel() >= B * k * k
    assert G32 is None or G32.shape == (B, k, k)
    _check(load().cq_sgram_combine(_p(A), _p(P), _p(qscale), B, k, _p(bound), float(out_scale), _p(Gh), _p(Gl),
                                   _p(scale_out), _p(inv_out), _p(G32), _stream(P.device)), "cq_sgram_combine")


def residual_split(Ws, packed, qscale, bits, wmax, *, ycol=None, ycol_max=1.0, res=None, Y=None, hi=None, lo=None,
                   thi=None, tlo=None, scale=None, sq=None, ycol_hi=None, ycol_hi_max=1.0, scale_hi=None):
    """Fused LR-step residual (see include/caldera_hip.h cq_residual_split).  Ws (B, m, n).
    ycol_hi: hi/lo are the halves of res * ycol_hi (their scale in scale_hi) instead.
    Per-matrix weights: ycol / ycol_hi (B, n) with ycol_max / ycol_hi_max (B,) fp32 tensors."""
    _require_hip(Ws, packed, qscale, wmax, ycol, res, Y, hi, lo, thi, tlo, scale, sq, ycol_hi, scale_hi)
    B, m, n = Ws.shape
    dt = {torch.float16: CQ_F16, torch.float32: CQ_F32}[Ws.dtype]
    yst = max(_wst(ycol, B), _wst(ycol_hi, B))
    assert ycol is None or ycol_hi is None or ycol.shape == ycol_hi.shape
    ymv = ycol_max if torch.is_tensor(ycol_max) else None
    yhmv = ycol_hi_max if torch.is_tensor(ycol_hi_max) else None
    for t in (ymv, yhmv):
        assert t is None or (t.dtype == torch.float32 and t.numel() == B and t.is_contiguous() and t.is_cuda)
    lib = load()
    ws = workspace(lib.cq_residual_split_workspace(m, n, B), Ws.device) if sq is not None else None
    _check(lib.cq_residual_split(dt, _p(Ws), _p(packed), _p(qscale), int(bits), _p(ycol),
                                 1.0 if ymv is not None else float(ycol_max), _p(wmax),
                                 B, m, n, _p(res), _p(Y), _p(hi), _p(lo), _p(thi), _p(tlo), _p(scale), _p(sq),
                                 _p(ycol_hi), 1.0 if yhmv is not None else float(ycol_hi_max), _p(scale_hi), yst,
                                 _p(ymv), _p(yhmv), _p(ws),
                                 0 if ws is None else ws.numel(), _stream(Ws.device)), "cq_residual_split")


# ---------------------------------------------------------------------------- calibration
_ACT_DT = {torch.float32: CQ_F32, torch.float16: CQ_F16, torch.bfloat16: CQ_BF16}


def _act_2d(x: torch.Tensor):
    """(rows, cols) view with unit column stride, or a contiguous copy."""
    if x.dtype not in _ACT_DT:
        raise TypeError(f"activations must be fp32/fp16/bf16, got {x.dtype}")
    if x.dim() != 2:
        raise ValueError("activations must be 2-D (rows, cols)")
    if x.stride(1) != 1 or (x.shape[0] > 1 and x.stride(0) < x.shape[1]):
        x = x.contiguous()
    return x, (x.stride(0) if x.shape[0] > 1 else x.shape[1])


def act_sqsum_cols(x: torch.Tensor, out: torch.Tensor, *, accumulate: bool = True, post: float = 1.0):
    """out (cols,) fp64 <- ((accumulate ? out : 0) + sum_i x[i, :]^2) * post  (diag of X^T X)."""
    _require_hip(x, out)
    x, ld = _act_2d(x)
    rows, cols = x.shape
    assert out.dtype == torch.float64 and out.numel() == cols and out.is_contiguous()
    lib = load()
    nws = lib.cq_act_sqsum_workspace(rows, cols)
    ws = workspace(nws, x.device) if nws else None
    _check(lib.cq_act_sqsum_cols(_ACT_DT[x.dtype], _p(x) if rows else None, rows, cols, max(ld, cols), _p(out),
                                 int(bool(accumulate)), float(post), _p(ws), 0 if ws is None else ws.numel(),
                                 _stream(x.device)), "cq_act_sqsum_cols")
    return out


def act_sqsum_rows(x: torch.Tensor, out: torch.Tensor, *, accumulate: bool = True, post: float = 1.0):
    """out (rows,) fp64 <- ((accumulate ? out : 0) + sum_j x[:, j]^2) * post  (diag of X X^T)."""
    _require_hip(x, out)
    x, ld = _act_2d(x)
    rows, length = x.shape
    assert out.dtype == torch.float64 and out.numel() == rows and out.is_contiguous()
    _check(load().cq_act_sqsum_rows(_ACT_DT[x.dtype], _p(x) if length else None, rows, length, max(ld, length),
                                    _p(out), int(bool(accumulate)), float(post), _stream(x.device)),
           "cq_act_sqsum_rows")
    return out
