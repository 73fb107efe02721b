"""CPU-side checks: the C-ABI library loads and exports everything include/caldera_hip.h
declares (no device calls), and the drop-in Python surface mirrors the reference's names,
defaults and exceptions (RCR/src/caldera/utils/{dataclasses,quantization}.py)."""
import ctypes
import dataclasses
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "caldera_hip.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(cq_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    lib = K.load()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(K.EXPORTS), set(names) ^ set(K.EXPORTS)
    assert lib.cq_abi_version() == K.ABI_VERSION == 5
    assert isinstance(lib.cq_last_error(), bytes)


def header_param_counts():
    """{function: number of parameters} of every prototype in include/caldera_hip.h."""
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(cq_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", txt):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else args.count(",") + 1
    return out


def test_ctypes_signatures_match_header_arity():
    """Every ctypes declaration in _lib.py passes as many arguments as the header's prototype
    takes (ABI 5 added weight batch strides to twelve entries: a missed one would shift every
    later argument)."""
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    counts = header_param_counts()
    assert set(counts) == set(K.EXPORTS)
    for name, (_, args) in K._SIGS.items():
        assert len(args) == counts[name], (name, len(args), counts[name])


def _struct_fields(name):
    txt = open(HEADER).read()
    body = txt[txt.index(f"typedef struct {name}"):txt.index(f"}} {name};")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    return re.findall(r"([A-Za-z_][A-Za-z0-9_]*)\s*[;,]", body.split("{", 1)[1])


def test_gemm_args_struct_matches_header():
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    assert [f for f, _ in K.GemmArgs._fields_] == _struct_fields("cq_gemm_args")
    assert [f for f, _ in K.X3Args._fields_] == _struct_fields("cq_x3_args")


def test_q_update_list_workspace_fits_1gb():
    """The 2-bit list workspace of the bench batch (B = 256 x 4096^2, rank 128) stays within
    1 GB; the region capacities are the measured-density fractions of csrc/cq_x3.h."""
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    lib = K.load()
    assert lib.cq_q_update_workspace(4096, 4096, 256, 1) <= 1_000_000_000
    rows, capA, capB = K.q_update_list_geometry(4096, 4096, 128, both=True)
    groups = rows * 4096 // 8
    assert capA >= 0.155 * groups and capB >= 0.015 * groups


def test_caldera_params_defaults_match_reference():
    from src.caldera.utils.dataclasses import CalderaParams, CalderaDecomposition, QuantInfo
    p = CalderaParams()
    # dataclasses.py:11-84
    assert (p.compute_quantized_component, p.compute_low_rank_factors) == (True, True)
    assert (p.Q_bits, p.L_bits, p.R_bits, p.rank, p.iters, p.lplr_iters) == (2, 2, 2, 64, 20, 5)
    assert p.activation_aware_LR is True and p.update_order == [] and p.rand_svd is False
    assert p.sigma_reg == 0
    assert p.quant_factory_Q.method == "uniform" and p.quant_factory_Q.block_size == 64
    names = [f.name for f in dataclasses.fields(CalderaDecomposition)]
    assert names == ["Q", "L", "R", "W", "Q_idxs", "L_idxs", "R_idxs", "Q_scale", "L_scale",
                     "R_scale", "global_scale", "SU", "SV", "scaleWH", "errors"]
    d = CalderaDecomposition()
    assert d.Q_scale == 1 and d.global_scale == 1 and d.errors == {}
    assert QuantInfo().quant.num_bits == 2


def test_quantizer_exceptions_match_reference():
    from src.caldera.utils.quantization import LowMemoryQuantizer, QuantizerFactory
    with pytest.raises(AssertionError, match="Bit-width not supported!"):
        LowMemoryQuantizer(num_bits=3)
    with pytest.raises(NotImplementedError):
        LowMemoryQuantizer(method="lattice")
    with pytest.raises(ValueError):
        LowMemoryQuantizer(num_bits=2, method="nf4")
    with pytest.raises(ValueError):
        LowMemoryQuantizer(num_bits=4, method="nf2")
    with pytest.raises(ValueError):
        LowMemoryQuantizer(num_bits=2, method="bbint4")
    q = LowMemoryQuantizer(4, "uniform", 64)
    with pytest.raises(ValueError):
        q.quantize_block(torch.zeros(4, 4, 4))
    with pytest.raises(ValueError):
        q.quantize_block(torch.zeros(3, 5))
    f = QuantizerFactory("uniform", 32)
    assert str(f) == "QuantizerFactory(method=uniform, block_size=32)"
    assert f.get_quantizer(8).block_size == 32


def test_drop_in_module_star_exports():
    import src.caldera.decomposition.alg as alg
    for n in ("caldera", "CalderaParams", "CalderaDecomposition", "QuantInfo", "QuantizerFactory",
              "LowMemoryQuantizer", "AbstractQuantizer", "quantize_matrix", "get_quant_info"):
        assert hasattr(alg, n), n


@pytest.mark.skipif(torch.cuda.is_available(), reason="CPU-only behaviour")
def test_no_cpu_fallback():
    from src.caldera.decomposition.alg import caldera, CalderaParams
    with pytest.raises(RuntimeError, match="no HIP device"):
        caldera(CalderaParams(update_order=["Q"]), torch.randn(8, 8), device="cpu")


def test_diagonal_h_detection_and_weights():
    from ee274_convexcaldera_llm_quantization_amd.api import _diag_of
    from ee274_convexcaldera_llm_quantization_amd.engine import EngineParams, _Weights
    h = torch.tensor([1.0, 0.0, 2.0, 0.5])
    assert torch.equal(_diag_of(torch.diag(h), 4), h)
    H = torch.diag(h)
    H[0, 1] = 1e-3
    assert _diag_of(H, 4) is not None and _diag_of(H, 4).dim() == 2  # dense H goes through whole
    with pytest.raises(ValueError):
        _diag_of(torch.eye(3), 4)
    # alg.py:59-64: shift by sigma_reg - lambda_min when lambda_min < sigma_reg (fp32 arithmetic)
    w = _Weights(h, 4, EngineParams(sigma_reg=1e-8, activation_aware_LR=True), "cpu")
    shift = torch.tensor(1e-8, dtype=torch.float32) - h.min()
    assert torch.equal(w.err, h + shift)
    assert torch.equal(w.ycol, torch.sqrt(h + shift))
    # identity fast path (alg.py:11-21): eigenvalues exactly one, H itself unchanged
    w2 = _Weights(torch.full((4,), 1.0 + 1e-7), 4, EngineParams(), "cpu")
    assert w2.ycol is None and w2.rinv is None and torch.all(w2.err == 1.0 + 1e-7)
    # not data-aware: H_sqrt = H -> lplr weights h^2, activation error weights h
    w3 = _Weights(h, 4, EngineParams(activation_aware_LR=False), "cpu")
    assert torch.equal(w3.lplr, h * h) and torch.equal(w3.err, h)


def test_default_parts_policy():
    """Batches of 16 matrices and more are decomposed as two interleaved parts by default
    (overlap.default_parts: +13-14 % at B = 16 / 32, +5-9 % on configs 2-5), smaller ones as one
    (they rely on split-K, which interleaving turns off: B = 8 / 4 measured slower)."""
    from ee274_convexcaldera_llm_quantization_amd.overlap import default_parts
    assert [default_parts(b) for b in (1, 4, 8, 15)] == [1, 1, 1, 1]
    assert [default_parts(b) for b in (16, 32, 64, 256)] == [2, 2, 2, 2]
