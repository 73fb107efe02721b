"""NF4/NF2 and bbint4/bbint2 HIP quantisers (csrc/cq_codebook.hip) through the C-ABI and the
drop-in LowMemoryQuantizer, against the reference's own outputs (tests/golden/quant_kat.npz)
and the CPU oracle (oracle/caldera_oracle.py) on larger, ragged and batched inputs.
Bar: bit-exact codes, scales, mins, outlier lists and dequantised values."""
import os

import numpy as np
import pytest
import torch

from oracle import caldera_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
METHODS = (("nf4", 4), ("nf2", 2), ("bbint4", 4), ("bbint2", 2))


@pytest.fixture(scope="module")
def K():
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    K.load()
    return K


@pytest.fixture(scope="module")
def Q():
    from src.caldera.utils.quantization import LowMemoryQuantizer
    return LowMemoryQuantizer


def _inputs(kat):
    return [k[3:] for k in kat.files if k.startswith("in_")]


def _check_against(method, codes, prm, deq, exp_codes, exp_prm, exp_deq, key):
    np.testing.assert_array_equal(np.asarray(codes), exp_codes, err_msg=key)
    if method.startswith("bbint"):
        for a, b, what in zip(prm, exp_prm, ("min", "scale", "ovals", "oidx")):
            np.testing.assert_array_equal(np.asarray(a), b, err_msg=f"{key} {what}")
    else:
        np.testing.assert_array_equal(np.asarray(prm), exp_prm, err_msg=key)
    np.testing.assert_array_equal(np.asarray(deq), exp_deq, err_msg=key)


@pytest.mark.parametrize("method,bits", METHODS)
def test_kat_drop_in_bit_exact(Q, kat, method, bits, tmp_path, monkeypatch):
    """quantize_block / dequantize_block of the drop-in (CPU tensors in and out, as the
    reference is called) reproduce the reference's codes, params and dequant bit for bit."""
    monkeypatch.chdir(tmp_path)  # bbint appends to ./outlier_log.csv like the reference
    n = 0
    for name in _inputs(kat):
        x = kat["in_" + name]
        for bs in (64, "all"):
            key = f"{method}_b{bits}_bs{bs}_{name}"
            if key + "_codes" not in kat.files:
                continue
            q = Q(bits, method, x.size if bs == "all" else bs)
            c, prm, shape = q.quantize_block(torch.from_numpy(x.copy()))
            assert c.device.type == "cpu"
            d = q.dequantize_block(c, prm, shape)
            if method.startswith("bbint"):
                exp = tuple(kat[key + s] for s in ("_min", "_scale", "_ovals", "_oidx"))
                assert c.dtype == torch.uint8 and prm[3].dtype == torch.int64
                prm = tuple(t.numpy() for t in prm)
            else:
                exp = kat[key + "_scale"]
                prm = prm.numpy()
            _check_against(method, c.numpy(), prm, d.numpy(), kat[key + "_codes"], exp, kat[key + "_deq"], key)
            n += 1
    assert n > 0
    if method.startswith("bbint"):
        assert os.path.exists("outlier_log.csv")
        rows = open("outlier_log.csv").read().strip().splitlines()
        assert rows[0] == "Call_ID,Num_Outliers" and len(rows) == n + 1


def _planted(m, n, seed, n_out=40):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((m, n)) * 0.02).astype(np.float32)
    idx = rng.integers(0, m * n, n_out)
    x.reshape(-1)[idx] = (rng.choice([-1.0, 1.0], n_out) * rng.uniform(0.2, 0.5, n_out)).astype(np.float32)
    return x


@pytest.mark.parametrize("method,bits", METHODS)
@pytest.mark.parametrize("shape,bs", [((512, 1024), "all"), ((256, 384), 96), ((64, 256), 8192), ((33, 20), 4),
                                      ((128, 128), 256), ((96, 96), 1152)])
def test_against_oracle_shapes(K, method, bits, shape, bs):
    """Large whole-matrix blocks (multi-chunk reductions), ragged block sizes (rest path of
    the torch-order mean), tiny blocks; bit-exact against the oracle restatement."""
    x = _planted(*shape, seed=bits * 7 + shape[0])
    b = x.size if bs == "all" else bs
    if method.startswith("bbint") and b % (8 // bits):
        pytest.skip("packing needs block_size % (8/bits) == 0 (reference raises)")
    q = O.LowMemoryQuantizer(bits, method, b)
    c_ref, p_ref, _ = q.quantize_block(x)
    d_ref = q.dequantize_block(c_ref, p_ref, x.shape)
    xt = torch.from_numpy(x).to(DEV).view(1, -1)
    if method.startswith("nf"):
        out = K.quantize_nf(xt, b, bits)
        np.testing.assert_array_equal(out["idx"].cpu().numpy().reshape(-1, b), c_ref)
        np.testing.assert_array_equal(out["scale"].cpu().numpy().reshape(-1, 1), p_ref)
        np.testing.assert_array_equal(out["deq"].cpu().numpy().reshape(x.shape), d_ref)
    else:
        out = K.quantize_bbint(xt, b, bits)
        np.testing.assert_array_equal(out["packed"].cpu().numpy().reshape(c_ref.shape), c_ref)
        np.testing.assert_array_equal(out["bmin"].cpu().numpy().reshape(-1, 1), p_ref[0])
        np.testing.assert_array_equal(out["bscale"].cpu().numpy().reshape(-1, 1), p_ref[1])
        np.testing.assert_array_equal(out["vals"].cpu().numpy(), p_ref[2])
        np.testing.assert_array_equal(out["idx"].cpu().numpy(), p_ref[3])
        np.testing.assert_array_equal(out["deq"].cpu().numpy().reshape(x.shape), d_ref)
        d2 = K.dequantize_bbint(out["packed"], bits, out["bmin"], out["bscale"], out["vals"], out["idx"], b)
        np.testing.assert_array_equal(d2.cpu().numpy().reshape(x.shape), d_ref)


@pytest.mark.parametrize("method,bits", METHODS)
def test_batched_whole_matrix_with_error(K, method, bits):
    """B matrices quantised whole (quantize_matrix, alg.py:245-250) in one call: per-matrix
    results equal the single-matrix oracle; the weighted error equals sum w (deq - x)^2."""
    B, m, n = 3, 256, 512
    xs = [_planted(m, n, seed=100 + b, n_out=10 * (b + 1)) for b in range(B)]
    w = np.random.default_rng(5).uniform(0.5, 2.0, n).astype(np.float32)
    xt = torch.from_numpy(np.stack(xs)).to(DEV).view(B, -1)
    wt = torch.from_numpy(w).to(DEV)
    err = torch.empty(B, dtype=torch.float64, device=DEV)
    if method.startswith("nf"):
        out = K.quantize_nf(xt, m * n, bits, err_w=wt, err_ncols=n, err_out=err)
    else:
        out = K.quantize_bbint(xt, m * n, bits, err_w=wt, err_ncols=n, err_out=err)
    off = 0
    for b in range(B):
        q = O.LowMemoryQuantizer(bits, method, m * n)
        c_ref, p_ref, _ = q.quantize_block(xs[b])
        d_ref = q.dequantize_block(c_ref, p_ref, (m, n))
        np.testing.assert_array_equal(out["deq"][b].cpu().numpy().reshape(m, n), d_ref)
        if method.startswith("bbint"):
            k = out["n_out"][b]
            assert k == p_ref[2].size
            np.testing.assert_array_equal(out["vals"][off:off + k].cpu().numpy(), p_ref[2])
            np.testing.assert_array_equal(out["idx"][off:off + k].cpu().numpy(), p_ref[3])
            off += k
        e_ref = float((((d_ref.astype(np.float64) - xs[b]) ** 2) * w).sum())
        assert abs(float(err[b]) - e_ref) <= 1e-6 * max(e_ref, 1e-30)  # (deq - x)^2 squared in fp32, summed in fp64
