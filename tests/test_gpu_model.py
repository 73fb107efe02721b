"""GPU parity of the §8(f) callers: the Hessian calibration kernels and HessianCalibrator
(main.py:268-319) against the numpy oracle / golden vectors, and the layer-replacement
caller apply_caldera_quantization (main.py:135-251) against per-layer caldera() calls and
the CPU oracle.  Tolerances: fp64 sums of exact fp64 squares differ from numpy only by
summation order (rtol 1e-12); Q + L R within the north-star 1e-4 relative Frobenius."""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import caldera_oracle as O
from test_model_host import TinyLlava

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _K():
    from ee274_convexcaldera_llm_quantization_amd import _lib as K
    return K


def _np64(x):
    return x.detach().float().cpu().numpy().astype(np.float64)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("rows,cols", [(0, 96), (1, 7), (37, 100), (1000, 896), (4096, 4864)])
def test_act_sqsum_cols(dtype, rows, cols):
    K = _K()
    g = torch.Generator(device="cpu").manual_seed(rows * 7 + cols)
    x = (torch.randn(rows, cols, generator=g) * 3).to(dtype).to(DEV)
    out = torch.full((cols,), 5.0, dtype=torch.float64, device=DEV)
    K.act_sqsum_cols(x, out, accumulate=True, post=0.5)
    exp = (5.0 + (_np64(x) ** 2).sum(0)) * 0.5
    np.testing.assert_allclose(out.cpu().numpy(), exp, rtol=1e-12, atol=0)
    K.act_sqsum_cols(x, out, accumulate=False)
    np.testing.assert_allclose(out.cpu().numpy(), (_np64(x) ** 2).sum(0), rtol=1e-12, atol=0)


def test_act_sqsum_cols_strided_and_misaligned():
    K = _K()
    base = torch.randn(300, 260, device=DEV)
    for x in (base[:, :256], base[:, 1:257], base[5:, 3:203]):  # ld > cols; 4-byte offset (scalar path)
        out = torch.empty(x.shape[1], dtype=torch.float64, device=DEV)
        K.act_sqsum_cols(x, out, accumulate=False)
        np.testing.assert_allclose(out.cpu().numpy(), (_np64(x) ** 2).sum(0), rtol=1e-12)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
@pytest.mark.parametrize("rows,length", [(96, 5), (96, 0), (3, 1000), (4864, 1)])
def test_act_sqsum_rows(dtype, rows, length):
    K = _K()
    x = (torch.randn(rows, length) * 2).to(dtype).to(DEV)
    out = torch.full((rows,), 2.0, dtype=torch.float64, device=DEV)
    K.act_sqsum_rows(x, out, accumulate=True, post=1.0 / 3)
    exp = (2.0 + (_np64(x) ** 2).sum(1)) / 3
    np.testing.assert_allclose(out.cpu().numpy(), exp, rtol=1e-12, atol=0)


def _golden_samples():
    g = load_golden("calib_ref.npz")
    D, Ts = int(g["D"]), [int(t) for t in g["Ts"]]
    flat, off, samples = g["acts"], 0, []
    for T in Ts:
        samples.append(torch.from_numpy(flat[off:off + T * D].reshape(1, T, D).copy()))
        off += T * D
    return D, samples, g["H"]


def test_calibrator_reference_mode_golden():
    """main.py's arithmetic (view(D, -1), running /(idx+1)) on the golden vectors; each
    sample first runs an extra forward that the reference's hook overwrites."""
    from ee274_convexcaldera_llm_quantization_amd.calibration import HessianCalibrator
    D, samples, H_ref = _golden_samples()
    lin = torch.nn.Linear(D, 8).to(DEV)
    model = torch.nn.Sequential(lin)
    cal = HessianCalibrator(model, mode="reference", full=True, diag=True)
    with cal:
        for a in samples:
            model(torch.randn(1, 9, D, device=DEV))  # overwritten by the next call (main.py:51)
            model(a.to(DEV))
            cal.end_sample()
    Hd = cal.hessians()["0"]
    Hf = cal.hessians(full=True)["0"]
    np.testing.assert_allclose(Hf.cpu().numpy(), H_ref, rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(Hd.cpu().numpy(), np.diag(H_ref), rtol=1e-12)
    assert Hd.dtype == torch.float64


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_calibrator_mean_mode(dtype):
    from ee274_convexcaldera_llm_quantization_amd.calibration import HessianCalibrator
    torch.manual_seed(3)
    model = torch.nn.Sequential(torch.nn.Linear(200, 300), torch.nn.GELU(), torch.nn.Linear(300, 64)).to(DEV, dtype)
    seen = {"0": [], "2": []}
    hooks = [model[i].register_forward_hook(lambda m, inp, out, k=str(i): seen[k].append(inp[0].detach().clone()))
             for i in (0, 2)]
    cal = HessianCalibrator(model, mode="mean", full=True)
    with cal, torch.no_grad():
        for T in (1, 17, 256):
            model(torch.randn(2, T, 200, device=DEV, dtype=dtype))
            cal.end_sample()
    for h in hooks:
        h.remove()
    for k in ("0", "2"):
        blocks = [_np64(a) for a in seen[k]]
        np.testing.assert_allclose(cal.hessians()[k].cpu().numpy(), O.hessian_mean(blocks, diag_only=True),
                                   rtol=1e-12)
        np.testing.assert_allclose(cal.hessians(full=True)[k].cpu().numpy(), O.hessian_mean(blocks),
                                   rtol=1e-11, atol=1e-13)
    cal2 = HessianCalibrator(model, names=["2"])
    with pytest.raises(ValueError):
        cal2.hessians(full=True)


def _tiny_model(seed=0):
    torch.manual_seed(seed)
    m = TinyLlava(n_layers=19, h=512, i=640)
    for p in m.parameters():
        torch.nn.init.normal_(p, std=0.02)
    return m.to(DEV)


def _params(rank=16, iters=2):
    from ee274_convexcaldera_llm_quantization_amd.model import driver_params
    p = driver_params(rank)
    p.iters = iters
    return p


def test_caller_matches_per_layer_caldera_and_oracle():
    """Each replaced weight = Q + L R of caldera(W, diag_embed(h), scale_W=False) (what
    main.py:186-198 computes), and one layer against the CPU oracle within 1e-4."""
    from ee274_convexcaldera_llm_quantization_amd.model import apply_caldera_quantization, select_layers
    from src.caldera.decomposition.alg import caldera
    m = _tiny_model()
    g = torch.Generator().manual_seed(11)
    names = [j[0] for j in select_layers(m)[0]]
    hess = {n: (torch.rand(dict(m.named_modules())[n].weight.shape[1], generator=g, dtype=torch.float64) + 0.05)
            for n in names}
    W0 = {n: dict(m.named_modules())[n].weight.data.clone() for n in names}
    qp = _params()
    rep = apply_caldera_quantization(m, hess, qp)
    assert [o.name for o in rep.layers] == names and all(o.applied for o in rep.layers)
    for i, n in enumerate(names):
        d = caldera(_params(), W0[n], torch.diag_embed(hess[n].float()).to(DEV), device=DEV, use_tqdm=False,
                    scale_W=False)
        exp = (d.Q.double() + d.L.double() @ d.R.double()).float()
        got = dict(m.named_modules())[n].weight.data
        rel = float(torch.linalg.norm(got - exp) / torch.linalg.norm(exp))
        assert rel < 1e-5, (n, rel)
        err = float(torch.linalg.norm(W0[n] - got) / torch.linalg.norm(W0[n]))
        assert abs(err - rep.layers[i].rel_error) < 1e-6
        if i == 0:
            ref = O.caldera(O.Params(Q_bits=2, L_bits=16, R_bits=16, rank=16, iters=2, update_order=["Q", "LR"],
                                     sigma_reg=1e-8), W0[n].cpu().numpy(), np.diag(hess[n].numpy().astype(np.float32)),
                            scale_W=False)
            o = ref.Q.astype(np.float64) + ref.L.astype(np.float64) @ ref.R.astype(np.float64)
            assert np.linalg.norm(got.cpu().numpy() - o) / np.linalg.norm(o) < 1e-4
    assert rep.quantized_param_count == sum(W0[n].numel() for n in names)


def test_caller_threshold_and_hadamard():
    from ee274_convexcaldera_llm_quantization_amd.model import (apply_caldera_quantization, hadamard_transform,
                                                                  select_layers)
    # Hadamard transform on the device: orthogonal round trip (main.py:108-133)
    W = torch.randn(300, 700, device=DEV)
    T, shp = hadamard_transform(W)
    assert T.shape == (512, 1024) and shp == (300, 700)
    back = hadamard_transform(T, inverse=True, original_shape=shp)
    assert float(torch.linalg.norm(back - W) / torch.linalg.norm(W)) < 1e-5
    m = _tiny_model(1)
    names = [j[0] for j in select_layers(m)[0]]
    W0 = {n: dict(m.named_modules())[n].weight.data.clone() for n in names}
    rep = apply_caldera_quantization(m, None, _params(), hadamard=True)
    # main.py:221-240: the Hadamard branch writes back unconditionally and counts nothing
    skipped_only = select_layers(_tiny_model(1))[1].unquantized_language_param_count
    assert rep.quantized_param_count == 0 and rep.unquantized_language_param_count == skipped_only
    rep_gate0 = apply_caldera_quantization(_tiny_model(1), None, _params(), hadamard=True, error_threshold=0.0)
    assert all(o.applied for o in rep_gate0.layers) and rep_gate0.quantized_param_count == 0
    for o in rep.layers:
        assert o.applied and 0.0 < o.rel_error < 0.99
        if o.shape == (512, 512):  # no padding: the orthogonal transform keeps the error
            assert abs(o.rel_error - min(o.errors["LR"])) < 1e-4
        got = dict(m.named_modules())[o.name].weight.data
        assert got.shape == W0[o.name].shape
    # threshold 0: nothing applied, weights restored and counted unquantised
    m2 = _tiny_model(2)
    W2 = {n: dict(m2.named_modules())[n].weight.data.clone() for n in names}
    rep2 = apply_caldera_quantization(m2, None, _params(), error_threshold=0.0)
    assert rep2.quantized_param_count == 0 and not any(o.applied for o in rep2.layers)
    for n in names:
        assert torch.equal(dict(m2.named_modules())[n].weight.data, W2[n])


def test_calibrate_then_quantize_end_to_end(tmp_path):
    """main.py's whole flow on a tiny LLaVA-shaped model: hook-based calibration (reference
    mode) saved in the diag_Hessians.pt layout, reloaded with the safe loader, then the layer
    replacement with those Hessians; every replaced layer matches caldera() with
    diag_embed(Hall[name]) (main.py:163-196)."""
    from ee274_convexcaldera_llm_quantization_amd.calibration import HessianCalibrator
    from ee274_convexcaldera_llm_quantization_amd.model import apply_caldera_quantization, select_layers
    from src.caldera.decomposition.alg import caldera
    m = _tiny_model(4)
    names = [j[0] for j in select_layers(m)[0]]
    mods = dict(m.named_modules())
    cal = HessianCalibrator(m, names=names, mode="reference")
    with cal, torch.no_grad():
        for s in range(3):
            for n in names:  # drive each selected layer with its own calibration activations
                lin = mods[n]
                lin(torch.randn(1, 5 + s, lin.in_features, device=DEV))
            cal.end_sample()
    path = tmp_path / "diag_Hessians.pt"
    cal.save(str(path))
    Hall = torch.load(str(path), weights_only=True)
    assert set(Hall) == set(names) and all(v.dtype == torch.float64 and v.dim() == 1 for v in Hall.values())
    W0 = {n: mods[n].weight.data.clone() for n in names}
    rep = apply_caldera_quantization(m, Hall, _params())
    assert all(o.applied for o in rep.layers)
    for n in names[:3]:
        d = caldera(_params(), W0[n], torch.diag_embed(Hall[n].float()).to(DEV), device=DEV, use_tqdm=False,
                    scale_W=False)
        exp = d.Q.double() + d.L.double() @ d.R.double()
        got = mods[n].weight.data.double()
        assert float(torch.linalg.norm(got - exp) / torch.linalg.norm(exp)) < 1e-5
