"""Host-side tests of the layer-replacement caller (main.py:135-251) and the calibration
oracle (main.py:296-308): selection, counters and bit accounting, Hadamard matrices, and the
oracle against the golden calibration vectors.  No GPU."""
import numpy as np
import pytest
import scipy.linalg
import torch

from conftest import load_golden
from oracle import caldera_oracle as O
from ee274_convexcaldera_llm_quantization_amd import model as M


class _Block(torch.nn.Module):
    def __init__(self, h, i):
        super().__init__()
        self.self_attn = torch.nn.Module()
        self.self_attn.q_proj = torch.nn.Linear(h, h, bias=False)
        self.self_attn.k_proj = torch.nn.Linear(h, 128, bias=False)  # <= 500 rows: skipped
        self.mlp = torch.nn.Module()
        self.mlp.up_proj = torch.nn.Linear(h, i, bias=False)
        self.mlp.down_proj = torch.nn.Linear(i, h, bias=False)
        self.input_layernorm = torch.nn.LayerNorm(h)


class TinyLlava(torch.nn.Module):
    """Module names shaped like LlavaOnevision's (language_model.model.layers.N..., vision_tower...)."""

    def __init__(self, n_layers=20, h=512, i=640):
        super().__init__()
        self.language_model = torch.nn.Module()
        self.language_model.model = torch.nn.Module()
        self.language_model.model.layers = torch.nn.ModuleList([_Block(h, i) for _ in range(n_layers)])
        self.language_model.lm_head = torch.nn.Linear(h, 600, bias=False)
        self.vision_tower = torch.nn.Module()
        self.vision_tower.fc1 = torch.nn.Linear(64, 64)


def _expected(model, layers, limit=10000, min_dim=500):
    """main.py:146-251's walk written out directly."""
    sel, q, u, v = [], 0, 0, 0
    counter = 1
    for name, mod in model.named_modules():
        if hasattr(mod, "weight") and "language" in name:
            if (any(k in name for k in M.PROJ_KEYS) and mod.weight.size(0) > min_dim and mod.weight.size(1) > min_dim
                    and any(f"layers.{i}" in name for i in layers) and counter <= limit):
                counter += 1
                sel.append(name)
            else:
                u += mod.weight.numel()
        elif hasattr(mod, "weight"):
            v += mod.weight.numel()
    return sel, u, v


@pytest.mark.parametrize("layers,limit", [(range(17, 24), 10000), ((1,), 10000), ((17, 18), 3), ((), 10000)])
def test_selection_matches_main_py(layers, limit):
    m = TinyLlava()
    sel = M.LayerSelection(layers=tuple(layers), limit=limit)
    jobs, rep = M.select_layers(m, None, sel)
    exp, u, v = _expected(m, tuple(layers), limit)
    assert [j[0] for j in jobs] == exp
    assert rep.unquantized_language_param_count == u and rep.vision_param_count == v
    if tuple(layers) == (1,):  # the reference's substring match: 'layers.1' also hits 10..19
        assert any("layers.17." in n for n in exp) and any("layers.1." in n for n in exp)
    if limit == 3:
        assert len(exp) == 3


def test_missing_hessian_raises_keyerror():
    m = TinyLlava(n_layers=18)
    with pytest.raises(KeyError):
        M.select_layers(m, {}, M.LayerSelection())


def test_caller_accounting_with_stub_decomposer(monkeypatch):
    """Threshold gate and counters (main.py:212-220), with a stand-in decomposition whose
    error is known; the HIP reconstruct / error helpers are replaced by torch on CPU here
    (the GPU test runs the real ones)."""
    m = TinyLlava(n_layers=20, h=512, i=640)
    for p in m.parameters():
        torch.nn.init.normal_(p, std=0.02)
    names = [n for n, _, _ in M.select_layers(m, None)[0]]
    bad = {names[1]}

    class Dec:
        def __init__(self, W, scale):
            self.Q, self.L, self.R = W.float() * scale, torch.zeros(W.shape[0], 1), torch.zeros(1, W.shape[1])
            self.errors = {"Q": [0.1]}

    calls = []

    def decompose(qp, Ws, H):
        calls.append((len(Ws), H))
        return [Dec(W, 0.0 if any(W.data_ptr() == dict(m.named_modules())[n].weight.data_ptr() for n in bad) else 0.5) for W in Ws]

    monkeypatch.setattr(M, "_reconstruct", lambda dec, dev: dec.Q + dec.L @ dec.R)
    monkeypatch.setattr(M, "_rel_error", lambda W, out: float(torch.linalg.norm(W.float() - out) / torch.linalg.norm(W.float())))
    before = {n: dict(m.named_modules())[n].weight.data.clone() for n in names}
    rep = M.apply_caldera_quantization(m, None, object(), decompose=decompose, device="cpu")
    assert [o.name for o in rep.layers] == names
    for o in rep.layers:
        W = dict(m.named_modules())[o.name].weight.data
        if o.name in bad:
            assert not o.applied and abs(o.rel_error - 1.0) < 1e-6
            assert torch.equal(W, before[o.name])
        else:
            assert o.applied and abs(o.rel_error - 0.5) < 1e-6
            assert torch.allclose(W, before[o.name] * 0.5)
    exp_sel, u, v = _expected(m, range(17, 24))
    nq = sum(before[n].numel() for n in names if n not in bad)
    assert rep.quantized_param_count == nq
    assert rep.unquantized_language_param_count == u + sum(before[n].numel() for n in bad)
    assert rep.total_bits == nq * 2 + rep.unquantized_language_param_count * 4
    assert rep.prior_total_bits == (nq + rep.unquantized_language_param_count) * 4
    # same-shape layers with H = None share a batch
    assert sum(c[0] for c in calls) == len(names) and max(c[0] for c in calls) > 1


def test_hadamard_matches_scipy():
    for n in (1, 2, 8, 64):
        Hm = M.normalized_hadamard(n, "cpu", torch.float64).numpy()
        np.testing.assert_allclose(Hm, scipy.linalg.hadamard(n) / np.sqrt(n), rtol=0, atol=1e-15)
    with pytest.raises(ValueError):
        M.normalized_hadamard(12, "cpu")


def test_calibration_oracle_against_golden():
    g = load_golden("calib_ref.npz")
    D, Ts = int(g["D"]), [int(t) for t in g["Ts"]]
    flat, off, samples = g["acts"], 0, []
    for T in Ts:
        samples.append(flat[off:off + T * D].reshape(1, T, D))
        off += T * D
    H = O.hessian_reference(samples)
    np.testing.assert_allclose(H, g["H"], rtol=1e-13, atol=0)
    np.testing.assert_allclose(O.hessian_reference(samples, diag_only=True), np.diag(g["H"]), rtol=1e-13)
    # mean mode: sum over tokens of a a^T / count
    Hm = O.hessian_mean(samples)
    X = np.concatenate([s.reshape(-1, D) for s in samples]).astype(np.float64)
    np.testing.assert_allclose(Hm, X.T @ X / X.shape[0], rtol=1e-12, atol=1e-14)
