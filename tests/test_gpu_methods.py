"""caldera() with the codebook quantisers (nf4 / nf2 / bbint4 / bbint2) for Q and for the
quantised low-rank factors, against the CPU oracle on the same W.

Bar: the first Q update quantises W/gs (no float solve in between), so its error matches
to 1e-6; the first LR update (SVD of W - Q) to 1e-4; with quantised factors the LPLR loop
(lstsq + 2/4-bit codes) is chaotic after its first step, so those errors
are compared at 2e-2 and the API layout is checked exactly."""
import numpy as np
import pytest
import torch

from oracle import caldera_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module")
def api():
    from src.caldera.decomposition.alg import caldera, CalderaParams, QuantizerFactory
    return caldera, CalderaParams, QuantizerFactory


def _W(m=256, n=512, seed=0):
    torch.manual_seed(seed)
    return (torch.randn(m, n) * 0.02).half()


@pytest.mark.parametrize("method,bits", [("nf4", 4), ("nf2", 2), ("bbint4", 4), ("bbint2", 2)])
def test_codebook_Q(api, method, bits, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    caldera, CP, QF = api
    W = _W()
    d = caldera(CP(Q_bits=bits, L_bits=16, R_bits=16, rank=16, iters=2, update_order=["Q", "LR"],
                   sigma_reg=1e-8, quant_factory_Q=QF(method, 64)), W.to(DEV), None, device=DEV, use_tqdm=False)
    ref = O.caldera(O.Params(Q_bits=bits, L_bits=16, R_bits=16, rank=16, iters=2, update_order=["Q", "LR"],
                             sigma_reg=1e-8, method_Q=method), W.numpy())
    assert abs(d.errors["Q"][0] - ref.errors["Q"][0]) < 1e-6, (d.errors, ref.errors)
    assert abs(d.errors["LR"][0] - ref.errors["LR"][0]) < 1e-4, (d.errors, ref.errors)
    for k in ("Q", "LR"):
        np.testing.assert_allclose(d.errors[k], ref.errors[k], rtol=0, atol=1e-3)
    out = (d.Q.double() + d.L.double() @ d.R.double()).cpu().numpy()
    exp = ref.Q.astype(np.float64) + ref.L.astype(np.float64) @ ref.R.astype(np.float64)
    assert np.linalg.norm(out - exp) / np.linalg.norm(exp) < 2e-3
    # layout of the reference's return values
    m, n = W.shape
    if method.startswith("nf"):
        assert d.Q_idxs.dtype == torch.uint8 and d.Q_idxs.shape == (1, m * n)
        assert d.Q_scale.shape == (1, 1)
    else:
        cb = 4 if method == "bbint4" else 2
        assert d.Q_idxs.dtype == torch.uint8 and d.Q_idxs.shape == (1, m * n * cb // 8)
        mn, sc, vals, idx = d.Q_scale
        assert mn.shape == (1, 1) and sc.shape == (1, 1) and idx.shape == (vals.numel(), 2)
        assert idx.dtype == torch.int64
        # the stored Q is the dequantisation of the stored codes + params
        from src.caldera.utils.quantization import LowMemoryQuantizer
        q = LowMemoryQuantizer(bits, method, m * n)
        Qre = q.dequantize_block(d.Q_idxs, d.Q_scale, (m, n))
        assert torch.equal(Qre.cpu(), d.Q.cpu())


@pytest.mark.parametrize("method", ["nf4", "bbint4", "uniform"])
def test_quantized_factors_methods(api, method, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    caldera, CP, QF = api
    W = _W(256, 256, seed=3)
    r = 16
    d = caldera(CP(Q_bits=2, L_bits=4, R_bits=4, rank=r, iters=2, lplr_iters=3, update_order=["Q", "LR"],
                   sigma_reg=1e-8, quant_factory_LR=QF(method, 64)), W.to(DEV), None, device=DEV,
                use_tqdm=False)
    ref = O.caldera(O.Params(Q_bits=2, L_bits=4, R_bits=4, rank=r, iters=2, lplr_iters=3,
                             update_order=["Q", "LR"], sigma_reg=1e-8, method_LR=method), W.numpy())
    assert abs(d.errors["Q"][0] - ref.errors["Q"][0]) < 1e-6
    np.testing.assert_allclose(d.errors["LR"], ref.errors["LR"], rtol=0, atol=2e-2)
    m, n = W.shape
    if method == "nf4":
        assert d.L_idxs.shape == (1, r * m) and d.L_idxs.dtype == torch.uint8
        assert d.R_idxs.shape == (1, r * n) and d.L_scale.shape == (1, 1)
    elif method == "bbint4":
        assert d.L_idxs.shape == (1, r * m // 2) and d.R_idxs.shape == (1, r * n // 2)
        assert len(d.L_scale) == 4 and len(d.R_scale) == 4
    # L is the dequantisation of L_idxs in L^T order (alg.py:171-172)
    from src.caldera.utils.quantization import LowMemoryQuantizer
    q = LowMemoryQuantizer(4, method, r * m)
    Lt = q.dequantize_block(d.L_idxs, d.L_scale, (r, m))
    assert torch.equal(Lt.t().cpu(), d.L.cpu())


def test_method_bit_checks(api):
    caldera, CP, QF = api
    W = _W(64, 128)
    with pytest.raises(ValueError):
        caldera(CP(Q_bits=2, rank=8, iters=1, update_order=["Q"], quant_factory_Q=QF("nf4", 64)),
                W.to(DEV), None, device=DEV, use_tqdm=False)
    with pytest.raises(AssertionError):
        caldera(CP(Q_bits=3, rank=8, iters=1, update_order=["Q"]), W.to(DEV), None, device=DEV, use_tqdm=False)


def _dense_H(n, k, seed, ridge):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(n, k, generator=g) / k ** 0.5
    return (X @ X.T + ridge * torch.eye(n)).float()


@pytest.mark.parametrize("ridge", [0.1, 0.0])  # 0.0: rank-deficient H -> sigma_reg shift (alg.py:59-64)
def test_dense_H_activation_aware(api, ridge):
    """Non-diagonal H (alg.py:44-68): eigh setup, Y = res H_sqrt V, R = S Vh diag(1/sqrt lam) V^T,
    tr(E H E^T) errors.  First errors to 1e-5 (fp32 eigh vs the oracle's dense GEMMs),
    Q + LR to 1e-4 relative Frobenius."""
    caldera, CP, _ = api
    W = _W(256, 512, seed=4)
    H = _dense_H(512, 96, seed=9, ridge=ridge)
    d = caldera(CP(Q_bits=2, L_bits=16, R_bits=16, rank=16, iters=2, update_order=["Q", "LR"], sigma_reg=1e-4),
                W.to(DEV), H.to(DEV), device=DEV, use_tqdm=False)
    ref = O.caldera(O.Params(Q_bits=2, L_bits=16, R_bits=16, rank=16, iters=2, update_order=["Q", "LR"],
                             sigma_reg=1e-4), W.numpy(), H.numpy())
    assert abs(d.errors["Q"][0] - ref.errors["Q"][0]) < 1e-5, (d.errors, ref.errors)
    assert abs(d.errors["LR"][0] - ref.errors["LR"][0]) < 1e-4, (d.errors, ref.errors)
    for k in ("Q", "LR"):
        np.testing.assert_allclose(d.errors[k], ref.errors[k], rtol=0, atol=1e-3)
    out = (d.Q.double() + d.L.double() @ d.R.double()).cpu().numpy()
    exp = ref.Q.astype(np.float64) + ref.L.astype(np.float64) @ ref.R.astype(np.float64)
    assert np.linalg.norm(out - exp) / np.linalg.norm(exp) < 1e-4


def test_dense_H_quantized_factors_and_not_aware(api):
    """Dense H with 4-bit factors, data-aware and not (H_sqrt = H, alg.py:47-49)."""
    caldera, CP, _ = api
    W = _W(128, 256, seed=6)
    H = _dense_H(256, 64, seed=2, ridge=0.05)
    for aware in (True, False):
        kw = dict(Q_bits=2, L_bits=4, R_bits=4, rank=8, iters=2, lplr_iters=2, update_order=["Q", "LR"],
                  sigma_reg=1e-6, activation_aware_LR=aware)
        d = caldera(CP(**kw), W.to(DEV), H.to(DEV), device=DEV, use_tqdm=False)
        ref = O.caldera(O.Params(**kw), W.numpy(), H.numpy())
        assert abs(d.errors["Q"][0] - ref.errors["Q"][0]) < 1e-5, (aware, d.errors, ref.errors)
        np.testing.assert_allclose(d.errors["LR"], ref.errors["LR"], rtol=0, atol=2e-2)


def test_notebook_recipe(api, nb):
    """caldera_playbook.ipynb cells 3-5 (tests/golden/e2e_nb.npz): fp32 1024^2 W, H = X X^T of
    rank 128 (diagonal here; sigma_reg shift of its zero eigenvalues), Q4/L4/R4, rank 16, 20 iters."""
    caldera, CP, QF = api
    torch.manual_seed(42)
    W = torch.randn(1024, 1024)
    X = torch.eye(1024, 128)
    H = X @ X.T
    d = caldera(CP(Q_bits=4, L_bits=4, R_bits=4, rank=16, iters=20, lplr_iters=5, update_order=["Q", "LR"],
                   quant_factory_Q=QF("uniform", 64), quant_factory_LR=QF("uniform", 64), sigma_reg=1e-8),
                W.to(DEV), H.to(DEV), device=DEV, use_tqdm=False)
    assert abs(d.global_scale - float(nb["global_scale"])) == 0
    assert abs(d.errors["Q"][0] - nb["errors_Q"][0]) < 1e-6
    assert abs(d.errors["LR"][0] - nb["errors_LR"][0]) < 1e-3
    np.testing.assert_allclose(d.errors["Q"], nb["errors_Q"], rtol=0, atol=2e-2)
    np.testing.assert_allclose(d.errors["LR"], nb["errors_LR"], rtol=0, atol=2e-2)
    assert min(d.errors["LR"]) <= min(nb["errors_LR"]) + 2e-2


def test_rand_svd(api):
    """rand_svd=True: torch.svd_lowrank(Y, 2r, niter=2) (alg.py:213-216).  Random sketches differ
    from the reference's, so the errors are compared with the oracle's own svd_lowrank run
    (statistical agreement) and bounded below by the exact-SVD error."""
    caldera, CP, _ = api
    g = torch.Generator().manual_seed(1)
    W = ((torch.randn(384, 32, generator=g) @ torch.randn(32, 512, generator=g)) * 0.01
         + torch.randn(384, 512, generator=g) * 0.01).half()
    kw = dict(Q_bits=4, L_bits=16, R_bits=16, rank=16, iters=2, update_order=["Q", "LR"], sigma_reg=1e-8)
    d = caldera(CP(rand_svd=True, **kw), W.to(DEV), None, device=DEV, use_tqdm=False)
    ref_r = O.caldera(O.Params(rand_svd=True, **kw), W.numpy())
    ref_x = O.caldera(O.Params(**kw), W.numpy())
    assert abs(d.errors["Q"][0] - ref_x.errors["Q"][0]) < 1e-6
    np.testing.assert_allclose(d.errors["LR"], ref_r.errors["LR"], rtol=0, atol=5e-3)
    assert d.errors["LR"][0] >= ref_x.errors["LR"][0] - 1e-4
    for (m, n) in ((512, 384),):  # tall: the non-transposed branch
        Wt = W.t().contiguous()
        dt = caldera(CP(rand_svd=True, **kw), Wt.to(DEV), None, device=DEV, use_tqdm=False)
        rt = O.caldera(O.Params(rand_svd=True, **kw), Wt.numpy())
        np.testing.assert_allclose(dt.errors["LR"], rt.errors["LR"], rtol=0, atol=5e-3)


def test_rank_deficient_lplr(api):
    """W of exact rank 4 < rank 8 with 4-bit factors: the LPLR normal equations are singular
    (R from LR_init has 4 zero-energy rows); the dropped pivots reproduce gelsy's
    least-squares error (alg.py:162-177) without NaN."""
    caldera, CP, _ = api
    g = torch.Generator().manual_seed(5)
    W = ((torch.randn(128, 4, generator=g) @ torch.randn(4, 256, generator=g)) * 0.05).half()
    kw = dict(Q_bits=8, L_bits=4, R_bits=4, rank=8, iters=2, lplr_iters=2, update_order=["LR", "Q"], sigma_reg=1e-8)
    d = caldera(CP(**kw), W.to(DEV), None, device=DEV, use_tqdm=False)
    ref = O.caldera(O.Params(**kw), W.numpy())
    assert all(np.isfinite(d.errors["LR"])) and torch.isfinite(d.L).all() and torch.isfinite(d.R).all()
    np.testing.assert_allclose(d.errors["LR"], ref.errors["LR"], rtol=0, atol=2e-2)
