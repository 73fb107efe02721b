"""HIP kernels (through the C-ABI) against the reference fixtures and fp64 references."""
import math

import numpy as np
import pytest
import torch

from oracle import caldera_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def K():
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    K.load()
    return K


DEV = "cuda:0"


def _inputs(kat):
    return [k[3:] for k in kat.files if k.startswith("in_")]


@pytest.mark.parametrize("bits", [2, 4, 8, 16])
def test_uniform_quantizer_kat_bit_exact(K, kat, bits):
    for name in _inputs(kat):
        x = kat["in_" + name]
        for bs in (64, "all"):
            key = f"uniform_b{bits}_bs{bs}_{name}"
            b = x.size if bs == "all" else bs
            xt = torch.from_numpy(x.copy()).to(DEV).view(1, -1)
            out = K.quantize_uniform(xt, b, bits, 1e-8, codes=True, deq=True)
            np.testing.assert_array_equal(out["codes"].cpu().numpy().reshape(-1, b), kat[key + "_codes"], err_msg=key)
            np.testing.assert_array_equal(out["scale"].cpu().numpy().reshape(-1, 1), kat[key + "_scale"], err_msg=key)
            np.testing.assert_array_equal(out["deq"].cpu().numpy().reshape(x.shape), kat[key + "_deq"], err_msg=key)
            deq2 = K.dequantize_uniform(out["codes"], out["scale"].view(-1), bits)
            np.testing.assert_array_equal(deq2.cpu().numpy().reshape(x.shape), kat[key + "_deq"], err_msg=key)


def _tie_matrix(m, n, seed):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((m, n)).astype(np.float32)
    mx = float(np.abs(x).max())
    # plant exact ties for k = 1 and k = 7 relative to the true max
    idx = rng.integers(0, m * n, 200)
    x.reshape(-1)[idx[:100]] = np.float32(mx * 0.5)
    x.reshape(-1)[idx[100:]] = np.float32(-mx * 3.5 / 7)
    return x


@pytest.mark.parametrize("bits", [2, 4, 8, 16])
@pytest.mark.parametrize("shape", [(1024, 1024), (512, 2048), (4, 8)])
def test_whole_matrix_quantize_large_and_packed(K, bits, shape):
    x = _tie_matrix(*shape, seed=bits)
    c_ref, s_ref = O.quantize_uniform(x, bits, x.size)
    d_ref = O.dequantize_uniform(c_ref, s_ref, bits, x.shape)
    xt = torch.from_numpy(x).to(DEV).view(1, -1)
    out = K.quantize_uniform(xt, x.size, bits, codes=True, packed=bits <= 4, deq=True,
                             err_w=torch.ones(shape[1], device=DEV), err_ncols=shape[1])
    np.testing.assert_array_equal(out["codes"].cpu().numpy().reshape(x.shape), c_ref.reshape(x.shape))
    np.testing.assert_array_equal(out["scale"].cpu().numpy().reshape(1, 1), s_ref)
    np.testing.assert_array_equal(out["deq"].cpu().numpy().reshape(x.shape), d_ref)
    err = float(out["err"].item())
    exp = float(((d_ref.astype(np.float64) - x) ** 2).sum())
    assert abs(err - exp) <= 1e-9 * max(1.0, exp)
    if bits <= 4:
        un = K.unpack_codes(out["packed"], x.size, bits)
        np.testing.assert_array_equal(un.cpu().numpy().reshape(x.shape), c_ref.reshape(x.shape))
        dq = K.dequantize_uniform(out["packed"], out["scale"].view(-1), bits, packed=True, numel=x.size)
        np.testing.assert_array_equal(dq.cpu().numpy().reshape(x.shape), d_ref)


def test_known_max_path_matches(K):
    x = _tie_matrix(256, 512, 3)
    xt = torch.from_numpy(x).to(DEV).view(1, -1)
    mx = torch.tensor([np.abs(x).max()], dtype=torch.float32, device=DEV).view(torch.int32)
    packed = torch.empty((1, x.size // 4), dtype=torch.uint8, device=DEV)
    scale = torch.empty(1, device=DEV)
    K.quantize_known_max(xt, mx, 2, packed=packed, scale=scale)
    c_ref, s_ref = O.quantize_uniform(x, 2, x.size)
    np.testing.assert_array_equal(K.unpack_codes(packed, x.size, 2).cpu().numpy().reshape(-1), c_ref.reshape(-1))


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_rms_scale_matches_oracle(K, dtype):
    for seed, (m, n) in enumerate([(512, 512), (300, 128), (64, 1000)]):
        torch.manual_seed(seed)
        W = (torch.randn(2, m, n) * (0.02 if seed % 2 == 0 else 1.3)).to(dtype)
        gs, Ws = K.rms_scale(W.to(DEV), True)
        for b in range(2):
            w = W[b].numpy()
            g = O.global_scale_of(w)
            if dtype == torch.float16:
                assert float(gs[b]) == g
                np.testing.assert_array_equal(Ws[b].cpu().numpy(), O.scale_weight(w, g))
            else:
                assert abs(float(gs[b]) - g) <= 2e-7 * g
        gs1, Ws1 = K.rms_scale(W.to(DEV), False)
        assert torch.all(gs1 == 1) and torch.equal(Ws1.cpu(), W)


def _ref_mm(A, B, ta, tb):
    A = A.double()
    B = B.double()
    if ta:
        A = A.transpose(-1, -2)
    if tb:
        B = B.transpose(-1, -2)
    return A @ B


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("MNK", [(1, 1, 1), (37, 53, 29), (128, 128, 16), (300, 260, 1000), (64, 512, 3)])
def test_gemm_linear(K, ta, tb, MNK):
    M, N, Kd = MNK
    torch.manual_seed(M + N + Kd)
    Bt = 3
    A = torch.randn(Bt, Kd, M) if ta else torch.randn(Bt, M, Kd)
    Bm = torch.randn(Bt, N, Kd) if tb else torch.randn(Bt, Kd, N)
    C0 = torch.randn(Bt, M, N)
    D = torch.randn(Bt, M, N)
    C = C0.clone().to(DEV)
    al = torch.tensor([0.5, -1.0, 2.0], device=DEV)
    K.gemm(A.to(DEV), Bm.to(DEV), ta=ta, tb=tb, C=C, alpha_v=al, beta=0.25, D=D.to(DEV), gamma=-1.5)
    ref = al.cpu().double().view(-1, 1, 1) * _ref_mm(A, Bm, ta, tb) + 0.25 * C0.double() - 1.5 * D.double()
    err = (C.cpu().double() - ref).abs().max().item()
    scale = (_ref_mm(A.abs(), Bm.abs(), ta, tb).abs().max().item() + 1.0)
    assert err <= 2e-6 * scale, (err, scale)


def test_gemm_resid_and_werr(K):
    torch.manual_seed(5)
    B, m, n, r = 2, 200, 300, 24
    L = torch.randn(B, m, r)
    R = torch.randn(B, r, n)
    W = (torch.randn(B, m, n) * 3).half()
    C = torch.empty(B, m, n, device=DEV)
    am = torch.zeros(B, dtype=torch.int32, device=DEV)
    K.gemm(L.to(DEV), R.to(DEV), C=C, D=W.to(DEV), epi=K.EPI_RESID, absmax=am)
    ref = W.double() - L.double() @ R.double()
    assert (C.cpu().double() - ref).abs().max().item() < 1e-4
    mx = am.view(torch.float32).cpu()
    for b in range(B):
        assert mx[b].item() == C[b].abs().max().item()
    w = torch.rand(n) + 0.5
    err = torch.empty(B, dtype=torch.float64, device=DEV)
    X = torch.randn(B, m, n)
    K.gemm(L.to(DEV), R.to(DEV), D=X.to(DEV), epi=K.EPI_WERR, w=w.to(DEV), err_out=err)
    refe = (((X.double() - L.double() @ R.double()) ** 2) * w.double()).sum(dim=(1, 2))
    assert torch.allclose(err.cpu(), refe, rtol=1e-5)


@pytest.mark.parametrize("ta,tb", [(False, False), (True, True), (False, True)])
def test_gram_f64(K, ta, tb):
    torch.manual_seed(1)
    Kd, M, N = 4096, 96, 130
    A = torch.randn(2, M, Kd) if ta else torch.randn(2, Kd, M)
    Bm = torch.randn(2, N, Kd) if tb else torch.randn(2, Kd, N)
    C = K.gram_f64(A.to(DEV), Bm.to(DEV), ta=ta, tb=tb)
    a = A.double().transpose(-1, -2) if not ta else A.double()
    b = Bm.double() if not tb else Bm.double().transpose(-1, -2)
    ref = a @ b
    assert (C.cpu() - ref).abs().max().item() < 1e-9


@pytest.mark.parametrize("tk", [False, True])
@pytest.mark.parametrize("M,N,Kd,sym", [(192, 192, 4096, True), (130, 96, 1000, False), (190, 190, 333, True),
                                        (256, 256, 4096, True), (64, 200, 1004, False)])
def test_gram_f64_mfma_paths(K, M, N, Kd, sym, tk):
    """Grams on the fp64 MFMA path, both operand orientations (tk: C = A B^T with K contiguous,
    the LPLR loop's R R^T); symmetric Grams skip and mirror the lower tiles.  Ragged K (not a
    multiple of the 32-deep slice or of 4) included."""
    g = torch.Generator().manual_seed(M + Kd)
    A = torch.randn(3, M, Kd, generator=g) if tk else torch.randn(3, Kd, M, generator=g)
    Bm = A if sym else (torch.randn(3, N, Kd, generator=g) if tk else torch.randn(3, Kd, N, generator=g))
    Ad = A.to(DEV)
    C = K.gram_f64(Ad, Ad if sym else Bm.to(DEV), ta=tk, tb=tk)
    ref = (A.double() @ Bm.double().transpose(1, 2)) if tk else (A.double().transpose(1, 2) @ Bm.double())
    assert ((C.cpu() - ref).abs().max() / ref.abs().max()).item() < 1e-13
    if sym:
        assert torch.equal(C, C.transpose(1, 2))
        # the mirrored lower tiles are the same bits the full product computes for them: a
        # copy of A takes the non-symmetric path, which computes every tile
        Cf = K.gram_f64(Ad, Ad.clone(), ta=tk, tb=tk)
        assert torch.equal(C, Cf)


def test_spd_whiten_and_jacobi(K):
    torch.manual_seed(2)
    p = 96
    X = torch.randn(3, 400, p, dtype=torch.float64)
    S = X.transpose(1, 2) @ X
    Wt32, Wt64, info = K.spd_whiten(S.clone().to(DEV))
    assert torch.all(info == 0)
    Wt = Wt64.cpu()
    I = Wt.transpose(1, 2) @ S @ Wt
    assert (I - torch.eye(p, dtype=torch.float64)).abs().max().item() < 1e-10
    assert torch.equal(torch.triu(Wt), Wt)
    ev, V32, V64, sw = K.jacobi_eigh(S.clone().to(DEV), want64=True)
    ref = torch.linalg.eigvalsh(S).flip(-1)
    assert torch.allclose(ev.cpu(), ref, rtol=1e-12, atol=1e-9)
    # p <= 192: eigenvector matrix accumulated in fp32 registers (orthogonal to ~1e-6)
    V = V64.cpu()
    assert (V.transpose(1, 2) @ V - torch.eye(p, dtype=torch.float64)).abs().max() < 2e-5
    res = S @ V - V * ev.cpu().unsqueeze(1)
    assert res.abs().max().item() < 2e-5 * S.abs().max().item()
    # odd size and a (near-)degenerate spectrum
    A = torch.diag(torch.tensor([3.0, 1.0, 1.0, 2.0, 2.0 + 1e-12, 0.5, 7.0], dtype=torch.float64)).unsqueeze(0)
    Q, _ = torch.linalg.qr(torch.randn(7, 7, dtype=torch.float64))
    A = Q @ A @ Q.T
    ev, _, V64, _ = K.jacobi_eigh(A.clone().to(DEV), want64=True)
    assert torch.allclose(ev.cpu()[0], torch.tensor([7.0, 3.0, 2.0 + 1e-12, 2.0, 1.0, 1.0, 0.5], dtype=torch.float64), atol=1e-12)
    V = V64.cpu()[0]
    assert (V.T @ V - torch.eye(7, dtype=torch.float64)).abs().max() < 1e-6


def test_build_residual_exact(K):
    torch.manual_seed(3)
    B, m, n = 2, 64, 128
    W = (torch.randn(B, m, n) * 0.7).half()
    for bits in (2, 4, 8, 16):
        x = torch.randn(B, m * n, device=DEV)
        q = K.quantize_uniform(x.contiguous(), m * n, bits, codes=True, packed=bits <= 4, deq=True)
        col = torch.rand(n, device=DEV) + 0.1
        Y = torch.empty(B, m, n, device=DEV)
        res = torch.empty(B, m, n, device=DEV)
        codes = q["packed"] if bits <= 4 else q["codes"]
        K.build_residual(W.to(DEV), codes, q["scale"].view(-1), bits, col, Y=Y, res=res)
        exp_res = W.to(DEV).float() - q["deq"].view(B, m, n)
        assert torch.equal(res, exp_res)
        assert torch.equal(Y, exp_res * col)


def test_ritz_residual(K):
    torch.manual_seed(4)
    X = torch.randn(2, 300, 40, device=DEV)
    Z = torch.randn(2, 300, 40, device=DEV)
    th = torch.rand(2, 40, dtype=torch.float64, device=DEV) + 1.0
    out = K.ritz_residual(X, Z, th, 10)
    ref = ((Z.double() - X.double() * th.view(2, 1, 40)) ** 2).sum(1).sqrt()[:, :10].max(1).values / th[:, 0]
    assert torch.allclose(out.double(), ref, rtol=1e-5)


def test_jacobi_block_path_p256(K):
    """p = 256 (> 192) runs the multi-workgroup block Jacobi (cq_bjacobi.hip, fp64):
    eigenvalues to ~1e-5 relative of ||T||, V orthogonal."""
    torch.manual_seed(9)
    p = 256
    X = torch.randn(2, 1024, p, dtype=torch.float64)
    S = X.transpose(1, 2) @ X
    ev, V32, V64, sw = K.jacobi_eigh(S.clone().to(DEV), want64=True)
    ref = torch.linalg.eigvalsh(S).flip(-1)
    nrm = ref[:, 0:1]
    assert ((ev.cpu() - ref).abs() / nrm).max().item() < 1e-5
    V = V64.cpu()
    assert (V.transpose(1, 2) @ V - torch.eye(p, dtype=torch.float64)).abs().max() < 1e-10
    D = V.transpose(1, 2) @ S @ V
    off = D - torch.diag_embed(torch.diagonal(D, dim1=1, dim2=2))
    assert off.abs().max().item() < 1e-5 * nrm.max().item()


@pytest.mark.parametrize("near_diag", [False, True])
def test_jacobi_global_path_p384(K, near_diag):
    """p = 384 (rank-256 Rayleigh-Ritz, config 5) runs the block Jacobi over many workgroups
    with threshold rotations: pairs below tol / (2 sqrt p) of sqrt|a_ii a_jj| are skipped,
    which must not stop the off-norm test from passing (cold and warm / near-diagonal)."""
    torch.manual_seed(10)
    p = 384
    X = torch.randn(1, 2048, p, dtype=torch.float64)
    S = X.transpose(1, 2) @ X
    if near_diag:  # a warm Rayleigh-Ritz matrix: eigenbasis of S perturbed by 1e-4
        _, U = torch.linalg.eigh(S)
        Qp, _ = torch.linalg.qr(U + 1e-4 * torch.randn_like(U))
        S = Qp.transpose(1, 2) @ S @ Qp
        S = 0.5 * (S + S.transpose(1, 2))
    ref = torch.linalg.eigvalsh(S).flip(-1)
    nrm = ref[:, 0:1]
    for tol in (1e-7, 1e-13):
        ev, V32, V64, sw = K.jacobi_eigh(S.clone().to(DEV), tol=tol, want64=True)
        assert int(sw.max()) < 30
        assert ((ev.cpu() - ref).abs() / nrm).max().item() < max(tol * tol * 1e4, 1e-12)
        V = V64.cpu()
        assert (V.transpose(1, 2) @ V - torch.eye(p, dtype=torch.float64)).abs().max() < 1e-10
        D = V.transpose(1, 2) @ S @ V
        off = D - torch.diag_embed(torch.diagonal(D, dim1=1, dim2=2))
        assert off.norm().item() <= 2 * tol * D.norm().item() + 1e-12 * nrm.max().item()
        # values only: the same rotations of A without the eigenvector updates
        ev2, V2, _, _ = K.jacobi_eigh(S.clone().to(DEV), tol=tol, want_vectors=False)
        assert V2 is None and torch.equal(ev2.cpu(), ev.cpu())


@pytest.mark.parametrize("p", [200, 288, 300])
def test_jacobi_block_path_ragged_batch(K, p):
    """Block Jacobi on p not a multiple of its 32-wide blocks (a partial last block, an odd
    block count rounded up with a virtual block; p = 288 is main.py's rank 200), in a batch
    whose matrices converge after different sweep counts (cold, near-diagonal, diagonal)."""
    torch.manual_seed(p)
    X = torch.randn(3, 1024, p, dtype=torch.float64)
    S = X.transpose(1, 2) @ X
    _, U = torch.linalg.eigh(S[1])
    Qp, _ = torch.linalg.qr(U + 1e-5 * torch.randn_like(U))
    S[1] = 0.5 * ((Qp.T @ S[1] @ Qp) + (Qp.T @ S[1] @ Qp).T)
    S[2] = torch.diag(torch.rand(p, dtype=torch.float64) + 0.5)
    ref = torch.linalg.eigvalsh(S).flip(-1)
    ev, V32, V64, sw = K.jacobi_eigh(S.clone().to(DEV), tol=1e-12, want64=True)
    assert int(sw[2]) == 0 and int(sw[1]) <= int(sw[0]) < 30
    assert ((ev.cpu() - ref).abs() / ref[:, 0:1]).max().item() < 1e-12
    V = V64.cpu()
    assert (V.transpose(1, 2) @ V - torch.eye(p, dtype=torch.float64)).abs().max() < 1e-12
    res = S @ V - V * ev.cpu().unsqueeze(1)
    assert res.abs().max().item() < 1e-10 * ref.max().item()


@pytest.mark.parametrize("want_vectors", [True, False])
def test_jacobi_block_staged_equals_one_shot(K, want_vectors):
    """cq_jacobi_eigh_staged (begin + 2 sweeps, then 2 at a time while the device count of
    unconverged matrices is nonzero, then end) runs the same kernel sequence as the one-shot
    cq_jacobi_eigh: eigenvalues, vectors and per-matrix sweep counts are identical, and the
    pending count reaches 0 no later than the slowest matrix's sweep count."""
    torch.manual_seed(41)
    p = 288
    X = torch.randn(3, 1024, p, dtype=torch.float64)
    S = X.transpose(1, 2) @ X
    _, U = torch.linalg.eigh(S[1])
    Qp, _ = torch.linalg.qr(U + 1e-5 * torch.randn_like(U))
    S[1] = 0.5 * ((Qp.T @ S[1] @ Qp) + (Qp.T @ S[1] @ Qp).T)
    ev1, V1, _, sw1 = K.jacobi_eigh(S.clone().to(DEV), tol=1e-9, want_vectors=want_vectors)
    bj = K.BlockJacobi(S.clone().to(DEV), 1e-9, want_vectors)
    left = bj.sweeps(2, begin=True)
    while left and bj.swept < 30:
        left = bj.sweeps(2)
    ev2, V2, _, sw2 = bj.finish()
    assert left == 0 and bj.swept - int(sw1.max()) in (0, 1)
    assert torch.equal(ev1, ev2) and torch.equal(sw1, sw2)
    assert (V1 is None and V2 is None) or torch.equal(V1, V2)


@pytest.mark.parametrize("want_vectors", [True, False])
@pytest.mark.parametrize("p", [2, 33, 64, 96, 192])
def test_jacobi_block_staged_small_p(K, p, want_vectors):
    """Small batches route every p (also p <= 192) to the staged block Jacobi
    (solver.BJ_SMALL_SUBPROBLEMS): one matrix (B = 1: a single pair block at p <= 64, so the
    values-only solve has no off-diagonal update), odd p (a ragged last block) and the
    1024-thread subproblem solve.  Eigenvalues against LAPACK to fp64 accuracy; vectors
    orthonormal and satisfying S V = V diag(ev) to fp32 accuracy."""
    torch.manual_seed(100 + p)
    X = torch.randn(1, 4 * p + 8, p, dtype=torch.float64)
    S = X.transpose(1, 2) @ X
    bj = K.BlockJacobi(S.clone().to(DEV), 1e-9, want_vectors)
    left = bj.sweeps(2, begin=True)
    while left and bj.swept < 40:
        left = bj.sweeps(2)
    ev, V32, _, sw = bj.finish()
    assert left == 0
    ref = torch.linalg.eigvalsh(S).flip(-1)
    ev = ev.cpu()
    assert ((ev - ref).abs() / ref[:, 0:1]).max().item() < 1e-12
    if not want_vectors:
        assert V32 is None
        return
    V = V32.cpu().double()
    assert (V.transpose(1, 2) @ V - torch.eye(p, dtype=torch.float64)).abs().max() < 2e-5
    assert (S @ V - V * ev.unsqueeze(1)).abs().max().item() < 2e-5 * ref.max().item()


@pytest.mark.parametrize("p", [64, 128, 180, 192])
def test_jacobi_register_path_accuracy(K, p):
    """p <= 192: fp64 A in LDS + fp32 V in registers (the solver's Rayleigh-Ritz path):
    eigenvalues to fp64 accuracy, V orthogonal to ~1e-6, residual ~1e-6 ||S||."""
    torch.manual_seed(11 + p)
    X = torch.randn(2, 1024, p, dtype=torch.float64)
    S = X.transpose(1, 2) @ X
    ev, V32, V64, sw = K.jacobi_eigh(S.clone().to(DEV), want64=True)
    ref = torch.linalg.eigvalsh(S).flip(-1)
    assert ((ev.cpu() - ref).abs() / ref[:, 0:1]).max().item() < 1e-13
    V = V64.cpu()
    assert (V.transpose(1, 2) @ V - torch.eye(p, dtype=torch.float64)).abs().max() < 2e-5
    res = S @ V - V * ev.cpu().unsqueeze(1)
    assert res.abs().max().item() < 2e-5 * ref.max().item()
    assert torch.equal(V32.cpu().double(), V)


@pytest.mark.parametrize("p", [8, 64, 128, 192, 288, 384])   # > 192: T read in place from L2
def test_extreme_eigs_lanczos(K, p):
    """cq_extreme_eigs, the filter bounds of the solver's cheap outer iterations: both ends of
    the spectrum approached from inside — to 5e-6 of the spread on Wishart spectra, inside a flat
    top cluster (a Ritz-like spectrum, 1 + 1e-3 u) to its width (its spread-out bottom to 1e-4);
    exact up to the fp32 copy of T
    when p <= steps (the Lanczos iteration breaks down on the whole space); T untouched; a NaN
    gives NaN ends."""
    torch.manual_seed(5 + p)
    X = torch.randn(4, 1024, p, dtype=torch.float64)
    S = X.transpose(1, 2) @ X
    Q, _ = torch.linalg.qr(torch.randn(p, p, dtype=torch.float64))
    lam = torch.cat([1 + 1e-3 * torch.rand(p - p // 3, dtype=torch.float64), 0.5 * torch.rand(p // 3, dtype=torch.float64)])
    S[2] = Q @ torch.diag(lam) @ Q.T
    S[3, 1, 2] = math.nan
    Sd = S.to(DEV)
    before = Sd.clone()
    ends = K.extreme_eigs(Sd, 40).cpu()
    assert torch.equal(Sd.view(torch.int64), before.view(torch.int64))   # (bitwise: matrix 3 holds a NaN)
    assert torch.isnan(ends[3]).all()
    ref = torch.linalg.eigvalsh(0.5 * (S[:3] + S[:3].transpose(1, 2)))
    spread = ref[:, -1] - ref[:, 0]
    hi_err = (ref[:, -1] - ends[:3, 0]) / spread
    lo_err = (ends[:3, 1] - ref[:, 0]) / spread
    # from inside, up to the fp32 rounding of the LDS copy of T (~6e-8 of its norm)
    assert (hi_err > -5e-7).all() and (lo_err > -5e-7).all(), (hi_err, lo_err)
    exact = p <= 40
    for b in range(3):
        tol_hi = 5e-7 if exact else (2e-3 if b == 2 else 5e-6)
        # (the Wishart bottom edge at p / N = 288 / 1024, 384 / 1024 is a slower Lanczos end:
        # 40 steps reach 4e-5 / 5e-4 of the spread there -- ample for a filter cut)
        tol_lo = 5e-7 if exact else (1e-4 if b == 2 else (5e-6 if p <= 192 else 2e-3))
        assert hi_err[b] < tol_hi and lo_err[b] < tol_lo, (b, hi_err[b].item(), lo_err[b].item())


@pytest.mark.parametrize("p", [256, 384])  # panel 32 / panel 16
def test_whiten_blocked(K, p):
    torch.manual_seed(10)
    X = torch.randn(2, 2048, p, dtype=torch.float64) * torch.logspace(0, 3, p, dtype=torch.float64)
    S = X.transpose(1, 2) @ X
    Wt32, Wt64, info = K.spd_whiten(S.clone().to(DEV))
    assert torch.all(info == 0)
    Wt = Wt64.cpu()
    I = Wt.transpose(1, 2) @ S @ Wt
    assert (I - torch.eye(p, dtype=torch.float64)).abs().max().item() < 1e-9
    assert torch.equal(torch.triu(Wt), Wt)


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("n", [100, 256, 300])
def test_gemm_syrk_mode(K, ta, n):
    torch.manual_seed(n)
    Kd = 777
    Y = torch.randn(2, Kd, n) if ta else torch.randn(2, n, Kd)
    C = torch.full((2, n, n), float("nan"), device=DEV)
    Yd = Y.to(DEV)
    K.gemm(Yd, Yd, ta=ta, tb=not ta, C=C, syrk=True)
    Y64 = Y.double()
    ref = Y64.transpose(1, 2) @ Y64 if ta else Y64 @ Y64.transpose(1, 2)
    Cc = C.cpu().double()
    assert torch.isfinite(Cc).all()
    assert (Cc - ref).abs().max().item() < 1e-5 * ref.abs().max().item()
    assert torch.equal(Cc, Cc.transpose(1, 2))


# ------------------------------------------------------------------ split-fp16 (f16x3) products
def _x3_split_ref(x, s):
    xs = x * s
    hi = xs.half()
    lo = (xs - hi.float()).half()
    return hi, lo


@pytest.mark.parametrize("rows,cols", [(200, 130), (256, 192), (328, 100), (4096, 192)])
def test_transpose_split_exact(K, rows, cols):
    # (200, 130): the per-element path (cols % 4 != 0); the others take the 16-byte path
    # (rows % 8 == 0, cols % 4 == 0), with partial 64 x 64 tiles at (328, 100)
    g = torch.Generator(device=DEV).manual_seed(3)
    X = torch.randn(3, rows, cols, device=DEV, generator=g)
    Y = torch.empty(3, cols, rows, device=DEV)
    hi = torch.empty(3, cols, rows, device=DEV, dtype=torch.float16)
    lo = torch.empty_like(hi)
    K.transpose_split(X, out=Y, hi=hi, lo=lo, scale=64.0)
    assert torch.equal(Y, X.transpose(1, 2))
    rh, rl = _x3_split_ref(X.transpose(1, 2).contiguous(), 64.0)
    assert torch.equal(hi, rh) and torch.equal(lo, rl)
    if rows % 32 == 0:   # K-blocked halves (the filter's A operand), without the fp32 output
        bh, bl = torch.empty_like(hi), torch.empty_like(lo)
        K.transpose_split(X, hi=bh, lo=bl, scale=64.0, blocked=True)
        assert torch.equal(bh, _kblock(rh)) and torch.equal(bl, _kblock(rl))
    # hi + lo carries x * s to 2^-22 relative
    rec = (hi.double() + lo.double()) / 64.0
    # (plus the fp16 subnormal spacing of lo, 2^-24, for the smallest entries)
    xt = X.transpose(1, 2).double()
    assert ((rec - xt).abs() <= 2.0 ** -21 * xt.abs() + 2.0 ** -24 / 64.0).all()


def test_sym_split_scale_and_halves(K):
    g = torch.Generator(device=DEV).manual_seed(4)
    Y = torch.randn(2, 96, 300, device=DEV, generator=g) * torch.tensor([0.01, 3.0], device=DEV).view(2, 1, 1)
    G = torch.matmul(Y, Y.transpose(1, 2)).contiguous()
    hi, lo, s, inv = K.sym_split_f16(G, 64.0)
    for b in range(2):
        mx = torch.diagonal(G[b]).max().item()
        sb = s[b].item()
        assert math.log2(sb) == int(math.log2(sb))          # power of two
        assert 2.0 ** 13 <= mx * sb < 2.0 ** 14 + 1e-3       # hi halves stay <= 2^14
        assert inv[b].item() == pytest.approx(1.0 / (sb * 64.0), rel=0, abs=0)
        rh, rl = _x3_split_ref(G[b], sb)
        assert torch.equal(hi[b], rh) and torch.equal(lo[b], rl)
    # upper-only input (lower triangle garbage) gives the same split
    Gu = torch.triu(G) + torch.tril(torch.full_like(G, 7.0), -1)
    hu, lu, su, _ = K.sym_split_f16(Gu, 64.0, upper_only=True)
    assert torch.equal(hu, hi) and torch.equal(lu, lo) and torch.equal(su, s)
    # K-blocked layout: (i, j) at (j // 32) * n * 32 + i * 32 + j % 32
    hb, lb, _, _ = K.sym_split_f16(G, 64.0, blocked=True)
    n = G.shape[1]
    ref_b = hi.view(2, n, n // 32, 32).permute(0, 2, 1, 3).reshape(2, n, n)
    assert torch.equal(hb, ref_b)


def test_gemm_x3_blocked_b_matches_rowmajor(K):
    g = torch.Generator(device=DEV).manual_seed(8)
    Y = torch.randn(2, 320, 96, device=DEV, generator=g)
    G = torch.matmul(Y, Y.transpose(1, 2)).contiguous()
    gh, gl, gs, ginv = K.sym_split_f16(G, 64.0)
    bh, bl, _, _ = K.sym_split_f16(G, 64.0, blocked=True)
    X = torch.randn(2, 200, 320, device=DEV, generator=g)
    xh, xl = _x3_split_ref(X, 64.0)
    C1 = torch.empty(2, 200, 320, device=DEV)
    C2 = torch.empty_like(C1)
    K.gemm_x3(xh, xl, gh, gl, ginv, C1)
    K.gemm_x3(xh, xl, bh, bl, ginv, C2, b_blocked=True)
    assert torch.equal(C1, C2)


@pytest.mark.parametrize("M,N,Kd", [(192, 256, 512), (96, 320, 256), (200, 520, 1024)])
def test_gemm_x3_matches_fp64(K, M, N, Kd):
    """C = A B^T from fp16 halves, fp32-grade: column errors within 3x the fp32 GEMM's
    (unsymmetric B checks the row/column placement)."""
    Bt = 3
    g = torch.Generator(device=DEV).manual_seed(M + N)
    A = torch.randn(Bt, M, Kd, device=DEV, generator=g) * 0.1
    Bm = torch.randn(Bt, N, Kd, device=DEV, generator=g) * 5.0
    sa, sb = 2.0 ** 6, 2.0 ** 10
    Ah, Al = _x3_split_ref(A, sa)
    Bh, Bl = _x3_split_ref(Bm, sb)
    inv = torch.full((Bt,), 1.0 / (sa * sb), device=DEV)
    C = torch.empty(Bt, M, N, device=DEV)
    K.gemm_x3(Ah.contiguous(), Al.contiguous(), Bh.contiguous(), Bl.contiguous(), inv, C)
    ref = torch.matmul(A.double(), Bm.double().transpose(1, 2))
    c32 = torch.matmul(A, Bm.transpose(1, 2)).double()
    err = ((C.double() - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
    err32 = ((c32 - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
    assert err < max(3 * err32, 1e-6), (err, err32)


@pytest.mark.parametrize("M,N,Kd,blocked", [(256, 1024, 4096, True), (256, 1024, 512, True), (512, 256, 256, False),
                                            (256, 4096, 128, False)])
def test_gemm_x3_square_tile_bit_identical(K, M, N, Kd, blocked):
    """The 256 x 256 tile (gemm_x3s_kernel: rank-256 products, config 5's LPLR loop and normal
    equations) against the 192 x 384 kernel on the same operands: an N a multiple of 384 but
    not of 256 (N + 128) keeps the 192 x 384 tiling, whose first N columns must be the same
    bits (same fragments, MFMA order per 16 x 16 block and epilogue roundings); and fp32-grade
    against fp64.  ksplit = 1 on both calls: the square kernel only runs one-pass products (a
    small batch's long-K products would otherwise take split-K on both sides and compare split-K
    with split-K), so the blocked long-K cases pin gemm_x3s_kernel itself -- the production path
    of config 5's LPLR products under interleaving (overlap.py turns split-K off)."""
    Bt = 2
    g = torch.Generator(device=DEV).manual_seed(M + N + Kd)
    A = torch.randn(Bt, M, Kd, device=DEV, generator=g) * 0.1
    Bm = torch.randn(Bt, N + 128, Kd, device=DEV, generator=g) * 5.0
    assert (N + 128) % 384 == 0 and (N + 128) % 256 != 0
    Ah, Al = K.split_f16(A.contiguous(), 2.0 ** 6, blocked=blocked)
    Bh, Bl = K.split_f16(Bm.contiguous(), 2.0 ** 10, blocked=blocked)
    inv = torch.full((Bt,), 2.0 ** -16, device=DEV)
    C_wide = torch.full((Bt, M, N + 128), float("nan"), device=DEV)
    K.gemm_x3(Ah, Al, Bh, Bl, inv, C_wide, a_blocked=blocked, b_blocked=blocked, ksplit=1)
    if blocked:   # the first N rows of B in the K-blocked layout [K/32][rows][32]
        Bh_n = Bh.view(Bt, Kd // 32, N + 128, 32)[:, :, :N].contiguous().view(Bt, N, Kd)
        Bl_n = Bl.view(Bt, Kd // 32, N + 128, 32)[:, :, :N].contiguous().view(Bt, N, Kd)
    else:
        Bh_n, Bl_n = Bh[:, :N].contiguous(), Bl[:, :N].contiguous()
    C = torch.full((Bt, M, N), float("nan"), device=DEV)
    K.gemm_x3(Ah, Al, Bh_n, Bl_n, inv, C, a_blocked=blocked, b_blocked=blocked, ksplit=1)
    assert torch.equal(C, C_wide[:, :, :N])
    ref = torch.matmul(A.double(), Bm[:, :N].double().transpose(1, 2))
    err = ((C.double() - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
    assert err < 1e-6, err


@pytest.mark.parametrize("M,N,Kd,blocked", [(192, 4096, 4096, True), (100, 1000, 32, False), (192, 400, 64, True),
                                            (250, 770, 96, False), (192, 384, 128, True)])
def test_gemm_x3_single_product_matches_fp64(K, M, N, Kd, blocked):
    """single mode (the filter's low-precision steps, 4-slot hi-only ring): C = Ah Bh^T * inv
    with fp32 accumulation -- pinned against fp64 of the same fp16 operands, short K (ring
    prologue deeper than the loop), ragged tiles and the K-blocked layouts included."""
    Bt = 2
    g = torch.Generator(device=DEV).manual_seed(M + N + Kd)
    A = torch.randn(Bt, M, Kd, device=DEV, generator=g)
    Bm = torch.randn(Bt, N, Kd, device=DEV, generator=g) * 3.0
    Ah, Al = K.split_f16(A.contiguous(), 2.0 ** 10, blocked=blocked)
    Bh, Bl = K.split_f16(Bm.contiguous(), 2.0 ** 8, blocked=blocked)
    inv = torch.full((Bt,), 2.0 ** -18, device=DEV)
    C = torch.full((Bt, M, N), float("nan"), device=DEV)
    K.gemm_x3(Ah, Al, Bh, Bl, inv, C, a_blocked=blocked, b_blocked=blocked, single=True)
    if blocked:  # back to row-major for the reference
        Ah = Ah.view(Bt, Kd // 32, M, 32).permute(0, 2, 1, 3).reshape(Bt, M, Kd)
        Bh = Bh.view(Bt, Kd // 32, N, 32).permute(0, 2, 1, 3).reshape(Bt, N, Kd)
    ref = torch.matmul(Ah.double(), Bh.double().transpose(1, 2)) * 2.0 ** -18
    err = ((C.double() - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
    assert err < 2e-6, err


@pytest.mark.parametrize("Bt,M,N,Kd,lda", [(2, 128, 4096, 4096, 192), (3, 100, 1000, 32, 104),
                                             (2, 192, 400, 64, 192), (2, 250, 776, 96, 256),
                                             (2, 64, 384, 160, 96)])
def test_gemm_x3_exact_b_matches_three_products(K, Bt, M, N, Kd, lda):
    """b_exact (B exactly fp16, Bl = 0 not read, 3-stage ring of A hi | A lo | B hi): the same
    bits as the three-product kernel given Bl = 0, with the gamma epilogue of R = U^T W - s U^T c,
    A rows lda > M (the block's first r columns), short K (ring prologue deeper than the loop)
    and ragged tiles."""
    g = torch.Generator(device=DEV).manual_seed(M + N + Kd)
    A = torch.randn(Bt, lda, Kd, device=DEV, generator=g)
    Wm = (torch.randn(Bt, N, Kd, device=DEV, generator=g) * 0.05).half().float()
    Ah, Al = K.split_f16(A.contiguous(), 2.0 ** 10, blocked=True)
    Bh, Bl = K.split_f16(Wm.contiguous(), 2.0 ** 14, blocked=True)
    assert int(Bl.view(torch.int16).abs().max()) == 0
    inv = torch.full((Bt,), 2.0 ** -24, device=DEV)
    D = torch.randn(Bt, M, N, device=DEV, generator=g)
    gam = torch.randn(Bt, device=DEV, generator=g)
    C3 = torch.full((Bt, M, N), float("nan"), device=DEV)
    C2 = torch.full_like(C3, float("nan"))
    K.gemm_x3(Ah, Al, Bh, Bl, inv, C3, a_blocked=True, b_blocked=True, lda=lda, M=M, D=D, gamma_v=gam, ksplit=1)
    K.gemm_x3(Ah, Al, Bh, None, inv, C2, a_blocked=True, b_blocked=True, lda=lda, M=M, D=D, gamma_v=gam, ksplit=1,
              b_exact=True)
    assert torch.equal(C2, C3)
    # split-K (the automatic choice for a batch with few tiles) sums the same partials
    C2k = torch.full_like(C3, float("nan"))
    K.gemm_x3(Ah, Al, Bh, None, inv, C2k, a_blocked=True, b_blocked=True, lda=lda, M=M, D=D, gamma_v=gam,
              b_exact=True)
    C3k = torch.full_like(C3, float("nan"))
    K.gemm_x3(Ah, Al, Bh, Bl, inv, C3k, a_blocked=True, b_blocked=True, lda=lda, M=M, D=D, gamma_v=gam)
    assert torch.equal(C2k, C3k)


@pytest.mark.parametrize("M,N", [(4096, 192), (1000, 64), (777, 160), (130, 32), (11008, 128), (300, 100),
                                 (520, 300), (96, 384)])
def test_gemm_b_triu_matches_plain(K, M, N):
    """b_triu (CholQR's X Wt with Wt upper triangular, zeros stored): the same bits as the
    plain product -- the skipped K slices only meet exact zeros of B.  N % 32 == 0 and
    N <= 192 take gemm_triu_kernel (ragged M included), the rest gemm_f32_kernel<TRIU>."""
    g = torch.Generator(device=DEV).manual_seed(M + N)
    A = torch.randn(3, M, N, device=DEV, generator=g)
    Bt = torch.triu(torch.randn(3, N, N, device=DEV, generator=g))
    C0 = K.gemm(A, Bt, C=torch.empty(3, M, N, device=DEV))
    C1 = K.gemm(A, Bt, C=torch.full((3, M, N), float("nan"), device=DEV), b_triu=True)
    assert torch.equal(C0, C1)


@pytest.mark.parametrize("M,p", [(4096, 192), (1024, 96), (352, 32), (11008, 128), (160, 160)])
def test_gemm_triu_split_matches_two_kernels(K, M, p):
    """cq_gemm_triu_split (CholQR's X Wt writing the Rayleigh-Ritz operand, the K-blocked split
    of its transpose, in the same pass): the same bits as the b_triu product followed by the
    blocked transpose-split."""
    g = torch.Generator(device=DEV).manual_seed(M + p)
    X = torch.randn(3, M, p, device=DEV, generator=g)
    Wt = torch.triu(torch.randn(3, p, p, device=DEV, generator=g))
    C0 = K.gemm(X, Wt, C=torch.empty(3, M, p, device=DEV), b_triu=True)
    h0 = torch.empty(3, p, M, device=DEV, dtype=torch.float16)
    l0 = torch.empty_like(h0)
    K.transpose_split(C0, hi=h0, lo=l0, scale=64.0, blocked=True)
    C1 = torch.full((3, M, p), float("nan"), device=DEV)
    h1 = torch.full_like(h0, float("nan"))
    l1 = torch.full_like(l0, float("nan"))
    assert K.triu_split_ok(M, p)
    K.gemm_triu_split(X, Wt, C1, h1, l1, 64.0)
    assert torch.equal(C0, C1)
    assert torch.equal(h0, h1) and torch.equal(l0, l1)


def test_residual_split_ycol_hi_matches_two_passes(K):
    """ycol_hi (the weighted Gram's operand): one pass writes the transposed halves and ||Y||^2
    with ycol and the column-blocked halves of res * ycol^2 at their own scale -- the same bits
    as two separate passes."""
    g = torch.Generator(device=DEV).manual_seed(9)
    B, m, n = 2, 96, 320
    W = (torch.randn(B, m, n, device=DEV, generator=g) * 0.3).half()
    ycol = torch.rand(n, device=DEV, generator=g) * 2.0 + 0.1
    y2 = (ycol * ycol).contiguous()
    ymax = float(ycol.max())
    wmax = K.absmax(W)
    e = lambda: torch.empty(B, m, n, dtype=torch.float16, device=DEV)  # noqa: E731
    hi, lo, thi, tlo = e(), e(), e(), e()
    sc, sc2 = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    sq = torch.empty(B, dtype=torch.float64, device=DEV)
    K.residual_split(W, None, None, 2, wmax, ycol=ycol, ycol_max=ymax, thi=thi, tlo=tlo, scale=sc, sq=sq, hi=hi, lo=lo,
                     ycol_hi=y2, ycol_hi_max=ymax * ymax, scale_hi=sc2)
    rhi, rlo, rthi, rtlo = e(), e(), e(), e()
    rsc, rsc2 = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    rsq = torch.empty(B, dtype=torch.float64, device=DEV)
    K.residual_split(W, None, None, 2, wmax, ycol=ycol, ycol_max=ymax, thi=rthi, tlo=rtlo, scale=rsc, sq=rsq)
    K.residual_split(W, None, None, 2, wmax, ycol=y2, ycol_max=ymax * ymax, hi=rhi, lo=rlo, scale=rsc2)
    for a, b in ((hi, rhi), (lo, rlo), (thi, rthi), (tlo, rtlo), (sc, rsc), (sc2, rsc2), (sq, rsq)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("Bt,ks", [(3, 1), (1, None)])
def test_gemm_x3_colw_epilogue(K, Bt, ks):
    """colw (R = (U^T W) diag(ycol) - s U^T c diag(ycol)): the product term times colw[j], then
    gamma D -- the same bits as scaling the plain product's columns afterwards, in the one-pass
    kernel and in the split-K epilogue (ks None: automatic split-K for a single matrix)."""
    g = torch.Generator(device=DEV).manual_seed(31 + Bt)
    M, N, Kd, lda = 128, 1024, 2048, 192
    A = torch.randn(Bt, lda, Kd, device=DEV, generator=g)
    Wm = (torch.randn(Bt, N, Kd, device=DEV, generator=g) * 0.05).half().float()
    Ah, Al = K.split_f16(A.contiguous(), 2.0 ** 10, blocked=True)
    Bh, _ = K.split_f16(Wm.contiguous(), 2.0 ** 14, blocked=True)
    inv = torch.full((Bt,), 2.0 ** -24, device=DEV)
    D = torch.randn(Bt, M, N, device=DEV, generator=g)
    gam = torch.randn(Bt, device=DEV, generator=g)
    w = torch.rand(N, device=DEV, generator=g) + 0.5
    C = torch.full((Bt, M, N), float("nan"), device=DEV)
    K.gemm_x3(Ah, Al, Bh, None, inv, C, a_blocked=True, b_blocked=True, lda=lda, M=M, D=D, gamma_v=gam,
              b_exact=True, colw=w, ksplit=ks)
    C0 = torch.full_like(C, float("nan"))
    K.gemm_x3(Ah, Al, Bh, None, inv, C0, a_blocked=True, b_blocked=True, lda=lda, M=M, b_exact=True, ksplit=ks)
    ref = C0 * w.view(1, 1, N) + gam.view(Bt, 1, 1) * D
    assert torch.equal(C, ref)


def test_residual_split_exact_w_skips_lo(K):
    """fp16 W without codes or column weights: scale >= 1 (also for max|W| >= 2^14), hi = W * s
    exactly, lo / tlo optional (zero when written)."""
    g = torch.Generator(device=DEV).manual_seed(5)
    B, m, n = 2, 96, 320
    W = (torch.randn(B, m, n, device=DEV, generator=g) * torch.tensor([0.02, 1e4], device=DEV).view(B, 1, 1)).half()
    wmax = K.absmax(W)
    hi, lo, thi, tlo = (torch.empty(B, m, n, dtype=torch.float16, device=DEV) for _ in range(4))
    sc = torch.empty(B, device=DEV)
    K.residual_split(W, None, None, 2, wmax, hi=hi, lo=lo, thi=thi, tlo=tlo, scale=sc)
    assert float(sc[1]) == 1.0 and float(sc[0]) > 1.0
    assert int(lo.view(torch.int16).abs().max()) == 0 and int(tlo.view(torch.int16).abs().max()) == 0
    h_ref, _ = K.split_f16(W.float().contiguous(), sc, blocked=True)
    assert torch.equal(hi, h_ref)
    hi2, thi2 = torch.empty_like(hi), torch.empty_like(hi)
    sc2 = torch.empty_like(sc)
    K.residual_split(W, None, None, 2, wmax, hi=hi2, thi=thi2, scale=sc2)
    assert torch.equal(hi2, hi) and torch.equal(thi2, thi) and torch.equal(sc2, sc)


def test_gemm_x3_tri_upper_exact(K):
    """tri mode: the upper triangle of Y Y^T equals the full product's bit for bit."""
    g = torch.Generator(device=DEV).manual_seed(21)
    Y = torch.randn(2, 600, 320, device=DEV, generator=g)
    s = K.pow2_scale(Y, 14)
    yh, yl = K.split_f16(Y, s)
    inv = 1.0 / (s * s)
    full = torch.empty(2, 600, 600, device=DEV)
    K.gemm_x3(yh, yl, yh, yl, inv, full)
    up = torch.full_like(full, float("nan"))
    K.gemm_x3(yh, yl, yh, yl, inv, up, tri=True)
    iu = torch.triu_indices(600, 600, device=DEV)
    assert torch.equal(up[:, iu[0], iu[1]], full[:, iu[0], iu[1]])


def test_gemm_x3_recurrence_epilogue_and_split(K):
    Bt, M, N, Kd = 2, 192, 256, 256
    g = torch.Generator(device=DEV).manual_seed(9)
    A = torch.randn(Bt, M, Kd, device=DEV, generator=g)
    Bm = torch.randn(Bt, N, Kd, device=DEV, generator=g)
    P = torch.randn(Bt, M, N, device=DEV, generator=g)
    D = torch.randn(Bt, M, N, device=DEV, generator=g)
    Ah, Al = _x3_split_ref(A, 1.0)
    Bh, Bl = _x3_split_ref(Bm, 1.0)
    inv = torch.ones(Bt, device=DEV)
    al = torch.tensor([0.5, 2.0], device=DEV)
    be = torch.tensor([-1.0, 0.25], device=DEV)
    ga = torch.tensor([0.125, -3.0], device=DEV)
    C = P.clone()  # in place: prev is overwritten by the new iterate
    Oh = torch.empty(Bt, M, N, device=DEV, dtype=torch.float16)
    Ol = torch.empty_like(Oh)
    ovf = torch.zeros(Bt, dtype=torch.int32, device=DEV)
    K.gemm_x3(Ah, Al, Bh, Bl, inv, C, P=C, D=D, alpha_v=al, beta_v=be, gamma_v=ga, out_h=Oh, out_l=Ol,
              out_scale=4.0, overflow=ovf)
    prod = torch.matmul(A.double(), Bm.double().transpose(1, 2))
    ref = al.double().view(-1, 1, 1) * prod + be.double().view(-1, 1, 1) * P.double() + ga.double().view(-1, 1, 1) * D.double()
    assert ((C.double() - ref).abs().max() / ref.abs().max()).item() < 2e-6
    rh, rl = _x3_split_ref(C, 4.0)
    assert torch.equal(Oh, rh) and torch.equal(Ol, rl)
    assert ovf.tolist() == [0, 0]
    # overflow of the fp16 split is flagged per batch
    K.gemm_x3(Ah, Al, Bh, Bl, inv, C, alpha_v=torch.tensor([1.0, 1e6], device=DEV), out_h=Oh, out_l=Ol,
              out_scale=4.0, overflow=ovf)
    assert ovf.tolist() == [0, 1]


def test_pow2_scale_and_split(K):
    g = torch.Generator(device=DEV).manual_seed(5)
    X = torch.randn(3, 100, 64, device=DEV, generator=g) * torch.tensor([1e-3, 1.0, 0.0], device=DEV).view(3, 1, 1)
    s = K.pow2_scale(X, 14)
    assert s[2].item() == 2.0 ** 14  # all-zero matrix: max 0 -> e = 0
    for b in range(2):
        mx = X[b].abs().max().item()
        assert 2.0 ** 13 <= mx * s[b].item() < 2.0 ** 14
    hi, lo = K.split_f16(X, s)
    rh, rl = _x3_split_ref(X, s.view(3, 1, 1))
    assert torch.equal(hi, rh) and torch.equal(lo, rl)
    Y = torch.empty(3, 64, 100, device=DEV)
    th = torch.empty(3, 64, 100, device=DEV, dtype=torch.float16)
    tl = torch.empty_like(th)
    K.transpose_split(X, out=Y, hi=th, lo=tl, scale=s)
    assert torch.equal(th, rh.transpose(1, 2)) and torch.equal(tl, rl.transpose(1, 2))


@pytest.mark.parametrize("bits", [2, 4, 8, 16])
def test_q_update_x3_without_lr_is_exact(K, bits):
    """r = 0 (first Q update, alg.py:262 with no LR): res = W, so the fused kernel must match
    the standalone whole-matrix quantiser bit for bit (codes, packed bytes, scale)."""
    g = torch.Generator(device=DEV).manual_seed(bits)
    W = (torch.randn(3, 200, 392, device=DEV, generator=g) * 0.02).half()
    ref = K.quantize_uniform(W.float().view(3, -1), 200 * 392, bits, codes=True)
    codes = torch.empty(3, 200 * 392, dtype=K.code_dtype(bits), device=DEV)
    scale = torch.empty(3, device=DEV)
    err = torch.empty(3, dtype=torch.float64, device=DEV)
    K.q_update_x3(W, None, None, bits, codes=codes, scale=scale, err_out=err)
    assert torch.equal(codes, ref["codes"].view(3, -1))
    assert torch.equal(scale, ref["scale"].view(3))
    if bits <= 4:
        packed = torch.empty(3, 200 * 392 * bits // 8, dtype=torch.uint8, device=DEV)
        K.q_update_x3(W, None, None, bits, packed=packed, scale=scale)
        assert torch.equal(K.unpack_codes(packed, 200 * 392, bits).view(3, -1).to(codes.dtype), codes)
    # the kernel's arithmetic: deq = (c / k) * s and d = deq - x in fp32, d^2 summed in fp64
    deq = (codes.float() / float(2 ** (bits - 1) - 1)) * scale.view(3, 1)
    d = deq - W.float().view(3, -1)
    e_ref = (d * d).double().sum(1)
    # torch fp32 division vs the IEEE one in-kernel: visible at 16 bits, where the error is tiny
    assert torch.allclose(err, e_ref, rtol=1e-4 if bits == 16 else 1e-6, atol=0)


def _near_tie(x64, scale64, bits, tol=1e-4):
    """x / max|x| * k within `tol` code units of a rounding boundary (quantization.py:95, 266)."""
    s = x64 / scale64 * float(2 ** (bits - 1) - 1)
    return (torch.abs(torch.abs(s - torch.floor(s)) - 0.5) < tol)


@pytest.mark.parametrize("m,n,r,bits,dt", [
    (300, 520, 64, 2, torch.float16),    # m % 16 != 0: the 192 x 384 tile kernel
    (320, 544, 96, 2, torch.float16),    # row-panel kernel: partial panel, K = 96 (3 of 4 MFMA steps)
    (640, 1024, 128, 4, torch.float16),  # row-panel kernel, 4-bit packing
    (336, 512, 256, 2, torch.float16),   # row-panel kernel, K = 256 (2 row blocks per wave)
    (320, 544, 64, 8, torch.float32),    # fp32 W, int8 codes
    (320, 544, 128, 16, torch.float32),  # fp32 W, int16 codes
])
def test_q_update_x3_with_lr_matches_fp64_residual(K, m, n, r, bits, dt):
    """Codes of res = W - L R equal those of the exact (fp64) residual everywhere except where
    the exact value lies within 1e-4 code units of a rounding boundary; scale to fp32
    rounding; the weighted error to 1e-4 relative."""
    g = torch.Generator(device=DEV).manual_seed(3 + m + r)
    B = 2
    W = (torch.randn(B, m, n, device=DEV, generator=g) * 0.02).to(dt)
    L = torch.linalg.qr(torch.randn(B, m, r, device=DEV, generator=g))[0].contiguous()
    R = (torch.randn(B, r, n, device=DEV, generator=g) * 0.01).contiguous()
    packed = torch.empty(B, m * n * bits // 8, dtype=torch.uint8, device=DEV) if bits <= 4 else None
    codes = torch.empty(B, m * n, dtype=K.code_dtype(bits), device=DEV)
    scale = torch.empty(B, device=DEV)
    err = torch.empty(B, dtype=torch.float64, device=DEV)
    w = torch.rand(n, device=DEV, generator=g) + 0.5
    K.q_update_x3(W, L, R, bits, packed=packed, codes=codes, scale=scale, err_w=w, err_out=err)
    res = W.double() - L.double() @ R.double()
    s64 = res.abs().amax((1, 2))
    assert torch.allclose(scale.double(), s64, rtol=1e-6, atol=0)
    k = float(2 ** (bits - 1) - 1)
    c = codes.view(B, m, n).double()
    if packed is not None:
        assert torch.equal(K.unpack_codes(packed, m * n, bits).view(B, m, n).double(), c)
    c_ref = torch.round(res / s64.view(B, 1, 1) * k)
    flips = c != c_ref
    # near-tie width in code units: 1e-4, or an fp32-grade residual's ~4e-6 relative error
    # expressed in code units at high bit widths (k = 32767 at 16 bits)
    tol = max(1e-4, 4e-6 * k)
    assert not (flips & ~_near_tie(res, s64.view(B, 1, 1), bits, tol)).any(), int(flips.sum())
    deq = c / k * scale.double().view(B, 1, 1)
    e_ref = (((deq - res) ** 2) * w.double()).sum((1, 2))
    assert torch.allclose(err, e_ref, rtol=1e-4, atol=0)


def test_q_update_with_lr_on_reference_inputs(K, trace):
    """The second Q update of the reference trace (alg.py:262 + quantize_matrix), replayed on
    the reference's own W/gs, L and R (its dequantised 4-bit factors after update_LR): the
    fused split-fp16 kernel's codes equal the reference's codes except where the reference's
    fp32 residual lies within 1e-4 code units of a rounding boundary (0 such flips seen)."""
    kinds = list(trace["kinds"])
    iu = kinds.index("update_lr")
    iq = kinds.index("quantize", iu)
    Ws = torch.from_numpy(trace["W_scaled"]).to(DEV)[None]
    L = torch.from_numpy(trace[f"c{iu}_L"]).to(DEV)[None].contiguous()
    R = torch.from_numpy(trace[f"c{iu}_R"]).to(DEV)[None].contiguous()
    A = torch.from_numpy(trace[f"c{iq}_A"]).double()
    m, n = A.shape
    bits = int(trace[f"c{iq}_bits"])
    packed = torch.empty(1, m * n * bits // 8, dtype=torch.uint8, device=DEV)
    scale = torch.empty(1, device=DEV)
    K.q_update_x3(Ws, L, R, bits, packed=packed, scale=scale)
    ref_scale = float(trace[f"c{iq}_scale"].reshape(-1)[0])
    assert abs(scale.item() - ref_scale) <= 1e-6 * ref_scale
    codes = K.unpack_codes(packed, m * n, bits).view(m, n).cpu()
    ref = torch.from_numpy(trace[f"c{iq}_A_idxs"]).view(m, n)
    flips = codes.to(ref.dtype) != ref
    ties = _near_tie(A, A.abs().max(), bits)
    assert not (flips & ~ties).any(), int((flips & ~ties).sum())
    print(f"reference second-Q replay: {int(flips.sum())} code flips of {m * n} (near-ties {int(ties.sum())})")


def test_q_update_with_lr_full_size_exact_residual(K):
    """Config 2 shape (4096 x 4096, r = 128) with L, R from the engine's own first LR step:
    fused Q-with-LR codes vs the codes of the exact fp64 residual, flips only at near-ties."""
    from src.caldera.decomposition.alg import caldera
    from src.caldera.utils.dataclasses import CalderaParams
    torch.manual_seed(0)
    W = (torch.randn(4096, 4096) * 0.02).to(torch.float16)
    d = caldera(CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=1, update_order=["Q", "LR"],
                              sigma_reg=1e-8), W.to(DEV), None, device=DEV, use_tqdm=False)
    Ws = d.W.to(DEV)[None]
    L, R = d.L.to(DEV)[None].contiguous(), d.R.to(DEV)[None].contiguous()
    packed = torch.empty(1, 4096 * 4096 // 4, dtype=torch.uint8, device=DEV)
    scale = torch.empty(1, device=DEV)
    K.q_update_x3(Ws, L, R, 2, packed=packed, scale=scale)
    res = Ws[0].double() - L[0].double() @ R[0].double()
    s64 = res.abs().max()
    assert abs(scale.item() - s64.item()) <= 1e-6 * s64.item()
    c = K.unpack_codes(packed, 4096 * 4096, 2).view(4096, 4096).double()
    flips = c != torch.round(res / s64)
    bad = flips & ~_near_tie(res, s64, 2)
    assert not bad.any(), int(bad.sum())
    print(f"full-size Q-with-LR: {int(flips.sum())} code flips of {4096 * 4096}, all at near-ties")


def _kblock(x):
    """(B, R, K) row-major -> the K-blocked operand layout [K/32][R][32] (same storage size)."""
    B, R, Kd = x.shape
    return x.view(B, R, Kd // 32, 32).permute(0, 2, 1, 3).contiguous().view(B, R, Kd)


def test_blocked_operand_layouts(K):
    """split_f16 / transpose_split blocked outputs equal the K-blocked permutation of the
    row-major halves; a product on blocked A and B equals the row-major product bit for bit,
    and a blocked split output feeds the next product like a row-major one."""
    g = torch.Generator(device=DEV).manual_seed(12)
    Y = torch.randn(2, 224, 320, device=DEV, generator=g)
    s = K.pow2_scale(Y, 14)
    h, l = K.split_f16(Y, s)
    hb, lb = K.split_f16(Y, s, blocked=True)
    assert torch.equal(hb, _kblock(h)) and torch.equal(lb, _kblock(l))
    X = torch.randn(2, 320, 96, device=DEV, generator=g)   # (k, p) -> X^T (p, k) halves
    _, th, tl = K.transpose_split(X, hi=torch.empty(2, 96, 320, dtype=torch.float16, device=DEV),
                                  lo=torch.empty(2, 96, 320, dtype=torch.float16, device=DEV), scale=64.0)
    _, tbh, tbl = K.transpose_split(X, hi=torch.empty_like(th), lo=torch.empty_like(tl), scale=64.0, blocked=True)
    assert torch.equal(tbh, _kblock(th)) and torch.equal(tbl, _kblock(tl))
    inv = 1.0 / (s * s)
    C1 = torch.empty(2, 224, 224, device=DEV)
    C2 = torch.empty_like(C1)
    K.gemm_x3(h, l, h, l, inv, C1)
    K.gemm_x3(hb, lb, hb, lb, inv, C2, a_blocked=True, b_blocked=True)
    assert torch.equal(C1, C2)
    # blocked split output (C = X^T Y^T: 96 x 224, K = 320)
    Yt = Y.transpose(1, 2).contiguous()          # (320, 224): B operand rows = 224
    yth, ytl = K.split_f16(Y, s)                  # Y (224, 320) rows are K-contiguous for B
    C3 = torch.empty(2, 96, 224, device=DEV)
    oh = torch.empty(2, 96, 224, dtype=torch.float16, device=DEV)
    ol = torch.empty_like(oh)
    ohb, olb = torch.empty_like(oh), torch.empty_like(ol)
    ovf = torch.zeros(2, dtype=torch.int32, device=DEV)
    inv2 = 1.0 / (64.0 * s)
    K.gemm_x3(th, tl, yth, ytl, inv2, C3, out_h=oh, out_l=ol, out_scale=4.0, overflow=ovf)
    K.gemm_x3(tbh, tbl, yth, ytl, inv2, C3, out_h=ohb, out_l=olb, out_scale=4.0, overflow=ovf,
              a_blocked=True, o_blocked=True)
    assert torch.equal(ohb, _kblock(oh)) and torch.equal(olb, _kblock(ol))


@pytest.mark.parametrize("bits,weighted", [(2, False), (4, True), (8, False)])
def test_residual_split_matches_unfused(K, bits, weighted):
    """cq_residual_split == build_residual + split (both blocked layouts) at the kernel's
    power-of-two scale, which bounds max|Y|; ||Y||^2 to fp64 rounding."""
    g = torch.Generator(device=DEV).manual_seed(bits)
    B, m, n = 2, 96, 320
    W = (torch.randn(B, m, n, device=DEV, generator=g) * 0.5).half()
    q = K.quantize_uniform(W.float().view(B, -1) * 0.9, m * n, bits, codes=True)
    if bits <= 4:
        codes = K.quantize_uniform(W.float().view(B, -1) * 0.9, m * n, bits, packed=True)["packed"]
    else:
        codes = q["codes"].view(B, -1).contiguous()
    qs = q["scale"].view(B).contiguous()
    ycol = (torch.rand(n, device=DEV, generator=g) + 0.5) if weighted else None
    wmax = K.absmax(W)
    assert torch.equal(wmax, W.float().abs().amax((1, 2)))
    res_ref = torch.empty(B, m, n, device=DEV)
    Y_ref = torch.empty(B, m, n, device=DEV) if weighted else None
    K.build_residual(W, codes, qs, bits, ycol, Y=Y_ref, res=res_ref)
    Ysrc = Y_ref if weighted else res_ref
    res = torch.empty_like(res_ref)
    Y = torch.empty_like(res_ref) if weighted else None
    hi = torch.empty(B, m, n, dtype=torch.float16, device=DEV)
    lo, thi, tlo = torch.empty_like(hi), torch.empty_like(hi), torch.empty_like(hi)
    sc = torch.empty(B, device=DEV)
    sq = torch.empty(B, dtype=torch.float64, device=DEV)
    K.residual_split(W, codes, qs, bits, wmax, ycol=ycol, ycol_max=float(ycol.max()) if weighted else 1.0,
                     res=res, Y=Y, hi=hi, lo=lo, thi=thi, tlo=tlo, scale=sc, sq=sq)
    assert torch.equal(res, res_ref)
    if weighted:
        assert torch.equal(Y, Y_ref)
    assert (Ysrc.abs().amax((1, 2)) * sc < 2.0 ** 14).all()
    h_ref, l_ref = K.split_f16(Ysrc.contiguous(), sc, blocked=True)
    assert torch.equal(hi, h_ref) and torch.equal(lo, l_ref)
    th_ref, tl_ref = K.split_f16(Ysrc.transpose(1, 2).contiguous(), sc, blocked=True)
    # the transposed halves are (B, n, m) operands stored in (B, m, n)-shaped buffers
    assert torch.equal(thi.view(B, n, m), th_ref) and torch.equal(tlo.view(B, n, m), tl_ref)
    assert torch.allclose(sq, (Ysrc.double() ** 2).sum((1, 2)), rtol=1e-12, atol=0)


@pytest.mark.parametrize("p", [1, 17, 32, 33, 96, 200, 256, 384])
def test_spd_whiten_shapes(K, p):
    """Blocked LDL^T whitening (MFMA panels of 32): Wt^T S Wt = I and Wt upper triangular for
    ragged last panels, a single pivot, and p > 192 (the LPLR normal equations at rank 200 /
    256, the p = 384 CholQR); per-matrix results independent of the batch."""
    g = torch.Generator().manual_seed(p)
    X = torch.randn(3, 4 * p + 8, p, dtype=torch.float64, generator=g)
    X[1] *= 1e3
    S = X.transpose(1, 2) @ X
    Wt32, Wt64, info = K.spd_whiten(S.clone().to(DEV))
    assert torch.all(info == 0)
    Wt = Wt64.cpu()
    I = Wt.transpose(1, 2) @ S @ Wt
    assert (I - torch.eye(p, dtype=torch.float64)).abs().max().item() < 1e-9
    assert torch.equal(torch.triu(Wt), Wt)
    assert torch.equal(Wt32.cpu(), Wt.float())
    _, W1, _ = K.spd_whiten(S[2:3].clone().to(DEV))
    assert torch.equal(W1.cpu()[0], Wt[2])


@pytest.mark.parametrize("p", [24, 200, 300, 384, 700])  # blocked nb 32 / nb 16, unblocked
def test_spd_whiten_rank_deficient_is_gelsy_basic_solution(K, p):
    """lstsq through the normal equations with dependent columns (alg.py:162-177 with a
    rank-deficient factor, e.g. a 2-bit L with an all-zero column): the dropped pivots give a
    finite basic solution (dependent coefficients 0) at the least-squares optimum.  (torch's
    gelsy returns huge cancelling coefficients on exactly dependent fp32 columns, whose fp64
    residual is above the optimum, so the optimum is taken from an fp64 SVD lstsq.)"""
    rng = np.random.default_rng(p)
    m = 4 * p
    A = rng.standard_normal((m, p)).astype(np.float32)
    A[:, 5] = 0.0                       # zero column
    A[:, 7] = 2.0 * A[:, 3]             # exactly dependent column
    y = rng.standard_normal((m, 3)).astype(np.float32)
    M = torch.from_numpy(A.astype(np.float64).T @ A.astype(np.float64)).to(DEV).unsqueeze(0)
    rc = np.finfo(np.float32).eps * m
    Wt32, Wt64, info = K.spd_whiten(M, rcond2=rc * rc)
    assert int(info[0]) == 2
    Wt = Wt64[0].cpu().numpy()
    x = Wt @ Wt.T @ (A.T.astype(np.float64) @ y)
    assert np.all(np.isfinite(x)) and np.all(x[5] == 0) and np.all(x[7] == 0)
    ref = np.linalg.lstsq(A.astype(np.float64), y.astype(np.float64), rcond=None)[0]
    r_ours = np.linalg.norm(A.astype(np.float64) @ x - y)
    r_ref = np.linalg.norm(A.astype(np.float64) @ ref - y)
    assert abs(r_ours - r_ref) <= 1e-6 * r_ref


@pytest.mark.parametrize("n,kd", [(416, 320), (4096, 256)])
def test_gram_sym_split_output(K, n, kd):
    """Gram Y Y^T in sym_out mode (the solver's path): its K-blocked halves are exactly
    symmetric and equal the blocked split of the fp32 upper-triangle Gram (cq_sym_split_f16)
    up to the power-of-two scale, which comes from the ||Y||_F^2 bound."""
    g = torch.Generator(device=DEV).manual_seed(21)
    B = 2
    Y = torch.randn(B, n, kd, device=DEV, generator=g) * 0.03
    ys = K.pow2_scale(Y, 14)
    yh, yl = K.split_f16(Y, ys, blocked=True)
    yinv = 1.0 / (ys * ys)
    G = torch.empty(B, n, n, device=DEV)
    K.gemm_x3(yh, yl, yh, yl, yinv, G, tri=True, a_blocked=True, b_blocked=True)
    rh, rl, rs, rinv = K.sym_split_f16(G, 64.0, upper_only=True, blocked=True)
    ysq = K.weighted_sqsum(Y, None, kd)
    hh = torch.full((B, n, n), float("nan"), device=DEV, dtype=torch.float16)
    hl = hh.clone()
    s = torch.empty(B, device=DEV)
    inv = torch.empty(B, device=DEV)
    K.gemm_x3(yh, yl, yh, yl, yinv, None, tri=True, a_blocked=True, b_blocked=True, out_h=hh, out_l=hl,
              out_scale=64.0, sym_bound=ysq, scale_out=s, inv_out=inv)
    assert not torch.isnan(hh.float()).any() and not torch.isnan(hl.float()).any()  # every entry written

    def unblock(t):
        return t.view(B, n // 32, n, 32).permute(0, 2, 1, 3).reshape(B, n, n)

    for b in range(B):
        e = math.frexp(float(ysq[b]))[1]
        assert float(s[b]) == 2.0 ** (14 - e) and float(inv[b]) == pytest.approx(1 / (float(s[b]) * 64), rel=1e-7)
        H = unblock(hh)[b].double() + unblock(hl)[b].double()
        assert torch.equal(H, H.T)
        Gr = (unblock(rh)[b].double() + unblock(rl)[b].double()) / float(rs[b])
        # same fp32 values split at another power-of-two scale: equal up to the fp16 subnormal
        # resolution of the small entries' lo halves (2^-24 / s absolute)
        tol = 2.0 ** -24 / min(float(s[b]), float(rs[b]))
        assert float((H / float(s[b]) - Gr).abs().max()) <= tol
        assert tol <= 2.0 ** -22 * float(Gr.abs().max())  # still fp32-grade


@pytest.mark.parametrize("weighted", [True, False])
@pytest.mark.parametrize("n", [1040, 1024, 4096])
@pytest.mark.parametrize("bits", [2, 4, 8, 16])
@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
def test_q_update_known_absmax_stream(K, bits, dtype, n, weighted):
    """First Q step with max|W| known (streaming kernel, one pass) == the two-pass fused
    update: identical codes, packed codes and scale, error equal to fp64 summation order.
    n = 1024 / 4096: the grid stride is a whole number of rows (each thread's error weights
    loaded once); n = 1040: it is not (weights loaded per group).  Unweighted: the kernel's
    no-weights instantiation (2-bit codes packed by FMAs, W two groups ahead)."""
    g = torch.Generator(device=DEV).manual_seed(5)
    B, m = 3, 192
    W = (torch.randn(B, m, n, device=DEV, generator=g) * 0.02).to(dtype)
    W[1, 7, 33] = 0.5  # a planted maximum
    ew = torch.rand(n, device=DEV, generator=g) + 0.5
    if not weighted:
        ew = None
    packed = bits <= 4
    outs = []
    for amax in (None, K.absmax(W)):
        codes = torch.empty(B, m * n, dtype=K.code_dtype(bits), device=DEV)
        pk = torch.empty(B, m * n * bits // 8, dtype=torch.uint8, device=DEV) if packed else None
        sc = torch.empty(B, device=DEV)
        err = torch.empty(B, dtype=torch.float64, device=DEV)
        K.q_update_x3(W, None, None, bits, codes=codes, packed=pk, scale=sc, err_w=ew, err_out=err, absmax_in=amax)
        outs.append((codes, pk, sc, err))
    (c0, p0, s0, e0), (c1, p1, s1, e1) = outs
    assert torch.equal(c0, c1) and torch.equal(s0, s1)
    if packed:
        assert torch.equal(p0, p1)
    assert torch.allclose(e0, e1, rtol=1e-12, atol=0)
    # codes against the oracle's uniform quantiser of the same W
    for b in range(B):
        x = W[b].float().cpu().numpy().reshape(1, -1)
        ref_c, ref_s = O.quantize_uniform(x, bits, block_size=m * n)
        assert np.array_equal(c1[b].cpu().numpy().reshape(1, -1), ref_c.reshape(1, -1))
        assert float(s1[b]) == float(np.asarray(ref_s).reshape(-1)[0])


@pytest.mark.parametrize("bits", [2, 4, 8, 16])
def test_q_update_kernels_kat_bit_exact(K, kat, bits):
    """The fused Q-update kernels (two-pass and the known-max streaming pass, both with the
    one-divisor correctly rounded division) reproduce the reference's whole-matrix KAT codes,
    scale and quantisation error bit for bit, ties included; inputs are zero-padded to a
    multiple of 16 columns (zeros change neither the max nor the other codes)."""
    for name in _inputs(kat):
        x = kat["in_" + name].reshape(-1).astype(np.float32)
        key = f"uniform_b{bits}_bsall_{name}"
        npad = -(-x.size // 16) * 16
        xp = np.zeros(npad, np.float32)
        xp[: x.size] = x
        W = torch.from_numpy(xp).to(DEV).view(1, 1, npad)
        d32 = (kat[key + "_deq"].reshape(-1).astype(np.float32) - x).astype(np.float32)
        e_ref = float((d32 * d32).astype(np.float64).sum())
        for amax in (None, K.absmax(W)):
            codes = torch.empty(1, npad, dtype=K.code_dtype(bits), device=DEV)
            sc = torch.empty(1, device=DEV)
            err = torch.empty(1, dtype=torch.float64, device=DEV)
            K.q_update_x3(W, None, None, bits, codes=codes, scale=sc, err_out=err, absmax_in=amax)
            np.testing.assert_array_equal(codes.cpu().numpy()[0, : x.size], kat[key + "_codes"].reshape(-1), err_msg=key)
            assert float(sc[0]) == float(kat[key + "_scale"].reshape(-1)[0]), key
            # the kernels sum d^2 in fp32 within runs of 4 elements, in fp64 across runs
            assert float(err[0]) == pytest.approx(e_ref, rel=1e-6, abs=1e-30), key


@pytest.mark.parametrize("single", [False, True])
@pytest.mark.parametrize("Bt,M,N,Kd,ks", [(1, 192, 4096, 4096, 16), (3, 128, 1000, 1024, 5), (2, 200, 520, 2048, 64)])
def test_gemm_x3_split_k_matches_one_pass(K, single, Bt, M, N, Kd, ks):
    """Split-K (ksplit chunks of the K loop by separate workgroups, partials summed in chunk
    order by the epilogue kernel: small batches, one caldera() call) against the one-pass
    kernel: the full epilogue -- alpha/beta/gamma, P and D, the K-blocked split output and its
    overflow flag, an inactive matrix passing D through -- within fp32 summation-order noise,
    and bit-exact where the output is pass-through."""
    g = torch.Generator(device=DEV).manual_seed(M + N + ks)
    A = torch.randn(Bt, M, Kd, device=DEV, generator=g)
    Bm = torch.randn(Bt, N, Kd, device=DEV, generator=g)
    Ah, Al = K.split_f16(A.contiguous(), 2.0 ** 10, blocked=True)
    Bh, Bl = K.split_f16(Bm.contiguous(), 2.0 ** 8, blocked=True)
    inv = torch.full((Bt,), 2.0 ** -18, device=DEV)
    P = torch.randn(Bt, M, N, device=DEV, generator=g)
    D = torch.randn(Bt, M, N, device=DEV, generator=g)
    al = torch.rand(Bt, device=DEV, generator=g) * 1e-2
    be = torch.rand(Bt, device=DEV, generator=g)
    ga = torch.rand(Bt, device=DEV, generator=g)
    active = torch.ones(Bt, dtype=torch.int32, device=DEV)
    active[-1] = 0 if Bt > 1 else 1
    outs = []
    for split in (1, ks):
        C = torch.full((Bt, M, N), float("nan"), device=DEV)
        oh = torch.empty((Bt, M, N), dtype=torch.float16, device=DEV)
        ol = torch.empty_like(oh)
        ovf = torch.zeros(Bt, dtype=torch.int32, device=DEV)
        K.gemm_x3(Ah, Al, Bh, Bl, inv, C, P=P, D=D, alpha_v=al, beta_v=be, gamma_v=ga, out_h=oh, out_l=ol,
                  out_scale=64.0, overflow=ovf, active=active, a_blocked=True, b_blocked=True, o_blocked=N % 32 == 0,
                  single=single, ksplit=split)
        outs.append((C, oh.float() + ol.float(), ovf))
    (c1, h1, o1), (c2, h2, o2) = outs
    for b in range(Bt):
        if active[b]:
            assert torch.allclose(c1[b], c2[b], rtol=0, atol=2e-6 * c1[b].abs().max().item())
            assert torch.allclose(h1[b], h2[b], rtol=0, atol=64 * 2e-6 * c1[b].abs().max().item())
        else:
            assert torch.equal(c1[b], D[b]) and torch.equal(c2[b], D[b]) and torch.equal(h1[b], h2[b])
    assert torch.equal(o1, o2)


@pytest.mark.parametrize("ks", [1, 5])
@pytest.mark.parametrize("Bt,M,N,Kd", [(3, 192, 4096, 1024), (2, 200, 520, 2048), (2, 136, 1002, 512)])
def test_gemm_x3_transposed_output(K, Bt, M, N, Kd, ks):
    """Ct (C^T written by the same epilogue: the solver's filter and Rayleigh-Ritz products hand
    back X's k x p layout without a transpose pass) is C transposed bit for bit -- with the full
    filter epilogue (P, D, alpha/beta/gamma, split output, an inactive matrix), one pass and
    split-K, and a ragged N (the scalar epilogue path)."""
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + ks)
    A = torch.randn(Bt, M, Kd, device=DEV, generator=g)
    Bm = torch.randn(Bt, N, Kd, device=DEV, generator=g)
    Ah, Al = K.split_f16(A.contiguous(), 2.0 ** 10, blocked=True)
    bb = N % 8 == 0   # a ragged N (1002) takes row-major B and the scalar epilogue
    Bh, Bl = K.split_f16(Bm.contiguous(), 2.0 ** 8, blocked=bb)
    inv = torch.full((Bt,), 2.0 ** -18, device=DEV)
    P = torch.randn(Bt, M, N, device=DEV, generator=g)
    D = torch.randn(Bt, M, N, device=DEV, generator=g)
    al = torch.rand(Bt, device=DEV, generator=g) * 1e-2
    be = torch.rand(Bt, device=DEV, generator=g)
    ga = torch.rand(Bt, device=DEV, generator=g)
    active = torch.ones(Bt, dtype=torch.int32, device=DEV)
    active[-1] = 0
    outs = []
    for with_t in (False, True):
        C = torch.full((Bt, M, N), float("nan"), device=DEV)
        Ct = torch.full((Bt, N, M), float("nan"), device=DEV) if with_t else None
        oh = torch.empty((Bt, M, N), dtype=torch.float16, device=DEV)
        ol = torch.empty_like(oh)
        ovf = torch.zeros(Bt, dtype=torch.int32, device=DEV)
        K.gemm_x3(Ah, Al, Bh, Bl, inv, C, P=P, D=D, alpha_v=al, beta_v=be, gamma_v=ga, out_h=oh, out_l=ol,
                  out_scale=64.0, overflow=ovf, active=active, a_blocked=True, b_blocked=bb,
                  o_blocked=N % 32 == 0, ksplit=ks if N % 4 == 0 else 1, Ct=Ct)
        outs.append((C, oh, ol, Ct))
    (c0, h0, l0, _), (c1, h1, l1, t1) = outs
    assert torch.equal(c0, c1) and torch.equal(h0, h1) and torch.equal(l0, l1)
    assert torch.equal(t1, c1.transpose(1, 2))
    # plain product (no epilogue terms) on the same operands
    C = torch.empty((Bt, M, N), device=DEV)
    Ct = torch.empty((Bt, N, M), device=DEV)
    K.gemm_x3(Ah, Al, Bh, Bl, inv, C, a_blocked=True, b_blocked=bb, Ct=Ct, ksplit=1)
    assert torch.equal(Ct, C.transpose(1, 2))


@pytest.mark.parametrize("M,N,Kd,Bt,ksplit", [(192, 768, 256, 2, 1),      # 192 x 384 one-pass kernel
                                               (192, 768, 4096, 2, 8),     # split-K epilogue
                                               (256, 1024, 512, 2, 1),     # 256 x 256 square tile
                                               (100, 1000, 64, 3, 1)])     # ragged tiles
def test_absmax_out_gives_pow2_scale_of_C(K, M, N, Kd, Bt, ksplit):
    """gemm_x3's absmax_out epilogue (the LPLR split scales rely on it, engine.lplr_rhs and
    lplr_R_step): pow2_from_absmax(absmax_out) equals pow2_scale(C) bit for bit on the plain,
    split-K and 256 x 256 paths; and a quantiser's scale taken as the bound (the r_bound /
    l_bound shortcut) equals pow2_scale of its dequantised output, whose max |.| it attains."""
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + Kd)
    A = torch.randn(Bt, M, Kd, device=DEV, generator=g) * torch.tensor([1e-3, 1.0, 37.0][:Bt], device=DEV).view(Bt, 1, 1)
    Bm = torch.randn(Bt, N, Kd, device=DEV, generator=g)
    sA = K.pow2_scale(A.contiguous(), 14)
    sB = K.pow2_scale(Bm.contiguous(), 14)
    Ah, Al = K.split_f16(A.contiguous(), sA)
    Bh, Bl = K.split_f16(Bm.contiguous(), sB)
    C = torch.empty(Bt, M, N, device=DEV)
    amx = torch.empty(Bt, dtype=torch.int32, device=DEV)
    K.gemm_x3(Ah, Al, Bh, Bl, 1.0 / (sA * sB), C, absmax_out=amx, ksplit=ksplit)
    assert torch.equal(K.pow2_from_absmax(amx), K.pow2_scale(C, 14))
    # quantiser scale as the bound of its own dequantised output (uniform, whole matrix)
    for bits in (2, 4):
        q = K.quantize_uniform(C.view(Bt, -1).contiguous(), M * N, bits, codes=True, deq=True)
        assert torch.equal(K.pow2_from_absmax(q["scale"].view(Bt).clone()),
                           K.pow2_scale(q["deq"].view(Bt, M, N).contiguous(), 14))
