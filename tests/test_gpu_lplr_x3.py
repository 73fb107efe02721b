"""Split-fp16 products of the quantised-factor LPLR loop (alg.py:162-177) with H = I.

With unweighted Y (= res) the loop's two m x n x r products -- Y R^T of the L step and
L^T res of the R step -- run on split-fp16 MFMAs (cq_gemm_x3 from the K-blocked halves
cq_residual_split writes) instead of fp32 MFMA GEMMs.  Each product is pinned here against
fp64 at fp32 grade, and the whole L / R steps (lstsq solutions) against the fp32-GEMM path;
config 5 (tests/test_gpu_configs.py) runs the engine with the split products on.
"""
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _halves(res):
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    B, m, n = res.shape
    ys = K.pow2_scale(res, 14)
    yh, yl = K.split_f16(res, ys, blocked=True)
    f16 = torch.float16
    yth = torch.empty((B, n, m), dtype=f16, device=DEV)
    ytl = torch.empty((B, n, m), dtype=f16, device=DEV)
    K.transpose_split(res, hi=yth, lo=ytl, scale=ys, blocked=True)
    return ys, yh, yl, yth, ytl


def _engine():
    from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams
    return CalderaEngine(EngineParams(Q_bits=2, L_bits=4, R_bits=4, rank=64, lplr_iters=2,
                                      update_order=["Q", "LR"], sigma_reg=1e-8))


@pytest.mark.parametrize("m,n,r", [(512, 1024, 96), (1024, 768, 256)])
def test_lplr_split_products_vs_fp64(m, n, r):
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    g = torch.Generator(device="cpu").manual_seed(11)
    B = 2
    res = torch.randn(B, m, n, generator=g) * 0.02
    res[1] *= 3.0e3                                       # per-matrix scales
    res = res.to(DEV).contiguous()
    R = (torch.randn(B, r, n, generator=g) * 0.1).to(DEV).contiguous()
    L = (torch.randn(B, m, r, generator=g) * 0.1).to(DEV).contiguous()
    ys, yh, yl, yth, ytl = _halves(res)
    eng = _engine()
    wts = types.SimpleNamespace(dense=False, ycol=None)
    f16 = torch.float16
    hv = dict(yh=yh, yl=yl, ys=ys, yth=yth, ytl=ytl,
              rwh=torch.empty((B, r, n), dtype=f16, device=DEV), rwl=torch.empty((B, r, n), dtype=f16, device=DEV),
              lth=torch.empty((B, r, m), dtype=f16, device=DEV), ltl=torch.empty((B, r, m), dtype=f16, device=DEV))
    # ---- Y R^T
    Bm, _ = eng.lplr_rhs(R, res, wts, torch.empty((B, m, r), device=DEV), hv)
    Bm32, _ = eng.lplr_rhs(R, res, wts, torch.empty((B, m, r), device=DEV), None)
    exp = res.double() @ R.double().transpose(1, 2)
    for b in range(B):
        e = exp[b]
        rel = ((Bm[b].double() - e).norm() / e.norm()).item()
        rel32 = ((Bm32[b].double() - e).norm() / e.norm()).item()
        assert rel < 2e-6, (b, rel, rel32)
    # ---- L^T res (inside the R step) and the R-step solution
    Rx = torch.empty((B, r, n), device=DEV)
    R32 = torch.empty((B, r, n), device=DEV)
    tmp = torch.empty((B, r, n), device=DEV)
    eng.lplr_R_step(L, res, Rx, tmp, halves=hv)
    ct = tmp.clone()
    eng.lplr_R_step(L, res, R32, torch.empty((B, r, n), device=DEV))
    exp = L.double().transpose(1, 2) @ res.double()
    for b in range(B):
        e = exp[b]
        assert ((ct[b].double() - e).norm() / e.norm()).item() < 2e-6
        # lstsq solutions of the two paths agree to fp32 grade
        rel = ((Rx[b] - R32[b]).double().norm() / R32[b].double().norm()).item()
        assert rel < 1e-5, (b, rel)


def test_lplr_loop_split_vs_fp32_engine(monkeypatch):
    """The engine end to end on H = I with quantised factors: split-fp16 LPLR products (and
    normal-equation GEMMs) on (default) and off give final errors within 1e-3 relative (the loop itself is chaotic --
    tests/test_gpu_lplr_teacher.py)."""
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams
    calls = []
    orig = K.gemm_x3

    def counting(Ah, Al, Bh, Bl, inv_scale, C, **kw):
        if C is not None and tuple(C.shape) in ((2, 512, 64), (2, 64, 1024)):
            calls.append(tuple(C.shape))
        return orig(Ah, Al, Bh, Bl, inv_scale, C, **kw)

    monkeypatch.setattr(K, "gemm_x3", counting)
    torch.manual_seed(3)
    W = (torch.randn(2, 512, 1024) * 0.02).half().to(DEV)
    errs = {}
    for x3 in (True, False):
        eng = CalderaEngine(EngineParams(Q_bits=2, L_bits=4, R_bits=4, rank=64, iters=2, lplr_iters=3,
                                         update_order=["Q", "LR"], sigma_reg=1e-8))
        eng.lplr_x3 = x3
        calls.clear()
        out = eng.run(W)
        # per LR update: lplr_iters + 1 Y R^T products and 2 lplr_iters normal-equation GEMMs
        # (Bm Wr, T1 Wr^T) with m x r outputs; lplr_iters L^T res, LR_init's U^T Y (from the
        # same Y^T halves) and 2 lplr_iters normal-equation GEMMs (Wl^T Ct, Wl T2), r x n
        assert (calls.count((2, 512, 64)), calls.count((2, 64, 1024))) == ((2 * 10, 2 * 10) if x3 else (0, 0))
        errs[x3] = np.array([o["errors"]["LR"][-1] for o in out], dtype=np.float64)
    np.testing.assert_allclose(errs[True], errs[False], rtol=1e-3)
