"""Sparse-code helpers of the LR step (cq_sgram.hip: cq_codes_transpose, cq_codes_matmul,
cq_codes_ysq_corr, cq_transpose_f16) against plain torch restatements on the unpacked codes:
integer work bit-exact, the fp32 products against fp64 (order-independent bound), the fp64
norm correction against the fp64 sum over the dense residual."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _codes(B, m, n, density, seed):
    """Packed 2-bit codes with ~density nonzeros (+-1) and their int8 form."""
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(B, m, n, generator=g)
    c = torch.zeros(B, m, n, dtype=torch.int8)
    c[u < density / 2] = -1
    c[(u >= density / 2) & (u < density)] = 1
    W = torch.randn(B, m, n, generator=g).half()
    packed = torch.empty(B, m * n // 4, dtype=torch.uint8, device=DEV)
    # quantise W' = c (exact codes): scale 1, |x| = 1 -> +-1, 0 -> 0
    K.q_update_x3(c.float().half().to(DEV), None, None, 2, packed=packed, scale=torch.empty(B, device=DEV))
    assert torch.equal(K.unpack_codes(packed, m * n, 2).cpu().view(B, m, n), c)
    return packed, c, W


@pytest.mark.parametrize("B,m,n", [(2, 4096, 4096), (3, 11008 // 16 * 16, 512), (1, 48, 80), (2, 272, 4096)])
def test_codes_transpose(B, m, n):
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    packed, c, _ = _codes(B, m, n, 0.02, m + n)
    t = K.codes_transpose(packed, m, n)
    got = K.unpack_codes(t, m * n, 2).cpu().view(B, n, m)
    assert torch.equal(got, c.transpose(1, 2))


@pytest.mark.parametrize("trans", [False, True])
@pytest.mark.parametrize("B,rows,cols,r,ldx,density", [(2, 4096, 4096, 128, 192, 0.01), (2, 200, 1040, 200, 256, 0.3),
                                                       (3, 64, 4096, 64, 64, 0.0), (1, 96, 2048, 33, 40, 1.0)])
def test_codes_matmul(trans, B, rows, cols, r, ldx, density):
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    packed, c, _ = _codes(B, rows, cols, density, rows * 7 + cols)
    g = torch.Generator().manual_seed(r)
    X = torch.randn(B, cols, ldx, generator=g)
    w = torch.rand(cols, generator=g) + 0.5
    for colw in (None, w):
        out = torch.empty((B, r, rows) if trans else (B, rows, r), device=DEV)
        K.codes_matmul(packed, rows, cols, X.to(DEV), r, out, colw=None if colw is None else colw.to(DEV), trans=trans)
        cw = c.double() * (1.0 if colw is None else colw.double())
        ref = cw @ X[:, :, :r].double()
        if trans:
            ref = ref.transpose(1, 2)
        # fp32 accumulation over a row's k nonzero terms: |err| <= k u sum |terms| (u = 2^-24)
        k = (c != 0).sum(-1, keepdim=True).double() + 1
        bound = (cw.abs() @ X[:, :, :r].double().abs()) * k * 2.0 ** -24 + 1e-30
        if trans:
            bound = bound.transpose(1, 2)
        assert ((out.cpu().double() - ref).abs() <= bound).all()


def test_codes_matmul_deterministic():
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    packed, c, _ = _codes(2, 512, 4096, 0.05, 5)
    X = torch.randn(2, 4096, 128, device=DEV)
    a = K.codes_matmul(packed, 512, 4096, X, 128, torch.empty(2, 512, 128, device=DEV))
    b = K.codes_matmul(packed, 512, 4096, X, 128, torch.empty(2, 512, 128, device=DEV))
    assert torch.equal(a, b)


@pytest.mark.parametrize("weighted", [False, True])
def test_codes_ysq_corr(weighted):
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    B, m, n = 3, 1024, 2048
    packed, c, W = _codes(B, m, n, 0.03, 11)
    s = torch.tensor([2.5, 3.0, 0.75])
    w = (torch.rand(n) + 0.1) if weighted else None
    got = K.codes_ysq_corr(packed, W.to(DEV), s.to(DEV), None if w is None else w.to(DEV)).cpu()
    Wd = W.double()
    wd = torch.ones(n, dtype=torch.float64) if w is None else w.double()
    full = ((Wd - s.double().view(B, 1, 1) * c.double()) ** 2 * wd).sum((1, 2))
    base = (Wd ** 2 * wd).sum((1, 2))
    ref = full - base
    assert torch.allclose(got, ref, rtol=1e-9, atol=1e-6 * base.max().item() * 1e-6)


@pytest.mark.parametrize("B,rows,cols", [(2, 4096, 4096), (1, 11008, 4096), (2, 100, 37)])
def test_transpose_f16(B, rows, cols):
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    X = torch.randn(B, rows, cols, device=DEV).half()
    assert torch.equal(K.transpose_f16(X), X.transpose(1, 2).contiguous())
