"""The sparse-code Gram (csrc/cq_sgram.hip, sgram.py) against fp64: G = Y Y^T for
Y = (W - Q) diag(ycol), Q = s c the 2-bit whole-matrix codes of the LR step (alg.py:211-217,
quantization.py:93-105), assembled as A - s (P + P^T) with A = W diag(w) W^T (split-fp16 Gram
of W) and P = (W - (s/2) c) diag(w) c^T over the sliced-ELL codes.  Checked: the per-row
nonzero counts (exact), the fp32 G and its K-blocked split halves (fp32-grade against fp64,
and against the dense split-fp16 Gram of Y that it replaces), for every LDS slab height
(R = 8 / 4 / 2 rows of E by contraction length) and with and without column weights."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _unblock(h, k):
    B = h.shape[0]
    return h.view(B, k // 32, k, 32).permute(0, 2, 1, 3).reshape(B, k, k)


@pytest.mark.parametrize("B,m,n,weighted", [(3, 256, 512, False), (2, 512, 512, True), (2, 256, 4608, False),
                                            (2, 128, 6400, True), (2, 64, 12800, False), (2, 256, 11008, False),
                                            (1, 4096, 11008, True)])
def test_sparse_gram_matches_fp64(B, m, n, weighted):
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    from ee274_convexcaldera_llm_quantization_amd import sgram
    from ee274_convexcaldera_llm_quantization_amd.solver import X3_SCALE
    g = torch.Generator(device=DEV).manual_seed(m + n + weighted)
    W = (torch.randn(B, m, n, device=DEV, generator=g) * 0.7).half()
    ycol = (torch.rand(n, device=DEV, generator=g) + 0.5) if weighted else None
    w = ycol * ycol if weighted else None
    q = K.quantize_uniform(W.float().reshape(B, -1), m * n, 2, codes=True, packed=True, deq=False)
    codes, packed, s = q["codes"].view(B, m, n), q["packed"], q["scale"].view(B)
    Y = (W.double() - codes.double() * s.double().view(B, 1, 1)) * (ycol.double() if weighted else 1.0)
    G64 = Y @ Y.transpose(1, 2)
    ysq = (Y * Y).sum(dim=(1, 2))

    assert sgram.applicable(m, n, W, 2, True, False)
    SG = sgram.SparseGram(B, m, n, DEV)
    SG.count(packed)
    nnz = (codes != 0).sum(dim=2).to(torch.int32).reshape(-1)
    assert torch.equal(SG.row_nnz, nnz)
    # rows sorted by count (descending, ties in row order) per matrix
    perm = SG.perm.view(B, m).long()
    ref = torch.stack([torch.sort(-nnz.view(B, m)[b].long() * m + torch.arange(m, device=DEV))[1] for b in range(B)])
    assert torch.equal(perm, ref)
    print(f"density (padded ELL) {SG.density:.4f}, nonzero codes {float((codes != 0).float().mean()):.4f}")

    wmax = K.absmax(W)
    A = torch.empty(B, m, m, device=DEV)
    Gh = torch.empty(B, m, m, device=DEV, dtype=torch.float16)
    Gl = torch.empty_like(Gh)
    yh = torch.empty(B, m, n, device=DEV, dtype=torch.float16)
    yl = torch.empty_like(yh)
    sgram.gram_A(W, ycol, float(ycol.max()) if weighted else 1.0, wmax, A, Gh, Gl, X3_SCALE, yh, yl)
    if not weighted:  # A from one fp16 product (lo = 0) equals the three-product Gram bit for bit
        A3 = torch.zeros_like(A)
        ys0 = torch.empty(B, device=DEV)
        K.residual_split(W, None, None, 2, wmax, hi=yh, lo=yl, scale=ys0)
        assert int(yl.view(torch.int16).abs().max()) == 0
        t = torch.empty(B, device=DEV)
        K.gemm_x3(yh, yl, yh, yl, 1.0 / (ys0 * ys0), A3, tri=True, a_blocked=True, b_blocked=True,
                  out_h=Gh, out_l=Gl, out_scale=X3_SCALE, sym_bound=torch.full((B,), 2.0 ** 60, device=DEV,
                                                                          dtype=torch.float64),
                  scale_out=t, inv_out=t.clone())
        up = torch.ones(m, m, dtype=torch.bool, device=DEV).triu()
        assert torch.equal(A[:, up], A3[:, up])
    gs = torch.empty(B, device=DEV)
    ginv = torch.empty(B, device=DEV)
    G32 = torch.empty(B, m, m, device=DEV)
    assert SG.gram(W, packed, s, w, A, ysq, Gh, Gl, gs, ginv, X3_SCALE, G32=G32, max_density=1.0)
    scale = G64.abs().amax(dim=(1, 2))
    err32 = ((G32.double() - G64).abs().amax(dim=(1, 2)) / scale).max().item()
    Gs = (_unblock(Gh, m).double() + _unblock(Gl, m).double()) / gs.double().view(B, 1, 1)
    errs = ((Gs - G64).abs().amax(dim=(1, 2)) / scale).max().item()
    Uh = _unblock(Gh, m)
    assert torch.equal(G32, G32.transpose(1, 2)) and torch.equal(Uh, Uh.transpose(1, 2))
    assert torch.allclose(ginv, 1.0 / (gs * X3_SCALE))

    # the dense split-fp16 Gram of Y it replaces (cq_residual_split halves + cq_gemm_x3 sym_out)
    ys = torch.empty(B, device=DEV)
    K.residual_split(W, packed, s, 2, wmax, ycol=ycol, ycol_max=float(ycol.max()) if weighted else 1.0,
                     hi=yh, lo=yl, scale=ys)
    Dh, Dl = torch.empty_like(Gh), torch.empty_like(Gl)
    ds, di = torch.empty(B, device=DEV), torch.empty(B, device=DEV)
    K.gemm_x3(yh, yl, yh, yl, 1.0 / (ys * ys), None, tri=True, a_blocked=True, b_blocked=True, out_h=Dh, out_l=Dl,
              out_scale=X3_SCALE, sym_bound=ysq, scale_out=ds, inv_out=di)
    assert torch.equal(ds, gs)
    Gd = (_unblock(Dh, m).double() + _unblock(Dl, m).double()) / ds.double().view(B, 1, 1)
    errd = ((Gd - G64).abs().amax(dim=(1, 2)) / scale).max().item()
    print(f"B={B} m={m} n={n} w={weighted}: max|G - G64| / max|G64|: sparse fp32 {err32:.2e}, sparse halves "
          f"{errs:.2e}, dense split Gram {errd:.2e}")
    # fp32-grade: within 1.5x (+2e-7) of the dense split-fp16 Gram's own error, on every shape
    assert err32 < 1.5 * errd + 2e-7 and errs < 1.5 * errd + 2e-7


def _expected_ell_rows(codes, perm, row_nnz, lo=0, hi=None):
    """The sliced-ELL entry order (cq_sgram.hip, sgram_fill_kernel) restated on the host: per
    sorted position p (row j = perm[p]) the nonzero codes (l << 2 | code + 1) with l in [lo, hi)
    (one part of an l-split row; default all), grouped by residue l mod 16 in increasing l;
    rows of at most 256 entries in total take residue (p + t) mod 16 at step t while it has
    entries left, else the residue with the most left (ties: the smaller); longer rows the
    residues in the order p, p + 1, ... (mod 16)."""
    out = []
    for p, j in enumerate(perm):
        row = codes[j]
        ls = [l for l in np.nonzero(row != 0)[0] if lo <= l < (len(row) if hi is None else hi)]
        ent = {u: [int((l << 2) | (row[l] + 1)) for l in ls if l % 16 == u] for u in range(16)}
        q = p & 15
        seq = []
        if row_nnz[j] > 256:   # SG_FILL_CAP
            for i in range(16):
                seq += ent[(q + i) & 15]
        else:
            taken = [0] * 16
            for t in range(len(ls)):
                d = (q + t) & 15
                if taken[d] < len(ent[d]):
                    u = d
                else:
                    u = max(range(16), key=lambda v: (len(ent[v]) - taken[v], -v))
                seq.append(ent[u][taken[u]])
                taken[u] += 1
        out.append(seq)
    return out


@pytest.mark.parametrize("k,L,dens", [(200, 1024, 0.03), (64, 4096, 0.004), (200, 10240, 0.01), (128, 11008, 0.012)])
def test_sparse_gram_ell_order(k, L, dens):
    """The ELL fill (sgram_count + sgram_fill) against the host restatement of its entry order:
    counts, row sort, per-row entry sequence (bank-group rotation, greedy fallback, rows past
    256 entries in residue-rotated order) and padding, entry for entry.  Contractions past
    9600 (L = 10240, 11008) take the l-split layout (cq_sgram_split): per slice the first parts
    (l < Lh) in its first slice_w1 rows, padded with l = 0, then the second parts padded with
    l = Lh, each part ordered as above on its own entries."""
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    rng = np.random.default_rng(k + L)
    B = 2
    codes = np.where(rng.random((B, k, L)) < dens, rng.choice([-1, 1], size=(B, k, L)), 0).astype(np.int8)
    codes[0, 5, : L // 2] = 1          # a row past 256 entries
    codes[1, 7, :] = 0                 # an empty row
    off = (codes + 1).astype(np.uint8).reshape(B, k, L // 4, 4)
    packed = (off[..., 0] << 6) | (off[..., 1] << 4) | (off[..., 2] << 2) | off[..., 3]
    dev = "cuda:0"
    pk = torch.from_numpy(np.ascontiguousarray(packed).reshape(B, -1)).to(dev)
    ns = -(-k // 64)
    row_nnz = torch.empty(B * k, dtype=torch.int32, device=dev)
    perm = torch.empty(B * k, dtype=torch.int32, device=dev)
    slice_off = torch.empty(B * (ns + 1), dtype=torch.int64, device=dev)
    total = torch.empty(B, dtype=torch.int64, device=dev)
    Lh = K.sgram_split(k, L)
    assert (Lh < L) == (L > 9600)
    nz1 = torch.empty(B * k, dtype=torch.int32, device=dev)
    sw1 = torch.empty(B * ns, dtype=torch.int32, device=dev)
    K.sgram_count(pk, k, L, row_nnz, perm, slice_off, total, Lh=Lh, row_nnz1=nz1, slice_w1=sw1)
    stride = int(total.max().item()) + 64
    ell = torch.full((B * stride,), -7, dtype=torch.int32, device=dev)
    K.sgram_fill(pk, k, L, row_nnz, perm, slice_off, ell, stride, Lh=Lh, slice_w1=sw1)
    torch.cuda.synchronize()
    nz, pm, so = row_nnz.cpu().numpy().reshape(B, k), perm.cpu().numpy().reshape(B, k), slice_off.cpu().numpy()
    w1 = sw1.cpu().numpy().reshape(B, ns)
    el = ell.cpu().numpy().view(np.uint32).reshape(B, stride)
    for b in range(B):
        assert (nz[b] == (codes[b] != 0).sum(1)).all()
        assert sorted(pm[b].tolist()) == list(range(k))
        parts = [(0, Lh, 1)] + ([(Lh, L, (Lh << 2) | 1)] if Lh < L else [])
        exps = [_expected_ell_rows(codes[b], pm[b], nz[b], lo, hi) for lo, hi, _ in parts]
        sob = so[b * (ns + 1):(b + 1) * (ns + 1)]
        for p in range(k):
            s = p // 64
            width = int(sob[s + 1] - sob[s])
            cut = int(w1[b, s]) if Lh < L else width
            if Lh < L:   # the slice's part widths: its widest row's count in each part
                rows = pm[b][64 * s:64 * s + 64]
                c1 = [int((codes[b][j, :Lh] != 0).sum()) for j in rows]
                assert cut == max(c1) and width - cut == max(int(nz[b][j]) - c for j, c in zip(rows, c1))
            for (lo, hi, pad), exp, (t0, t1) in zip(parts, exps, [(0, cut), (cut, width)]):
                got = [int(el[b, (sob[s] + t) * 64 + p % 64]) for t in range(t0, t1)]
                want = exp[p] + [pad] * (t1 - t0 - len(exp[p]))
                assert got == want, (b, p, lo, got[:8], want[:8])


@pytest.mark.parametrize("m,n,weighted", [(1024, 2048, False), (1024, 2048, True), (2048, 1024, False),
                                          (1024, 1024, False)])
def test_lr_step_from_codes_matches_residual_pass(m, n, weighted):
    """The LR step without a pass over Y (R = U^T W - s U^T c, L = W V - s c V for m > n, and
    ||Y||^2 from ||W||^2 plus the codes' correction; tall shapes through the sparse-code Gram of
    W^T and c^T) against the same engine with the residual pass (r_from_codes off; for m > n
    also the dense Gram): same first-Q codes, errors and Q + L R to the solver tolerance (1e-5
    relative error of the rank-r projection: the two Grams' roundings differ, so the two solves'
    iterates and filter bounds do too)."""
    from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams
    ep = EngineParams(Q_bits=2, L_bits=16, R_bits=16, rank=64, iters=3, update_order=["Q", "LR"], sigma_reg=1e-8)
    g = torch.Generator().manual_seed(m + 3 * n + weighted)
    W = (torch.randn(2, m, n, generator=g) * 0.02).half().to(DEV)
    h = (torch.rand(n, generator=g) + 0.05).to(DEV) if weighted else None
    outs, engs = [], []
    for codes in (True, False):
        e = CalderaEngine(ep)
        e.r_from_codes = codes
        outs.append(e.run(W, h))
        engs.append(e)
    assert engs[0].lr_steps_from_codes == 3 and engs[1].lr_steps_from_codes == 0
    for a, b in zip(*outs):
        assert torch.equal(a["Q_idxs"], b["Q_idxs"]) or (a["Q_idxs"] != b["Q_idxs"]).sum() <= 2
        for k in ("Q", "LR"):
            assert max(abs(x - y) for x, y in zip(a["errors"][k], b["errors"][k])) < 1e-5, (k, a["errors"], b["errors"])
        qa = a["Q"].double() + a["L"].double() @ a["R"].double()
        qb = b["Q"].double() + b["L"].double() @ b["R"].double()
        assert float(torch.linalg.norm(qa - qb) / torch.linalg.norm(qb)) < 2e-5


@pytest.mark.parametrize("case", ["tall_not_aware_h", "wide_allclose_I", "tall_allclose_I", "rank_over_256"])
def test_lr_step_gates_write_what_the_error_reads(case):
    """Configurations the codes-only LR step must NOT take (round-4 advisor findings), run
    against the residual-pass engine (r_from_codes off):
    * m > n with activation_aware_LR=False and a non-unit diagonal H: the error weights are
      not Y's column weights, so the LR error is the fused GEMM on res (alg.py:286-302) --
      the codes-only step never writes res;
    * an H that passes allclose(H, I) (optimized_eigh: unit eigenvalues, Y = res) but is not
      exactly 1: the error keeps h, so again res must be written (wide and tall shapes);
    * rank > 256: cq_codes_matmul takes r <= 256, larger ranks keep the residual pass."""
    from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams
    m, n, rank, aware = {"tall_not_aware_h": (2048, 1024, 64, False), "wide_allclose_I": (1024, 2048, 64, True),
                         "tall_allclose_I": (2048, 1024, 64, True), "rank_over_256": (1024, 2048, 272, True)}[case]
    ep = EngineParams(Q_bits=2, L_bits=16, R_bits=16, rank=rank, iters=2, update_order=["Q", "LR"], sigma_reg=1e-8,
                      activation_aware_LR=aware)
    g = torch.Generator().manual_seed(len(case))
    W = (torch.randn(1, m, n, generator=g) * 0.02).half().to(DEV)
    if case == "tall_not_aware_h":
        h = (torch.rand(n, generator=g) + 0.05).to(DEV)
    elif case.endswith("allclose_I"):
        h = (1.0 + 2e-6 * (torch.rand(n, generator=g) - 0.5)).to(DEV)
    else:
        h = None
    outs = []
    for codes in (True, False):
        e = CalderaEngine(ep)
        e.r_from_codes = codes
        outs.append(e.run(W, h))
        assert e.lr_steps_from_codes == 0, (case, codes, e.lr_steps_from_codes)
    a, b = outs[0][0], outs[1][0]
    for k in ("Q", "LR"):
        assert all(math.isfinite(x) for x in a["errors"][k])
        assert max(abs(x - y) for x, y in zip(a["errors"][k], b["errors"][k])) < 2e-6, (k, a["errors"], b["errors"])
    # the LR errors against a direct fp64 evaluation of the final state's weighted error
    Ws = a["W"].double().to(DEV)
    E = Ws - a["Q"].double() - a["L"].double() @ a["R"].double()
    hw = torch.ones(n, dtype=torch.float64, device=DEV) if h is None else h.double()
    direct = math.sqrt(float((E * E * hw).sum() / (Ws * Ws * hw).sum()))
    # (the kept iterate is the one with the smallest error after both update kinds ran)
    assert min(abs(direct - x) for x in a["errors"]["LR"] + a["errors"]["Q"]) < 2e-6, (direct, a["errors"])
