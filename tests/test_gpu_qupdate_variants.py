"""The fused Q update (cq_q_update_x3: res = W - L R, alg.py:262, quantised whole-matrix,
quantization.py:260-268) reproduces the round-2 kernel bit for bit after round 3's changes to
it: pass 1 now gathers a row's 2-bit code bytes across four 32-column chunks and stores 32
contiguous bytes per row (instead of one 2-byte store per lane and chunk), and the opt-in pass-0
variants were removed from the library.

tests/golden/qupdate_r02_fingerprints.json holds the round-2 library's packed codes (SHA-256),
scales and error sums on the host-seeded inputs of tests/qupdate_cases.py (full config-2 shape,
a partial last code group, 4-bit packing, K = 256, fp32 W), recorded on an MI355X by
tools/ab_qupdate_r02.py, which runs both libraries in one process."""
import json
import os

import pytest
import torch

from conftest import GOLDEN
import qupdate_cases as C

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", C.CASES, ids=[c[0] for c in C.CASES])
def test_q_update_matches_round2_kernel(case):
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    ref = json.load(open(os.path.join(GOLDEN, "qupdate_r02_fingerprints.json")))["cases"][case[0]]
    got = C.run(K, case, torch.device("cuda:0"))
    assert got["packed_sha256"] == ref["packed_sha256"]
    assert got["scale"] == ref["scale"]
    assert got["err"] == ref["err"]


LIST_CASES = [c for c in C.CASES if c[5] == 2 and c[6] == torch.float16]


@pytest.mark.parametrize("kind", ["single", "multi"])
@pytest.mark.parametrize("extra", [-1, 0, 1], ids=["cap-1", "cap", "cap+1"])
def test_q_update_list_at_capacity(extra, kind):
    """A list region holding exactly its capacity of candidate groups is complete (no
    fallback) and one more overflows (fallback to the second recompute); both give the
    two-pass codes bit for bit.  Region 0 of matrix 0 gets cap + extra planted groups -- with
    one candidate element each (list A) or two (list B) -- region 1 a few, so a count one past
    the filled slots would read region 1's first entry."""
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    dev = torch.device("cuda:0")
    B, n, r = 2, 64, 32
    rows, cap_a, cap_b = K.q_update_list_geometry(8 * 48, n, r, both=True)
    cap = cap_a if kind == "single" else cap_b
    m = 8 * rows                          # 8 wave regions (the first panel)
    g = torch.Generator().manual_seed(4242)
    W = torch.randn(B, m, n, generator=g) * 0.01
    groups = [(i, 8 * c) for i in range(rows) for c in range(n // 8)]   # (row, first column) of region 0
    assert len(groups) >= cap + 1
    pick = torch.randperm(len(groups), generator=g)[: cap + extra].tolist()
    for t, j in enumerate(pick):          # candidate elements >= 0.5 per planted group; the first is the absmax
        i, c0 = groups[j]
        W[0, i, c0 + t % 8] = 1.0 if t == 0 else (0.5 + 0.4 * torch.rand((), generator=g)) * (1 if t % 3 else -1)
        if kind == "multi":
            W[0, i, c0 + (t + 3) % 8] = (0.5 + 0.4 * torch.rand((), generator=g)) * (-1 if t % 2 else 1)
    for t in range(5):                    # region 1
        W[0, rows + 3 * t, 8 * t % n] = 0.7
    W[1, 5, 9] = 1.0
    W = W.half().to(dev)
    L = (torch.randn(B, m, r, generator=g) * 1e-3).to(dev)
    R = (torch.randn(B, r, n, generator=g) * 1e-3).to(dev)

    def call(hint):
        packed = torch.empty(B, m * n // 4, dtype=torch.uint8, device=dev)
        scale = torch.empty(B, device=dev)
        err = torch.empty(B, dtype=torch.float64, device=dev)
        fb = torch.full((B,), -1, dtype=torch.int32, device=dev)
        K.q_update_x3(W, L, R, 2, packed=packed, scale=scale, err_out=err, scale_hint=hint, fallback_out=fb)
        torch.cuda.synchronize()
        return packed.cpu(), scale.cpu(), err.cpu(), fb.cpu()

    p0, s0, e0, _ = call(None)
    p, s, e, fb = call(s0.to(dev))
    assert fb.tolist() == [int(cap + extra > cap), 0], (cap, extra, fb.tolist())
    assert torch.equal(p, p0) and torch.equal(s, s0)
    for i in range(B):
        assert abs(e[i].item() - e0[i].item()) <= 1e-7 * e0[i].item()


@pytest.mark.parametrize("weighted", [False, True], ids=["unit", "err_w"])
@pytest.mark.parametrize("case", LIST_CASES, ids=[c[0] for c in LIST_CASES])
def test_q_update_single_recompute_matches_two_pass(case, weighted):
    """The 2-bit single-recompute path (scale_hint given: one L R recompute, candidate lists
    |res| >= 0.45 hint, codes from the lists) gives the two-pass kernel's packed codes and
    scales bit for bit and its error sums to 1e-7 relative (the same fp32 terms, summed in
    fp32 over runs of 4 by pass 1 and of 8 by the list path, whose nonzero codes' terms are
    corrected in fp64); matrices whose list cannot be
    complete (scale < 0.9 hint, an overflowing list, a non-finite hint) take pass 1 and give
    the two-pass codes and scales exactly and its error to fp64 summation order.  Mixed batches exercise both in one call, and the hint may
    alias the scale output (the engine's use: st.Qs is both)."""
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    tag, B, m, n, r, bits, dt = case
    dev = torch.device("cuda:0")
    W, L, R = C.make(B, m, n, r, dt, seed=sum(map(ord, tag)) + 7)
    W, L, R = W.to(dev), L.to(dev), R.to(dev)
    # error column weights (the activation-aware error, alg.py:286-302): h spanning 1e-3..10
    ew = (10.0 ** torch.empty(n).uniform_(-3, 1, generator=torch.Generator().manual_seed(n))).to(dev) if weighted else None

    def call(hint, alias=False):
        packed = torch.empty(B, m * n // 4, dtype=torch.uint8, device=dev)
        err = torch.empty(B, dtype=torch.float64, device=dev)
        fb = torch.full((B,), -1, dtype=torch.int32, device=dev)
        if alias and hint is not None:
            scale = hint.clone()
            K.q_update_x3(W, L, R, 2, packed=packed, scale=scale, err_out=err, err_w=ew, scale_hint=scale,
                          fallback_out=fb)
        else:
            scale = torch.empty(B, device=dev)
            K.q_update_x3(W, L, R, 2, packed=packed, scale=scale, err_out=err, err_w=ew, scale_hint=hint,
                          fallback_out=fb)
        torch.cuda.synchronize()
        return packed.cpu(), scale.cpu(), err.cpu(), fb.cpu()

    p0, s0, e0, f0 = call(None)
    assert (f0 == 0).all()
    s = s0.to(dev)
    variants = {
        "exact": (s, [0] * B),
        "hint 5% high": (s * 1.05, [0] * B),
        "hint 20% high": (s * 1.2, [1] * B),            # 2 tau = 1.08 s > s: list incomplete
        "hint 1e-3": (s * 1e-3, [1] * B),               # every element a candidate: overflow
        "hint nan": (torch.full_like(s, float("nan")), [1] * B),
        "mixed": (torch.stack([s[i] * (1.2 if i % 2 else 1.0) for i in range(B)]), [i % 2 for i in range(B)]),
    }
    for name, (hint, want_fb) in variants.items():
        for alias in (False, True):
            p, sc, e, fb = call(hint, alias)
            assert fb.tolist() == want_fb, (name, fb.tolist())
            assert torch.equal(p, p0), (name, alias, int((p != p0).sum()))
            assert torch.equal(sc, s0), name
            for i in range(B):
                if want_fb[i]:
                    # pass 1 again, on the list path's panel geometry (12 waves of 32 rows at
                    # K <= 128): the same fp32 terms, summed in fp64 over other panels
                    assert abs(e[i].item() - e0[i].item()) <= 1e-12 * e0[i].item(), (name, i)
                else:
                    assert abs(e[i].item() - e0[i].item()) <= 1e-7 * e0[i].item(), (name, i, e[i].item(), e0[i].item())


def test_q_update_list_path_nan_residual_falls_back():
    """A NaN residual (a NaN in W) on the single-recompute path: pass 2's |res| max skips NaN
    (v_max3 with |.| modifiers), so the matrix is sent to pass 1 through its NaN error sum,
    with a NaN absmax, as the two-pass form has it: same packed codes, a NaN scale and error
    for that matrix, the other matrices of the batch untouched and on the list path."""
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    tag, B, m, n, r, bits, dt = LIST_CASES[0]
    dev = torch.device("cuda:0")
    W, L, R = C.make(B, m, n, r, dt, seed=99)
    W, L, R = W.to(dev), L.to(dev), R.to(dev)
    W[0, 5, 17] = float("nan")

    def call(hint):
        packed = torch.empty(B, m * n // 4, dtype=torch.uint8, device=dev)
        err = torch.empty(B, dtype=torch.float64, device=dev)
        scale = torch.empty(B, device=dev)
        fb = torch.full((B,), -1, dtype=torch.int32, device=dev)
        K.q_update_x3(W, L, R, 2, packed=packed, scale=scale, err_out=err, scale_hint=hint, fallback_out=fb)
        torch.cuda.synchronize()
        return packed.cpu(), scale.cpu(), err.cpu(), fb.cpu()

    p0, s0, e0, _ = call(None)
    assert torch.isnan(s0[0]) and torch.isnan(e0[0])
    hint = torch.where(torch.isnan(s0), torch.ones_like(s0), s0).to(dev)
    p, s, e, fb = call(hint)
    assert fb.tolist() == [1] + [0] * (B - 1)
    assert torch.equal(p, p0)
    assert torch.isnan(s[0]) and torch.isnan(e[0])
    assert torch.equal(s[1:], s0[1:])
