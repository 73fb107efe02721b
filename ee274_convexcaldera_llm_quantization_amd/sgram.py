"""The LR step's Gram G = Y Y^T from the sparse 2-bit Q codes (csrc/cq_sgram.hip).

Y = (W - Q) diag(ycol) is the operand the reference's SVD factors (alg.py:211-217).  With
2-bit whole-matrix absmax codes (quantization.py:93-105: k = 1, Q = s c, c in {-1, 0, 1}) only
the elements with |x| > s/2 carry a nonzero code -- about 1 % at the bench's configuration --
so with w = ycol^2 and E = W - (s/2) c

    G = A - s (P + P^T),    A = W diag(w) W^T,    P = E diag(w) c^T.

A does not depend on Q: it is one split-fp16 Gram of W's halves per run (`gram_A`).  Every LR
step then costs the sparse product P and one elementwise pass instead of a dense Gram
(`sparse_gram`).  Scope: m <= n (G is m x m, the contraction runs over the n columns), fp16 W,
2-bit packed codes, diagonal or no H; anything else keeps the dense Gram."""
from __future__ import annotations

import torch

from . import _lib as K
from . import scratch

# l-split ELL for the long contractions (cq_sgram_split); False: the unsplit R = 2 layout (A/B)
L_SPLIT = True

# above this fraction of nonzero codes (padded sliced-ELL entries / (m n)) the dense Gram is
# cheaper (the sparse product's cost grows with the entries, the dense Gram's does not)
MAX_DENSITY = 0.03


def applicable(m: int, n: int, W: torch.Tensor, q_bits: int, packed: bool, dense_h: bool) -> bool:
    return (m <= n and m % 64 == 0 and n % 64 == 0 and W.dtype == torch.float16 and q_bits == 2 and packed
            and not dense_h and K.sgram_rows(n) > 0)


def gram_A(Ws: torch.Tensor, ycol, ycol_max: float, wmax: torch.Tensor, A: torch.Tensor, Gh, Gl, out_scale: float,
           yh: torch.Tensor, yl: torch.Tensor, ys=None, wth=None, wtl=None, wsq=None):
    """A (B, m, m) fp32 upper triangle = (W diag(ycol)) (W diag(ycol))^T on split-fp16 products
    (cq_gemm_x3 Gram, tri + sym_out).  H = I: the K-blocked halves of W written into yh are
    exact (fp16 W under a split scale >= 1, lo = 0) and one fp16 product gives the same bits as
    three.  Diagonal H: A = (W diag(ycol^2)) W^T from the split halves of W diag(ycol^2) (yh/yl)
    against W itself (fp16, exact: b_exact, two products instead of three; the B operand is W's
    row-major storage, no halves written).  Gh/Gl receive a split of A that the caller
    overwrites later.  The same work writes the exact halves of W^T (wth (B, n, m), K-blocked
    over m, lo = 0: the B operand of R = (U^T W) diag(ycol), run as gemm_x3 b_exact with the
    column weights in its epilogue) and ||W diag(ycol)||_F^2 (wsq, fp64), with the halves'
    scale in ys (B,)."""
    B, m, n = Ws.shape
    dev = Ws.device
    if ys is None:
        ys = torch.empty(B, dtype=torch.float32, device=dev)
    bound = torch.full((B,), 2.0 ** 60, dtype=torch.float64, device=dev)  # any bound >= max|A|: halves unused
    so = torch.empty(B, dtype=torch.float32, device=dev)
    io = torch.empty(B, dtype=torch.float32, device=dev)
    gram = dict(tri=True, a_blocked=True, out_h=Gh, out_l=Gl, out_scale=out_scale, sym_bound=bound, scale_out=so,
                inv_out=io)
    if ycol is None:
        assert Ws.dtype == torch.float16
        K.residual_split(Ws, None, None, 2, wmax, hi=yh, thi=wth, scale=ys, sq=wsq)
        # H = I: W's halves are W itself (fp16) and zeros -- one fp16 product gives the same bits
        K.gemm_x3(yh, yl, yh, yl, 1.0 / (ys * ys), A, b_blocked=True, single=True, **gram)
        return
    # one pass: W^T's exact halves (R = (U^T W) diag(ycol) takes the column weights in its
    # epilogue, gemm_x3 colw) and the Gram operand's halves of W diag(ycol^2) at their own
    # scale (ycol_hi); ||W diag(ycol)||^2 from the weighted square sum
    assert wtl is None
    y2 = (ycol * ycol).contiguous()
    ys2 = torch.empty(B, dtype=torch.float32, device=dev)
    K.residual_split(Ws, None, None, 2, wmax, thi=wth, scale=ys, hi=yh, lo=yl, ycol_hi=y2,
                     ycol_hi_max=ycol_max * ycol_max, scale_hi=ys2)
    if wsq is not None:
        wsq.copy_(K.weighted_sqsum(Ws, y2, n))
    K.gemm_x3(yh, yl, Ws, None, 1.0 / ys2, A, b_blocked=False, b_exact=True, **gram)


class SparseGram:
    """Per-batch workspace of the sparse Gram (row counts, ELL, P)."""

    def __init__(self, B: int, m: int, n: int, dev, split: bool = True):
        self.B, self.m, self.n = B, m, n
        self.ns = -(-m // 64)
        self.row_nnz = torch.empty(B * m, dtype=torch.int32, device=dev)
        self.perm = torch.empty(B * m, dtype=torch.int32, device=dev)
        self.slice_off = torch.empty(B * (self.ns + 1), dtype=torch.int64, device=dev)
        self.total = torch.empty(B, dtype=torch.int64, device=dev)
        # l-split ELL for the long contractions (cq_sgram_split: n = 11008 at k = 4096): four rows
        # of E staged half a contraction at a time instead of two over all of it.  split=False
        # (the engine's column-weighted Grams): the unsplit layout, whose SpMM measured faster
        # there (config 3: 32.9 vs 34.7 ms per B = 192 launch; unweighted config 4t: 10.97 vs
        # 10.53 ms per B = 64, profiles/r05i_kt3*, r05n_kt4t_*)
        self.Lh = K.sgram_split(m, n) if (L_SPLIT and split) else n
        self.row_nnz1 = torch.empty(B * m, dtype=torch.int32, device=dev) if self.Lh < n else None
        self.slice_w1 = torch.empty(B * self.ns, dtype=torch.int32, device=dev) if self.Lh < n else None
        self.density = None
        self.stats = {"sparse": 0, "dense": 0}
        self._corr_ws = None
        self.ysq_corr = None

    def count(self, packed: torch.Tensor, W=None, qscale=None, wcol=None) -> int:
        """ELL entries per matrix (max over the batch) -- one host read-back.  With W (the codes'
        layout, fp16) also self.ysq_corr (B,) fp64 = ||(W - s c) diag(ycol)||^2 - ||W diag(ycol)||^2
        (wcol = ycol^2)."""
        corr = {}
        if W is not None:
            if self._corr_ws is None:
                self._corr_ws = torch.empty(self.B * self.m, dtype=torch.float64, device=W.device)
            self.ysq_corr = torch.empty(self.B, dtype=torch.float64, device=W.device)
            corr = dict(W=W, qscale=qscale, wcol=wcol, corr_ws=self._corr_ws, corr_out=self.ysq_corr)
        K.sgram_count(packed, self.m, self.n, self.row_nnz, self.perm, self.slice_off, self.total, Lh=self.Lh,
                      row_nnz1=self.row_nnz1, slice_w1=self.slice_w1, **corr)
        mx = int(self.total.max().item())
        self.density = mx / float(self.m * self.n)
        return mx

    def gram(self, Ws, packed, qscale, w, A, bound, Gh, Gl, gscale, ginv, out_scale, G32=None,
             max_density: float = MAX_DENSITY, counted: bool = False) -> bool:
        """G's K-blocked split halves (and G32) from the codes; False (nothing written) when the
        codes are too dense for the sparse product to pay.  counted: count() already ran on
        these codes (the caller decided on its density)."""
        B, m, n = self.B, self.m, self.n
        dev = Ws.device
        if not counted:
            self.count(packed)
        elif self.density is None:
            raise RuntimeError("SparseGram.gram(counted=True) before count()")
        if self.density > max_density:
            self.stats["dense"] += 1
            return False
        # fixed capacity per matrix (a stable scratch shape across LR steps)
        stride = -(-int(max(MAX_DENSITY, self.density) * m * n) // 4096) * 4096
        ell = scratch.get("sgram.ell", (B * stride,), torch.int32, dev)
        K.sgram_fill(packed, m, n, self.row_nnz, self.perm, self.slice_off, ell, stride, Lh=self.Lh,
                     slice_w1=self.slice_w1)
        P = scratch.get("sgram.P", (B, m, m), torch.float32, dev)
        K.sgram_spmm(Ws, packed, qscale, w, ell, self.perm, self.slice_off, stride, P, Lh=self.Lh,
                     slice_w1=self.slice_w1)
        K.sgram_combine(A, P, qscale, bound, out_scale, Gh, Gl, gscale, ginv, G32=G32)
        self.stats["sparse"] += 1
        return True
