"""GPU-resident CALDERA engine (batched).  The hot path of the reference,
RCR/src/caldera/decomposition/alg.py:24-302, re-designed for MI355X:

  * B same-shape weight matrices are decomposed in lockstep, so the tall-skinny rank-r
    GEMMs and the one-workgroup-per-matrix p x p solvers fill the 256 CUs;
  * Q is never materialised in fp32 inside the loop: it lives as packed int2/int4 codes
    plus one scale, and is dequantised on the fly where it is consumed;
  * diagonal H (None, identity, or diag_embed(h) as main.py:163-165 passes) is a column
    weight vector — H_sqrt @ eigvecs (alg.py:66-68, :211) become exact column scalings;
  * the activation-aware error (alg.py:286-302) is fused into the producing kernel (the
    quantiser for Q updates, a GEMM epilogue for LR updates), accumulated in fp64;
  * the full SVD (alg.py:217) is replaced by RankRSolver (solver.py), warm-started
    across outer iterations.

State per matrix follows CalderaDecomposition (dataclasses.py:87-106).  Selection of the
best iterate reproduces alg.py:105-107 exactly (strict <, only once every update kind in
update_order has run).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from . import _lib as K
from .overlap import run_to_end
from .solver import RankRSolver


@dataclass
class EngineParams:
    """Subset of CalderaParams (dataclasses.py:11-84) the engine consumes."""
    compute_quantized_component: bool = True
    compute_low_rank_factors: bool = True
    Q_bits: int = 2
    L_bits: int = 2
    R_bits: int = 2
    rank: int = 64
    iters: int = 20
    lplr_iters: int = 5
    activation_aware_LR: bool = True
    update_order: list = field(default_factory=list)
    method_Q: str = "uniform"
    method_LR: str = "uniform"
    rand_svd: bool = False
    sigma_reg: float = 0.0

    @classmethod
    def from_caldera_params(cls, qp):
        return cls(compute_quantized_component=qp.compute_quantized_component,
                   compute_low_rank_factors=qp.compute_low_rank_factors,
                   Q_bits=qp.Q_bits, L_bits=qp.L_bits, R_bits=qp.R_bits, rank=qp.rank,
                   iters=qp.iters, lplr_iters=qp.lplr_iters,
                   activation_aware_LR=qp.activation_aware_LR,
                   update_order=list(qp.update_order),
                   method_Q=qp.quant_factory_Q.method.lower(),
                   method_LR=qp.quant_factory_LR.method.lower(),
                   rand_svd=qp.rand_svd, sigma_reg=qp.sigma_reg)


def _uniform_k(bits):
    return 2 ** (bits - 1) - 1


class _Weights:
    """Column weights derived from a diagonal H (alg.py:44-68 for diagonal H).

    err   : diag of the H used by activation_aware_error (after the sigma_reg shift)
    ycol  : diag of H_sqrt (data-aware) — Y = residual * ycol  (alg.py:211)
    rinv  : 1/sqrt(eigenvalues) in original column order (alg.py:223)
    lplr  : weights of ||(res - L R) H_sqrt||^2 (alg.py:182): ycol^2 (aware) / h^2 (not)
    """

    def __init__(self, h: torch.Tensor | None, n: int, p: EngineParams, dev):
        f32 = torch.float32
        if h is None:
            h = torch.ones(n, dtype=f32, device=dev)
        h = h.to(device=dev, dtype=f32)
        if not p.activation_aware_LR:
            self.err = h
            self.ycol = None
            self.ycol_max = 1.0
            self.rinv = None
            self.lplr = h * h
            self.identity = False
            return
        # optimized_eigh (alg.py:11-23): allclose(H, I) -> eigenvalues exactly 1
        ident = bool(torch.all(torch.abs(h - 1.0) <= 1e-8 + 1e-5).item())
        lam = torch.ones_like(h) if ident else h.clone()
        herr = h.clone()
        lmin = lam.min()
        if float(lmin.item()) < p.sigma_reg:  # alg.py:59-64 (fp32 arithmetic, as torch)
            shift = torch.tensor(p.sigma_reg, dtype=f32, device=dev) - lmin
            herr = herr + shift
            lam = lam + shift
        self.identity = ident and bool(torch.all(lam == 1.0).item())
        self.err = herr
        sq = torch.sqrt(lam)
        self.ycol = None if self.identity else sq
        self.ycol_max = 1.0 if self.identity else float(sq.max().item())
        self.rinv = None if self.identity else 1.0 / sq
        self.lplr = None if self.identity else lam  # ||Y - L (R*ycol)||^2 uses unit weights


class BatchState:
    def __init__(self, B, m, n, r, p: EngineParams, dev):
        self.B, self.m, self.n, self.r = B, m, n, r
        f32 = torch.float32
        numel = m * n
        self.q_packed = p.Q_bits <= 4 and numel % 4 == 0
        self.qcode_numel = numel * p.Q_bits // 8 if self.q_packed else numel
        qdt = torch.uint8 if self.q_packed else K.code_dtype(p.Q_bits)
        self.Qc = torch.zeros((B, self.qcode_numel), dtype=qdt, device=dev)  # codes (Q=0: see has_Q)
        self.Qs = torch.zeros(B, dtype=f32, device=dev)
        self.has_Q = False
        self.L = torch.zeros((B, m, r), dtype=f32, device=dev)
        self.R = torch.zeros((B, r, n), dtype=f32, device=dev)
        self.has_LR = False
        self.L_idxs = self.R_idxs = None
        self.L_scale = self.R_scale = None

    def snapshot_into(self, dst: "BatchState", sel: list[int]):
        """Copy the state of matrices `sel` into dst (one gather/scatter per tensor)."""
        B = self.B
        if dst.L.shape != self.L.shape:
            dst.L = torch.zeros_like(self.L)
            dst.R = torch.zeros_like(self.R)
        if self.L_idxs is not None and (dst.L_idxs is None or dst.L_idxs.shape != self.L_idxs.shape):
            dst.L_idxs = torch.zeros_like(self.L_idxs)
            dst.R_idxs = torch.zeros_like(self.R_idxs)
            dst.L_scale = torch.zeros_like(self.L_scale)
            dst.R_scale = torch.zeros_like(self.R_scale)
        pairs = [(dst.Qc, self.Qc), (dst.Qs, self.Qs), (dst.L, self.L), (dst.R, self.R)]
        if self.L_idxs is not None:
            pairs += [(dst.L_idxs, self.L_idxs), (dst.R_idxs, self.R_idxs),
                      (dst.L_scale, self.L_scale), (dst.R_scale, self.R_scale)]
        if len(sel) == B:
            for d, s in pairs:
                d.copy_(s)
        else:
            idx = torch.tensor(sel, dtype=torch.long, device=self.Qc.device)
            for d, s in pairs:
                d.index_copy_(0, idx, s.index_select(0, idx))
        for b in sel:
            dst.flag_Q[b] = self.has_Q
            dst.flag_LR[b] = self.has_LR


class CalderaEngine:
    """Decomposes a batch of B weight matrices (B, m, n) with shared params and H."""

    def __init__(self, params: EngineParams, *, solver_tol: float = 5e-6, solver_p: int | None = None,
                 filter_precision: str = "f16x3", profile: bool = False, solver_kwargs: dict | None = None):
        self.p = params
        self.solver_kwargs = dict(solver_kwargs or {})
        self.solver_tol = solver_tol
        self.solver_p = solver_p
        self.filter_precision = filter_precision
        self.profile = profile
        self.timings = {}
        self.solver = None
        for meth in (params.method_Q, params.method_LR):
            if meth != "uniform":
                raise NotImplementedError(f"quantizer method '{meth}' is not yet available on MI355X")
        if params.rand_svd:
            raise NotImplementedError("rand_svd=True is not yet available on MI355X")

    # ------------------------------------------------------------------ pieces
    def _q_update(self, st: BatchState, Ws, res_buf, wts: _Weights, den):
        """maybe_update_Q / update_Q_non_data_aware (alg.py:253-283) + error (:286-302)."""
        p = self.p
        B, m, n = st.B, st.m, st.n
        Kdim = st.L.shape[-1] if (p.compute_low_rank_factors and st.has_LR) else 0
        if Kdim % 32 == 0:
            # fused: res = W - L R recomputed per tile on split-fp16 products, never stored
            err = torch.empty(B, dtype=torch.float64, device=Ws.device)
            Lm = st.L if Kdim else None
            Rm = st.R if Kdim else None
            if st.q_packed:
                K.q_update_x3(Ws, Lm, Rm, p.Q_bits, packed=st.Qc, scale=st.Qs, err_w=wts.err, err_out=err)
            else:
                K.q_update_x3(Ws, Lm, Rm, p.Q_bits, codes=st.Qc, scale=st.Qs, err_w=wts.err, err_out=err)
            st.has_Q = True
            return err
        absmax = torch.zeros(B, dtype=torch.int32, device=Ws.device)  # |res| max as uint32 bits
        Lm = st.L[:, :, :Kdim]
        Rm = st.R[:, :Kdim, :]
        # res = W - L R  (alg.py:262; RESID epilogue also produces |res| max for the quantiser)
        K.gemm(Lm, Rm, C=res_buf, D=Ws, epi=K.EPI_RESID, absmax=absmax, batch=B)
        err = torch.empty(B, dtype=torch.float64, device=Ws.device)
        x = res_buf.view(B, m * n)
        if st.q_packed:
            K.quantize_known_max(x, absmax, p.Q_bits, packed=st.Qc, scale=st.Qs, err_w=wts.err,
                                 err_ncols=n, err_out=err)
        else:
            K.quantize_known_max(x, absmax, p.Q_bits, codes=st.Qc, scale=st.Qs, err_w=wts.err,
                                 err_ncols=n, err_out=err)
        st.has_Q = True
        return err

    def _lr_update(self, st: BatchState, Ws, Y, res, wts: _Weights, den):
        """maybe_update_LR / update_LR / LR_init (alg.py:115-235) + error (:286-302)."""
        p = self.p
        B, m, n = st.B, st.m, st.n
        dev = Ws.device
        quantized = p.L_bits < 16 or p.R_bits < 16
        weighted = p.activation_aware_LR and wts.ycol is not None
        if self.solver is None:
            self.solver = RankRSolver(B, m, n, p.rank, dev, tol=self.solver_tol, p=self.solver_p,
                                      filter_precision=self.filter_precision, **self.solver_kwargs)
        sv = self.solver
        y_split = None
        ysq = None
        if sv.x3 and not sv.direct and m % 32 == 0 and n % 64 == 0 and st.q_packed:
            # one pass: res / Y (fp32), the solver's Gram operand halves and ||Y||^2
            if self._yh is None:
                self._yh = torch.empty((B, m, n), dtype=torch.float16, device=dev)
                self._yl = torch.empty_like(self._yh)
                self._ys = torch.empty(B, dtype=torch.float32, device=dev)
            ysq = torch.empty(B, dtype=torch.float64, device=dev)
            halves = dict(hi=self._yh, lo=self._yl) if sv.left else dict(thi=self._yh, tlo=self._yl)
            K.residual_split(Ws, st.Qc if st.has_Q else None, st.Qs if st.has_Q else None, p.Q_bits, self._wmax,
                             ycol=wts.ycol if weighted else None, ycol_max=wts.ycol_max if weighted else 1.0,
                             res=res, Y=Y if weighted else None, scale=self._ys, sq=ysq, **halves)
            y_split = (self._yh, self._yl, self._ys)
        else:
            K.build_residual(Ws, st.Qc if st.has_Q else None, st.Qs if st.has_Q else None, p.Q_bits,
                             wts.ycol, Y=Y if weighted else None, res=res)
        Ysrc = Y if weighted else res  # Y = res * sqrt(h) (alg.py:211); identity H: Y = res
        Y = Ysrc
        vecs, theta = yield from sv.solve_iter(Ysrc, y_split=y_split)
        r = sv.r
        S = torch.sqrt(theta.clamp_min(0.0))  # singular values (fp64)
        S32 = S.float()
        tiny = (S32 <= S32[:, :1] * 1e-30) | (S32 == 0)
        L = torch.empty((B, m, r), dtype=torch.float32, device=dev)
        R = torch.empty((B, r, n), dtype=torch.float32, device=dev)
        if sv.left:
            U = vecs  # (B, m, r) view, ld p
            if p.activation_aware_LR:
                L.copy_(U)
                # R = (U^T Y) diag(1/sqrt(lam))   (alg.py:219-225)
                K.gemm(U, Ysrc, ta=True, C=R)
                if wts.rinv is not None:
                    K.scale_rc(R, colscale=wts.rinv, out=R)
            else:
                sq = torch.sqrt(S32)
                K.scale_rc(U, colscale=sq, out=L)  # L = U sqrt(S)
                K.gemm(U, Ysrc, ta=True, C=R)      # S Vh
                rs = torch.where(tiny, torch.zeros_like(sq), 1.0 / sq.clamp_min(1e-30))
                K.scale_rc(R, rowscale=rs, out=R)  # R = sqrt(S) Vh
        else:
            V = vecs  # (B, n, r)
            inv = torch.where(tiny, torch.zeros_like(S32), 1.0 / S32.clamp_min(1e-30))
            if p.activation_aware_LR:
                K.gemm(Ysrc, V, C=L)                 # Y V
                K.scale_rc(L, colscale=inv, out=L)   # U = Y V / S
                K.scale_rc(V, trans=True, rowscale=S32, colscale=wts.rinv, out=R)  # S V^T diag(rinv)
            else:
                sq = torch.sqrt(S32)
                K.gemm(Ysrc, V, C=L)
                K.scale_rc(L, colscale=torch.where(tiny, torch.zeros_like(sq), 1.0 / sq.clamp_min(1e-30)), out=L)
                K.scale_rc(V, trans=True, rowscale=sq, out=R)
        if quantized:
            L, R = yield from self._lplr(st, Y, res, L, R, wts)
        st.L, st.R = L, R
        st.has_LR = True
        # activation-aware error: sum_j h_j (res - L R)^2  (alg.py:286-302, diagonal H)
        if sv.left and p.activation_aware_LR and not quantized:
            # L = U (orthonormal columns), L R = U U^T Y diag(1/sqrt(h)) with h the error
            # weights, so the weighted residual is (I - U U^T) Y and, by Pythagoras,
            # sum_j h_j (res - L R)_ij^2 = ||Y||^2 - ||U^T Y||^2 = ||Y||^2 - sum_j h_j R_ij^2
            # (two fp64 reductions instead of an m x n x r product; U orthonormal to ~1e-7)
            ysq = K.weighted_sqsum(Ysrc, None, n) if ysq is None else ysq
            return ysq - K.weighted_sqsum(R, wts.err if wts.ycol is not None else None, n)
        err = torch.empty(B, dtype=torch.float64, device=dev)
        K.gemm(L, R, D=res, epi=K.EPI_WERR, w=wts.err, err_out=err)
        return err

    def _solve_normal(self, M64):
        """Whitening of the r x r SPD normal matrix; Wt Wt^T = M^{-1}."""
        Wt32, _, info = K.spd_whiten(M64)
        return Wt32, info

    def _lplr(self, st, Y, res, L0, R0, wts: _Weights):
        """Quantised-factor LPLR loop, alg.py:144-195 (data-aware lstsq in normal-equation form
        with fp64 Grams; quantise L^T and R as whole matrices, alg.py:171-180)."""
        p = self.p
        B, m, n = st.B, st.m, st.n
        r = R0.shape[1]
        dev = res.device
        aware = p.activation_aware_LR
        R = R0
        best_err = torch.full((B,), float("inf"), dtype=torch.float64, device=dev)
        best = dict(L=torch.zeros((B, m, r), device=dev), R=torch.zeros((B, r, n), device=dev),
                    Lc=torch.zeros((B, m * r), dtype=K.code_dtype(p.L_bits), device=dev),
                    Rc=torch.zeros((B, r * n), dtype=K.code_dtype(p.R_bits), device=dev),
                    Ls=torch.zeros(B, device=dev), Rs=torch.zeros(B, device=dev))
        Ysrc = Y if aware else res
        tmp_mr = torch.empty((B, m, r), dtype=torch.float32, device=dev)
        L = torch.empty((B, m, r), dtype=torch.float32, device=dev)
        tmp_rn = torch.empty((B, r, n), dtype=torch.float32, device=dev)
        Rn = torch.empty((B, r, n), dtype=torch.float32, device=dev)
        err = torch.empty(B, dtype=torch.float64, device=dev)
        for _ in range(p.lplr_iters):
            # --- L = lstsq((R H_sqrt)^T, (res H_sqrt)^T)^T = (Y Rw^T)(Rw Rw^T)^{-1}   (alg.py:162-169)
            Rw = K.scale_rc(R, colscale=wts.ycol) if (aware and wts.ycol is not None) else R
            Bm = K.gemm(Ysrc, Rw, tb=True, C=tmp_mr)            # m x r
            Mr = K.gram_f64(Rw, Rw, ta=True, tb=True)          # r x r
            Wr, info = self._solve_normal(Mr)
            T1 = K.gemm(Bm, Wr, C=torch.empty_like(tmp_mr))     # (Y Rw^T) Wr
            K.gemm(T1, Wr, tb=True, C=L)                       # ... Wr^T
            # --- quantise L^T as one block (alg.py:171-172); codes kept in L layout
            qL = K.quantize_uniform(L.view(B, m * r), m * r, p.L_bits, codes=True, deq=True)
            L = qL["deq"].view(B, m, r)
            # --- R = lstsq(L, res) = (L^T L)^{-1} L^T res   (alg.py:175-177, unweighted)
            Ml = K.gram_f64(L, L)                              # r x r
            Wl, info2 = self._solve_normal(Ml)
            Ct = K.gemm(L, res, ta=True, C=tmp_rn)             # r x n
            T2 = K.gemm(Wl, Ct, ta=True, C=torch.empty_like(tmp_rn))
            K.gemm(Wl, T2, C=Rn)
            qR = K.quantize_uniform(Rn.view(B, r * n), r * n, p.R_bits, codes=True, deq=True)
            R = qR["deq"].view(B, r, n)
            # --- error ||(res - L R) H_sqrt||_F  (alg.py:182)
            if aware:
                Rw2 = K.scale_rc(R, colscale=wts.ycol) if wts.ycol is not None else R
                K.gemm(L, Rw2, D=Y, epi=K.EPI_WERR, err_out=err)
            else:
                K.gemm(L, R, D=res, epi=K.EPI_WERR, w=wts.lplr, err_out=err)
            e32 = torch.sqrt(err).float().double()  # torch.linalg.matrix_norm in fp32
            better = e32 < best_err
            yield
            better = better.tolist()
            sel = [b for b in range(B) if better[b]]
            for b in sel:
                best["L"][b].copy_(L[b])
                best["R"][b].copy_(R[b])
                best["Lc"][b].copy_(qL["codes"][b].view(m, r).t().reshape(-1))  # L^T order
                best["Rc"][b].copy_(qR["codes"][b])
                best["Ls"][b] = qL["scale"][b, 0]
                best["Rs"][b] = qR["scale"][b, 0]
                best_err[b] = e32[b]
        st.L_idxs, st.R_idxs = best["Lc"], best["Rc"]
        st.L_scale, st.R_scale = best["Ls"], best["Rs"]
        return best["L"], best["R"]

    # ------------------------------------------------------------------ driver
    def run(self, W: torch.Tensor, h: torch.Tensor | None = None, scale_W: bool = True,
            use_tqdm: bool = False):
        """W (B, m, n) fp16/fp32 on a HIP device; h: (n,) diagonal of H or None.
        Returns a list of per-matrix result dicts (see api.py for the dataclass view)."""
        return run_to_end(self.run_iter(W, h, scale_W, use_tqdm))

    def run_iter(self, W: torch.Tensor, h: torch.Tensor | None = None, scale_W: bool = True,
                 use_tqdm: bool = False):
        """Generator form of run(): yields before each host synchronisation, so several
        engines can be interleaved on their own streams (overlap.run_interleaved)."""
        p = self.p
        if W.dim() == 2:
            W = W.unsqueeze(0)
        B, m, n = W.shape
        dev = W.device
        if W.dtype not in (torch.float16, torch.float32):
            W = W.float()
        if n % 4:
            raise NotImplementedError("caldera-mi355x: W.shape[1] must be a multiple of 4")
        gs, Ws = K.rms_scale(W, scale_W)
        wts = _Weights(h, n, p, dev)
        self._wmax = K.absmax(Ws)  # bound for the split scale of the LR-step residual
        self._yh = self._yl = self._ys = None
        den = K.weighted_sqsum(Ws, wts.err, n)
        r = p.rank
        st = BatchState(B, m, n, r, p, dev)
        best = BatchState(B, m, n, r, p, dev)
        best.flag_Q = [False] * B
        best.flag_LR = [False] * B
        errors = {mtx: [[] for _ in range(B)] for mtx in p.update_order}
        min_err = [math.inf] * B
        updated = {mtx: False for mtx in p.update_order}
        work = torch.empty((B, m, n), dtype=torch.float32, device=dev)  # Y / Q-residual buffer
        need_res = any(x == "LR" for x in p.update_order)
        res = torch.empty((B, m, n), dtype=torch.float32, device=dev) if need_res else None
        to_iter = range(p.iters)
        if use_tqdm:
            from tqdm import tqdm
            to_iter = tqdm(to_iter)
        for _ in to_iter:
            for mtx in p.update_order:
                num = None
                if mtx == "LR" and p.compute_low_rank_factors:
                    num = yield from self._lr_update(st, Ws, work, res, wts, den)
                elif mtx == "Q" and p.compute_quantized_component:
                    num = self._q_update(st, Ws, work, wts, den)
                updated[mtx] = True
                if num is None:  # no update: error of the unchanged state
                    num = self._state_error(st, Ws, work, wts)
                e = torch.sqrt((num.float() / den.float()))  # fp32 ratio + sqrt (alg.py:297-301)
                yield
                e = e.tolist()
                for b in range(B):
                    errors[mtx][b].append(float(e[b]))
                if all(updated.values()):
                    sel = [b for b in range(B) if e[b] < min_err[b]]
                    for b in sel:
                        min_err[b] = e[b]
                    if sel:
                        st.snapshot_into(best, sel)
        if self.solver is not None:
            self.solver.release()  # G, halves, blocks: ~300 MB per 4096^2 matrix
        self._yh = self._yl = None
        return self._finalize(best, st, W, Ws, gs, errors, wts)

    def _state_error(self, st, Ws, work, wts):
        B, m, n = st.B, st.m, st.n
        K.build_residual(Ws, st.Qc if st.has_Q else None, st.Qs if st.has_Q else None, self.p.Q_bits,
                         None, res=work)
        err = torch.empty(B, dtype=torch.float64, device=Ws.device)
        K.gemm(st.L, st.R, D=work, epi=K.EPI_WERR, w=wts.err, err_out=err)
        return err

    def _finalize(self, best, st, W, Ws, gs, errors, wts):
        p = self.p
        B, m, n = best.B, best.m, best.n
        dev = W.device
        out = []
        gsl = gs.tolist()
        qs = best.Qs.tolist()
        # compact (storage / gather) form: packed codes as kept by the engine
        self.last_packed = [dict(codes=best.Qc[b].clone(), Q_scale=qs[b], L=best.L[b].clone(),
                                 R=best.R[b].clone(), global_scale=gsl[b],
                                 errors={k: v[b] for k, v in errors.items()})
                            for b in range(B)]
        for b in range(B):
            d = {}
            if best.flag_Q[b]:
                qc = best.Qc[b:b + 1]
                codes = K.unpack_codes(qc, m * n, p.Q_bits) if best.q_packed else qc.clone()
                # dequantize_block (quantization.py:103-105) on the reference int codes
                d["Q"] = K.dequantize_uniform(codes, best.Qs[b:b + 1], p.Q_bits).view(m, n)
                d["Q_idxs"] = codes.view(1, m * n)
                d["Q_scale"] = best.Qs[b].view(1, 1).clone()
            else:
                d["Q"] = torch.zeros((m, n), dtype=torch.float32, device=dev)
                d["Q_idxs"] = None
                d["Q_scale"] = 1
            d["L"] = best.L[b].clone()
            d["R"] = best.R[b].clone()
            if best.L_idxs is not None and best.flag_LR[b]:
                d["L_idxs"] = best.L_idxs[b].view(1, -1).clone()
                d["R_idxs"] = best.R_idxs[b].view(1, -1).clone()
                d["L_scale"] = best.L_scale[b].view(1, 1).clone()
                d["R_scale"] = best.R_scale[b].view(1, 1).clone()
            else:
                d["L_idxs"] = d["R_idxs"] = None
                d["L_scale"] = d["R_scale"] = 1
            d["W"] = Ws[b]
            d["global_scale"] = gsl[b] if True else 1
            d["errors"] = {k: v[b] for k, v in errors.items()}
            out.append(d)
        return out
