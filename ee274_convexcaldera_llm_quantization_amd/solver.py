"""Batched rank-r truncated SVD on MI355X: Chebyshev-filtered subspace iteration (ChFSI).

Replaces the full LAPACK SVD of RCR/src/caldera/decomposition/alg.py:217
(`torch.linalg.svd(Y, full_matrices=False)`, of which LR_init keeps only the top `rank`
triplets, :219-225).  Exact to tolerance, not randomized: the near-degenerate spectrum at
the rank boundary of CALDERA residuals (sigma_128/sigma_129 - 1 ~ 3e-4)
rules out fixed-iteration sketches, so iteration runs until every wanted Ritz pair has
relative residual <= tol.

Algorithm, for a batch of B same-shape matrices Y (m x n) in lockstep:
  k = min(m, n); G = Y Y^T (m <= n) or Y^T Y (fp32 MFMA GEMM)           [1 big GEMM]
  X = random k x p (p = block, ~2r) or the previous call's Ritz block (warm start)
  X <- CholQR2(X); Rayleigh-Ritz
  repeat:   X <- T_d(filter damping [0, c]) X   (scaled 3-term recurrence, d GEMMs G X)
            X <- CholQR2(X)                       (fp64 Gram + symmetric elimination)
            Z = G X; T = X^T Z (fp64); T = V diag(theta) V^T (Jacobi); X <- X V, Z <- Z V
            c <- theta_p (cut);  stop when max_{i<r} ||Z_i - theta_i X_i|| / theta_0 <= tol
The filter products G X run as split-fp16 MFMA products (cq_gemm_x3: each fp32 operand
carried as two fp16 halves, three v_mfma_f32_32x32x16_f16 per product, fp32 accumulation;
measured error at or below the fp32 MFMA GEMM's) on X^T so both operands are K-contiguous;
should a filter iterate ever overflow the fp16 range, the outer iteration is redone with
the fp32 filter.  The Rayleigh-Ritz product and everything that decides convergence run on
cq_gemm_f32 (v_mfma_f32_32x32x2_f32); the p x p problems run one workgroup per matrix
(cq_gram_f64 / cq_spd_whiten / cq_jacobi_eigh).  The per-matrix
filter coefficients are passed as per-batch vectors, so the whole batch stays on device;
the only host synchronisation is the convergence test once per outer iteration.
"""
from __future__ import annotations

import math
import warnings

import numpy as np
import torch

from . import _lib as K
from . import scratch
from .overlap import run_to_end



# the filter's last step and the Rayleigh-Ritz product write X's k x p layout from their epilogue
# (gemm_x3 Ct) instead of a transpose_split pass; False: the transpose passes (A/B, bench.py
# --no-transposed-output)
TRANSPOSED_OUT = True

class _EventProbe:
    """HIP-event timing of the dominant kernel (the G X filter GEMM) on the stream it is
    launched on; used by bench.py inside its timed region (roofline.achieved).  The event
    pairs are created up front (hipEventCreate per launch costs more than the launch) and
    the first `max_pairs` filter launches of the timed region are sampled.

    Launches of several kernels may be probed (the split-fp16 and the single-product filter
    steps): summary() reports the kernel with the most probed time at the top level, per-kernel
    groups under "kernels", and "aggregate" -- the algorithmic bytes of every probed launch on
    every stream divided by the union of their [start, end] windows (a reference event recorded
    at enable() puts all streams on one clock): the chip-level rate of interleaved parts, where
    a per-launch rate only says how fast one launch ran while sharing the chip."""

    def __init__(self):
        self.on = False
        self.pool = []
        self.used = 0
        self.meta = []
        self.ref = None

    def enable(self, on: bool, max_pairs: int = 96):
        self.on = on
        if on:
            self.pool = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                         for _ in range(max_pairs)]
            self.used = 0
            self.meta = []
            self.ref = torch.cuda.Event(enable_timing=True)
            self.ref.record()

    def start(self, flops, nbytes=0.0, kernel=""):
        if not self.on or self.used >= len(self.pool):
            return None
        ev = self.pool[self.used]
        self.used += 1
        ev[0].record()
        self.meta.append((flops, nbytes, kernel))
        return ev

    def stop(self, ev):
        if ev is not None:
            ev[1].record()

    def summary(self):
        if not self.used:
            return {"count": 0}
        torch.cuda.synchronize()
        pairs = self.pool[: self.used]
        ms = [a.elapsed_time(b) for a, b in pairs]
        groups = {}
        for t, (fl, nb, kn) in zip(ms, self.meta):
            g = groups.setdefault(kn, {"count": 0, "ms": 0.0, "flops_per_launch": fl, "bytes_per_launch": nb})
            g["count"] += 1
            g["ms"] += t
        for g in groups.values():
            g["avg_ms"] = g["ms"] / g["count"]
        top = max(groups, key=lambda k: groups[k]["ms"])
        g = groups[top]
        out = {"count": g["count"], "avg_ms": g["avg_ms"], "flops_per_launch": g["flops_per_launch"],
               "bytes_per_launch": g["bytes_per_launch"], "kernel": top, "kernels": groups}
        if self.ref is not None:
            iv = sorted((self.ref.elapsed_time(a), self.ref.elapsed_time(b)) for a, b in pairs)
            union, cur_s, cur_e = 0.0, None, None
            for s0, e0 in iv:
                if cur_e is None or s0 > cur_e:
                    if cur_e is not None:
                        union += cur_e - cur_s
                    cur_s, cur_e = s0, e0
                else:
                    cur_e = max(cur_e, e0)
            union += cur_e - cur_s
            out["aggregate"] = {"launches": len(iv), "bytes": float(sum(nb for _, nb, _ in self.meta)),
                                "busy_ms": union, "window_ms": iv[-1][1] - iv[0][0] if iv else 0.0}
        return out


EVENT_PROBE = _EventProbe()


class _GroupProbe:
    """HIP-event timing of the fused Q-update launches (the quantise kernel: both passes of
    cq_q_update_x3 on its stream), grouped by kind (first Q step without L R, and with the
    rank-r recompute); used by bench.py for the quantise kernel's roofline."""

    def __init__(self):
        self.on = False
        self.pool = []
        self.meta = []

    def enable(self, on: bool, max_pairs: int = 64):
        self.on = on
        if on:
            self.pool = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                         for _ in range(max_pairs)]
            self.meta = []

    def start(self, kind, flops, nbytes):
        if not self.on or len(self.meta) >= len(self.pool):
            return None
        ev = self.pool[len(self.meta)]
        self.meta.append((kind, flops, nbytes))
        return ev  # recorded by the caller around the kernel launches (_lib.q_update_x3 events=)

    def summary(self):
        if not self.meta:
            return {}
        torch.cuda.synchronize()
        out = {}
        for (a, b), (kind, fl, nb) in zip(self.pool, self.meta):
            g = out.setdefault(kind, {"count": 0, "ms": 0.0, "flops_per_launch": fl, "bytes_per_launch": nb})
            g["count"] += 1
            g["ms"] += a.elapsed_time(b)
        for g in out.values():
            g["avg_ms"] = g.pop("ms") / g["count"]
        return out


QUANT_PROBE = _GroupProbe()
LPLR_PROBE = _GroupProbe()  # the LPLR loop's m x n x r GEMMs (alg.py:162-177), bench roofline_lplr
GRAM_PROBE = _GroupProbe()  # the split-fp16 Gram G = Y Y^T (or Y^T Y) of every solve, bench roofline_gram


X3_SCALE = 2.0 ** 6  # power-of-two scale of the filter iterates' fp16 halves (entries <= ~1)
FILTER_MAX_AMP = 2.0e5  # bound on T_d(t0): config 2's degree-12 steps (T_12(1.6) ~ 1.4e5) stay uncapped
MAX_OUTER = 40  # outer iterations per solve (the schedule's last degree repeats until converged)


JACOBI_MAX_SWEEPS = 30
# block Jacobi (p > 192) runs in caller-driven stages (cq_jacobi_eigh_staged, each stage
# stream-ordered): a first batch of sweeps sized from the previous call, then BJ_STEP more at a
# time while the device count of unconverged matrices (one int read back) is nonzero
BJ_FIRST, BJ_MIN_FIRST, BJ_STEP = 6, 2, 2
BJ_SMALL_SUBPROBLEMS = 256  # batches with at most this many 64 x 64 block-Jacobi subproblems take it at every p
STALL_RATIO = 0.98
LATENCY_BATCH = 8  # batches up to this size (one caldera() call) take the latency-first variants
# B <= this (an outer iteration latency-bound: its eigensolve and read-back cost more than filter
# products): a warm solve's cheap iteration is segmented too (its bounds are the previous call's
# converged ones), and every segment runs the whole capped degree (above: the last one only the
# rest of the requested degree).  tools/tune_main.py: main.py's layer set (batches of 7-14) 174 ->
# 203 matrices/s with both, 189 with remainder segments; config 5 (B = 256) 93.5 whole, 95.1
# remainder, 96.3 unsegmented; config 3 (B = 192) 219 with its warm cheap iteration segmented, 243 without
SEGMENTS_SMALL_BATCH = 32
SEGMENTS_MAX = 4  # filter segments per outer iteration at most (segment_capped; tools/tune_main.py: 1 -> 113, 3 -> 198, 4 -> 200, 6 -> 145, 16 -> 104 matrices/s on main.py's layer set)
VALUES_LANCZOS = 40  # Lanczos steps for the cheap iterations' filter bounds (0: values-only Jacobi)


class SolverStats:
    def __init__(self):
        self.outer = 0
        self.matvecs = 0
        self.x3_fallbacks = 0
        self.jacobi_unconverged = 0  # Rayleigh-Ritz eigensolves that used all JACOBI_MAX_SWEEPS
        self.bj_readbacks = 0        # block-Jacobi stage read-backs (one int each)
        self.stalls = 0              # matrices whose solve ended at the products' precision floor
        self.refines = 0             # refinement outer iterations run after convergence
        self.segments = 0            # extra filter segments run (segment_capped), over the batch
        self.calls = 0
        self.max_resid = 0.0
        self.resid_hist = []
        self.history = []  # per solve call: (cold, degrees used, residual after each)

    def as_dict(self):
        return dict(outer=self.outer, matvecs=self.matvecs, calls=self.calls,
                    jacobi_unconverged=self.jacobi_unconverged, bj_readbacks=self.bj_readbacks, stalls=self.stalls,
                    max_resid=self.max_resid, x3_fallbacks=self.x3_fallbacks, refines=self.refines,
                    segments=self.segments)


class RankRSolver:
    """Top-r eigenpairs of the Gram of a batch of matrices, warm-started across calls."""

    def __init__(self, B: int, m: int, n: int, r: int, device, *, p: int | None = None,
                 tol: float = 1e-5, deg_cold=(6, 12, 12, 12, 12, 12, 12), deg_warm=(10, 7, 6, 6, 6, 6),
                 seed: int = 0x5EED, jacobi_tol: float = 1e-7, filter_precision: str = "f16x3",
                 cheap_cold: int = 3, cheap_warm: int = 1, skip_warm_cheap_rr: bool | None = None,
                 jacobi_tol_values: float = 1e-2, criterion: str = "product",
                 jacobi_values_sweeps: int = 30, values_lanczos: int | None = None, ns_second: bool | None = None,
                 segment_capped: bool = True, cheap_one_pass: bool = True):
        self.B, self.m, self.n = B, m, n
        self.k = min(m, n)
        self.left = m <= n  # G = Y Y^T -> eigenvectors are left singular vectors
        self.r = min(r, self.k)
        if p is None:
            # block size ~1.4 r rounded up to a multiple of 32: at r = 128 this is p = 192,
            # the largest block whose fp64 Rayleigh-Ritz matrix fits the 160 KB LDS of one CU
            # (cq_jacobi_eigh register/LDS path) and one 192-wide GEMM tile; same GEMM cost to
            # tolerance as p = 2r (solver tuning).
            p = max(int(1.4 * self.r) + 4, self.r + 16)
            p = (p + 31) // 32 * 32
        p = p + (p & 1)
        self.direct = p >= self.k or self.k <= 256  # small problem: Jacobi on the full Gram
        self.p = self.k if self.direct else p
        self.tol = tol
        if criterion not in ("product", "theta0"):
            raise ValueError(f"criterion must be 'product' or 'theta0', got {criterion!r}")
        self.criterion = criterion
        self.deg_cold, self.deg_warm = tuple(deg_cold), tuple(deg_warm)
        self.device = device
        self.seed = seed
        # Jacobi off-norm tolerances (relative to the diagonal), tuned at config 2 B = 256
        # (profiles/r01i_tune_jacobi_tol*.log): the full Rayleigh-Ritz at 1e-7 (1e-5 stalls the
        # Ritz residuals, 1e-6 leaves a thin margin), the values-only one at 1e-2 (eigenvalue
        # errors ~1e-4 relative are ample for filter bounds): 243 -> 259 matrices/s
        self.jacobi_tol = jacobi_tol
        self.jacobi_tol_values = jacobi_tol_values
        # sweep cap of the values-only eigensolves (cheap iterations: the Ritz values only set
        # the next filter's bounds)
        self.jacobi_values_sweeps = int(jacobi_values_sweeps)
        # the cheap iterations' filter bounds (the two ends of the Ritz spectrum) from this many
        # Lanczos steps on T (cq_extreme_eigs, one launch, no read-back) instead of a values-only
        # eigensolve; 0: the eigensolve (p > 512 always)
        self.values_lanczos = int(VALUES_LANCZOS if values_lanczos is None else values_lanczos)
        self.refine = ()   # extra full outer iterations after convergence (per call; engine.py)
        self.X = None      # warm-start Ritz block (B, k, p)
        self.theta = None  # its Ritz values (B, p) fp64: filter bounds for the next call
        self.stats = SolverStats()
        self.valid_k = self.k  # rows >= valid_k of the eigenproblem are zero padding (engine.py)
        # Rayleigh-Ritz sweep budget: fixed for the one-workgroup Jacobi (its sweep loop runs
        # inside one kernel), adaptive for the block Jacobi (each sweep is a set of launches)
        # block Jacobi over many workgroups where one CU cannot hold the problem (p > 192), and
        # for batches whose 64 x 64 subproblems (p / 64 per matrix) do not outnumber the CUs,
        # where the one-workgroup-per-matrix kernel (~4 ms per 192 x 192 eigensolve on one CU)
        # would leave most of the chip idle: one caldera() call, config 4's batches of 64, the
        # 8-GPU model run's batches of 16
        nblk = -(-self.p // 32)
        self.block_jacobi = self.p > 192 or B * ((nblk + (nblk & 1)) // 2) <= BJ_SMALL_SUBPROBLEMS
        self.bj_first = BJ_FIRST  # block Jacobi: sweeps launched before the first read-back
        self._bufs = None
        self._G = None
        self._yh = self._yl = None
        self._halves_of = None   # the block whose X^T halves the last CholQR product wrote
        if filter_precision not in ("f16x3", "f32"):
            raise ValueError(f"filter_precision must be 'f16x3' or 'f32', got {filter_precision!r}")
        # split-fp16 filter needs K (= k) a multiple of 32 and 16-byte aligned rows
        self.x3 = filter_precision == "f16x3" and not self.direct and self.k % 32 == 0
        self._g_blocked = True  # K-blocked G halves: each K step of a tile is one contiguous run
        self._x3f = True        # split-fp16 filter for the current outer iteration
        # the first `cheap_cold` outer iterations of a cold solve and the first `cheap_warm`
        # of a warm one filter with one fp16 product (hi x hi, ~2^-11 relative, half the G
        # bytes, a third of the MFMAs): their residual targets (1e-1 ... 4e-4) sit above the
        # ~1.5e-4 floor of that filter, and the following split-fp16 steps damp its error like
        # any other unwanted component; the Rayleigh-Ritz products stay split-fp16, so the
        # convergence test is exact (tools/tune_solver.py, config 2: (10, 7) warm degrees with
        # one cheap outer iteration converge in two outer iterations per call, 6% faster)
        self.cheap_cold = int(cheap_cold)
        self.cheap_warm = int(cheap_warm)
        # a warm solve's cheap outer iterations skip Rayleigh-Ritz: their filter bounds are the
        # previous call's converged Ritz values (the residual moved by <1%), their convergence
        # test could never pass (single-product floor), and the subspace does not depend on the
        # basis, so the G X product, Jacobi and rotations of that step are dropped.  Off by
        # default: measured at config 2 (B = 256) the stale bounds cost later warm calls a third
        # outer iteration (131 vs 121 G products per step, 243.6 vs 244.1 matrices/s)
        # (None: on for latency batches, below)
        self.latency = B <= LATENCY_BATCH
        self.skip_warm_cheap_rr = self.latency if skip_warm_cheap_rr is None else bool(skip_warm_cheap_rr)
        # CholQR2's second pass (and the final re-orthonormalisation) as Newton-Schulz steps
        # X <- X (3 I - X^T X) / 2 (fp64 Gram, one fp32 product each) instead of a whitening: the
        # block after one CholQR pass is orthonormal to ~eps32 cond(X) <= ~1e-2, two steps take that
        # to the fp32 floor (error^2 per step) -- the same subspace without the whitening's chain of
        # 32-pivot panels on one CU (0.2 ms at p = 192): for latency batches, where that chain is
        # the critical path (one caldera() call), not for large ones (there the whitening costs
        # less than the two Grams and products that replace it)
        self.ns_second = self.latency if ns_second is None else bool(ns_second)
        # a requested filter degree the amplification cap cuts runs as several segments with a
        # CholQR pass between them, inside one outer iteration (round 6; False: the cut degree
        # and more outer iterations, as through round 5)
        self.segment_capped = bool(segment_capped)
        # cheap (values-only) outer iterations: one CholQR pass instead of two -- the block only
        # feeds the next filter and the two ends of a Lanczos spectrum, for which orthonormality
        # to eps32 * cond(filtered block) is plenty (fp64 Gram).  Config 2: +1.7-2.0 % (320.9 ->
        # 326.4, 323.3 -> 329.8 matrices/s), pinned / exact-LR / held-out parity at B = 256
        # unchanged at 11/16, 15/16, 27/32 (tools/ab_solver_kw.py, profiles/r06ba_*, r06bb_*);
        # at B = 64 (test_gpu_holdout.py) the held-out classes move from 26 / 30 / 2 misses to
        # 28 / 28 / 2 misses (bit-exact vs the reference / vs exact LR / in no class:
        # profiles/r06bi_holdout.log, r06bc_gpu_suite_onepass.log) -- two more seeds on the
        # reference's own codes
        self.cheap_one_pass = bool(cheap_one_pass)

    # ------------------------------------------------------------------ buffers
    def _alloc(self, dev):
        B, k, p = self.B, self.k, self.p
        if self._bufs is None:
            # 5 buffers: an outer iteration keeps its input alive until its overflow check
            # large work buffers: cached scratch (scratch.py), reused by later solves
            f32, f16 = torch.float32, torch.float16
            self._bufs = [scratch.get(f"solver.blk{i}", (B, k, p), f32, dev) for i in range(5)]
            # the warm start of an earlier solve may be one of the cached blocks (the final
            # swap below): it must not also serve as scratch
            self._bufs = [torch.empty_like(t) if t is self.X else t for t in self._bufs]
            # fp32 G only for the fp32 products (the split-fp16 path keeps G as its halves and
            # allocates it on an fp16 overflow fallback)
            self._G = None if self.x3 else torch.empty((B, k, k), dtype=f32, device=dev)
            if self.x3:
                self._Gh = scratch.get("solver.Gh", (B, k, k), f16, dev)
                self._Gl = scratch.get("solver.Gl", (B, k, k), f16, dev)
                self._gscale = torch.empty(B, dtype=f32, device=dev)
                self._ginv = torch.empty(B, dtype=f32, device=dev)
                self._xt = [scratch.get(f"solver.xt{i}", (B, p, k), f32, dev) for i in range(2)]
                self._xh = [scratch.get(f"solver.xh{i}", (B, p, k), f16, dev) for i in range(2)]
                self._xl = [scratch.get(f"solver.xl{i}", (B, p, k), f16, dev) for i in range(2)]
                self._ovf = torch.zeros(B, dtype=torch.int32, device=dev)
            self._active = torch.ones(B, dtype=torch.int32, device=dev)

    def _free(self, *used):
        for b in self._bufs:
            if all(b is not u for u in used):
                return b
        raise RuntimeError("solver buffer pool exhausted")

    def release(self):
        """Drop the large per-call work buffers (G and its halves, Y halves, blocks); the warm
        start (X, theta) and the statistics stay."""
        self._bufs = None
        self._G = None
        self._yh = self._yl = None
        self._halves_of = None
        for name in ("_Gh", "_Gl", "_xt", "_xh", "_xl"):
            if hasattr(self, name):
                setattr(self, name, None)

    def split_block_t(self, X):
        """K-blocked split-fp16 halves of X^T (B, p, k) at X3_SCALE, in the solver's iterate
        buffers (valid until the next solve)."""
        self._halves_of = None
        K.transpose_split(X, hi=self._xh[0], lo=self._xl[0], scale=X3_SCALE, blocked=True)
        return self._xh[0], self._xl[0]

    def _fill_G(self, Y):
        """fp32 G = Y Y^T (m <= n) or Y^T Y: from the Gram operand's split halves when the
        caller provided them (Y itself may not exist in fp32), else on the fp32 MFMA GEMM."""
        if self._gram_fill is not None:  # caller-formed G (sgram.py): its fp32 form
            self._gram_fill(self._Gh, self._Gl, self._gscale, self._ginv, G32=self._G)
            return
        if self._y_halves is not None:
            yh, yl, ys = self._y_halves
            K.gemm_x3(yh, yl, yh, yl, 1.0 / (ys * ys), self._G, tri=True, a_blocked=True, b_blocked=True)
            self._G.copy_(torch.triu(self._G) + torch.triu(self._G, 1).transpose(1, 2))
            return
        if self.left:
            K.gemm(Y, Y, tb=True, C=self._G, syrk=True)
        else:
            K.gemm(Y, Y, ta=True, C=self._G, syrk=True)

    # ------------------------------------------------------------------ steps
    def _cholqr(self, X, *keep, halves=False):
        """halves: the Rayleigh-Ritz step follows -- the product also writes its operand, the
        K-blocked split of out^T, into the iterate halves (cq_gemm_triu_split: one pass instead
        of the product and a transpose-split pass, the same bits)."""
        out = self._free(X, *keep)
        M = K.gram_f64(X, X)
        Wt32, _, info = K.spd_whiten(M)
        self._halves_of = None
        if halves and self.x3 and self._x3f and K.triu_split_ok(self.k, self.p):
            K.gemm_triu_split(X, Wt32, out, self._xh[0], self._xl[0], X3_SCALE)
            self._halves_of = out
        else:
            K.gemm(X, Wt32, C=out, b_triu=True)  # Wt upper triangular (zeros stored)
        return out, info

    def _ns(self, X, *keep, steps=2):
        """Newton-Schulz re-orthonormalisation of a nearly orthonormal block (see ns_second)."""
        self._halves_of = None
        eye = None
        for _ in range(steps):
            out = self._free(X, *keep)
            M = K.gram_f64(X, X)
            if eye is None:
                eye = torch.eye(self.p, dtype=torch.float64, device=X.device)
            N = (1.5 * eye - 0.5 * M).float()
            K.gemm(X, N, C=out)
            X = out
        return X, None

    def _orth2(self, X, *keep, halves=False):
        """CholQR2's second pass: CholQR, or Newton-Schulz steps for latency batches."""
        if self.ns_second:
            return self._ns(X, *keep)
        return self._cholqr(X, *keep, halves=halves)

    def _rr(self, X, *keep, single=False, values_only=False):
        """Rayleigh-Ritz on the block X (generator: yields before the block Jacobi's read-backs).  single: Z = G X with one fp16 product (cheap outer
        iterations: the Ritz values only set the next filter's bounds, and the residuals it
        reports sit at the ~1.5e-4 floor of that product, far above the tolerance, so no
        matrix can be declared converged on them).  values_only: Ritz values only, X returned
        unrotated and Z = None — the next filter sees the same subspace either way, so a
        cheap iteration needs no eigenvectors, rotations or residuals."""
        G = self._G
        Z = self._free(X, *keep)
        if self.x3:  # Z = G X on split-fp16 products (X orthonormal: no overflow possible)
            if self._halves_of is not X:   # (else the CholQR product wrote them)
                K.transpose_split(X, hi=self._xh[0], lo=self._xl[0], scale=X3_SCALE, blocked=True)
            self._halves_of = None
            K.gemm_x3(self._xh[0], self._xl[0], self._Gh, self._Gl, self._ginv, self._xt[0], b_blocked=self._g_blocked,
                      a_blocked=True, single=single and self._x3f, Ct=Z if TRANSPOSED_OUT else None)
            if not TRANSPOSED_OUT:
                K.transpose_split(self._xt[0], out=Z)
        else:
            K.gemm(G, X, ta=True, C=Z)  # Z = G X  (G symmetric: G^T's layout stages faster)
        self.stats.matvecs += 1
        T = K.gram_f64(X, Z)
        if values_only and self.values_lanczos > 0 and self.p <= 512:
            # only theta_0 and theta_{p-1} are read (filter bounds): Lanczos ends, the rest NaN
            ends = K.extreme_eigs(T, self.values_lanczos)
            theta = torch.full((self.B, self.p), math.nan, dtype=torch.float64, device=T.device)
            theta[:, 0] = ends[:, 0]
            theta[:, self.p - 1] = ends[:, 1]
            self._last_sw = torch.zeros(self.B, dtype=torch.int32, device=T.device)
            return theta, X, None
        if values_only:
            # eigenvalue errors are O(off-norm^2): a loose off-norm tolerance still gives the
            # filter bounds to ~1e-8 relative, in fewer sweeps
            theta, _, _, sw = yield from self._eigh(T, self.jacobi_tol_values, want_vectors=False,
                                                    max_sweeps=self.jacobi_values_sweeps)
            self._last_sw = sw
            return theta, X, None
        theta, V32, _, sw = yield from self._eigh(T, self.jacobi_tol)
        self._last_sw = sw
        Xo = self._free(X, Z, *keep)
        K.gemm(X, V32, C=Xo)
        Zo = self._free(X, Z, Xo, *keep)
        K.gemm(Z, V32, C=Zo)
        return theta, Xo, Zo

    def _eigh(self, T, tol, want_vectors=True, max_sweeps=None):
        """Rayleigh-Ritz eigensolve (descending).  p <= 192: one launch to convergence (A in
        one CU's LDS).  p > 192: block Jacobi in stages -- bj_first sweeps, then BJ_STEP at a
        time while matrices remain unconverged (one int read back per stage); bj_first follows
        what the last call needed, so a warm call usually reads back once.  Generator: yields
        before each read-back, so batches interleaved on other streams (overlap.py) keep
        issuing while this one waits."""
        if not self.block_jacobi:
            return K.jacobi_eigh(T, max_sweeps=max_sweeps or JACOBI_MAX_SWEEPS, tol=tol, want_vectors=want_vectors)
        bj = K.BlockJacobi(T, tol, want_vectors)
        first = min(self.bj_first, JACOBI_MAX_SWEEPS)
        bj.launch(first, begin=True)
        yield
        left = bj.pending_count()
        while left and bj.swept < JACOBI_MAX_SWEEPS:
            bj.launch(min(BJ_STEP, JACOBI_MAX_SWEEPS - bj.swept))
            yield
            left = bj.pending_count()
        self.bj_first = bj.swept if bj.swept > first else max(BJ_MIN_FIRST, first - 1)
        self.stats.bj_readbacks += 1 + (bj.swept - first + BJ_STEP - 1) // BJ_STEP
        return bj.finish()

    def _cheb_coeffs(self, ends, deg, dev, limit=None):
        """Coefficients of the scaled 3-term recurrence, from the host copy of the Ritz values
        ends = [(theta_0, theta_{p-1}) per matrix] (fp64, as read back at the convergence
        check).  Returns a (deg, 3, B) fp32 device tensor: step i computes
        X_{i+1} = a_i G X_i + b_i X_{i-1} + c_i X_i.  limit: optional per-matrix degree bound
        below the cap (a segment's remainder, _more_segments); the table then only sets
        self._eff_deg when limit is None."""
        ref = ends[:, 0]
        live = np.isfinite(ref) & (ref > 0)
        # G is positive semi-definite: a Ritz value below 0 (or a few ulps of theta_0 above it) is
        # the rounding of the products on a spectrum whose bottom is ~0 relative to its top -- a
        # widely spread one -- so the damped interval ends just above 0 (the degree cap then holds
        # the amplification); a flat block (theta_{p-1} ~ theta_0) damps [0, theta_0 / 2].  Either
        # way the recurrence stays scaled to 1 at theta_0: unscaled, G's top (1e7 on an
        # activation-weighted Y) overflows the iterates within a few steps.
        c = np.where(live, np.maximum(ends[:, 1], ref * 1e-6), 0.0)
        ok = live & (ref > c * (1 + 1e-6))
        c = np.where(live & ~ok, ref / 2.0, c)
        e = np.where(live, c / 2.0, 1.0)
        ctr = np.where(live, c / 2.0, 0.0)
        t0 = np.where(live, (ref - ctr) / e, 2.0)
        # per-matrix degree cap: the filter amplifies the top of the wanted band by up to
        # T_d(t0) against its bottom (~1); beyond ~1/eps of the products the wanted directions
        # near theta_r drown in the top ones and the block degenerates.  Widely spread spectra
        # (activation-weighted Y, theta_0/theta_r ~ 20 at config 3) thus get low degrees and more
        # outer iterations; near-flat ones (config 2, t0 ~ 1.6) keep the full schedule.
        cap = np.maximum(1, np.floor(np.arccosh(FILTER_MAX_AMP) / np.arccosh(np.maximum(t0, 1.0 + 1e-12))))
        if limit is None:
            self._eff_deg = np.minimum(cap, deg).astype(np.int64)   # per matrix (segment_capped)
        else:
            cap = np.minimum(cap, np.maximum(limit, 1))
        deg = int(min(deg, cap.max()))
        s = 1.0 / t0
        rows = [(s / e, np.zeros_like(s), -s * ctr / e)]
        for i in range(1, deg):
            sn = 1.0 / (2.0 * t0 - s)
            run = i < cap  # past its cap a matrix's iterate passes through: X_{i+1} = X_i
            rows.append((np.where(run, 2 * sn / e, 0.0), np.where(run, -sn * s, 0.0),
                         np.where(run, -2 * sn * ctr / e, 1.0)))
            s = np.where(run, sn, s)
        tab = torch.from_numpy(np.asarray(rows, dtype=np.float64).astype(np.float32))
        return tab.to(dev)

    def _more_segments(self, Xf, X, d, coef, single, ends):
        """The segments after the first of an outer iteration's filter (segment_capped): matrix
        b runs ceil(d / its capped degree) segments of its capped degree (the last one the
        remainder of d), each after a CholQR pass; a matrix whose segments are done sits out the
        rest (its block is restored from before the segment, and it passes through the filter),
        so its result does not depend on its batch-mates' spectra.  Returns the filtered block."""
        if not self.segment_capped:
            return Xf
        eff = np.maximum(self._eff_deg, 1)
        segs = np.minimum(SEGMENTS_MAX, -(-d // eff))
        dev = X.device
        for j in range(1, int(segs.max())):
            cont = segs > j
            self.stats.segments += 1
            # large batches: the last segment runs only the remainder of the requested degree
            # (config 5: d = 12 capped at 7-11 -- a whole capped-degree segment there costs more
            # than it gains); small ones keep whole segments (SEGMENTS_SMALL_BATCH)
            rem = eff if self.B <= SEGMENTS_SMALL_BATCH else np.where(cont, np.minimum(d - j * eff, eff), eff)
            cj = coef if (rem >= eff).all() else self._cheb_coeffs(ends, d, dev, limit=rem)
            Xs, _ = self._cholqr(Xf, X)
            saved = None
            if not cont.all():
                saved = self._active.clone()
                self._active.mul_(torch.from_numpy(cont.astype(np.int32)).to(dev))
            Xn = self._filter(Xs, cj, single=single, keep=(X, Xf))
            if saved is not None:
                self._active.copy_(saved)
                idx = torch.from_numpy(np.nonzero(~cont)[0]).to(dev)
                Xn.index_copy_(0, idx, Xf.index_select(0, idx))
            Xf = Xn
        return Xf

    def _filter(self, X, coef, single=False, keep=()):
        """X <- p_d(G) X, p_d = Chebyshev polynomial of degree d = len(coef) damping [0, c],
        c = theta_p, scaled to 1 at theta_0 (scaled 3-term recurrence).  Returns a buffer
        other than X's (X is left intact)."""
        if self.x3 and self._x3f:
            return self._filter_x3(X, coef, single, keep)
        G = self._G
        deg = coef.shape[0]
        X0 = self._free(X, *keep)  # the recurrence overwrites its buffers: keep the input intact
        X0.copy_(X)
        Y1 = self._free(X, X0, *keep)
        fl = 2.0 * self.k * self.k * self.p * self.B
        nb = float(self.B) * (4.0 * self.k * self.k + 16.0 * self.p * self.k)
        kn = "gemm_f32_kernel (fp32 G X, Chebyshev filter)"
        ev = EVENT_PROBE.start(fl, nb, kn)
        K.gemm(G, X0, ta=True, C=Y1, D=X0, alpha_v=coef[0, 0], gamma_v=coef[0, 2])
        EVENT_PROBE.stop(ev)
        self.stats.matvecs += 1
        prev, cur = X0, Y1
        for i in range(1, deg):
            # prev <- a G cur + b prev + c cur
            ev = EVENT_PROBE.start(fl, nb, kn)
            K.gemm(G, cur, ta=True, C=prev, D=cur, alpha_v=coef[i, 0], beta_v=coef[i, 1], gamma_v=coef[i, 2])
            EVENT_PROBE.stop(ev)
            self.stats.matvecs += 1
            prev, cur = cur, prev
        return cur

    def _filter_x3(self, X, coef, single=False, keep=()):
        """Same recurrence on X^T with split-fp16 products (cq_gemm_x3; single: one fp16
        product per step); X is left intact."""
        deg = coef.shape[0]
        xt, xh, xl = self._xt, self._xh, self._xl
        self._halves_of = None
        # iterates' halves are K-blocked (each 32-deep step of a tile is one contiguous run)
        K.transpose_split(X, out=xt[0], hi=xh[0], lo=xl[0], scale=X3_SCALE, blocked=True)
        fl = 2.0 * self.k * self.k * self.p * self.B
        # bytes a recurrence step moves: G halves (4 B/elem) + X^T halves + prev, cur in,
        # new out (fp32) + new halves out
        nb = float(self.B) * (4.0 * self.k * self.k + 20.0 * self.p * self.k)
        kn = "gemm_x3v_kernel<0> (split-fp16 G X, Chebyshev filter)"
        # the probe (bench.py's roofline) times both kinds of step, each with its own bytes: a
        # single-product step moves G's hi half and one iterate half per matrix, 2k^2 + 18pk
        if single:
            nb = float(self.B) * (2.0 * self.k * self.k + 18.0 * self.p * self.k)
            kn = "gemm_x3v_kernel<1> (single fp16 product G X, Chebyshev filter)"
        probe = EVENT_PROBE.start
        # the last step also writes its result in X's own k x p layout (Ct): no transpose pass
        out = self._free(X, *keep)
        ct = out if TRANSPOSED_OUT else None
        last = deg == 1
        ev = probe(fl, nb, kn)
        K.gemm_x3(xh[0], xl[0], self._Gh, self._Gl, self._ginv, xt[1], D=xt[0], alpha_v=coef[0, 0],
                  gamma_v=coef[0, 2], out_h=None if last else xh[1], out_l=None if last else xl[1],
                  out_scale=X3_SCALE, overflow=self._ovf, b_blocked=self._g_blocked, active=self._active,
                  a_blocked=True, o_blocked=True, single=single, Ct=ct if last else None)
        EVENT_PROBE.stop(ev)
        self.stats.matvecs += 1
        prev, cur = 0, 1
        for i in range(1, deg):
            last = i == deg - 1
            ev = probe(fl, nb, kn)
            K.gemm_x3(xh[cur], xl[cur], self._Gh, self._Gl, self._ginv, xt[prev], P=xt[prev], D=xt[cur],
                      alpha_v=coef[i, 0], beta_v=coef[i, 1], gamma_v=coef[i, 2],
                      out_h=None if last else xh[prev], out_l=None if last else xl[prev],
                      out_scale=X3_SCALE, overflow=self._ovf, b_blocked=self._g_blocked,
                      active=self._active, a_blocked=True, o_blocked=True, single=single,
                      Ct=ct if last else None)
            EVENT_PROBE.stop(ev)
            self.stats.matvecs += 1
            prev, cur = cur, prev
        if ct is None:
            K.transpose_split(xt[cur], out=out)
        return out

    # ------------------------------------------------------------------ main entry
    def solve(self, Y: torch.Tensor, warm: bool = True):
        """Y (B, m, n) fp32 -> (vecs (B, k, r), theta (B, r) fp64 eigenvalues of G, descending)."""
        return run_to_end(self.solve_iter(Y, warm))

    def solve_iter(self, Y: torch.Tensor, warm: bool = True, y_split=None, gram=None):
        """Generator form of solve(): yields before each host synchronisation (overlap.py).
        y_split: optional (hi, lo, scale, sq) K-blocked split-fp16 halves of the Gram operand (Y
        for m <= n, Y^T otherwise) and ||Y||_F^2 (fp64, or None) already produced by the caller
        (cq_residual_split).  gram: optional dict(fill, ysq) -- the caller forms G itself
        (sgram.py): fill(Gh, Gl, gscale, ginv, G32=None) writes G's K-blocked split halves
        (and fp32 G when asked), ysq = ||Y||_F^2; Y is then not read."""
        B, k, p = self.B, self.k, self.p
        dev = Y.device
        self.stats.calls += 1
        if self.direct:
            Gd = K.gram_f64(Y, Y, ta=True, tb=True) if self.left else K.gram_f64(Y, Y)
            theta, V32, _, _ = K.jacobi_eigh(Gd)
            return V32[:, :, : self.r], theta[:, : self.r]
        self._alloc(dev)
        self._g_upper_only = False
        self._Y = Y
        self._y_halves = None
        g_split = False
        self._gram_fill = None
        if gram is not None:
            assert self.x3, "solver: a caller-formed Gram needs the split-fp16 path"
            self._gram_fill = gram["fill"]
            self._ysq = gram["ysq"]
            # algorithmic bytes of the sparse Gram: W and its codes once (E slabs), P written
            # and read back, A's upper triangle, G's split halves written
            kk, nn = k, Y.shape[1] + Y.shape[2] - k
            gev = GRAM_PROBE.start("gram_sparse", 0.0, B * (2.25 * kk * nn + 14.0 * kk * kk))
            if gev is not None:
                gev[0].record()
            self._gram_fill(self._Gh, self._Gl, self._gscale, self._ginv)
            if gev is not None:
                gev[1].record()
            g_split = True
        elif self.x3 and (self.n if self.left else self.m) % 32 == 0:
            # G = Y Y^T (or Y^T Y) on split-fp16 products, Y scaled per matrix by a power of two;
            # the Gram writes G's K-blocked split halves itself (scale from ||Y||_F^2 >= max|G|)
            ysq = None
            if y_split is not None:
                yh, yl, ys, ysq = y_split
                # the Gram operand: Y (k x n) when m <= n, Y^T (k x m) otherwise
                assert yh.shape == (B, k, Y.shape[1] + Y.shape[2] - k), "solver: Gram operand halves misshaped"
            else:
                if self._yh is None:
                    yshape = (B, k, Y.shape[1] + Y.shape[2] - k)
                    self._yh = scratch.get("solver.yh", yshape, torch.float16, dev)
                    self._yl = scratch.get("solver.yl", yshape, torch.float16, dev)
                    self._ys = torch.empty(B, dtype=torch.float32, device=dev)
                yh, yl, ys = self._yh, self._yl, self._ys
                K.pow2_scale(Y, 14, out=ys)
                if self.left:
                    K.split_f16(Y, ys, hi=yh, lo=yl, blocked=True)
                else:
                    K.transpose_split(Y, hi=yh, lo=yl, scale=ys, blocked=True)
            yinv = 1.0 / (ys * ys)
            self._y_halves = (yh, yl, ys)
            if ysq is None:
                ysq = K.weighted_sqsum(Y, None, Y.shape[2])
            self._ysq = ysq
            # fp16 MFMA work issued: 3 products x k^2 n (the upper half of the symmetric 2 k^2 n)
            kk, nn = k, yh.shape[2]
            gev = GRAM_PROBE.start("gram", 3.0 * kk * kk * nn * B, 4.0 * kk * nn * B + 4.0 * kk * kk * B)
            if gev is not None:
                gev[0].record()
            K.gemm_x3(yh, yl, yh, yl, yinv, None, tri=True, a_blocked=True, b_blocked=True,
                      out_h=self._Gh, out_l=self._Gl, out_scale=X3_SCALE, sym_bound=ysq,
                      scale_out=self._gscale, inv_out=self._ginv)
            if gev is not None:
                gev[1].record()
            g_split = True
        elif not self.x3:
            self._fill_G(Y)  # Y Y^T (upper tiles + mirror) or Y^T Y
        self._active.fill_(1)
        if not g_split:
            self._ysq = K.weighted_sqsum(Y, None, Y.shape[2])  # trace(G) for the product-error test
        if self.x3:
            if not g_split:
                if self._G is None:
                    self._G = torch.empty((B, k, k), dtype=torch.float32, device=dev)
                self._fill_G(Y)
                K.sym_split_f16(self._G, X3_SCALE, hi=self._Gh, lo=self._Gl, scale=self._gscale,
                                inv_scale=self._ginv, upper_only=False, blocked=self._g_blocked)
            self._g_fp32_valid = not g_split
            self._ovf.zero_()
        cold = not (warm and self.X is not None)
        if cold:
            # same start block for every matrix: a matrix's result does not depend on its
            # position in the batch or on how the batch is split across streams
            X = self._bufs[0]
            g = torch.Generator(device=dev)
            g.manual_seed(self.seed)
            X.copy_(torch.randn((1, k, p), generator=g, device=dev, dtype=torch.float32).expand(B, k, p))
            if self.valid_k < k:  # zero-padded columns of W (engine.py): keep the block out of them
                X[:, self.valid_k:, :] = 0.0
            X, _ = self._cholqr(X)
            X, _ = self._orth2(X, halves=True)
            theta, X, Z = yield from self._rr(X, single=self.cheap_cold > 0, values_only=self.cheap_cold > 0)
            ends = torch.stack([theta[:, 0], theta[:, p - 1]], 1)
            yield
            ends = ends.cpu().numpy()
            degs = self.deg_cold
        else:
            # previous Ritz block (kept in self.X, never handed out by the pool) and values:
            # orthonormal, and its Ritz values bound the new spectrum closely (the residual
            # changes in <1% of its entries between updates)
            X = self.X
            theta = self.theta
            ends = self._ends
            Z = None
            degs = self.deg_warm
        self.stats.resid_hist = []
        # refinement: after every matrix passed the test, `refine` more full outer iterations
        # (filter of degree refine[i], CholQR2, Rayleigh-Ritz) for the whole batch -- set per
        # call by the engine (its first LR steps decide the kept Q's codes)
        refine = list(self.refine or ())
        used = []
        hist = []                               # per-matrix test values of the full iterations
        stalled = np.zeros(B, dtype=bool)
        # matrices that passed the test (or stalled) are FROZEN until every matrix has: the
        # filter passes their block through (active = 0) and the CholQR / Rayleigh-Ritz steps that
        # still run batch-wide are undone for them by restoring the state they froze with.  A
        # matrix's result then does not depend on how long its batch-mates take: it is the same
        # in any batch of the same size (main.py's layers, each with its own Hessian, batched).
        frz = None                              # (host mask, device index, X, Z, theta, ends, resid)
        n_outer = 0
        while n_outer < MAX_OUTER:
            d = degs[min(n_outer, len(degs) - 1)]
            n_outer += 1
            self.stats.outer += 1
            cheap = n_outer <= (self.cheap_cold if cold else self.cheap_warm)
            if cheap and not cold and self.skip_warm_cheap_rr:
                coef = self._cheb_coeffs(ends, d, dev)
                Xf = self._filter(X, coef, single=True)
                if B <= SEGMENTS_SMALL_BATCH:
                    Xf = self._more_segments(Xf, X, d, coef, True, ends)
                Xa, _ = self._cholqr(Xf, X)
                Xb, _ = self._orth2(Xa, X)
                ok = True
                if self.x3:  # an fp16 overflow of a single-product iterate: redo this outer
                    ovf = self._ovf.max()  # iteration on the regular path below (fp32 fallback)
                    yield
                    ok = int(ovf.item()) == 0
                    self._ovf.zero_()
                if ok:
                    X = Xb
                    used.append(d)
                    continue
            while True:
                coef = self._cheb_coeffs(ends, d, dev)
                # a widely spread spectrum caps the degree (FILTER_MAX_AMP): in the full
                # iterations the rest of the requested degree runs as further segments, each after
                # a CholQR pass that re-conditions the block (the same subspace), instead of as
                # further outer iterations with a Rayleigh-Ritz eigensolve and a read-back each.
                # (Not in the cheap ones: their bounds are a cold block's or the previous call's,
                # and a cold block's loose ends cap flat spectra too -- config 2's first iterations)
                Xf = self._filter(X, coef, single=cheap)
                # (a warm solve's cheap iteration too in small batches, SEGMENTS_SMALL_BATCH)
                if not cheap or (not cold and B <= SEGMENTS_SMALL_BATCH):
                    Xf = self._more_segments(Xf, X, d, coef, cheap, ends)
                Xa, _ = self._cholqr(Xf, X)
                Xb = Xa if (cheap and self.cheap_one_pass) else self._orth2(Xa, X, halves=True)[0]
                theta_n, Xn, Zn = yield from self._rr(Xb, X, single=cheap, values_only=cheap)
                # (B,) per-matrix max residual; a cheap iteration cannot converge (see _rr)
                # stopping test: estimated relative error of the rank-r projection of Y (a
                # residual relative to theta_0 over-converges flat spectra and under-converges
                # activation-weighted ones); "theta0": the max Ritz residual / theta_0
                if cheap:
                    res = torch.full((B,), math.inf, dtype=torch.float64, device=dev)
                elif self.criterion == "product" and self.r < p:
                    res = K.ritz_product_error(Xn, Zn, theta_n, self.r, self._ysq).double()
                else:
                    res = K.ritz_residual(Xn, Zn, theta_n, self.r).double()
                ovf = (self._ovf.max().double() if self.x3 and self._x3f
                       else torch.zeros((), dtype=torch.float64, device=dev))
                # matrices whose Jacobi used all JACOBI_MAX_SWEEPS (read back with the residuals)
                unconv = (self._last_sw >= JACOBI_MAX_SWEEPS).sum().double().view(1)
                chk = torch.cat([ovf.view(1), theta_n[:, 0], theta_n[:, p - 1], res, unconv])
                yield
                chk = chk.cpu().numpy()
                n_unconv = int(chk[-1])
                chk = chk[:-1]
                if frz is not None and Zn is not None:
                    # restore the frozen matrices' block, products, values and test (batch-wide
                    # CholQR / Rayleigh-Ritz rotated them; an overflow redo keeps them frozen too)
                    fm, fi, fX, fZ, fth, fends, fres = frz
                    Xn.index_copy_(0, fi, fX)
                    Zn.index_copy_(0, fi, fZ)
                    theta_n = theta_n.index_copy(0, fi, fth)
                    chk[1:1 + B][fm] = fends[fm, 0]
                    chk[1 + B:1 + 2 * B][fm] = fends[fm, 1]
                    chk[1 + 2 * B:][fm] = fres[fm]
                self.stats.jacobi_unconverged += n_unconv
                if self.x3 and self._x3f and chk[0] != 0:
                    # an fp16 half overflowed (a Ritz value far below the true top of the
                    # spectrum, cold start): redo this outer iteration with the fp32 filter
                    self._x3f = False
                    self._ovf.zero_()
                    self.stats.x3_fallbacks += 1
                    if not self._g_fp32_valid:  # the fp32 products need G itself
                        if self._G is None:
                            self._G = torch.empty((B, k, k), dtype=torch.float32, device=dev)
                        self._fill_G(self._Y)
                        self._g_fp32_valid = True
                    continue
                break
            self._x3f = True
            theta, X, Z = theta_n, Xn, Zn
            ends = np.stack([chk[1:1 + B], chk[1 + B:1 + 2 * B]], 1)
            resid = chk[1 + 2 * B:]
            mr = float(resid.max())
            self.stats.max_resid = mr
            self.stats.resid_hist.append(mr)
            used.append(d)
            if math.isfinite(mr) or np.isfinite(resid).any():
                hist.append(resid.copy())
            # precision floor (split-fp16 products), decided per matrix: a matrix whose test has
            # not improved at all over its last two outer iterations (best of the two above
            # STALL_RATIO x its best before them) is done; one still converging, however
            # slowly, keeps iterating (the filter gains far more than 2 % per outer iteration
            # unless the products' rounding dominates)
            if len(hist) >= 3:
                Hh = np.stack(hist)
                before = np.min(Hh[:-2], axis=0)
                recent = np.min(Hh[-2:], axis=0)
                new_stall = (~stalled) & (resid > self.tol) & np.isfinite(before) & (recent > STALL_RATIO * before)
                self.stats.stalls += int(new_stall.sum())
                if new_stall.any():
                    # the split-fp16 products' precision floor sits above the tolerance for these
                    # matrices (an input whose dynamic range erodes the fp32-grade margin): the
                    # rank-r projection is then only as accurate as the residual reached
                    warnings.warn(f"rank-r solver: {int(new_stall.sum())} matrices stopped at the product "
                                  f"precision floor above tolerance {self.tol:g} (residual estimate "
                                  f"{float(resid[new_stall].max()):.2e})", RuntimeWarning, stacklevel=2)
                stalled |= new_stall
            # converged (or stalled) matrices sit out the remaining filter products (X passes through)
            live = (resid > self.tol) & ~stalled
            if not live.any() and refine:
                degs = (refine.pop(0),)
                n_outer = max(n_outer, self.cheap_cold if cold else self.cheap_warm)  # a full iteration
                live = np.ones(B, dtype=bool)
                self.stats.refines += 1
            self._active.copy_(torch.from_numpy(live.astype(np.int32)))
            if not live.any():
                break
            if (~live).any() and (frz is None or (frz[0] != ~live).any()):
                # the frozen set grew (or a refinement reopened it): snapshot the frozen rows
                fm = ~live
                fi = torch.from_numpy(np.nonzero(fm)[0]).to(dev)
                frz = (fm, fi, X.index_select(0, fi), Z.index_select(0, fi), theta.index_select(0, fi),
                       ends.copy(), resid.copy())
            elif live.all():
                frz = None
        if Z is None:  # left the loop on a values-only iteration (MAX_OUTER): rotate once
            theta, X, Z = yield from self._rr(X)
        self.stats.history.append((cold, used, list(self.stats.resid_hist)))
        # Ritz rotations are accumulated in fp32 by the Jacobi kernel (orthogonal to ~1e-6):
        # one CholQR pass restores orthonormality without moving the converged subspace (latency
        # batches: one Newton-Schulz step, error 1e-6 -> the fp32 floor)
        X, _ = self._ns(X, steps=1) if self.ns_second else self._cholqr(X)
        # the final block becomes the warm start by a swap with the pool (no copy): X's pool
        # slot takes the previous warm-start buffer (a fresh one on the first call)
        i = next(j for j, t in enumerate(self._bufs) if t is X)
        old = self.X
        if old is None or any(t is old for t in self._bufs):  # never two pool slots on one tensor
            old = torch.empty((B, k, p), dtype=torch.float32, device=dev)
        self._bufs[i], self.X = old, X
        self.theta = theta.clone()
        self._ends = ends
        return self.X[:, :, : self.r], theta[:, : self.r]


class RandSVD:
    """`torch.svd_lowrank(Y, q, niter=2)` of LR_init's rand_svd branch (alg.py:213-216,
    :228-231; q = min(2 rank, min(m, n))), restated on the HIP kernels for a batch in
    lockstep: Halko et al. Algorithm 5 with the same structure as torch/_lowrank.py — a
    Gaussian sketch, `niter` power iterations re-orthonormalised after every product, a
    wide Y (m < n) processed as Y^T — with CholQR2 (fp64 Gram + symmetric
    elimination) in place of Householder QR (same subspaces) and the small SVD through the
    Jacobi eigensolver of the q x q Gram.  The sketch is random, as in the reference, so
    results agree with it statistically, not bitwise (oracle/caldera_oracle.py:svd_lowrank is
    pinned to torch.svd_lowrank on a shared sketch, tests/test_oracle_golden.py).

    solve_iter returns (U (B, m, r), theta = S^2 (B, r)) and sets `self.SVh` = diag(S) Vh
    restricted to the top r (B, r, n): LR_init's R before the H scaling.  As in torch the
    transposed variant's S Vh carries the projection onto the sketch (A Q Q^T), so R is not
    re-fitted as U^T Y."""

    left = True
    direct = False
    x3 = False

    def __init__(self, B: int, m: int, n: int, r: int, device, *, niter: int = 2, seed: int = 0x5EED):
        self.B, self.m, self.n = B, m, n
        self.k = min(m, n)
        self.r = min(r, self.k)
        self.q = min(2 * r, self.k)
        self.niter = niter
        self.device = device
        self.gen = torch.Generator(device=device)
        self.gen.manual_seed(seed)
        self.stats = SolverStats()
        self.SVh = None

    def release(self):
        self.SVh = None

    @staticmethod
    def _orth(X):
        for _ in range(2):  # CholQR2
            M = K.gram_f64(X, X)
            Wt32, _, _ = K.spd_whiten(M)
            X = K.gemm(X, Wt32, C=torch.empty_like(X), b_triu=True)
        return X

    def solve_iter(self, Y: torch.Tensor, warm: bool = True, y_split=None):
        B, m, n, q, r = self.B, self.m, self.n, self.q, self.r
        dev = Y.device
        f32 = torch.float32
        self.stats.calls += 1
        transposed = m < n  # torch: "assume that A is tall", a wide A is processed as A^T
        if transposed:  # basis of range(Y^T): Q (n x q)
            R0 = torch.randn((B, m, q), generator=self.gen, device=dev, dtype=f32)
            Qb = self._orth(K.gemm(Y, R0, ta=True, C=torch.empty((B, n, q), dtype=f32, device=dev)))
            for _ in range(self.niter):
                Qm = self._orth(K.gemm(Y, Qb, C=torch.empty((B, m, q), dtype=f32, device=dev)))
                Qb = self._orth(K.gemm(Y, Qm, ta=True, C=torch.empty((B, n, q), dtype=f32, device=dev)))
            Bt = K.gemm(Y, Qb, C=torch.empty((B, m, q), dtype=f32, device=dev))      # A Q
            T = K.gram_f64(Bt, Bt)                                                   # (A Q)^T (A Q)
            theta, Vb, _, _ = K.jacobi_eigh(T, tol=1e-12)
            S = torch.sqrt(theta[:, :r].clamp_min(0.0)).float()
            U = K.gemm(Bt, Vb[:, :, :r], C=torch.empty((B, m, r), dtype=f32, device=dev))
            inv = torch.where(S > 0, 1.0 / S.clamp_min(1e-30), torch.zeros_like(S))
            K.scale_rc(U, colscale=inv, out=U)                                       # U = A Q Vb / S
            V = K.gemm(Qb, Vb[:, :, :r], C=torch.empty((B, n, r), dtype=f32, device=dev))  # Q Vb
            self.SVh = K.scale_rc(V, trans=True, rowscale=S)                         # S V^T
        else:  # basis of range(Y): Q (m x q)
            R0 = torch.randn((B, n, q), generator=self.gen, device=dev, dtype=f32)
            Qm = self._orth(K.gemm(Y, R0, C=torch.empty((B, m, q), dtype=f32, device=dev)))
            for _ in range(self.niter):
                Qb = self._orth(K.gemm(Y, Qm, ta=True, C=torch.empty((B, n, q), dtype=f32, device=dev)))
                Qm = self._orth(K.gemm(Y, Qb, C=torch.empty((B, m, q), dtype=f32, device=dev)))
            Bm = K.gemm(Qm, Y, ta=True, C=torch.empty((B, q, n), dtype=f32, device=dev))  # Q^T A
            T = K.gram_f64(Bm, Bm, ta=True, tb=True)                                # B B^T
            theta, Ub, _, _ = K.jacobi_eigh(T, tol=1e-12)
            U = K.gemm(Qm, Ub[:, :, :r], C=torch.empty((B, m, r), dtype=f32, device=dev))
            self.SVh = K.gemm(Ub[:, :, :r], Bm, ta=True, C=torch.empty((B, r, n), dtype=f32, device=dev))
        self.stats.outer += 1
        if False:
            yield
        return U, theta[:, :r]
