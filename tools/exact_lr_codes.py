"""CPU tool: do the reference's final Q codes on config 2 follow exact arithmetic, or its fp32
rounding?  

For config-2 seeds (4096^2 fp16 randn * 0.02, torch host RNG, rank 128, Q 2-bit, iters 5, H = I)
the alternating minimisation of alg.py:24-112 is re-run with an EXACT rank-r step: the top-r
eigenpairs of G = Y Y^T in fp64 (LAPACK syevr on the upper r of the spectrum), L = U_r,
R = U_r^T Y -- the rank-r truncation of the SVD of Y = W - Q to ~1e-12, i.e. what an infinitely
tight solver would return.  Two variants of the Q step:
  f64      res = W - L R in fp64, scale and codes from the fp64 quotient (exact arithmetic);
  f32lr    L, R rounded to fp32 (as the reference stores them), res = fp32(W - L R) with the
           product in fp64 (one rounding, like a well-behaved fp32 GEMM), fp32 quotient as
           quantization.py:260-268.
The final codes of the kept iterate are compared with the reference's own (fixture
tests/golden/final_codes.npz via tests/final_codes.py): bit-exact, or flips at the reference's
near-ties.  If exact arithmetic also disagrees with the reference where the GPU engine does, that
code is decided by the reference's fp32 rounding, not by the accuracy of our LR solve.

  python tools/exact_lr_codes.py 8 15 0 > profiles/r04_exact_lr_codes.jsonl
"""
import json
import math
import os
import sys
import time

import numpy as np
import scipy.linalg
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import caldera_oracle as O  # noqa: E402  (test infrastructure: the checker)
from final_codes import compare, fixture  # noqa: E402

M = N = 4096
RANK, ITERS = 128, 5
VARIANTS = tuple(os.environ.get("VARIANTS", "f64,f32lr").split(","))


def weights(seed):
    torch.manual_seed(seed)
    return (torch.randn(M, N) * 0.02).to(torch.float16).numpy()


def top_r(Y):
    G = Y @ Y.T
    w, U = scipy.linalg.eigh(G, subset_by_index=[M - RANK, M - 1], driver="evr", overwrite_a=True)
    U = U[:, ::-1].copy()
    return U, U.T @ Y


def quantise(res, variant):
    if variant == "f64":
        s = np.abs(res).max()
        c = np.rint(res / s)
        return c.astype(np.int8), s, c * s
    r32 = res.astype(np.float32)
    s = np.float32(np.abs(r32).max())
    c = np.rint((r32 / s).astype(np.float32))
    return c.astype(np.int8), float(s), (c.astype(np.float32) * s).astype(np.float64)


def run(seed, variant):
    W16 = weights(seed)
    gs = O.global_scale_of(W16)
    W = O.scale_weight(W16, gs).astype(np.float64)
    den = float((W * W).sum())
    L = np.zeros((M, RANK))
    R = np.zeros((RANK, N))
    best, best_err, errs = None, math.inf, []
    for it in range(ITERS):
        if variant == "f32lr":
            res = (W - L.astype(np.float32).astype(np.float64) @ R.astype(np.float32).astype(np.float64))
        else:
            res = W - L @ R
        codes, s, Q = quantise(res, variant)
        eq = math.sqrt(float(((res - Q) ** 2).sum()) / den)
        U, R = top_r(W - Q)
        L = U
        elr = math.sqrt(float(((W - Q - L @ R) ** 2).sum()) / den)
        errs.append((eq, elr))
        for e in (eq, elr) if it else (elr,):   # alg.py:105-107: selection once Q and LR have run
            if e < best_err:
                best_err, best = e, (codes.copy(), s, it)
    return best, errs


def main():
    fx = fixture()
    for seed in [int(a) for a in sys.argv[1:]]:
        tag = "cfg2" if seed == 0 else f"cfg2s{seed}"
        for variant in VARIANTS:
            t0 = time.perf_counter()
            (codes, s, it), errs = run(seed, variant)
            c = compare(tag, codes.reshape(-1), M, N)
            # where exact arithmetic and the reference disagree at the reference's near-ties
            tidx, tcode, tdist = fx[tag + "_ties_idx"], fx[tag + "_ties_code"], fx[tag + "_ties_dist"]
            d = codes.reshape(-1)[tidx] != tcode
            print(json.dumps({"seed": seed, "variant": variant, "kept_iteration": it, "scale": s,
                              "ref_scale": float(fx[tag + "_Q_scale"]), "final_codes_vs_reference": c,
                              "tie_positions_differing": [[int(i), float(x)] for i, x in zip(tidx[d], tdist[d])],
                              "errors_Q_LR": errs, "seconds": time.perf_counter() - t0}), flush=True)


if __name__ == "__main__":
    main()
