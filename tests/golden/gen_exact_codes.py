"""Generates tests/golden/exact_codes_cfg2.npz: the final 2-bit codes of config 2 (seeds 0-15,
4096^2 fp16 randn * 0.02 on the torch host RNG, rank 128, Q 2-bit, iters 5, H = I) when every LR
step is EXACT -- the top-128 eigenpairs of G = Y Y^T in fp64 (LAPACK syevr), L = U, R = U^T Y --
and the Q step follows the reference's fp32 arithmetic on those factors (L, R rounded to fp32,
res = fp32(W - L R) with the product in fp64, fp32 quotient, quantization.py:260-268).  Built from
the CPU oracle (oracle/caldera_oracle.py: global scale, scaled W); no reference code runs here.

Why: the reference's own final codes sit at its fp32 rounding floor on 5 of these
16 seeds -- the exact-LR run differs from them on seeds 2, 4, 8, 11, 14 at reference near-ties
(profiles/r04_exact_lr_codes.jsonl) -- so the codes a perfectly accurate rank-r solver would
produce are the second, sharper yardstick for the engine's final codes.

Per seed s: s{s}_sha256, s{s}_rowhash (64-bit blake2b per code row), s{s}_ties_idx / _code /
_dist (elements within 1e-3 code units of a rounding boundary in the kept Q update, their code
and distance), s{s}_kept_iteration, s{s}_Q_scale.   ~25 s per seed on 8 host threads.
    python tests/golden/gen_exact_codes.py             seeds 0-15  -> exact_codes_cfg2.npz
    python tests/golden/gen_exact_codes.py holdout     seeds 16-47 -> exact_codes_cfg2_holdout.npz
The held-out seeds are matrices the engine's schedules and tolerances were never tuned on
(round 6): the parity rates reported on them are out-of-sample."""
import hashlib
import math
import os
import sys
import time

import numpy as np
import scipy.linalg
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import caldera_oracle as O  # noqa: E402

M = N = 4096
RANK, ITERS, TIE_TOL = 128, 5, 1e-3
OUT = os.path.join(HERE, "exact_codes_cfg2.npz")
OUT_HOLDOUT = os.path.join(HERE, "exact_codes_cfg2_holdout.npz")
HOLDOUT_SEEDS = range(16, 48)


def rowhash(codes):
    a = np.ascontiguousarray(codes.reshape(M, N))
    return np.array([int.from_bytes(hashlib.blake2b(a[i].tobytes(), digest_size=8).digest(), "little")
                     for i in range(M)], dtype=np.uint64)


def exact_lr(Y):
    """Rank-r truncated SVD of Y to fp64 accuracy: L = U_r, R = U_r^T Y."""
    G = Y @ Y.T
    _, U = scipy.linalg.eigh(G, subset_by_index=[M - RANK, M - 1], driver="evr", overwrite_a=True)
    U = U[:, ::-1].copy()
    return U, U.T @ Y


def run(seed):
    torch.manual_seed(seed)
    W16 = (torch.randn(M, N) * 0.02).to(torch.float16).numpy()
    W = O.scale_weight(W16, O.global_scale_of(W16)).astype(np.float64)
    den = float((W * W).sum())
    L, R = np.zeros((M, RANK)), np.zeros((RANK, N))
    best, best_err = None, math.inf
    for it in range(ITERS):
        res = (W - L.astype(np.float32).astype(np.float64) @ R.astype(np.float32).astype(np.float64))
        r32 = res.astype(np.float32)
        s = np.float32(np.abs(r32).max())
        z = (r32 / s).astype(np.float32)
        codes = np.rint(z).astype(np.int8)
        Q = codes.astype(np.float64) * float(s)
        eq = math.sqrt(float(((res - Q) ** 2).sum()) / den)
        U, R = exact_lr(W - Q)
        L = U
        elr = math.sqrt(float(((W - Q - L @ R) ** 2).sum()) / den)
        for e in ((eq, elr) if it else (elr,)):  # alg.py:105-107 (selection once Q and LR ran)
            if e < best_err:
                d = np.abs(np.abs(z.astype(np.float64) - np.floor(z.astype(np.float64))) - 0.5).reshape(-1)
                tidx = np.nonzero(d < TIE_TOL)[0].astype(np.int64)
                best_err, best = e, dict(codes=codes.reshape(-1).copy(), s=float(s), it=it, tidx=tidx,
                                         tdist=d[tidx].astype(np.float32))
    return best


def main(seeds=range(16), out=OUT):
    o = {}
    for seed in seeds:
        t = time.time()
        b = run(seed)
        k = f"s{seed}"
        o[k + "_sha256"] = np.array(hashlib.sha256(b["codes"].tobytes()).hexdigest())
        o[k + "_rowhash"] = rowhash(b["codes"])
        o[k + "_ties_idx"] = b["tidx"]
        o[k + "_ties_code"] = b["codes"][b["tidx"]].astype(np.int8)
        o[k + "_ties_dist"] = b["tdist"]
        o[k + "_kept_iteration"] = np.array(b["it"])
        o[k + "_Q_scale"] = np.array(b["s"], dtype=np.float32)
        print(f"seed {seed}: kept iteration {b['it']}, {len(b['tidx'])} near-ties, {time.time() - t:.1f} s", flush=True)
        np.savez_compressed(out, **o)


if __name__ == "__main__":
    if sys.argv[1:] == ["holdout"]:
        main(HOLDOUT_SEEDS, OUT_HOLDOUT)
    else:
        main()
