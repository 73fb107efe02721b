"""CPU BASELINE — test/bench infrastructure only, never the product path.

The reference's own CPU path, restated on torch CPU tensors (fp32, MKL/LAPACK through
torch.linalg exactly as the reference calls them), so that `bench.py`'s `cpu_baseline` times
the arithmetic the reference runs rather than the numpy oracle (which is ~2x slower than
torch's MKL path on the same cores).  Scope: uniform quantisers, H = None / diagonal / dense,
deterministic SVD (rand_svd=False) — the configurations BASELINE.json quotes.

  caldera()          alg.py:24-112 (global scale in W's dtype, best iterate by strict <)
  _lr_update()       alg.py:115-198 (LR_init + the quantised-factor lstsq loop)
  _lr_init()         alg.py:201-235 (torch.linalg.svd, full_matrices=False)
  _quantize_whole()  alg.py:245-250 + quantization.py:244-307 (uniform, one block)
  _error()           alg.py:286-302

Only tests/ and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import math

import torch


def _quantize_whole(A: torch.Tensor, bits: int, eps: float = 1e-8):
    """Whole-matrix uniform absmax quantiser: (A_hat, codes, scale)."""
    k = 2 ** (bits - 1) - 1
    flat = A.reshape(1, -1)
    mx = torch.maximum(flat.abs().max(dim=1, keepdim=True)[0], torch.tensor([eps]))
    codes = torch.round(flat / mx * k).to(torch.int8 if bits <= 8 else torch.int16)
    A_hat = ((codes.float() / k) * mx).reshape(A.shape)
    return A_hat, codes, mx


def _eig_of(H: torch.Tensor, sigma_reg: float, aware: bool, n: int):
    """alg.py:44-68: (H used by the error, H_sqrt, eigenvalues, eigenvectors)."""
    if not aware:
        return H, H, torch.ones(n), H
    H = (H + H.T) / 2
    if torch.allclose(H, torch.eye(n), rtol=1e-5, atol=1e-8):
        lam, V = torch.ones(n), torch.eye(n)
    else:
        lam, V = torch.linalg.eigh(H)
    if lam.min() < sigma_reg:
        shift = sigma_reg - lam.min()
        H = H + shift * torch.eye(n)
        lam = lam + shift
    return H, V @ torch.diag(torch.sqrt(lam)) @ V.T, lam, V


def _lr_init(res, H_sqrt, lam, V, rank, aware):
    if aware:
        U, S, Vh = torch.linalg.svd(res @ H_sqrt @ V, full_matrices=False)
        return U[:, :rank], torch.diag(S[:rank]) @ Vh[:rank] @ torch.diag(1 / lam.sqrt()) @ V.T
    U, S, Vh = torch.linalg.svd(res, full_matrices=False)
    s = S[:rank].sqrt()
    return U[:, :rank] @ torch.diag(s), torch.diag(s) @ Vh[:rank]


def _lr_update(st, p, res, H_sqrt, lam, V):
    L, R = _lr_init(res, H_sqrt, lam, V, p["rank"], p["aware"])
    if p["L_bits"] < 16 or p["R_bits"] < 16:
        best = (L, R, None, None, math.inf)
        for _ in range(p["lplr_iters"]):
            if p["aware"]:
                L = torch.linalg.lstsq((R @ H_sqrt).T, (res @ H_sqrt).T)[0].T
            else:
                L = torch.linalg.lstsq(R.T, res.T)[0].T
            L, Lc, Ls = _quantize_whole(L.T, p["L_bits"])
            L = L.T
            R, Rc, Rs = _quantize_whole(torch.linalg.lstsq(L, res)[0], p["R_bits"])
            e = torch.linalg.matrix_norm((res - L @ R) @ H_sqrt)
            if e < best[-1]:
                best = (L, R, (Lc, Ls), (Rc, Rs), e)
        L, R = best[0], best[1]
        st["L_q"], st["R_q"] = best[2], best[3]
    st["L"], st["R"] = L, R


def _error(W, H, st, gs):
    E = (st["Q"] + st["L"] @ st["R"]) * gs - W
    return (torch.trace(E @ H @ E.T) / torch.trace(W @ H @ W.T)).sqrt().item()


def caldera(W: torch.Tensor, H: torch.Tensor | None = None, *, Q_bits=2, L_bits=2, R_bits=2, rank=64,
            iters=20, lplr_iters=5, update_order=("Q", "LR"), sigma_reg=1e-8, activation_aware_LR=True,
            scale_W=True):
    """W (m, n) fp16/fp32 CPU tensor; defaults as CalderaParams (dataclasses.py:11-84).
    Returns dict(Q, L, R, Q_idxs, Q_scale, errors, global_scale)."""
    gs = W.square().mean().sqrt().item() if scale_W else 1
    W = W / gs
    m, n = W.shape
    H = torch.eye(n) if H is None else H.float()
    p = dict(rank=rank, L_bits=L_bits, R_bits=R_bits, lplr_iters=lplr_iters, aware=activation_aware_LR)
    H, H_sqrt, lam, V = _eig_of(H, sigma_reg, activation_aware_LR, n)
    st = dict(Q=torch.zeros(m, n), L=torch.zeros(m, rank), R=torch.zeros(rank, n), Q_idxs=None, Q_scale=1)
    best, min_err = dict(st), math.inf
    errors = {k: [] for k in update_order}
    done = {k: False for k in update_order}
    Wf = W.float()
    for _ in range(iters):
        for k in update_order:
            if k == "LR":
                _lr_update(st, p, W - st["Q"], H_sqrt, lam, V)
            else:
                st["Q"], st["Q_idxs"], st["Q_scale"] = _quantize_whole(W - st["L"] @ st["R"], Q_bits)
            done[k] = True
            errors[k].append(_error(Wf, H, st, 1.0))
            if errors[k][-1] < min_err and all(done.values()):
                min_err, best = errors[k][-1], dict(st)
    best["errors"], best["global_scale"] = errors, gs
    return best
