"""Deterministic inputs of the fused Q-update fingerprint test (tests/test_gpu_qupdate_variants.py)
and of tools/ab_qupdate_r02.py, which recorded the round-2 kernel's outputs on them
(tests/golden/qupdate_r02_fingerprints.json).  Host RNG only, so the inputs are the same bytes
on every machine."""
import hashlib

import numpy as np
import torch

# (tag, B, m, n, r, bits, W dtype): full config-2 shape, a partial last 4-chunk code group
# (n = 544: 17 chunks of 32), 4-bit packing, K = 256, fp32 W
CASES = [
    ("cfg2_b4", 4, 4096, 4096, 128, 2, torch.float16),
    ("n544_r96", 2, 320, 544, 96, 2, torch.float16),
    ("b4bit", 2, 640, 1024, 128, 4, torch.float16),
    ("r256", 2, 336, 512, 256, 2, torch.float16),
    ("f32w", 2, 320, 544, 64, 2, torch.float32),
]


def make(B, m, n, r, dt, seed):
    g = torch.Generator().manual_seed(seed)
    W = (torch.randn(B, m, n, generator=g) * 0.02).to(dt)
    W = (W.float() / W.float().pow(2).mean().sqrt()).to(dt)      # unit RMS, like W / global_scale
    L = torch.linalg.qr(torch.randn(B, m, r, generator=g))[0].contiguous()
    R = (torch.randn(B, r, n, generator=g) * (0.3 * (m ** 0.5) / (r ** 0.5))).contiguous()
    return W, L, R


def digest(t):
    return hashlib.sha256(np.ascontiguousarray(t.detach().cpu().numpy()).tobytes()).hexdigest()


def run(K, case, dev):
    """Packed codes, scales and error sums of cq_q_update_x3 on the case's inputs."""
    tag, B, m, n, r, bits, dt = case
    W, L, R = make(B, m, n, r, dt, seed=sum(map(ord, tag)))
    W, L, R = W.to(dev), L.to(dev), R.to(dev)
    packed = torch.empty(B, m * n * bits // 8, dtype=torch.uint8, device=dev)
    scale = torch.empty(B, device=dev)
    err = torch.empty(B, dtype=torch.float64, device=dev)
    K.q_update_x3(W, L, R, bits, packed=packed, scale=scale, err_out=err)
    torch.cuda.synchronize()
    return {"packed_sha256": digest(packed), "scale": scale.cpu().tolist(), "err": err.cpu().tolist()}
