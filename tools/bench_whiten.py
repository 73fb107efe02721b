"""Times the solver's small p x p kernels on the config-2 block shape (p = 192) at B = 1 (one
drop-in caldera() call) and B = 256 (the bench batch) with HIP events: the SPD whitening of
CholQR (on a Gram of a Chebyshev-amplified block, condition ~1e10), the Lanczos filter bounds
and the values-only Jacobi they replace.  Prints a SHA-256 of the whitening's outputs so two
builds can be checked bit for bit (--lib loads another build: tools/probes/build_rev_lib.sh).

    python tools/bench_whiten.py [--lib path/to/lib.so]
"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import ee274_convexcaldera_llm_quantization_amd._lib as K  # noqa: E402

lib = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else None
K.load() if lib is None else K.load(lib)
tag = os.path.basename(lib) if lib else "tree"
dev = torch.device("cuda", 0)
p, k = 192, 4096


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for B in (1, 256):
    g = torch.Generator(device=dev).manual_seed(1)
    X = torch.randn(B, k, p, device=dev, generator=g) * torch.logspace(0, 5, p, device=dev)
    M = K.gram_f64(X, X)
    Mc = M.clone()
    Wt32, Wt64, info = K.spd_whiten(Mc)
    h = hashlib.sha256(Wt32.cpu().numpy().tobytes() + Wt64.cpu().numpy().tobytes()).hexdigest()[:16]
    ortho = (Wt64.transpose(1, 2) @ M @ Wt64 - torch.eye(p, dtype=torch.float64, device=dev)).abs().max().item()
    bufs = [M.clone() for _ in range(4)]
    it = iter(range(10 ** 9))
    t_w = timed(lambda: K.spd_whiten(bufs[next(it) % 4].copy_(M)))
    t_c = timed(lambda: bufs[next(it) % 4].copy_(M))
    T = K.gram_f64(X, X)
    t_l = timed(lambda: K.extreme_eigs(T, 40)) if hasattr(K, "extreme_eigs") else float("nan")
    print(f"[{tag}] B={B:3d} spd_whiten {t_w - t_c:.4f} ms (copy {t_c:.4f} excluded)  sha {h}  "
          f"max|Wt^T M Wt - I| {ortho:.2e}  info {int(info.max())}  extreme_eigs {t_l:.4f} ms", flush=True)
