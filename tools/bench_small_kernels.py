"""Times the solver's block kernels on the config-2 block shape (k = 4096, p = 192) with HIP
events: the symmetric fp64 Gram X^T X (CholQR), the fp64 Rayleigh-Ritz Gram X^T Z, CholQR's
X Wt (Wt upper triangular), a full rotation X V, and the two transpose-split forms the solver
uses (with and without the fp32 X^T).  --lib loads another build of the library, so two
builds can be compared on one box (tools/probes/build_rev_lib.sh).

    python tools/bench_small_kernels.py [B] [--lib tools/probes/lib_head.so]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import ee274_convexcaldera_llm_quantization_amd._lib as K  # noqa: E402

lib = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else None
K.load() if lib is None else K.load(lib)
args = [a for i, a in enumerate(sys.argv[1:], 1) if a != "--lib" and sys.argv[i - 1] != "--lib"]
B = int(args[0]) if args else 128
k, p = 4096, 192
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(B, k, p, device=dev, generator=g)
Z = torch.randn(B, k, p, device=dev, generator=g)
Wt = torch.triu(torch.randn(B, p, p, device=dev, generator=g))
V = torch.randn(B, p, p, device=dev, generator=g)
C = torch.empty(B, k, p, device=dev)
Xt = torch.empty(B, p, k, device=dev)
hi = torch.empty(B, p, k, device=dev, dtype=torch.float16)
lo = torch.empty_like(hi)

cases = {
    "gram_f64 sym (X^T X)": lambda: K.gram_f64(X, X),
    "gram_f64 (X^T Z)": lambda: K.gram_f64(X, Z),
    "gemm X Wt (b_triu)": lambda: K.gemm(X, Wt, C=C, b_triu=True),
    "gemm X V": lambda: K.gemm(X, V, C=C),
    "transpose_split (X^T + halves)": lambda: K.transpose_split(X, out=Xt, hi=hi, lo=lo, scale=64.0, blocked=True),
    "transpose_split (halves)": lambda: K.transpose_split(X, hi=hi, lo=lo, scale=64.0, blocked=True),
}
tag = os.path.basename(lib) if lib else "tree"
for name, fn in cases.items():
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    reps = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"[{tag}] B={B} {name:34s} {e0.elapsed_time(e1) / reps:.3f} ms", flush=True)
