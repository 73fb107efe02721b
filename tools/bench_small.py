"""Micro-benchmark of the p x p solver kernels (Jacobi, whitening, fp64 Gram) on one GPU."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ee274_convexcaldera_llm_quantization_amd._lib as K

dev = "cuda:0"
K.load()


def t(fn, n=3):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for p in (int(a) for a in (sys.argv[1:] or ["192"])):
    for B in (8, 32):
        torch.manual_seed(0)
        X = torch.randn(B, 4 * p, p, dtype=torch.float64, device=dev)
        S = X.transpose(1, 2) @ X
        Q, _ = torch.linalg.qr(torch.randn(p, p, dtype=torch.float64, device=dev))
        D = torch.diag_embed(torch.linspace(1, 2, p, dtype=torch.float64, device=dev)).expand(B, p, p).clone()
        Dn = D + 1e-3 * (lambda M: M + M.transpose(1, 2))(torch.randn(B, p, p, dtype=torch.float64, device=dev))
        sw = []
        def jac(A):
            ev, V32, _, s = K.jacobi_eigh(A.clone())
            sw.append(int(s.max()))
        tj = t(lambda: jac(S))
        tjn = t(lambda: jac(Dn))
        tw = t(lambda: K.spd_whiten(S.clone()))
        Xf = torch.randn(B, 4096, p, device=dev)
        tg = t(lambda: K.gram_f64(Xf, Xf))
        print(f"p={p} B={B}: jacobi cold {tj:.2f} ms (sweeps {sw[0]}), near-diag {tjn:.2f} ms (sweeps {sw[-1]}), "
              f"whiten {tw:.2f} ms, gram_f64(4096) {tg:.3f} ms", flush=True)
