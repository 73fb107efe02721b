"""Time the p <= 192 register Jacobi (cq_jacobi_eigh) on a batch of dense symmetric matrices
with a flat spectrum (the Rayleigh-Ritz matrices of config 2), vectors on; checks the
eigen-residual.  CQ_JAC_VARIANT selects the instantiation (cq_small.hip).
    CQ_JAC_VARIANT=a python tools/bench_jacobi.py 256 192"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import ee274_convexcaldera_llm_quantization_amd._lib as K

dev = "cuda:0"
B, p = int(sys.argv[1]), int(sys.argv[2])
g = torch.Generator(device=dev).manual_seed(0)
Q, _ = torch.linalg.qr(torch.randn(B, p, p, device=dev, dtype=torch.float64, generator=g))
lam = torch.linspace(3.0, 1.0, p, device=dev, dtype=torch.float64) ** 2
A0 = (Q * lam) @ Q.transpose(1, 2)
A0 = 0.5 * (A0 + A0.transpose(1, 2))
for tol, vec in ((1e-7, True), (1e-2, False)):
    K.jacobi_eigh(A0.clone(), tol=tol, want_vectors=vec)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    As = [A0.clone() for _ in range(3)]
    e0.record()
    for A in As:
        ev, V32, _, sw = K.jacobi_eigh(A, tol=tol, want_vectors=vec)
    e1.record()
    torch.cuda.synchronize()
    msg = ""
    if vec:
        V = V32.double()
        res = (A0 @ V - V * ev[:, None, :]).norm(dim=(1, 2)) / lam.max()
        orth = (V.transpose(1, 2) @ V - torch.eye(p, device=dev, dtype=torch.float64)).abs().max()
        msg = f" resid {res.max().item():.2e} orth {orth.item():.2e}"
    err = (ev - lam.flip(0).flip(0)).abs().max().item()
    print(f"[{os.environ.get('CQ_JAC_VARIANT', 'default')}] B={B} p={p} tol={tol:.0e} vectors={vec}: "
          f"{e0.elapsed_time(e1) / 3:.3f} ms/call sweeps {sw.float().mean().item():.1f} eval err {err:.2e}{msg}",
          flush=True)
