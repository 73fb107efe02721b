"""Time one fixed-sweep p=192 Jacobi per ablated build (see jacobi_ablate.sh)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ee274_convexcaldera_llm_quantization_amd._lib as K
A_ID = int(sys.argv[1])
K.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build_diag", f"libcq_abl{A_ID}.so"))
dev = "cuda:0"
p, B = 192, 64
A = torch.randn(B, p, p, device=dev, dtype=torch.float64)
A = A + A.transpose(1, 2)
K.jacobi_eigh(A.clone(), max_sweeps=2, tol=0.0); torch.cuda.synchronize()
t0 = time.perf_counter()
K.jacobi_eigh(A.clone(), max_sweeps=2, tol=0.0); torch.cuda.synchronize()
print(f"abl {A_ID}: {(time.perf_counter() - t0) * 1e3 / 2:.3f} ms per sweep")
