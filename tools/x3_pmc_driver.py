"""Runs the p=192 filter product (batch 128) a few times: target for rocprofv3 --pmc passes."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ee274_convexcaldera_llm_quantization_amd._lib as K
K.load()
dev = "cuda:0"
B, k, p = int(sys.argv[1]) if len(sys.argv) > 1 else 128, 4096, 192
g = torch.Generator(device=dev).manual_seed(0)
Gh = (torch.randn(B, k, k, device=dev, generator=g) * 100).half()
Gl = (torch.randn(B, k, k, device=dev, generator=g) * 0.05).half()
Xh = (torch.randn(B, p, k, device=dev, generator=g)).half()
Xl = (torch.randn(B, p, k, device=dev, generator=g) * 1e-3).half()
inv = torch.ones(B, device=dev)
C = torch.empty(B, p, k, device=dev)
for _ in range(3):
    K.gemm_x3(Xh, Xl, Gh, Gl, inv, C, b_blocked=True)
torch.cuda.synchronize()
print("ok")
