"""GPU A/B of the LPLR error: fused (normal-equation pieces) vs the m x n x r error GEMM, on a
config-5-like matrix; prints both per-iteration LPLR error traces and the caldera errors."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
r = int(sys.argv[2]) if len(sys.argv) > 2 else 64
torch.manual_seed(0)
W = (torch.randn(2, n, n) * 0.02).half().cuda()
ep = EngineParams(Q_bits=2, L_bits=4, R_bits=4, rank=r, iters=2, lplr_iters=10, update_order=["Q", "LR"],
                  sigma_reg=1e-8)
for fused in (False, True):
    e = CalderaEngine(ep)
    e.lplr_fused_err = fused
    e.lplr_trace = []
    out = e.run(W)
    print("fused" if fused else "gemm ", [round(float(x[0]), 4) for x in e.lplr_trace[:10]])
    print("   caldera errors", out[0]["errors"], out[1]["errors"]["LR"])
