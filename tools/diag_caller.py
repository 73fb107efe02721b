"""Reproduce the caller test's per-layer decompositions one shape at a time (diagnostics)."""
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "ee274_convexcaldera_llm_quantization_amd")
from src.caldera.decomposition.alg import caldera  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd.model import driver_params  # noqa: E402

DEV = "cuda:0"
g = torch.Generator().manual_seed(11)
for (m, n) in [(512, 512), (640, 512), (512, 640)]:
    for aware_h in (True,):
        torch.manual_seed(0)
        W = torch.randn(m, n) * 0.02
        h = torch.rand(n, generator=g, dtype=torch.float64) + 0.05
        p = driver_params(16)
        p.iters = 2
        print(f"=== {m}x{n} fp32 diagH", flush=True)
        t = time.time()
        d = caldera(p, W.to(DEV), torch.diag_embed(h.float()).to(DEV), device=DEV, use_tqdm=False, scale_W=False)
        print("ok", d.errors, time.time() - t, flush=True)
