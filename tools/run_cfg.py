"""One config-5 (or config-N) decomposition on the GPU, for rocprofv3 kernel stats:
    python tools/run_cfg.py 5"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
from src.caldera.decomposition.alg import caldera  # noqa: E402
from src.caldera.utils.dataclasses import CalderaParams  # noqa: E402

CFG = {5: dict(Q_bits=2, L_bits=4, R_bits=4, rank=256, iters=5, lplr_iters=10, update_order=["Q", "LR"],
               sigma_reg=1e-8)}
cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 5
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
torch.manual_seed(0)
W = (torch.randn(4096, 4096) * 0.02).to(torch.float16).to("cuda")
for i in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d = caldera(CalderaParams(**CFG[cfg]), W, None, device="cuda", use_tqdm=False)
    torch.cuda.synchronize()
    print(f"cfg{cfg} run {i}: {time.perf_counter() - t0:.3f} s  LR errors {d.errors['LR'][:2]}", flush=True)
