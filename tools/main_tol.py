"""GPU tool: the primary caller's configurations (tests/golden/main_caller.npz) vs solver
tolerance: relative Frobenius error of Q + L R against the reference run, and solver stats.
Usage: python tools/main_tol.py main_up 1e-5 1e-6"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
from ee274_convexcaldera_llm_quantization_amd.api import caldera_batch  # noqa: E402
from src.caldera.utils.dataclasses import CalderaParams  # noqa: E402

tag = sys.argv[1]
g = np.load(os.path.join(ROOT, "tests", "golden", "main_caller.npz"))
m, n = {"main_down": (896, 4864), "main_up": (4864, 896), "main_o": (896, 896)}[tag]
seed = {"main_down": 11, "main_up": 12, "main_o": 13}[tag]
torch.manual_seed(seed)
W = (torch.randn(m, n) * 0.02).to(torch.float16).cuda()
H = torch.diag_embed(torch.from_numpy(g[tag + "_h"])).cuda()
qp = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=200, iters=int(os.environ.get("ITERS", "5")), lplr_iters=5,
                   update_order=["Q", "LR"], sigma_reg=1e-8)
om = np.random.default_rng(1234).standard_normal((n, 16))
for tol in [float(x) for x in sys.argv[2:]]:
    outs, eng = caldera_batch(qp, [W], H, device="cuda", scale_W=False, return_engine=True,
                              engine_kwargs=dict(solver_tol=tol))
    d = outs[0]
    sk = (d.Q.double() + d.L.double() @ d.R.double()).cpu().numpy() @ om
    ref = g[tag + "_sketch_QLR"]
    rel = np.linalg.norm(sk - ref) / np.linalg.norm(ref)
    st = eng.solver.stats
    print(f"{tag} tol {tol:g}: rel {rel:.3e} LR0 {d.errors['LR'][0]:.8f} (ref {g[tag + '_errors_LR'][0]:.8f}) "
          f"matvecs {st.matvecs} outer {st.outer} max_resid {st.max_resid:.2e} hist {st.history}", flush=True)
