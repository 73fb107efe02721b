"""Diagnostic for config 3 (4096x11008, diag-H): our LR step vs an fp64 eigh of G = Y Y^T."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
import numpy as np
import torch
from ee274_convexcaldera_llm_quantization_amd.api import caldera_batch
from src.caldera.utils.dataclasses import CalderaParams

g = np.load(os.path.join(ROOT, "tests/golden/sum_large.npz"))
dev = "cuda:0"
torch.manual_seed(0)
W = (torch.randn(4096, 11008) * 0.02).half()
h = torch.from_numpy(g["cfg3_h"]).float().to(dev)
qp = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, update_order=["Q", "LR"], sigma_reg=1e-8)
outs, eng = caldera_batch(qp, [W.to(dev)], h, device=dev, return_engine=True)
d = outs[0]
print("ours Q ", d.errors["Q"])
print("ref  Q ", list(g["cfg3_errors_Q"]))
print("ours LR", d.errors["LR"])
print("ref  LR", list(g["cfg3_errors_LR"]))
st = eng.solver.stats
print("solver", st.as_dict(), st.history[:3])
# independent check of the first LR step: Y = (W/gs - Q1) * sqrt(h)
qp1 = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=1, update_order=["Q"], sigma_reg=1e-8)
d1 = caldera_batch(qp1, [W.to(dev)], h, device=dev)[0]
Ws = (W.to(dev).float() / d1.global_scale).half().float()
Y = (Ws - d1.Q) * torch.sqrt(h)
G = (Y.double() @ Y.double().T)
ev = torch.linalg.eigvalsh(G).flip(0)
tot = float((Y.double() ** 2).sum())
den = float(((Ws.double() ** 2) * h.double()).sum())
e_exact = np.sqrt((tot - float(ev[:128].sum())) / den)
print("exact first-LR error", e_exact, "ratio theta0/theta127", float(ev[0] / ev[127]), "theta127/theta128", float(ev[127] / ev[128]))
