import os, sys, json
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import numpy as np, torch
from conftest import load_golden
from test_gpu_configs import _W
from src.caldera.utils.dataclasses import CalderaParams as CP
from ee274_convexcaldera_llm_quantization_amd.api import caldera_batch
large = load_golden("sum_large.npz")
W = _W(4096, 4096)
outs = caldera_batch(CP(Q_bits=2, L_bits=4, R_bits=4, rank=256, iters=5, lplr_iters=10, update_order=["Q", "LR"], sigma_reg=1e-8), [W.to("cuda:0")], None, device="cuda:0")
d = outs[0]
print(os.environ.get("CQ_WHITEN_LEGACY", "mfma"), "LR", np.round(np.asarray(d.errors["LR"]) - large["cfg5_errors_LR"], 5).tolist(), "Q", np.round(np.asarray(d.errors["Q"]) - large["cfg5_errors_Q"], 5).tolist())
