"""A/B of the sparse-code Gram inside the engine: the same W through the engine with
sparse_gram on and off (and W^T, whose m > n shape keeps the dense Gram), reporting the error
histories, Q + L R distances and final-code flips.  python tools/diag_sgram.py [m n iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
import torch  # noqa: E402

from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams  # noqa: E402
from src.caldera.utils.dataclasses import CalderaParams  # noqa: E402

m, n, iters = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (4096, 11008, 2)
torch.manual_seed(0)
W = (torch.randn(m, n) * 0.02).to(torch.float16).cuda()
qp = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=iters, update_order=["Q", "LR"], sigma_reg=1e-8)


def run(Wx, sparse):
    eng = CalderaEngine(EngineParams.from_caldera_params(qp))
    eng.sparse_gram = sparse
    d = eng.run(Wx.unsqueeze(0))[0]
    st = eng.solver.stats.as_dict()
    return d, st


res = {}
for tag, Wx, sp in (("sparse", W, True), ("dense", W, False), ("dense_T", W.t().contiguous(), False)):
    d, st = run(Wx, sp)
    QLR = d["Q"].double() + d["L"].double() @ d["R"].double()
    if tag == "dense_T":
        QLR = QLR.t()
        codes = d["Q_idxs"].view(n, m).t().reshape(-1)
    else:
        codes = d["Q_idxs"].reshape(-1)
    res[tag] = (QLR, codes, d["errors"])
    print(tag, "errors", d["errors"], "solver", {k: st[k] for k in ("matvecs", "outer", "stalls", "max_resid")
                                                    if k in st}, flush=True)
for a, b in (("sparse", "dense"), ("dense", "dense_T"), ("sparse", "dense_T")):
    qa, ca, _ = res[a]
    qb, cb, _ = res[b]
    rel = float(torch.linalg.norm(qa - qb) / torch.linalg.norm(qb))
    print(f"{a} vs {b}: rel Q+LR {rel:.3e}, final-code flips {int((ca != cb).sum())}", flush=True)
