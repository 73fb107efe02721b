"""Per-seed diagnosis of config-2 parity (round 6): decompose the given seeds (host RNG, the
survey's recipe) in one batch with the engine and print, per seed, our error trajectory beside
the reference's (tests/golden/final_codes*.npz errors_Q / errors_LR), the kept iteration, and the
final codes against the reference and against the exact-LR step.
    python tools/diag_holdout.py 22 38 20 [--kw "deg_cold=(6,12,10)"] [--tol 1e-5] [--pad 0]
--pad P adds P device-RNG matrices to the batch (batch-size effects)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import torch

from final_codes import compare

ap = argparse.ArgumentParser()
ap.add_argument("seeds", type=int, nargs="+")
ap.add_argument("--kw", type=str, default="")
ap.add_argument("--tol", type=float, default=1e-5)
ap.add_argument("--pad", type=int, default=0)
args = ap.parse_args()

from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams
from src.caldera.utils.dataclasses import CalderaParams

dev = torch.device("cuda", 0)
gd = os.path.join(ROOT, "tests", "golden")
fx0 = np.load(os.path.join(gd, "final_codes.npz"), allow_pickle=False)
fx1 = np.load(os.path.join(gd, "final_codes_holdout.npz"), allow_pickle=False)
ex0 = np.load(os.path.join(gd, "exact_codes_cfg2.npz"), allow_pickle=False)
ex1 = np.load(os.path.join(gd, "exact_codes_cfg2_holdout.npz"), allow_pickle=False)
qp = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, update_order=["Q", "LR"], sigma_reg=1e-8)
B = len(args.seeds) + args.pad
Wb = torch.empty(B, 4096, 4096, dtype=torch.float16, device=dev)
for i, s in enumerate(args.seeds):
    torch.manual_seed(s)
    Wb[i].copy_((torch.randn(4096, 4096) * 0.02).to(torch.float16))
if args.pad:
    g = torch.Generator(device=dev).manual_seed(99)
    Wb[len(args.seeds):].copy_(torch.randn(args.pad, 4096, 4096, device=dev, generator=g) * 0.02)
kw = eval(f"dict({args.kw})")
eng = CalderaEngine(EngineParams.from_caldera_params(qp), solver_tol=args.tol, solver_kwargs=kw or None)
out = eng.run(Wb)
print(f"kw {kw} tol {args.tol} B {B}; solver {eng.solver.stats.as_dict() if eng.solver else None}")
for i, s in enumerate(args.seeds):
    fx, ex = (fx0, ex0) if s < 16 else (fx1, ex1)
    tag = "cfg2" if s == 0 else f"cfg2s{s}"
    d = out[i]
    eq, el = d["errors"]["Q"], d["errors"]["LR"]
    rq, rl = fx[f"{tag}_errors_Q"], fx[f"{tag}_errors_LR"]
    c = compare(tag, d["Q_idxs"], 4096, 4096, fx=fx)
    e = compare(f"s{s}", d["Q_idxs"], 4096, 4096, fx=ex)
    print(f"seed {s}: Q  ours {' '.join(f'{x:.7f}' for x in eq)}\n"
          f"          Q  ref  {' '.join(f'{x:.7f}' for x in rq)}\n"
          f"          LR ours {' '.join(f'{x:.7f}' for x in el)}\n"
          f"          LR ref  {' '.join(f'{x:.7f}' for x in rl)}\n"
          f"          scale ours {float(d['Q_scale'] if 'Q_scale' in d else float('nan')):.7f} ref "
          f"{float(fx[f'{tag}_Q_scale']):.7f} exact {float(ex[f's{s}_Q_scale']):.7f} (exact kept it "
          f"{int(ex[f's{s}_kept_iteration'])})\n"
          f"          vs ref {c}\n          vs exact {e}", flush=True)
