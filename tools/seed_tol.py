"""GPU tool: parity of the reference seeds inside a B = 256 config-2 batch vs solver tolerance.

For each Ritz-residual tolerance: one warm-up + one timed engine run of 256 config-2 matrices
(seeds 0-3 at positions 0/77/150/255, the rest random), relative Frobenius error of each
seed's Q + L R against the reference's golden sketch, number of first-iteration Q codes
that differ... (printed as JSON lines).
Usage: python tools/seed_tol.py 1e-5 3e-6 1e-6
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]


def main():
    from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams
    from src.caldera.utils.dataclasses import CalderaParams
    dev = "cuda:0"
    g = np.load(os.path.join(ROOT, "tests", "golden", "sum_large.npz"))
    qp = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, update_order=["Q", "LR"], sigma_reg=1e-8)
    B = int(os.environ.get("B", "256"))
    pos = {0: 0, 1: B // 3, 2: (2 * B) // 3 - 20, 3: B - 1}
    gen = torch.Generator(device=dev).manual_seed(123)
    Wb = (torch.randn(B, 4096, 4096, device=dev, generator=gen) * 0.02).half()
    for s, i in pos.items():
        torch.manual_seed(s)
        Wb[i].copy_((torch.randn(4096, 4096) * 0.02).half().to(dev))
    om = torch.from_numpy(np.random.default_rng(1234).standard_normal((4096, 16))).to(dev)
    for tol in [float(x) for x in sys.argv[1:]]:
        eng = CalderaEngine(EngineParams.from_caldera_params(qp), solver_tol=tol)
        eng.run(Wb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng = CalderaEngine(EngineParams.from_caldera_params(qp), solver_tol=tol)
        out = eng.run(Wb)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        rels = {}
        for s, i in pos.items():
            tag = "cfg2" if s == 0 else f"cfg2s{s}"
            d = out[i]
            sk = (d["Q"].double() @ om + d["L"].double() @ (d["R"].double() @ om)).cpu().numpy()
            ref = g[f"{tag}_sketch_QLR"]
            rels[s] = float(np.linalg.norm(sk - ref) / np.linalg.norm(ref))
        st = eng.solver.stats.as_dict() if eng.solver is not None else {}
        print(json.dumps(dict(tol=tol, B=B, seconds=el, matrices_per_s=B / el, rel=rels,
                              matvecs=st.get("matvecs"), outer=st.get("outer"), max_resid=st.get("max_resid"))),
              flush=True)
        del out, eng


if __name__ == "__main__":
    main()
