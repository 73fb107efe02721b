"""GPU tool: the segmented filter (solver.segment_capped) against the unsegmented path and a
tight-tolerance run of the same engine, on tests/test_gpu_solver_variants.py's inputs; prints the
per-iteration errors and the distance of Q + L R from the tight run's.

    python tools/seg_check.py [B] [weighted] [seed]
    python tools/seg_check.py solver [r]      (the solver alone on log-normally spread columns)
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]


def solver_check(r):
    from ee274_convexcaldera_llm_quantization_amd import solver as S
    g = torch.Generator().manual_seed(17 + r)
    m, n, B = 512, 1024, 4
    spread = torch.tensor([0.0, 1.0, 2.0, 3.0])
    Y = torch.randn(B, m, n, generator=g) * torch.exp(torch.randn(B, 1, n, generator=g) * spread[:, None, None])
    Y = (Y * 0.02).to("cuda:0")
    Yd = Y.double().cpu()
    for seg in (False, True):
        sv = S.RankRSolver(B, m, n, r, "cuda:0", tol=5e-6, segment_capped=seg)
        U, th = sv.solve(Y)
        rows = []
        for b in range(B):
            ev, V = torch.linalg.eigh(Yd[b] @ Yd[b].T)
            ev, V = ev.flip(0)[:r], V.flip(1)[:, :r]
            P1 = U[b].double().cpu() @ U[b].double().cpu().T
            rows.append({"ev_rel_max": float(((th[b].cpu() - ev).abs() / ev).max()),
                         "ev_rel_top": float(((th[b].cpu() - ev).abs() / ev[0]).max()),
                         "proj": float(torch.linalg.norm(P1 - V @ V.T) / r ** 0.5),
                         "ev_range": float(ev[0] / ev[-1])})
        print(json.dumps({"segment_capped": seg, "stats": sv.stats.as_dict(), "hist": [h[1:] for h in sv.stats.history],
                          "rows": rows}, default=str), flush=True)


def main():
    from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams
    if sys.argv[1:2] == ["solver"]:
        return solver_check(int(sys.argv[2]) if len(sys.argv) > 2 else 64)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    weighted = len(sys.argv) > 2 and sys.argv[2] == "1"
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 61 + B + weighted
    g = torch.Generator().manual_seed(seed)
    W = (torch.randn(B, 1024, 2048, generator=g) * 0.02).half().to("cuda:0")
    h = (torch.rand(2048, generator=g) + 0.05).to("cuda:0") if weighted else None
    ep = EngineParams(Q_bits=2, L_bits=16, R_bits=16, rank=64, iters=4, update_order=["Q", "LR"], sigma_reg=1e-8)
    runs = {}
    for name, tol, kw in [("tight", 1e-8, dict(segment_capped=False)), ("seg", 1e-5, {}),
                          ("noseg", 1e-5, dict(segment_capped=False)), ("tight_seg", 1e-8, {})]:
        eng = CalderaEngine(ep, solver_tol=tol, solver_kwargs=kw)
        torch.cuda.synchronize()
        runs[name] = eng.run(W, h)
    ref = runs["tight"]
    for name, out in runs.items():
        rows = []
        for a, b in zip(out, ref):
            if B > 4:
                qa = a["Q"].double() + a["L"].double() @ a["R"].double()
                qb = b["Q"].double() + b["L"].double() @ b["R"].double()
                rows.append(round(float(torch.linalg.norm(qa - qb) / torch.linalg.norm(qb)), 8))
                continue
            qa = a["Q"].double() + a["L"].double() @ a["R"].double()
            qb = b["Q"].double() + b["L"].double() @ b["R"].double()
            rows.append({"errQ": a["errors"]["Q"], "errLR": a["errors"]["LR"],
                         "rel_vs_tight": float(torch.linalg.norm(qa - qb) / torch.linalg.norm(qb)),
                         "code_diffs_vs_tight": int((a["Q_idxs"] != b["Q_idxs"]).sum())})
        print(json.dumps({name: rows}), flush=True)


if __name__ == "__main__":
    main()
