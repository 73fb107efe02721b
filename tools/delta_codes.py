"""GPU tool: how much the 2-bit Q codes change between consecutive Q updates of a config-2 run
(the premise of an incremental sparse-code Gram, VERDICT r05 "next" #3).  Per Q update after the
first: the fraction of elements whose code changed, the fraction of code rows (the Gram's
columns j of P = E c^T) holding any change, the nonzero-code density, and the relative change
of the whole-matrix scale s (the s-dependent part of G = A - s (W c^T + c W^T) + s^2 c c^T
changes with it everywhere).

    python tools/delta_codes.py [B]        (config 2, seeds 0..B-1, one engine run)
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]

import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams
    K.load()
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS["cfg2"]
    W = torch.stack([bench.synth_W(wl, s) for s in range(B)]).to(dev)
    m, n = W.shape[1:]
    ep = EngineParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, update_order=["Q", "LR"], sigma_reg=1e-8)
    eng = CalderaEngine(ep)
    hist = []
    orig = eng._q_update

    def rec(st, *a, **k):
        out = orig(st, *a, **k)
        codes = K.unpack_codes(st.Qc, m * n, 2).view(B, m, n).to(torch.int8)
        hist.append((codes, st.Qs.clone()))
        return out

    eng._q_update = rec
    eng.run(W)
    rows = []
    for i in range(1, len(hist)):
        (c0, s0), (c1, s1) = hist[i - 1], hist[i]
        ch = c0 != c1
        flips = ((c0 * c1) < 0).sum().item()
        rows.append({"q_update": i + 1, "changed_frac": ch.float().mean().item(),
                     "rows_touched_frac": ch.any(dim=2).float().mean().item(),
                     "sign_flips": flips, "nonzero_frac": (c1 != 0).float().mean().item(),
                     "rel_scale_change_max": ((s1 - s0).abs() / s0).max().item(),
                     "rel_scale_change_median": ((s1 - s0).abs() / s0).median().item()})
    print(json.dumps({"B": B, "m": m, "n": n, "first_nonzero_frac": (hist[0][0] != 0).float().mean().item(),
                      "steps": rows}, indent=1), flush=True)


if __name__ == "__main__":
    main()
