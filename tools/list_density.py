"""Candidate-list densities of the 2-bit single-recompute Q update on the bench batch (test
infrastructure: sizes the list capacities in csrc/cq_x3.h from measurements).

Runs the config-2 engine on the bench's B matrices and, at every Q update that gets a
scale hint, recomputes res = W - L R in fp32 (torch, outside the product path) and counts per
wave region (rows x n of one pass-2 wave, `cq_q_update_list_geometry`) the 8-element groups
holding exactly one |res| >= 0.45 hint (list A) and two or more (list B).  Prints the mean and
the maximum region fraction per Q update, the regions' capacities, and the matrices the call
reported as second recomputes.

  python tools/list_density.py [B] [--workload cfg2|cfg3|cfg4t]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import ee274_convexcaldera_llm_quantization_amd._lib as K  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd.overlap import run_to_end  # noqa: E402

wlname = "cfg2"
if "--workload" in sys.argv:
    i = sys.argv.index("--workload")
    wlname = sys.argv[i + 1]
    del sys.argv[i:i + 2]
wl = bench.WORKLOADS[wlname]
B = int(sys.argv[1]) if len(sys.argv) > 1 else wl["batch"]
dev = torch.device("cuda", 0)
K.load()
m, n, r = wl["m"], wl["n"], wl["rank"]
rows, capA, capB = K.q_update_list_geometry(m, n, r, both=True)
groups = rows * n // 8
print(f"{wlname} B={B} m={m} n={n} r={r}: region {rows} rows, {groups} groups; "
      f"cap A {capA} ({capA / groups:.4f}), cap B {capB} ({capB / groups:.4f})", flush=True)

orig = K.q_update_x3
calls = []


def wrapped(W, L, R, bits, **kw):
    hint = kw.get("scale_hint")
    hint = None if hint is None else hint.clone()   # the engine may pass the scale output itself
    out = orig(W, L, R, bits, **kw)
    fb = kw.get("fallback_out")
    if hint is None or L is None:
        return out
    tb = 0.45 * hint.float()
    fa, fbm, sd = [], [], []
    for b0 in range(0, W.shape[0], 16):
        res = W[b0:b0 + 16].float() - torch.bmm(L[b0:b0 + 16].float(), R[b0:b0 + 16].float())
        c = (res.abs() >= tb[b0:b0 + 16, None, None]).view(res.shape[0], m // rows, rows, n // 8, 8).sum(-1)
        one = (c == 1).sum(dim=(2, 3)).float() / groups
        many = (c >= 2).sum(dim=(2, 3)).float() / groups
        fa.append(one)
        fbm.append(many)
        sd.append(kw["scale"][b0:b0 + 16] / hint[b0:b0 + 16])
        del res, c
    fa, fbm, sd = torch.cat(fa), torch.cat(fbm), torch.cat(sd)
    nfb = int(fb.sum()) if fb is not None else -1
    calls.append((fa, fbm, sd, nfb))
    print(f"Q update {len(calls)}: A mean {fa.mean():.4f} max {fa.max():.4f} | B mean {fbm.mean():.4f} "
          f"max {fbm.max():.4f} | scale/hint min {sd.min():.4f} | over cap A {(fa * groups > capA).any(1).sum()} "
          f"B {(fbm * groups > capB).any(1).sum()} matrices | second recomputes {nfb}", flush=True)
    return out


K.q_update_x3 = wrapped
import ee274_convexcaldera_llm_quantization_amd.engine as E  # noqa: E402
E.K.q_update_x3 = wrapped
Wb = bench.synth_batch(wl, B, wl.get("seed0", 0), dev)
h = bench.make_h(wl)
h = None if h is None else h.to(dev)
ep = EngineParams.from_caldera_params(bench.make_params(wl))
run_to_end(CalderaEngine(ep).run_iter(Wb, h, True))
torch.cuda.synchronize()
allA = torch.stack([c[0] for c in calls]).max().item()
allB = torch.stack([c[1] for c in calls]).max().item()
print(f"max region fraction over all Q updates: A {allA:.4f} (cap {capA / groups:.4f}), "
      f"B {allB:.4f} (cap {capB / groups:.4f})", flush=True)
