"""Sweeps used by the Rayleigh-Ritz Jacobi calls during one engine run (bench config)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ee274_convexcaldera_llm_quantization_amd"))
import torch
import bench
import ee274_convexcaldera_llm_quantization_amd._lib as K
from ee274_convexcaldera_llm_quantization_amd import solver as S
from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams

calls = []
orig = K.jacobi_eigh


def wrapped(A, **kw):
    out = orig(A, **kw)
    calls.append(out[3])
    return out


S.K.jacobi_eigh = wrapped
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda", 0)
W = bench.synth_batch(B, 0, dev)
ep = EngineParams.from_caldera_params(bench.make_params())
import json
skw = json.loads(sys.argv[2]) if len(sys.argv) > 2 else {}
sp = skw.pop("p", None)
eng = CalderaEngine(ep, solver_kwargs=skw, solver_p=sp)
eng.run(W, None)
torch.cuda.synchronize()
for h in eng.solver.stats.history:
    print("solve cold=%s degs=%s resid=%s" % (h[0], h[1], ["%.2e" % r for r in h[2]]))
print("matvecs", eng.solver.stats.matvecs, "jacobi calls", len(calls))
W0 = bench.synth_batch(1, 0, dev)
d0 = CalderaEngine(ep, solver_kwargs=skw, solver_p=sp).run(W0, None)[0]
import numpy as np
g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "sum_large.npz"))
om = np.random.default_rng(1234).standard_normal((4096, 16))
sk = (d0["Q"].double() + d0["L"].double() @ d0["R"].double()).cpu().numpy() @ om
print("frob vs ref sketch", np.linalg.norm(sk - g["cfg2_sketch_QLR"]) / np.linalg.norm(g["cfg2_sketch_QLR"]))
if len(sys.argv) > 3:
    sys.exit(0)
for i, sw in enumerate(calls):
    s = sw.tolist()
    print(i, "sweeps min/mean/max", min(s), sum(s) / len(s), max(s))
# timing of one jacobi call at p=192 for cold-like and warm-like inputs
p = 192
A = torch.randn(B, p, p, device=dev, dtype=torch.float64)
A = A + A.transpose(1, 2)
D = torch.diag_embed(torch.linspace(100, 1, p, device=dev, dtype=torch.float64)).expand(B, p, p).contiguous()
Aw = D + 1e-3 * A
for name, M in (("random", A), ("near-diagonal", Aw)):
    orig(M.clone()); torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = orig(M.clone()); torch.cuda.synchronize()
    print(name, "ms", (time.perf_counter() - t0) * 1e3, "sweeps", out[3].tolist()[:4])
