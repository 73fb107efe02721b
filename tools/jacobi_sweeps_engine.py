"""Jacobi sweeps per Rayleigh-Ritz eigensolve inside a config-2 decomposition (diagnostic):
wraps _lib.jacobi_eigh, runs the engine on B bench matrices and prints, per call, p, the
tolerance, values-only or not, and the sweeps used (min / mean / max over the batch) with the
call's time (HIP events).
    python tools/jacobi_sweeps_engine.py [B]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import ee274_convexcaldera_llm_quantization_amd._lib as K  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd.overlap import run_to_end  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
wl = bench.WORKLOADS["cfg2"]
dev = torch.device("cuda", 0)
K.load()
orig = K.jacobi_eigh
log = []


def wrapped(A, max_sweeps=30, tol=1e-13, want64=False, want_vectors=True):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = orig(A, max_sweeps=max_sweeps, tol=tol, want64=want64, want_vectors=want_vectors)
    e1.record()
    log.append((A.shape[-1], tol, want_vectors, out[3], e0, e1))
    return out


K.jacobi_eigh = wrapped
Wb = bench.synth_batch(wl, B, 0, dev)
ep = EngineParams.from_caldera_params(bench.make_params(wl))
for rep in range(2):
    log.clear()
    run_to_end(CalderaEngine(ep).run_iter(Wb, None, True))
    torch.cuda.synchronize()
tot = 0.0
for p, tol, vec, sw, e0, e1 in log:
    ms = e0.elapsed_time(e1)
    tot += ms
    swf = sw.float()
    print(f"p {p} tol {tol:.0e} vectors {int(vec)}  sweeps min {int(sw.min())} mean {float(swf.mean()):.2f} "
          f"max {int(sw.max())}  {ms:.3f} ms", flush=True)
print(f"{len(log)} calls, {tot:.1f} ms", flush=True)
