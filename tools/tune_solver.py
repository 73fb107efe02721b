"""Solver tuning sweep on a bench workload: for each setting, time one batched step of B
matrices (after a warm-up step) and report the parity of seeds 0-3 (batch positions 0-3)
against the reference's golden sketches (bench.parity_of_timed_step).
    python tools/tune_solver.py cfg2 128 "tol=1e-5" "deg_cold=(8,12,12,12)" "cheap_cold=2"
    (--parts N: the batch as N interleaved parts, as bench.py's default two from 16 matrices)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch

import bench
from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams

dev = torch.device("cuda", 0)
parts = 1
if "--parts" in sys.argv:
    _i = sys.argv.index("--parts")
    parts = int(sys.argv[_i + 1])
    del sys.argv[_i:_i + 2]
name, B = sys.argv[1], int(sys.argv[2])
wl = bench.WORKLOADS[name]
ep = EngineParams.from_caldera_params(bench.make_params(wl))
Wb = bench.synth_batch(wl, B, 0, dev)
h = bench.make_h(wl)
h = None if h is None else h.to(dev)


def run(kw):
    tol = kw.pop("tol", 1e-5)
    from ee274_convexcaldera_llm_quantization_amd.overlap import run_interleaved
    engs = [CalderaEngine(ep, solver_tol=tol, solver_kwargs=dict(kw)) for _ in range(parts)]
    bnd = [B * i // parts for i in range(parts + 1)]
    outs = run_interleaved([e.run_iter(Wb[bnd[i]:bnd[i + 1]], h) for i, e in enumerate(engs)], dev)
    return [d for o in outs for d in o], engs[0]


for spec in sys.argv[3:]:
    kw = eval(f"dict({spec})")
    run(dict(kw))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    decs, eng = run(dict(kw))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    par = bench.parity_of_timed_step(name, decs, wl)
    st = eng.solver.stats
    rels = [v for k, v in par.items() if k.startswith("seed") and isinstance(v, float)]
    fc = par.get("final_codes_summary", {})
    fx = par.get("final_codes_vs_exact_lr", {})
    print(f"{spec:44s} {B / el:7.1f} matrices/s {1000 * el:8.1f} ms  matvecs {st.matvecs:4d} outer {st.outer:3d}  "
          f"stalls {st.stalls}  rel(seeds) max {max(rels):.2e} median {sorted(rels)[len(rels) // 2]:.2e}  "
          f"codes bit-exact {fc.get('bit_exact')}/{fc.get('matrices')} near-tie flips {fc.get('flips_at_near_ties')} "
          f"unexplained rows {fc.get('rows_unexplained')}  vs exact LR {fx.get('bit_exact')}/{fx.get('matrices')}", flush=True)
    del decs, eng
    torch.cuda.empty_cache()
