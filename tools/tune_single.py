"""GPU tool: one drop-in caldera() call (B = 1, main.py:189-196's pattern) on config 2 under
solver schedules given as JSON dicts of RankRSolver keyword arguments; per schedule the median
latency, the outer iterations / products / eigensolves per call, and the parity of the seed-0..3
results (relative Frobenius of Q + L R to the reference's sketch, final codes vs the reference
and vs an exact rank-r step).
    python tools/tune_single.py '{"deg_warm": [14, 10]}' '{...}' ...     (first: the default {})"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from ee274_convexcaldera_llm_quantization_amd import api
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    from final_codes import compare, exact_fixture, fixture
    K.load()
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS["cfg2"]
    qp = bench.make_params(wl)
    seeds = range(4)
    Ws = [bench.synth_W(wl, s).to(dev) for s in seeds]
    fx, ex = fixture(), exact_fixture()
    scheds = [{}] + [json.loads(a) for a in sys.argv[1:]]
    for sk in scheds:
        kw = {"solver_kwargs": sk}
        api.caldera_batch(qp, [Ws[0]], device=dev, engine_kwargs=kw)  # warm-up
        ts, par = [], []
        stats = None
        for i, W in enumerate(Ws):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out, eng = api.caldera_batch(qp, [W], device=dev, engine_kwargs=kw, return_engine=True)
            torch.cuda.synchronize()
            ts.append(1000.0 * (time.perf_counter() - t0))
            d = out[0]
            tag = "cfg2" if i == 0 else f"cfg2s{i}"
            skt = bench._sketch(d.Q.to(dev), d.L.to(dev), d.R.to(dev), 4096)
            ref = fx[f"{tag}_sketch_QLR"].astype(np.float64)
            c = compare(tag, d.Q_idxs, 4096, 4096)
            e = compare(f"s{i}", d.Q_idxs, 4096, 4096, fx=ex)
            par.append({"rel": float(np.linalg.norm(skt - ref) / np.linalg.norm(ref)), "ref_exact": c["sha_equal"],
                        "flips": c["flips"], "unexpl": c["rows_unexplained"], "exact_lr": e["sha_equal"]})
            st = eng.solver.stats.as_dict() if eng.solver is not None else {}
            stats = {k: st.get(k) for k in ("outer", "matvecs", "calls")}
        print(json.dumps({"sched": sk, "ms": sorted(ts)[len(ts) // 2], "ms_all": ts, "stats_last": stats,
                          "parity": par}), flush=True)


if __name__ == "__main__":
    main()
