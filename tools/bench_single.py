"""GPU tool: latency of single drop-in caldera() calls (B = 1, the reference's calling pattern,
main.py:189-196) on config-2 matrices, optionally per phase (engine.profile timings).
  python tools/bench_single.py [calls] [workload]   (cfg2 default; run under rocprofv3 for kernels)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    name = sys.argv[2] if len(sys.argv) > 2 else "cfg2"
    wl = bench.WORKLOADS[name]
    from src.caldera.decomposition.alg import caldera
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    K.load()
    dev = torch.device("cuda", 0)
    qp = bench.make_params(wl)
    h = bench.make_h(wl)
    H = None if h is None else torch.diag_embed(h).to(dev)
    Ws = [bench.synth_W(wl, wl.get("seed0", 0) + i).to(dev) for i in range(calls + 1)]
    caldera(qp, Ws[0], H, device=dev, use_tqdm=False)
    ts = []
    for W in Ws[1:]:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d = caldera(qp, W, H, device=dev, use_tqdm=False)
        torch.cuda.synchronize()
        ts.append(1000.0 * (time.perf_counter() - t0))
        del d
    print(json.dumps({"workload": name, "ms_per_call": ts, "median_ms": sorted(ts)[len(ts) // 2]}), flush=True)


if __name__ == "__main__":
    main()
