"""Per-step time and allocator state of the config-3 workload (bench.py --workload cfg3) with
the 2-bit single-recompute Q update on and off:  python tools/diag/cfg3_mem.py [B]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 192
dev = "cuda:0"
wl = bench.WORKLOADS["cfg3"]
Wb = bench.synth_batch(wl, B, 0, dev)
h = bench.make_h(wl).to(dev)
ep = EngineParams.from_caldera_params(bench.make_params(wl))
for single in (True, False, True):
    for it in range(2):
        eng = CalderaEngine(ep)
        eng.q_single_recompute = single
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = eng.run(Wb, h)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"single={single} step {it}: {dt:.3f} s ({B / dt:.1f} matrices/s); reserved "
              f"{torch.cuda.memory_reserved() / 2**30:.1f} GiB, max allocated "
              f"{torch.cuda.max_memory_allocated() / 2**30:.1f} GiB, fallbacks {eng.q_fallbacks}", flush=True)
        del out, eng
