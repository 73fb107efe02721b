"""Per-config latency: the MI355X engine (one matrix, caldera() drop-in) next to the CPU
baseline (the numpy/LAPACK oracle, `kind: port`) on the same host, for BASELINE configs 1, 2,
3, 5 and the three Llama-2-7B shapes of config 4 (SURVEY.md §8(d) "CPU baseline timing":
config 4 = one matrix per shape, extrapolated x32 layers).  Run on the GPU box:
    python tools/cpu_gpu_configs.py > gpurun_out/cpu_gpu_configs.json
A heartbeat line goes to stderr every 30 s while the CPU runs (long LAPACK calls)."""
import json
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]

from oracle import caldera_oracle as O  # noqa: E402  (CPU baseline leg only)
from src.caldera.decomposition.alg import caldera  # noqa: E402
from src.caldera.utils.dataclasses import CalderaParams  # noqa: E402
from src.caldera.utils.quantization import QuantizerFactory  # noqa: E402

DEV = "cuda:0"


def W_of(m, n, seed=0):
    torch.manual_seed(seed)
    return (torch.randn(m, n) * 0.02).to(torch.float16)


def heartbeat(stop):
    t0 = time.time()
    while not stop.wait(30):
        print(f"[cpu_gpu_configs] still running, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)


def run(name, m, n, kw, h=None, seed=0):
    W = W_of(m, n, seed)
    qf = {"quant_factory_Q": QuantizerFactory("uniform", 64), "quant_factory_LR": QuantizerFactory("uniform", 64)}
    Hd = None if h is None else torch.diag_embed(torch.from_numpy(h).float())
    caldera(CalderaParams(**kw, **qf), W.to(DEV), None if Hd is None else Hd.to(DEV), device=DEV, use_tqdm=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d = caldera(CalderaParams(**kw, **qf), W.to(DEV), None if Hd is None else Hd.to(DEV), device=DEV, use_tqdm=False)
    torch.cuda.synchronize()
    tg = time.perf_counter() - t0
    t0 = time.perf_counter()
    ref = O.caldera(O.Params(**kw), W.numpy(), None if h is None else np.diag(h.astype(np.float32)))
    tc = time.perf_counter() - t0
    out = (d.Q.double() + d.L.double() @ d.R.double()).cpu().numpy()
    exp = ref.Q.astype(np.float64) + ref.L.astype(np.float64) @ ref.R.astype(np.float64)
    rel = float(np.linalg.norm(out - exp) / np.linalg.norm(exp))
    row = {"config": name, "shape": [m, n], "gpu_s": tg, "cpu_s": tc, "speedup": tc / tg,
           "rel_frob_QLR_vs_oracle": rel, "errors_LR_gpu": d.errors.get("LR"), "errors_LR_cpu": ref.errors.get("LR")}
    print(json.dumps(row), flush=True)
    return row


def main():
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    stop = threading.Event()
    threading.Thread(target=heartbeat, args=(stop,), daemon=True).start()
    base = dict(update_order=["Q", "LR"], sigma_reg=1e-8)
    g = np.load(os.path.join(ROOT, "tests", "golden", "sum_large.npz"), allow_pickle=False)
    rows = [
        run("cfg1 512x512 r16 Q4 (L/R 2-bit, lplr 5) iters 3", 512, 512,
            dict(Q_bits=4, L_bits=2, R_bits=2, rank=16, iters=3, lplr_iters=5, **base)),
        run("cfg2 4096x4096 r128 Q2 L/R16 iters 5", 4096, 4096,
            dict(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, **base)),
        run("cfg3 4096x11008 diag-H r128 Q2 L/R16 iters 5", 4096, 11008,
            dict(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, **base), h=g["cfg3_h"].astype(np.float64)),
        run("cfg5 4096x4096 r256 Q2 L/R4 lplr 10 iters 5", 4096, 4096,
            dict(Q_bits=2, L_bits=4, R_bits=4, rank=256, iters=5, lplr_iters=10, **base)),
        run("cfg4 gate/up 11008x4096 r128 Q2 iters 5", 11008, 4096,
            dict(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, **base), seed=4),
    ]
    stop.set()
    by = {r["config"].split()[0] + ("_tall" if r["shape"][0] > r["shape"][1] else ""): r for r in rows}
    # config 4 on one host: 32 layers x (4 x 4096^2 + 2 x 11008x4096 + 1 x 4096x11008), one matrix per shape
    per_layer_cpu = 4 * by["cfg2"]["cpu_s"] + 2 * by["cfg4_tall"]["cpu_s"] + by["cfg3"]["cpu_s"]
    summary = {"cfg4_cpu_extrapolated_s": 32 * per_layer_cpu,
               "cfg4_note": "CPU: one matrix per shape x 32 layers (4096x11008 timed with cfg3's diag H); GPU: "
                            "tools/bench_model.py (batched, interleaved)",
               "cpu_threads": torch.get_num_threads(), "cpu_kind": "port (numpy/LAPACK oracle)"}
    print(json.dumps(summary), flush=True)


if __name__ == "__main__":
    main()
