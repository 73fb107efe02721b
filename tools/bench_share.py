"""One rank's share of config 4 (BASELINE configs[3]) at world W, on one GPU: the 28 matrices
shard_indices(224, 8, r) gives rank r at 8 GPUs, batched and interleaved exactly as
bench.py --workload model --emulate-world does, plus the packing for the gather.  Steps are
separated by a 50 ms idle gap so a kernel trace (rocprofv3 --kernel-trace) splits into steps
(tools/timeline.py).

  python tools/bench_share.py [--world 8] [--rank 0] [--steps 3] [--warmup 1] [--group 4] [--max-batch 16]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd"))

from ee274_convexcaldera_llm_quantization_amd import sharding as S  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd.overlap import run_interleaved  # noqa: E402
import ee274_convexcaldera_llm_quantization_amd._lib as K  # noqa: E402
from src.caldera.utils.dataclasses import CalderaParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--max-batch", type=int, default=16)
    ap.add_argument("--group", type=int, default=4)
    ap.add_argument("--rr", action="store_true", help="plain round-robin interleaving (overlap.run_interleaved)")
    ap.add_argument("--no-splitk", action="store_true", help="_lib.AUTO_SPLIT_K = False (one-pass products)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    K.load()
    if args.no_splitk:
        K.AUTO_SPLIT_K = False
    qp = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, update_order=["Q", "LR"], sigma_reg=1e-8)
    ep = EngineParams.from_caldera_params(qp)
    items = S.llama2_7b_matrices(32)
    mine = [items[i] for i in S.shard_indices(len(items), args.world, args.rank)]
    Wd = {}
    for name, m, n, seed in mine:
        torch.manual_seed(seed)
        Wd[name] = (torch.randn(m, n) * 0.02).to(torch.float16).to(dev)

    def run_all(batches):
        res = []
        for g0 in range(0, len(batches), args.group):
            grp = batches[g0:g0 + args.group]
            engines = [CalderaEngine(ep) for _ in grp]
            run_interleaved([e.run_iter(torch.stack([Wd[it[0]] for it in b])) for e, b in zip(engines, grp)], dev,
                            ready_first=not args.rr)
            res += [S.MatrixResult(name, m, n, d["L"].shape[1], qp.Q_bits, d["codes"], d["Q_scale"], d["L"], d["R"],
                                   d["global_scale"], d["errors"])
                    for b, e in zip(grp, engines) for (name, m, n, _), d in zip(b, e.last_packed)]
        return res

    def dec(batch_items):
        return run_all([batch_items])
    dec.run_all = run_all

    def step():
        res = S.decompose_sharded(items, dec, rank=args.rank, world=args.world, max_batch=args.max_batch,
                                  gather=False, device=dev)
        return S.pack_results(res, device=dev)

    ts = []
    for i in range(args.warmup + args.steps):
        torch.cuda.synchronize()
        time.sleep(0.05)
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        if i >= args.warmup:
            ts.append(time.perf_counter() - t0)
    print(json.dumps({"world": args.world, "rank": args.rank, "matrices": len(mine), "max_batch": args.max_batch,
                      "group": args.group, "rr": args.rr, "no_splitk": args.no_splitk, "share_s": ts, "median_s": sorted(ts)[len(ts) // 2]}), flush=True)


if __name__ == "__main__":
    main()
