"""Config 4 (BASELINE.json configs[3]): Llama-2-7B's linear weights (random-init fp16, the
survey's per-matrix seeds) decomposed by the MI355X engine, matrix-sharded round-robin over
the ranks, packed results gathered to rank 0 (sharding.py).  Secondary measurement (the
headline bench is config 2 in bench.py).

  python tools/bench_model.py --layers 4            # one GPU: 28 matrices = one rank's share at 8 GPUs
  torchrun --nproc-per-node N tools/bench_model.py --layers 32

Weights are generated before the timed region (on the host with the survey's recipe, then
copied to HBM); the timed region is decomposition + packing + (N > 1) the RCCL gather."""
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
from src.caldera.utils.dataclasses import CalderaParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--max-batch", type=int, default=16)
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--sequential", action="store_true",
                    help="one batch after another (default: all shape batches at once, each engine on "
                         "its own HIP stream, overlap.py)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    items = S.llama2_7b_matrices(args.layers)
    mine = [items[i] for i in S.shard_indices(len(items), world, rank)]
    qp = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, update_order=["Q", "LR"], sigma_reg=1e-8)
    by_shape = {}
    for it in mine:
        by_shape.setdefault((it[1], it[2]), []).append(it)
    batches = []
    for shape, grp in by_shape.items():  # weights: survey recipe per seed, resident in HBM
        for s in range(0, len(grp), args.max_batch):
            part = grp[s:s + args.max_batch]
            ws = []
            for name, m, n, seed in part:
                torch.manual_seed(seed)
                ws.append((torch.randn(m, n) * 0.02).to(torch.float16))
            batches.append((part, torch.stack(ws).to(dev)))
    eng_params = EngineParams.from_caldera_params(qp)
    # warm-up: one small decomposition per shape class compiles nothing (AOT kernels) but
    # primes the allocator and the HIP module
    CalderaEngine(eng_params).run(batches[0][1][:1])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    results = []
    per_shape = {}
    if not args.sequential:
        from ee274_convexcaldera_llm_quantization_amd.overlap import run_interleaved
        engines = [CalderaEngine(eng_params) for _ in batches]
        run_interleaved([e.run_iter(W) for e, (_, W) in zip(engines, batches)], dev)
        for eng, (part, W) in zip(engines, batches):
            for (name, m, n, seed), d in zip(part, eng.last_packed):
                results.append(S.MatrixResult(name, m, n, d["L"].shape[1], qp.Q_bits, d["codes"], d["Q_scale"],
                                              d["L"], d["R"], d["global_scale"], d["errors"]))
        torch.cuda.synchronize()
        batches_seq = []
    else:
        batches_seq = batches
    for part, W in batches_seq:
        ts = time.perf_counter()
        eng = CalderaEngine(eng_params)
        eng.run(W)
        for (name, m, n, seed), d in zip(part, eng.last_packed):
            results.append(S.MatrixResult(name, m, n, d["L"].shape[1], qp.Q_bits, d["codes"], d["Q_scale"],
                                          d["L"], d["R"], d["global_scale"], d["errors"]))
        torch.cuda.synchronize()
        key = f"{part[0][1]}x{part[0][2]}"
        per_shape[key] = per_shape.get(key, 0.0) + time.perf_counter() - ts
    gathered = None
    if world > 1 and not args.no_gather:
        payload = S.pack_results(results)
        gathered = S.gather_to_rank0(payload, device=dev)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    tmax = torch.tensor([dt], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    if rank == 0:
        n_all = len(items)
        if gathered is not None:
            got = sum(len(S.unpack_results(p)) for p in gathered)
            assert got == n_all, (got, n_all)
        print(json.dumps({"workload": "BASELINE configs[3]: Llama-2-7B linear weights (random-init fp16), r=128, Q2, "
                                      "L/R 16, iters 5, H=I",
                          "layers": args.layers, "interleave": not args.sequential, "matrices": n_all, "n_gpus": world, "seconds": float(tmax.item()),
                          "matrices_per_s": n_all / float(tmax.item()),
                          "rank0_seconds_by_shape": per_shape,
                          "extrapolated_full_model_s_at_this_world": float(tmax.item()) * 32 / args.layers,
                          "frob_err_last": {r.name: r.errors["LR"][-1] for r in results[:3]}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
