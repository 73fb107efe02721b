"""Child process of tests/test_gpu_rccl.py: a world-1 "nccl" (RCCL) process group initialised
before any other GPU call, then the sharded decomposition of two real matrices on the HIP
engine, the packed payload gathered to rank 0 over RCCL (HBM -> HBM), and the gathered
results compared byte for byte with the direct ones, and the same payload once more through the
asynchronous gather bench.py's N > 1 steps use.  Prints one JSON line; exit code 0 = equal."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dev = torch.device("cuda", 0)
    # the process group first: RCCL sees a device no kernel has touched yet
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        from ee274_convexcaldera_llm_quantization_amd import sharding as S
        from src.caldera.utils.dataclasses import CalderaParams
        qp = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=32, iters=2, update_order=["Q", "LR"],
                           sigma_reg=1e-8)
        items = [("model.layers.0.self_attn.q_proj", 512, 1024, 0), ("model.layers.0.self_attn.k_proj", 512, 1024, 1)]
        run = S.engine_decompose_batch(qp, dev)
        direct = S.decompose_sharded(items, run, rank=0, world=1, max_batch=2, device=dev)
        assert direct[0].L.is_cuda, "results must live in HBM"
        payloads = S.gather_to_rank0(S.pack_results(direct, device=dev), device=dev)
        assert payloads is not None and len(payloads) == 1 and payloads[0].is_cuda
        got = S.unpack_results(payloads[0])
        ok = [r.name for r in got] == [r.name for r in direct]
        for a, b in zip(direct, got):
            for x, y in ((a.codes, b.codes), (a.L, b.L), (a.R, b.R)):
                ok &= torch.equal(x.contiguous().view(-1).view(torch.uint8), y.contiguous().view(-1).view(torch.uint8))
            ok &= a.Q_scale == b.Q_scale and a.global_scale == b.global_scale and a.errors == b.errors
        # the asynchronous form bench.py's N > 1 steps use (round 6): issued, the payload reused
        # at once, compute queued behind it on the default stream, then retired stream-ordered
        pk = S.pack_results(direct, device=dev)
        ref = pk.clone()
        pend = S.gather_to_rank0_async(pk, device=dev, sizes=[pk.numel()])
        pk.zero_()
        x = torch.randn(2048, 2048, device=dev)
        y = x @ x   # noqa: F841  (compute beside the transfer)
        got2 = pend.wait()
        ok &= got2 is not None and len(got2) == 1 and torch.equal(got2[0], ref)
        torch.cuda.synchronize()
        print(json.dumps({"backend": dist.get_backend(), "world": dist.get_world_size(), "equal": bool(ok),
                          "payload_bytes": int(payloads[0].numel()), "matrices": len(got)}), flush=True)
        return 0 if ok else 1
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
