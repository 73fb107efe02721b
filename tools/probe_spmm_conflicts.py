"""Probe (no product change): how much of the sparse-Gram SpMM is LDS bank conflicts?  Times
sgram_spmm on the real ELL of the bench shape and on the same ELL with every entry's column
moved to residue (lane mod 16) of its own 16-column block -- the same entry count, FMAs and ELL
loads, but every ds_read_b128 group of a step on 16 different bank slots (results wrong by
design; timing only).

  python tools/probe_spmm_conflicts.py [B] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
import torch  # noqa: E402

import ee274_convexcaldera_llm_quantization_amd._lib as K  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd import scratch, sgram  # noqa: E402

dev = "cuda:0"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
for (m, n) in ((4096, 4096), (4096, 11008)):
    g = torch.Generator(device=dev).manual_seed(0)
    W = torch.empty(B, m, n, device=dev, dtype=torch.float16)
    for b in range(B):
        W[b] = (torch.randn(m, n, device=dev, generator=g) * 0.02).half()
    packed = torch.empty(B, m * n // 4, dtype=torch.uint8, device=dev)
    s = torch.empty(B, device=dev)
    K.q_update_x3(W, None, None, 2, packed=packed, scale=s)
    SG = sgram.SparseGram(B, m, n, dev)
    SG.count(packed)
    stride = -(-int(max(sgram.MAX_DENSITY, SG.density) * m * n) // 4096) * 4096
    ell = scratch.get("sgram.ell", (B * stride,), torch.int32, dev)
    P = scratch.get("sgram.P", (B, m, m), torch.float32, dev)
    K.sgram_fill(packed, m, n, SG.row_nnz, SG.perm, SG.slice_off, ell, stride)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timed(f):
        f()
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(reps):
            f()
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / reps

    t0 = timed(lambda: K.sgram_spmm(W, packed, s, None, ell, SG.perm, SG.slice_off, stride, P))
    lane = (torch.arange(ell.numel(), device=dev, dtype=torch.int32) % 64) & 15
    col = ell >> 2
    ell2 = (((col & ~15) | lane) << 2) | (ell & 3)
    t1 = timed(lambda: K.sgram_spmm(W, packed, s, None, ell2, SG.perm, SG.slice_off, stride, P))
    # the same with 32 residues (8-byte slab entries: ds_read_b64 over 32-lane groups)
    lane32 = (torch.arange(ell.numel(), device=dev, dtype=torch.int32) % 64) & 31
    ell3 = (((col & ~31) | lane32) << 2) | (ell & 3)
    t2 = timed(lambda: K.sgram_spmm(W, packed, s, None, ell3, SG.perm, SG.slice_off, stride, P))
    print(f"{m}x{n} B={B} density {SG.density:.4%}: spmm real ELL {t0:.3f} ms, residue = lane mod 16 "
          f"{t1:.3f} ms, residue = lane mod 32 {t2:.3f} ms", flush=True)
    del W, packed, SG, P, ell, ell2, ell3, col, lane, lane32
    scratch.release()
    torch.cuda.empty_cache()
