"""GPU micro-benchmark of the sparse-code Gram (sgram.py) at the bench shape: B x 4096 x 4096
fp16 W, 2-bit codes of W itself (~0.8 % nonzero, as at config 2), per phase with HIP events:
count (+ host read-back), ELL fill, sparse product P, combine (G's split halves); and the dense
split-fp16 Gram of Y it replaces.

  python tools/bench_sgram.py [B] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
import torch  # noqa: E402

import ee274_convexcaldera_llm_quantization_amd._lib as K  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd import scratch, sgram  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd.solver import X3_SCALE  # noqa: E402

dev = "cuda:0"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
m = n = 4096
g = torch.Generator(device=dev).manual_seed(0)
W = torch.empty(B, m, n, device=dev, dtype=torch.float16)
for b in range(B):
    W[b] = torch.randn(m, n, device=dev, generator=g).half()
packed = torch.empty(B, m * n // 4, dtype=torch.uint8, device=dev)
s = torch.empty(B, device=dev)
K.q_update_x3(W, None, None, 2, packed=packed, scale=s)
wmax = K.absmax(W)
A = torch.empty(B, m, m, device=dev)
Gh = torch.empty(B, m, m, device=dev, dtype=torch.float16)
Gl = torch.empty_like(Gh)
yh = torch.empty(B, m, n, device=dev, dtype=torch.float16)
yl = torch.empty_like(yh)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]


def timed(f, r=reps):
    f()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(r):
        f()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / r


t_a = timed(lambda: sgram.gram_A(W, None, 1.0, wmax, A, Gh, Gl, X3_SCALE, yh, yl), 1)
print(f"A = W W^T (split Gram of W, once per run): {t_a:.2f} ms", flush=True)
ysq = torch.full((B,), float(m * n), dtype=torch.float64, device=dev)
gs = torch.empty(B, device=dev)
gi = torch.empty(B, device=dev)
SG = sgram.SparseGram(B, m, n, dev)
SG.count(packed)
print(f"ELL density {SG.density:.4%}", flush=True)
stride = -(-int(max(sgram.MAX_DENSITY, SG.density) * m * n) // 4096) * 4096
ell = scratch.get("sgram.ell", (B * stride,), torch.int32, dev)
P = scratch.get("sgram.P", (B, m, m), torch.float32, dev)
t_c = timed(lambda: K.sgram_count(packed, m, n, SG.row_nnz, SG.perm, SG.slice_off, SG.total))
t_f = timed(lambda: K.sgram_fill(packed, m, n, SG.row_nnz, SG.perm, SG.slice_off, ell, stride))
t_p = timed(lambda: K.sgram_spmm(W, packed, s, None, ell, SG.perm, SG.slice_off, stride, P))
t_g = timed(lambda: K.sgram_combine(A, P, s, ysq, X3_SCALE, Gh, Gl, gs, gi))
t_all = timed(lambda: SG.gram(W, packed, s, None, A, ysq, Gh, Gl, gs, gi, X3_SCALE))
print(f"count {t_c:.3f} ms  fill {t_f:.3f} ms  spmm {t_p:.3f} ms  combine {t_g:.3f} ms  "
      f"whole sparse Gram (with read-back) {t_all:.3f} ms", flush=True)
nz = SG.density * m * n * B
print(f"spmm: {2 * nz * m / t_p / 1e9:.1f} GFLOP/s fp32 over the ELL entries; combine "
      f"{B * m * m * (4 + 4 + 4) / 2 / t_g / 1e6 + B * m * m * 4 / t_g / 1e6:.0f} GB/s algorithmic", flush=True)
ys = torch.empty(B, device=dev)
K.residual_split(W, packed, s, 2, wmax, hi=yh, lo=yl, scale=ys)
t_d = timed(lambda: K.gemm_x3(yh, yl, yh, yl, 1.0 / (ys * ys), None, tri=True, a_blocked=True, b_blocked=True,
                              out_h=Gh, out_l=Gl, out_scale=X3_SCALE, sym_bound=ysq, scale_out=gs, inv_out=gi))
print(f"dense split-fp16 Gram of Y: {t_d:.3f} ms", flush=True)
