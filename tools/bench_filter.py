"""Micro-benchmark of the solver's split-fp16 products at the bench shape (k = 4096, p = 192):
the Chebyshev filter step (blocked A/B, recurrence epilogue, blocked split output), the
upper-triangle Gram Y Y^T, and the fused Q update.  Run once per kernel variant:
    CQ_X3_KERNEL=w2 python tools/bench_filter.py 128     # 2-stage ring (BK 32)
    python tools/bench_filter.py 128                     # default kernel
    python tools/bench_filter.py 256 --lib tools/probes/lib_x.so   # another build (A/B on one box)
Prints ms per launch and the filter's algorithmic GB/s."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ee274_convexcaldera_llm_quantization_amd._lib as K

dev = "cuda:0"
_lib = None
if "--lib" in sys.argv:
    _i = sys.argv.index("--lib")
    _lib = sys.argv[_i + 1]
    del sys.argv[_i:_i + 2]
K.load() if _lib is None else K.load(_lib)


CLOCK = bool(os.environ.get("CQ_X3_CLOCK"))


def bench(fn, n=10):
    fn(); torch.cuda.synchronize()
    if CLOCK:
        K.x3_clock()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record(); torch.cuda.synchronize()
    if CLOCK:
        sh, rt = K.x3_clock()
        if rt:
            print(f"   avg shader clock over the workgroups: {sh / rt * 0.1:.3f} GHz", flush=True)
    return e0.elapsed_time(e1) / n


B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
k, p, xs = 4096, 192, 2.0 ** 6
tag = os.environ.get("CQ_X3_KERNEL", os.path.basename(_lib) if _lib else "default")
g = torch.Generator(device=dev).manual_seed(0)
Gh = torch.empty(B, k, k, device=dev, dtype=torch.float16)
Gl = torch.empty_like(Gh)
inv = torch.full((B,), 1.0 / xs / xs, device=dev)
for b in range(B):  # symmetric G, built one matrix at a time (bounded memory)
    Y = torch.randn(k, k // 4, device=dev, generator=g) * 0.05
    Gb = (Y @ Y.T).unsqueeze(0)
    h, l, _, _ = K.sym_split_f16(Gb, xs, blocked=True)
    Gh[b].copy_(h[0]); Gl[b].copy_(l[0])
del Y, Gb, h, l
X = torch.randn(B, k, p, device=dev, generator=g) / k ** 0.5
Xt = torch.empty(B, p, k, device=dev)
Xh = torch.empty(B, p, k, device=dev, dtype=torch.float16); Xl = torch.empty_like(Xh)
K.transpose_split(X, out=Xt, hi=Xh, lo=Xl, scale=xs, blocked=True)
Ct = torch.empty(B, p, k, device=dev)
Oh = torch.empty_like(Xh); Ol = torch.empty_like(Xh)
ovf = torch.zeros(B, dtype=torch.int32, device=dev)
a = torch.full((B,), 0.5, device=dev); bb = torch.full((B,), -0.25, device=dev); c = torch.full((B,), 0.1, device=dev)
Pv = Xt.clone()
filt = lambda: K.gemm_x3(Xh, Xl, Gh, Gl, inv, Ct, P=Pv, D=Xt, alpha_v=a, beta_v=bb, gamma_v=c, out_h=Oh, out_l=Ol,
                         out_scale=xs, overflow=ovf, b_blocked=True, a_blocked=True, o_blocked=True)
ms = bench(filt)
by = B * (4 * k * k + 20 * p * k)
print(f"[{tag}] filter B={B}: {ms:.3f} ms/launch  {by / ms / 1e6:.0f} GB/s algorithmic  "
      f"{2 * 3 * k * k * p * B / ms / 1e9:.0f} TFLOP/s fp16", flush=True)
plain = lambda: K.gemm_x3(Xh, Xl, Gh, Gl, inv, Ct, b_blocked=True, a_blocked=True)
ms2 = bench(plain)
print(f"[{tag}] plain X^T G B={B}: {ms2:.3f} ms/launch", flush=True)
single = lambda: K.gemm_x3(Xh, Xl, Gh, Gl, inv, Ct, P=Pv, D=Xt, alpha_v=a, beta_v=bb, gamma_v=c, out_h=Oh, out_l=Ol,
                           out_scale=xs, overflow=ovf, b_blocked=True, a_blocked=True, o_blocked=True, single=True)
ms6 = bench(single)
print(f"[{tag}] single-product filter B={B}: {ms6:.3f} ms/launch  "
      f"{B * (2 * k * k + 20 * p * k) / ms6 / 1e6:.0f} GB/s algorithmic", flush=True)
if tag.startswith("w4"):
    def reblock(t, n, kk):  # 32-blocked -> 16-blocked
        return t.view(-1, kk // 32, n, 32).permute(0, 2, 1, 3).reshape(-1, n, kk // 16, 16).permute(0, 2, 1, 3).contiguous().view(-1, n, kk)
    Gh16, Gl16 = reblock(Gh, k, k), reblock(Gl, k, k)
    Xh16, Xl16 = reblock(Xh, p, k), reblock(Xl, p, k)
    C16 = torch.empty_like(Ct)
    p16 = lambda: K.gemm_x3(Xh16, Xl16, Gh16, Gl16, inv, C16, b_blocked=2, a_blocked=2)
    ms5 = bench(p16)
    print(f"[{tag}] plain X^T G 16-blocked B={B}: {ms5:.3f} ms/launch  identical={torch.equal(C16, Ct)}", flush=True)
    del Gh16, Gl16, Xh16, Xl16, C16
# Gram of Y (m = n = k): upper-triangle tiles, K-blocked halves on both sides
Gout = torch.empty(B // 4, k, k, device=dev)
gram = lambda: K.gemm_x3(Gh[: B // 4], Gl[: B // 4], Gh[: B // 4], Gl[: B // 4], inv[: B // 4], Gout, tri=True,
                         a_blocked=True, b_blocked=True)
ms3 = bench(gram, n=3)
print(f"[{tag}] gram B={B // 4}: {ms3:.3f} ms/launch  {3 * k ** 3 * (B // 4) / ms3 / 1e9:.0f} TFLOP/s fp16 "
      f"(upper half)", flush=True)
ref = torch.empty_like(Ct)
filt(); torch.cuda.synchronize()
print(f"[{tag}] checksum {float(Ct.double().abs().sum()):.10e} {float(Oh.float().abs().sum()):.10e}", flush=True)
# fused Q update (two passes over W, K = r = 128)
del Gout
W = (torch.randn(B, k, k, device=dev, generator=g) * 0.02).half()
L = torch.randn(B, k, 128, device=dev, generator=g) * 0.01
R = torch.randn(B, 128, k, device=dev, generator=g) * 0.01
packed = torch.empty(B, k * k // 4, dtype=torch.uint8, device=dev)
qs = torch.empty(B, device=dev)
qe = torch.empty(B, dtype=torch.float64, device=dev)
qu = lambda: K.q_update_x3(W, L, R, 2, packed=packed, scale=qs, err_out=qe)
ms4 = bench(qu, n=5)
print(f"[{tag}] q_update B={B}: {ms4:.3f} ms/call (incl. factor splits)  "
      f"{B * (2 * k * k + k * k // 4) / ms4 / 1e6:.0f} GB/s (bytes_Q)", flush=True)
print(f"[{tag}] q checksum {int(packed.long().sum())} {float(qs.double().sum()):.10e} {float(qe.sum()):.10e}", flush=True)
