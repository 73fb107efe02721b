"""Micro-benchmark of the split-fp16 (f16x3) filter GEMM vs the fp32 MFMA GEMM on the
solver's shape: C^T (p x k) = X^T G for a batch of k x k symmetric G (k = 4096)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ee274_convexcaldera_llm_quantization_amd._lib as K

dev = "cuda:0"
K.load()


def bench(name, fn, flops, n=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"{name:50s} {ms:8.3f} ms {flops / ms / 1e9:8.1f} TFLOP/s (fp32-equivalent)", flush=True)
    return ms


B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
k = 4096
Y = torch.randn(B, k, k, device=dev) * 0.05
G = torch.empty(B, k, k, device=dev)
K.gemm(Y, Y, tb=True, C=G, syrk=True)
del Y
xs = 2.0 ** 6
Gh, Gl, gs, inv = K.sym_split_f16(G, xs, blocked=True)
for p in (192, 256, 384):
    X = torch.linalg.qr(torch.randn(B, k, p, device=dev))[0].contiguous()
    Xt = torch.empty(B, p, k, device=dev)
    Xh = torch.empty(B, p, k, device=dev, dtype=torch.float16); Xl = torch.empty_like(Xh)
    K.transpose_split(X, out=Xt, hi=Xh, lo=Xl, scale=xs)
    Ct = torch.empty(B, p, k, device=dev)
    Oh = torch.empty_like(Xh); Ol = torch.empty_like(Xh)
    ovf = torch.zeros(B, dtype=torch.int32, device=dev)
    a = torch.full((B,), 0.5, device=dev); b = torch.full((B,), -0.25, device=dev); c = torch.full((B,), 0.1, device=dev)
    fl = 2 * k * k * p * B
    bench(f"x3  C^T = X^T G  p={p}", lambda: K.gemm_x3(Xh, Xl, Gh, Gl, inv, Ct, b_blocked=True), fl)
    bench(f"x3  + cheb epilogue + split p={p}", lambda: K.gemm_x3(Xh, Xl, Gh, Gl, inv, Ct, P=Ct, D=Xt, alpha_v=a,
                                                               beta_v=b, gamma_v=c, out_h=Oh, out_l=Ol,
                                                               out_scale=xs, overflow=ovf, b_blocked=True), fl)
    Xhb = Xh.view(B, p, k // 32, 32).permute(0, 2, 1, 3).contiguous().view(B, p, k)
    Xlb = Xl.view(B, p, k // 32, 32).permute(0, 2, 1, 3).contiguous().view(B, p, k)
    bench(f"x3  A and B K-blocked p={p}", lambda: K.gemm_x3(Xhb, Xlb, Gh, Gl, inv, Ct, b_blocked=True, a_blocked=True), fl)
    Ctb = torch.empty_like(Ct)
    K.gemm_x3(Xhb, Xlb, Gh, Gl, inv, Ctb, b_blocked=True, a_blocked=True)
    K.gemm_x3(Xh, Xl, Gh, Gl, inv, Ct, b_blocked=True)
    print("   blocked-A result identical:", torch.equal(Ct, Ctb), flush=True)
    C = torch.empty(B, k, p, device=dev)
    bench(f"f32 G X ta  p={p}", lambda: K.gemm(G, X, ta=True, C=C), fl)
    K.gemm_x3(Xh, Xl, Gh, Gl, inv, Ct, b_blocked=True)
    K.gemm(G, X, ta=True, C=C)
    ref = torch.matmul(G.double(), X.double())
    e3 = ((Ct.transpose(1, 2).double() - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
    e32 = ((C.double() - ref).norm(dim=1) / ref.norm(dim=1)).max().item()
    print(f"   max column rel err: x3 {e3:.3e}   fp32 {e32:.3e}", flush=True)
bench("sym_split_f16 blocked", lambda: K.sym_split_f16(G, xs, hi=Gh, lo=Gl, scale=gs, inv_scale=inv, blocked=True), 0.0 + 1)
