"""Probe: is the filter product G X^T (gemm_x3v, 192 x 384 tiles, B = 256, k = 4096) bound by
HBM or by the per-CU LDS-DMA intake?  Times the product with 256 distinct G (streamed from
HBM) against the same launch with every matrix pointing at ONE G (stride 0: its panels come
from L2 / MALL), for the split (3-product), exact-B and single-product loops."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ee274_convexcaldera_llm_quantization_amd._lib as K

dev = "cuda:0"
lib = K.load()
B, k, p = int(sys.argv[1]) if len(sys.argv) > 1 else 256, 4096, 192
g = torch.Generator(device=dev).manual_seed(0)
Gh = (torch.randn(B, k, k, device=dev, generator=g) * 0.01).half()
Gl = (torch.randn(B, k, k, device=dev, generator=g) * 1e-5).half()
Xh = (torch.randn(B, p, k, device=dev, generator=g)).half()
Xl = (torch.randn(B, p, k, device=dev, generator=g) * 1e-3).half()
C = torch.empty(B, p, k, device=dev)
inv = torch.full((B,), 2.0 ** -20, device=dev)


def launch(shared, mode):
    a = K.X3Args()
    a.M, a.N, a.K, a.batch = p, k, k, B
    a.Ah, a.Al, a.lda, a.stride_a = Xh.data_ptr(), Xl.data_ptr(), k, p * k
    a.Bh, a.Bl, a.ldb, a.stride_b = Gh.data_ptr(), Gl.data_ptr(), k, 0 if shared else k * k
    a.inv_scale = inv.data_ptr()
    a.C, a.ldc, a.stride_c = C.data_ptr(), k, p * k
    a.b_blocked = 1
    a.single = int(mode == "single")
    a.b_exact = int(mode == "exact")
    K._check(lib.cq_gemm_x3(ctypes.byref(a), K._stream(torch.device(dev))), "cq_gemm_x3")


def bench(fn, n=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


print(f"CQ_X3_NT={os.environ.get('CQ_X3_NT', '(default)')}  B={B} p={p} k={k}", flush=True)
for mode, gb in (("split", 4.0), ("exact", 2.0), ("single", 2.0)):
    for shared in (False, True):
        ms = bench(lambda: launch(shared, mode))
        hbm = (gb * k * k * (1 if shared else B) + (4.0 if mode != "single" else 2.0) * p * k * B + 4.0 * p * k * B) / 1e9
        intake = (gb * k * k + (4.0 if mode != "single" else 2.0) * p * k * 11) * B / 1e9
        print(f"{mode:7s} shared_G={int(shared)}  {ms:7.3f} ms   HBM~{hbm / ms:6.2f} TB/s   "
              f"CU intake {intake / ms / 256 * 1e3:6.1f} GB/s per CU", flush=True)
