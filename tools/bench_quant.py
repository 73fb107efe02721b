"""Micro-benchmark of the quantise kernels at the bench shape (B x 4096 x 4096 fp16 W, 2-bit):
the first-Q streaming pass (max|W| known) with/without the error weights and error output,
and the standalone absmax pass."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import ee274_convexcaldera_llm_quantization_amd._lib as K

dev = "cuda:0"
K.load()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
m = n = 4096
g = torch.Generator(device=dev).manual_seed(0)
W = (torch.randn(B, m, n, device=dev, generator=g) * 0.02).half()
amax = K.absmax(W)
packed = torch.empty(B, m * n // 4, dtype=torch.uint8, device=dev)
sc = torch.empty(B, device=dev)
err = torch.empty(B, dtype=torch.float64, device=dev)
ew = torch.ones(n, device=dev)


def bench(name, fn, nbytes, n=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"{name:55s} {ms:7.3f} ms  {nbytes / ms / 1e6:7.0f} GB/s", flush=True)


bq = B * (2 * m * n + m * n // 4)
bench("stream quantise (known max), err + weights", lambda: K.q_update_x3(W, None, None, 2, packed=packed, scale=sc,
      err_w=ew, err_out=err, absmax_in=amax), bq)
bench("stream quantise (known max), err, no weights", lambda: K.q_update_x3(W, None, None, 2, packed=packed, scale=sc,
      err_out=err, absmax_in=amax), bq)
bench("stream quantise (known max), no err", lambda: K.q_update_x3(W, None, None, 2, packed=packed, scale=sc,
      absmax_in=amax), bq)
bench("two-pass fused (r = 0)", lambda: K.q_update_x3(W, None, None, 2, packed=packed, scale=sc, err_w=ew,
      err_out=err), bq)
bench("absmax pass", lambda: K.absmax(W), B * 2 * m * n)
bench("torch W.float().abs().amax()", lambda: W.view(B, -1).abs().amax(1), B * 2 * m * n, n=3)
