"""GPU micro-benchmark of the fused Q-with-LR update at the bench shape: B x 4096 x 4096 fp16 W,
r = 128 split-fp16 factors, 2-bit codes (cq_q_update_x3: absmax pass + quantise pass), timed
with HIP events for the current library and for the round-2 library (tools/ab/
libcaldera_hip_r02.so) in the same process, on the same inputs; the packed codes, scales and
error sums of both must be identical.

  python tools/bench_qupdate_lr.py [B] [reps]"""
import ctypes
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
import torch  # noqa: E402

import ee274_convexcaldera_llm_quantization_amd._lib as K  # noqa: E402

dev = "cuda:0"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
m = n = 4096
r = 128
K.load()
g = torch.Generator(device=dev).manual_seed(0)
W = torch.randn(B, m, n, device=dev, generator=g).half()
L = torch.linalg.qr(torch.randn(B, m, r, device=dev, generator=g))[0].contiguous()
R = (torch.randn(B, r, n, device=dev, generator=g) * 2.0).contiguous()
packed = torch.empty(B, m * n // 4, dtype=torch.uint8, device=dev)
sc = torch.empty(B, device=dev)
err = torch.empty(B, dtype=torch.float64, device=dev)


def run_lib(lib, tag):
    K._lib = lib
    K.q_update_x3(W, L, R, 2, packed=packed, scale=sc, err_out=err)
    torch.cuda.synchronize()
    digest = (hashlib.sha256(packed.cpu().numpy().tobytes()).hexdigest(), sc.cpu().tolist(), err.cpu().tolist())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        K.q_update_x3(W, L, R, 2, packed=packed, scale=sc, err_out=err)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{tag:8s} {ms:7.3f} ms per B = {B} call (both passes, incl. factor splits)", flush=True)
    return digest


cur = K._lib
d_new = run_lib(cur, "current")
old = ctypes.CDLL(os.path.join(ROOT, "tools", "ab", "libcaldera_hip_r02.so"))
for name, (res, args) in K._SIGS.items():
    if hasattr(old, name):
        getattr(old, name).restype, getattr(old, name).argtypes = res, args
d_old = run_lib(old, "round-2")
K._lib = cur
print("identical outputs:", d_new == d_old, flush=True)
sys.exit(0 if d_new == d_old else 1)
