"""GPU micro-benchmark of the solver's symmetric Gram (split-fp16 Y Y^T, upper tiles, K-blocked
split halves of G written mirrored) at the bench shape: B x 4096 x 4096, timed with HIP events
for the current library and the round-2 library (tools/ab/libcaldera_hip_r02.so) on the same
inputs; the G halves of both must be bit-identical (the tile order is the only difference).

  python tools/bench_gram.py [B] [reps]"""
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
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
k = 4096
K.load()
g = torch.Generator(device=dev).manual_seed(0)
Yh = torch.empty(B, k, k, device=dev, dtype=torch.float16)
Yl = torch.empty_like(Yh)
for b in range(B):
    y = torch.randn(1, k, k, device=dev, generator=g) * 0.05
    hs = (y * 64.0).half()
    Yh[b].copy_(hs[0].view(k, k // 32, 32).permute(1, 0, 2).reshape(k, k))
    Yl[b].copy_(((y * 64.0) - hs.float()).half()[0].view(k, k // 32, 32).permute(1, 0, 2).reshape(k, k))
del y, hs
inv = torch.full((B,), 1.0 / 64.0 / 64.0, device=dev)
bound = torch.full((B,), float(k) * k * 0.05 ** 2 * 4, device=dev, dtype=torch.float64)
Gh = torch.empty(B, k, k, device=dev, dtype=torch.float16)
Gl = torch.empty_like(Gh)
so = torch.empty(B, device=dev)
io = torch.empty(B, device=dev)


def run_lib(lib, tag):
    K._lib = lib
    f = lambda: K.gemm_x3(Yh, Yl, Yh, Yl, inv, None, tri=True, a_blocked=True, b_blocked=True, sym_bound=bound,
                          scale_out=so, inv_out=io, out_h=Gh, out_l=Gl, out_scale=1.0)
    Gh.zero_(); Gl.zero_()
    f()
    torch.cuda.synchronize()
    digest = hashlib.sha256(Gh.view(torch.int16).sum(dim=(1, 2)).cpu().numpy().tobytes() +
                            Gl.view(torch.int16).sum(dim=(1, 2)).cpu().numpy().tobytes() +
                            Gh[0].cpu().numpy().tobytes() + Gl[-1].cpu().numpy().tobytes()).hexdigest()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fl = 3 * 2 * k * k * k / 2 * B
    print(f"{tag:8s} gram {ms:8.3f} ms per B = {B} launch  {fl / ms / 1e9:.0f} TFLOP/s fp16 (upper half)", flush=True)
    return digest


cur = K._lib
d_new = run_lib(cur, "current")
same = True
for alt in os.environ.get("AB_LIB", "libcaldera_hip_r02.so").split(","):
    old = ctypes.CDLL(os.path.join(ROOT, "tools", "ab", alt))
    for name, (res, args) in K._SIGS.items():
        if hasattr(old, name):
            getattr(old, name).restype, getattr(old, name).argtypes = res, args
    d_old = run_lib(old, alt.replace("libcaldera_hip_", "").replace(".so", ""))
    same &= d_new == d_old
K._lib = cur
print("identical outputs:", same, flush=True)
sys.exit(0 if same else 1)
