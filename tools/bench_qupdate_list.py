"""GPU micro-benchmark of the 2-bit Q-with-LR update at the bench shape (B x 4096 x 4096 fp16
W, r = 128): the two-pass form (absmax pass + quantise pass, each recomputing L R) against
the single-recompute list path (scale_hint given: pass 2 + qp_codes_kernel), HIP events per
call; the packed codes and scales of both must be identical.  Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split.

  python tools/bench_qupdate_list.py [B] [reps] [--lib path/to/libcaldera_hip.so]
(--lib: another build of the library, e.g. tools/probes/build_rev.sh HEAD base, for an A/B on one box)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
import torch  # noqa: E402

import ee274_convexcaldera_llm_quantization_amd._lib as K  # noqa: E402

dev = "cuda:0"
lib = None
if "--lib" in sys.argv:
    i = sys.argv.index("--lib")
    lib = sys.argv[i + 1]
    del sys.argv[i:i + 2]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
m = n = 4096
r = 128
K.load() if lib is None else K.load(lib)
print("library:", lib or K.LIB_PATH)
g = torch.Generator(device=dev).manual_seed(0)
W = (torch.randn(B, m, n, device=dev, generator=g) * 0.5).half()
L = (torch.randn(B, m, r, device=dev, generator=g) / m ** 0.5).contiguous()  # ~orthonormal columns (no solver call: rocprofv3 --pmc and hipsolver do not mix)
R = (torch.randn(B, r, n, device=dev, generator=g) * 0.05).contiguous()
outs = {}
for tag in ("two-pass", "list"):
    packed = torch.empty(B, m * n // 4, dtype=torch.uint8, device=dev)
    sc = torch.empty(B, device=dev)
    err = torch.empty(B, dtype=torch.float64, device=dev)
    fb = torch.zeros(B, dtype=torch.int32, device=dev)
    K.q_update_x3(W, L, R, 2, packed=packed, scale=sc, err_out=err)   # scales for the hint
    hint = sc.clone() if tag == "list" else None
    K.q_update_x3(W, L, R, 2, packed=packed, scale=sc, err_out=err, scale_hint=hint, fallback_out=fb)
    torch.cuda.synchronize()
    outs[tag] = (packed.clone(), sc.clone(), err.clone())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        K.q_update_x3(W, L, R, 2, packed=packed, scale=sc, err_out=err, scale_hint=hint, fallback_out=fb)
    e1.record()
    torch.cuda.synchronize()
    print(f"{tag:9s} {e0.elapsed_time(e1) / reps:7.3f} ms per B = {B} call (incl. factor splits); "
          f"fallbacks {int(fb.sum())}", flush=True)
a, b = outs["two-pass"], outs["list"]
print("codes identical:", torch.equal(a[0], b[0]), " scales identical:", torch.equal(a[1], b[1]),
      " max rel err diff: %.2e" % float(((a[2] - b[2]).abs() / a[2]).max()))
