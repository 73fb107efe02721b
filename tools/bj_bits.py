"""GPU tool: SHA-256 and time of a small-batch block-Jacobi eigensolve (the single-call path:
B = 1 and 2, p = 192 and 288, values and vectors) so two builds can be compared bit for bit
(--lib loads another build: tools/probes/build_rev_lib.sh)."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import ee274_convexcaldera_llm_quantization_amd._lib as K  # noqa: E402

lib = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else None
K.load() if lib is None else K.load(lib)
tag = os.path.basename(lib) if lib else "tree"
dev = "cuda:0"
for B, p in ((1, 192), (2, 192), (1, 288)):
    g = torch.Generator(device=dev).manual_seed(7 + p)
    X = torch.randn(B, 2048, p, device=dev, dtype=torch.float64, generator=g)
    A0 = X.transpose(1, 2) @ X
    outs = []
    for it in range(4):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        bj = K.BlockJacobi(A0.clone(), 1e-7, True)
        bj.launch(6, begin=True)
        while bj.pending_count() and bj.swept < 30:
            bj.launch(2)
        ev, V32, V64, sw = bj.finish()
        e1.record()
        torch.cuda.synchronize()
        outs.append(e0.elapsed_time(e1))
    h = hashlib.sha256(ev.cpu().numpy().tobytes() + V32.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"[{tag}] B={B} p={p} sweeps {sw.tolist()} sha {h} ms {sorted(outs)[1]:.3f}", flush=True)
