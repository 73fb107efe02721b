"""Build-container tool: the reference's own thread-count sensitivity on config 2 seeds.

Runs the unmodified reference caldera() (RCR alg.py:24-112, imported read-only) on the
bench's seed 0-3 matrices with 4 torch threads and compares Q + L R (16-column sketch)
with the golden runs in tests/golden/sum_large.npz (generated with 8 threads), plus the
number of Q codes that differ.  Output: JSON on stdout.
"""
import json
import os
import sys
import tempfile

import numpy as np
import torch

REF = "/root/reference/rank-constrained-regression-main"


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from src.caldera.decomposition import alg
    from src.caldera.utils.dataclasses import CalderaParams
    g = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "sum_large.npz"))
    os.chdir(tempfile.mkdtemp())
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    torch.set_num_threads(threads)
    om = np.random.default_rng(1234).standard_normal((4096, 16))
    out = {"threads": threads, "golden_threads": 8, "seeds": {}}
    for s in (0, 1, 2, 3):
        tag = "cfg2" if s == 0 else f"cfg2s{s}"
        torch.manual_seed(s)
        W = (torch.randn(4096, 4096) * 0.02).to(torch.float16)
        p = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, update_order=["Q", "LR"], sigma_reg=1e-8)
        d = alg.caldera(p, W, None, device="cpu", use_tqdm=False)
        sk = (d.Q.double() + d.L.double() @ d.R.double()).numpy() @ om
        ref = g[f"{tag}_sketch_QLR"]
        out["seeds"][s] = dict(rel_frob_QLR_vs_golden=float(np.linalg.norm(sk - ref) / np.linalg.norm(ref)),
                               errors=d.errors, golden_errors={"Q": g[f"{tag}_errors_Q"].tolist(),
                                                               "LR": g[f"{tag}_errors_LR"].tolist()})
        print(s, out["seeds"][s]["rel_frob_QLR_vs_golden"], file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
