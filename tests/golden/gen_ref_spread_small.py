"""The reference's own run-to-run spread on the configurations whose GPU tests compare error
histories (test infrastructure; imports the unmodified reference read-only, like gen_golden.py).

The quantised-factor LPLR loop (alg.py:144-195) and the outer Q/LR alternation amplify
rounding differences: the same call of the reference with another torch thread count (MKL
gelsy / gesdd summation orders) lands on other codes and other error histories.  For each case
the reference is run with 8, 4, 2 and 1 threads and once more with 8; recorded are the largest
absolute difference of every error list between any two of those runs, of the first LR error,
and the largest relative Frobenius distance of Q + L R.  The GPU tests' bars are these
measured spreads (with a margin) instead of hand-picked tolerances.

  cfg1    BASELINE config 1: 512 x 512 fp16 (seed 0), r 16, Q4, L/R 2-bit, lplr 5, iters 3
  ragged4 tests/test_gpu_caldera.py::test_ragged_shapes_vs_oracle's 4-bit-factor case:
          333 x 517 fp16, diag H, r 20, Q2, L/R 4-bit, lplr 3, iters 2 (its generator recipe)
  cfg3    BASELINE config 3 (4096 x 11008, resampled diag H), 8 vs 4 threads only

Usage:  python tests/golden/gen_ref_spread_small.py [cfg1] [ragged4] [cfg3]
Output: tests/golden/ref_spread_small.json
"""
import itertools
import json
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402

OUT = os.path.join(HERE, "ref_spread_small.json")


def inputs(case):
    if case == "cfg1":
        torch.manual_seed(0)
        W = (torch.randn(512, 512) * 0.02).to(torch.float16)
        return W, None, dict(Q_bits=4, rank=16, iters=3)
    if case == "ragged4":
        m, n = 333, 517
        g = torch.Generator().manual_seed(m * 3 + n)
        W = (torch.randn(m, n, generator=g) * 0.02).to(torch.float16)
        h = torch.rand(n, generator=g) + 0.05
        return W, torch.diag_embed(h), dict(Q_bits=2, L_bits=4, R_bits=4, rank=20, iters=2, lplr_iters=3)
    if case == "cfg3":
        large = np.load(os.path.join(HERE, "sum_large.npz"))
        torch.manual_seed(0)
        W = (torch.randn(4096, 11008) * 0.02).to(torch.float16)
        h = torch.from_numpy(large["cfg3_h"]).float()
        return W, torch.diag_embed(h), dict(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5)
    raise ValueError(case)


def spread(alg, CP, case, threads):
    W, H, kw = inputs(case)
    runs = []
    for t in threads:
        torch.set_num_threads(t)
        d = alg.caldera(G._params(CP, None, **kw), W, H, device="cpu", use_tqdm=False)
        QLR = (d.Q.double() + d.L.double() @ d.R.double())
        runs.append((t, {k: list(v) for k, v in d.errors.items()}, QLR))
        print(case, t, d.errors, flush=True)
    torch.set_num_threads(8)
    out = {"threads": [t for t, _, _ in runs], "errors": [e for _, e, _ in runs],
           "max_abs_err_diff": {}, "first_LR_err_range": None, "max_rel_frob_QLR": 0.0}
    for k in runs[0][1]:
        out["max_abs_err_diff"][k] = max(float(np.max(np.abs(np.array(a[1][k]) - np.array(b[1][k]))))
                                         for a, b in itertools.combinations(runs, 2))
    lr0 = [r[1]["LR"][0] for r in runs]
    out["first_LR_err_range"] = [min(lr0), max(lr0)]
    for a, b in itertools.combinations(runs, 2):
        out["max_rel_frob_QLR"] = max(out["max_rel_frob_QLR"],
                                      float(torch.linalg.norm(a[2] - b[2]) / torch.linalg.norm(b[2])))
    return out


if __name__ == "__main__":
    what = sys.argv[1:] or ["cfg1", "ragged4", "cfg3"]
    alg, q, CP = G._import_ref()
    res = json.load(open(OUT)) if os.path.exists(OUT) else {}
    res["generated_by"] = "tests/golden/gen_ref_spread_small.py (unmodified reference, CPU)"
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp())
    try:
        for case in what:
            res[case] = spread(alg, CP, case, (8, 4) if case == "cfg3" else (8, 4, 2, 1, 8))
            json.dump(res, open(OUT, "w"), indent=1)
    finally:
        os.chdir(cwd)
