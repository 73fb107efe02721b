"""Is config 5 (r = 256, Q2, L/R 4-bit, lplr_iters 10) determined by its inputs to 1e-4?

Build-container tool (imports the unmodified reference, read-only, like
tests/golden/gen_golden.py; /root/reference does not exist on the GPU box).  Runs the
reference's caldera() (RCR/src/caldera/decomposition/alg.py:24-112) on the config-5 W three
times and compares the results:

  base      torch threads = 8
  repeat    the same call again (run-to-run determinism)
  threads4  torch threads = 4 (MKL/OpenMP reduction order differs)
  perturb   threads = 8, the first LR_init's L and R multiplied by (1 + 1e-7 * N(0,1)),
            i.e. perturbed below fp32 resolution of any SVD of this residual

For every run the first update_LR's LPLR loop is traced (alg.py:160-188): L^T and R codes of
each iteration, and ||(res - L R) H_sqrt|| per iteration.  Output: JSON with, per pair of
runs, the first LPLR iteration whose codes differ, flip counts, error-list differences and
the relative Frobenius distance of the final Q + L R.

Usage: python tools/ref_chaos.py [cfg5|mid] > profiles/r02_ref_chaos_cfg5.json
       python tools/ref_chaos.py spread profiles/r02_ref_chaos_cfg5.json > tests/golden/ref_spread_cfg5.json
       (the compact run-to-run spread the config-5 GPU test is held to)
"""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

REF = "/root/reference/rank-constrained-regression-main"
CFGS = {
    "cfg5": dict(m=4096, n=4096, Q_bits=2, L_bits=4, R_bits=4, rank=256, iters=5, lplr_iters=10),
    "mid": dict(m=1024, n=1024, Q_bits=2, L_bits=4, R_bits=4, rank=64, iters=3, lplr_iters=10),
}


def run(alg, CalderaParams, cfg, threads, perturb):
    torch.set_num_threads(threads)
    torch.manual_seed(0)
    W = (torch.randn(cfg["m"], cfg["n"]) * 0.02).to(torch.float16)
    p = CalderaParams(update_order=["Q", "LR"], sigma_reg=1e-8,
                      **{k: v for k, v in cfg.items() if k not in ("m", "n")})
    rec = dict(L=[], R=[], lplr_err=[], calls=0)
    o_init, o_q = alg.LR_init, alg.quantize_matrix
    state = {}

    def LR_init(ci, qp, H_sqrt, eigH, residual):
        L, R = o_init(ci, qp, H_sqrt, eigH, residual)
        rec["calls"] += 1
        if rec["calls"] == 1:
            state["res"] = residual
            if perturb:
                g = torch.Generator().manual_seed(99)
                L = L * (1 + 1e-7 * torch.randn(L.shape, generator=g))
                R = R * (1 + 1e-7 * torch.randn(R.shape, generator=g))
        return L, R

    def quantize_matrix(A, qp, qi=None):
        r = o_q(A, qp, qi)
        if rec["calls"] == 1 and "res" in state:
            if A.shape[0] == p.rank and A.shape[1] == cfg["m"] and len(rec["L"]) == len(rec["R"]):
                rec["L"].append(r.A_idxs.clone())
                state["Lhat"] = r.A_hat.T
            elif A.shape[0] == p.rank and len(rec["R"]) < len(rec["L"]):
                rec["R"].append(r.A_idxs.clone())
                e = torch.linalg.matrix_norm(state["res"] - state["Lhat"] @ r.A_hat)
                rec["lplr_err"].append(float(e))
        return r

    alg.LR_init, alg.quantize_matrix = LR_init, quantize_matrix
    try:
        t = time.time()
        d = alg.caldera(p, W, None, device="cpu", use_tqdm=False)
        el = time.time() - t
    finally:
        alg.LR_init, alg.quantize_matrix = o_init, o_q
    QLR = (d.Q.double() + d.L.double() @ d.R.double())
    return dict(seconds=el, errors={k: list(map(float, v)) for k, v in d.errors.items()},
                QLR=QLR, L=rec["L"], R=rec["R"], lplr_err=rec["lplr_err"])


def compare(a, b):
    first = None
    flips = []
    for i, (la, lb, ra, rb) in enumerate(zip(a["L"], b["L"], a["R"], b["R"])):
        fl, fr = int((la != lb).sum()), int((ra != rb).sum())
        flips.append([fl, fr])
        if first is None and (fl or fr):
            first = i
    rel = float(torch.linalg.matrix_norm(a["QLR"] - b["QLR"]) / torch.linalg.matrix_norm(a["QLR"]))
    return dict(first_lplr_iter_with_code_flips=first, code_flips_L_R_per_iter=flips,
                lplr_err_a=a["lplr_err"], lplr_err_b=b["lplr_err"],
                errors_a=a["errors"], errors_b=b["errors"],
                max_abs_err_diff={k: max(abs(x - y) for x, y in zip(a["errors"][k], b["errors"][k]))
                                  for k in a["errors"]},
                rel_frob_QLR=rel)


def spread(path):
    """Per-run error lists and pairwise distances of the reference runs in a ref_chaos JSON."""
    d = json.load(open(path))
    runs = {"base": d["base_vs_repeat"]["errors_a"]}
    pairs = {}
    for key in ("base_vs_repeat", "base_vs_threads4", "base_vs_perturb"):
        runs[key.split("_vs_")[1]] = d[key]["errors_b"]
        pairs[key] = dict(rel_frob_QLR=d[key]["rel_frob_QLR"], max_abs_err_diff=d[key]["max_abs_err_diff"],
                          best_lplr_err=[min(d[key]["lplr_err_a"]), min(d[key]["lplr_err_b"])])
    first_lr = [v["LR"][0] for v in runs.values()]
    return dict(source=os.path.basename(path), generated_by="tools/ref_chaos.py (unmodified reference, CPU)",
                config=d["config"], params=d["params"], errors=runs, pairs=pairs,
                first_LR_err_range=[min(first_lr), max(first_lr)],
                max_rel_frob_QLR=max(p["rel_frob_QLR"] for p in pairs.values()),
                max_abs_err_diff={k: max(p["max_abs_err_diff"][k] for p in pairs.values()) for k in ("Q", "LR")})


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "cfg5"
    if which == "spread":
        print(json.dumps(spread(sys.argv[2]), indent=1))
        return
    cfg = CFGS[which]
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from src.caldera.decomposition import alg
    from src.caldera.utils.dataclasses import CalderaParams
    os.chdir(tempfile.mkdtemp())
    runs = {"base": run(alg, CalderaParams, cfg, 8, False),
            "repeat": run(alg, CalderaParams, cfg, 8, False),
            "threads4": run(alg, CalderaParams, cfg, 4, False),
            "perturb": run(alg, CalderaParams, cfg, 8, True)}
    out = dict(config=which, params=cfg, torch=torch.__version__,
               seconds={k: v["seconds"] for k, v in runs.items()},
               base_vs_repeat=compare(runs["base"], runs["repeat"]),
               base_vs_threads4=compare(runs["base"], runs["threads4"]),
               base_vs_perturb=compare(runs["base"], runs["perturb"]))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
