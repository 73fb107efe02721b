"""Golden fixtures for the FINAL integer codes (Q_idxs, alg.py:280-283) of the reference.

Test infrastructure only: imports the unmodified reference (read-only) in the build
container, like gen_golden.py.  For every full-size configuration the reference's final
`Q_idxs` are pinned three ways, compactly enough to commit:

  <tag>_Q_idxs_sha256   SHA-256 of the final int8 codes (as gen_golden.py's sum_large);
  <tag>_rowhash         uint64 per row of the m x n code matrix (first 8 bytes of
                        blake2b(row bytes)): a mismatching row is localised;
  <tag>_ties_idx/_code/_dist
                        every element whose scaled value x / max|x| * k (quantization.py:95,
                        266) in the quantise call that produced the final codes lies within
                        1e-3 code units of a rounding boundary (flat index, the reference's code
                        there, the distance).  A row of ours that differs from the reference only
                        at such positions hashes equal once those positions carry the reference's
                        codes: every flip is then PROVEN to sit at a reference near-tie.

Config 2 is recorded for seeds 0-15 (the bench's timed batch holds seed i at position i),
with the reference's own 4- vs 8-thread spread per seed (relative Frobenius of Q + L R and
the number of final-code flips between the two runs).  Config 5 (the chaotic 4-bit LPLR
path, where two identical reference calls diverge in Q + L R) records the flips of the final
codes between two more reference runs of the same W (none: the kept iterate's Q is stable).

Held-out set (round 6): config 2 seeds 16-47 -- matrices the engine's solver schedules and
tolerances were never tuned on -- recorded the same way (final codes, near-ties, sketch, errors,
4- vs 8-thread spread) into separate files, so parity measured on them is out-of-sample.

Usage:  python tests/golden/gen_golden_codes.py [cfg2seeds] [cfg3] [cfg4t] [main] [cfg5] [cfg2holdout]
Output: tests/golden/final_codes.npz, tests/golden/ref_spread_cfg2_seeds16.json,
        (cfg2holdout) tests/golden/final_codes_holdout.npz, tests/golden/ref_spread_cfg2_holdout.json
"""
import hashlib
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402

OUT = os.path.join(HERE, "final_codes.npz")
SPREAD = os.path.join(HERE, "ref_spread_cfg2_seeds16.json")
OUT_HOLDOUT = os.path.join(HERE, "final_codes_holdout.npz")
SPREAD_HOLDOUT = os.path.join(HERE, "ref_spread_cfg2_holdout.json")
HOLDOUT_SEEDS = range(16, 48)
TIE_TOL = 1e-3
CFG2 = dict(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5)


def rowhash(codes, m, n):
    a = np.ascontiguousarray(codes.reshape(m, n))
    return np.array([int.from_bytes(hashlib.blake2b(a[i].tobytes(), digest_size=8).digest(), "little")
                     for i in range(m)], dtype=np.uint64)


def ties(A, bits, tol=TIE_TOL):
    a = A.detach().double().numpy().reshape(-1)
    mx = max(np.abs(a).max(), 1e-8)
    s = a / mx * (2 ** (bits - 1) - 1)
    d = np.abs(np.abs(s - np.floor(s)) - 0.5)
    idx = np.nonzero(d < tol)[0]
    return idx.astype(np.int64), d[idx].astype(np.float32)


def run(alg, CP, m, n, seed, H=None, scale_W=True, threads=8, **kw):
    """One reference caldera() call; returns (decomposition, final-Q quantise record, W)."""
    torch.set_num_threads(threads)
    torch.manual_seed(seed)
    W = (torch.randn(m, n) * 0.02).to(torch.float16)
    p = G._params(CP, None, **kw)
    t = time.time()
    with G.Tracer(alg) as tr:
        d = alg.caldera(p, W, H, device="cpu", use_tqdm=False, scale_W=scale_W)
    el = time.time() - t
    fin = [c for k, c in tr.rec if k == "quantize" and c["A"].shape == (m, n) and torch.equal(c["A_idxs"], d.Q_idxs)]
    assert fin, "final Q codes not produced by any traced quantise call"
    firstq = next(c for k, c in tr.rec if k == "quantize")
    return d, fin[-1], W, el, firstq


def record(o, tag, d, fin, W, el, m, n, bits):
    codes = d.Q_idxs.numpy().reshape(-1)
    o[tag + "_Q_idxs_sha256"] = np.array(G.sha(d.Q_idxs))
    o[tag + "_W_sha256"] = np.array(G.sha(W))
    o[tag + "_rowhash"] = rowhash(codes, m, n)
    idx, dist = ties(fin["A"], bits)
    o[tag + "_ties_idx"] = idx
    o[tag + "_ties_code"] = codes[idx].astype(np.int8)
    o[tag + "_ties_dist"] = dist
    o[tag + "_Q_scale"] = np.float32(d.Q_scale.reshape(-1)[0].item())
    o[tag + "_seconds"] = np.float64(el)
    print(f"{tag}: {el:.1f} s, {len(idx)} near-ties (< {TIE_TOL} code units)", flush=True)


def sketch(d, n):
    """16-column Gaussian sketch of Q + L R, stored in fp32 (the tests compare at >= 1e-5)."""
    return ((d.Q.double() + d.L.double() @ d.R.double()).numpy() @ G.sketch_omega(n)).astype(np.float32)


def gen_cfg2_seeds(alg, CP, o, seeds=range(16), spread_path=SPREAD, out_path=OUT):
    large = np.load(os.path.join(HERE, "sum_large.npz"))
    spread = {"generated_by": "tests/golden/gen_golden_codes.py cfg2seeds (unmodified reference, CPU, "
                              "4 vs 8 torch threads)", "tie_tol_code_units": TIE_TOL, "seeds": {}}
    for s in seeds:
        tag = "cfg2" if s == 0 else f"cfg2s{s}"
        d, fin, W, el, firstq = run(alg, CP, 4096, 4096, s, **CFG2)
        if f"{tag}_W_sha256" in large.files:   # seeds 0-3: the existing golden runs must reproduce
            assert G.sha(W) == str(large[f"{tag}_W_sha256"])
            sk_old = large[f"{tag}_sketch_QLR"]
            rel_old = float(np.linalg.norm(sketch(d, 4096) - sk_old) / np.linalg.norm(sk_old))
            print(f"{tag}: rerun vs sum_large golden sketch {rel_old:.2e}", flush=True)
            assert rel_old < 1e-6, rel_old   # the same run (fp32-stored sketch)
        record(o, tag, d, fin, W, el, 4096, 4096, 2)
        o[tag + "_sketch_QLR"] = sketch(d, 4096)
        o[tag + "_global_scale"] = np.float64(d.global_scale)
        o[tag + "_firstQ_idxs_sha256"] = np.array(G.sha(firstq["A_idxs"]))
        o[tag + "_firstQ_scale"] = firstq["scale"].numpy()
        for k, v in d.errors.items():
            o[tag + "_errors_" + k] = np.array(v, dtype=np.float64)
        # the reference's own spread: the same call on 4 threads
        d4, _, _, el4, _ = run(alg, CP, 4096, 4096, s, threads=4, **CFG2)
        sk8, sk4 = o[tag + "_sketch_QLR"], sketch(d4, 4096)
        c8, c4 = d.Q_idxs.numpy().reshape(-1), d4.Q_idxs.numpy().reshape(-1)
        flips = np.nonzero(c8 != c4)[0]
        at_ties = int(np.isin(flips, o[tag + "_ties_idx"]).sum())
        spread["seeds"][str(s)] = {
            "rel_frob_QLR_ref4_vs_ref8": float(np.linalg.norm(sk4 - sk8) / np.linalg.norm(sk8)),
            "final_code_flips_ref4_vs_ref8": int(flips.size), "flips_at_ref8_near_ties": at_ties,
            "errors_ref8": d.errors, "errors_ref4": d4.errors, "seconds_8": el, "seconds_4": el4}
        print(f"{tag}: ref4 vs ref8 {spread['seeds'][str(s)]['rel_frob_QLR_ref4_vs_ref8']:.2e}, "
              f"{flips.size} code flips ({at_ties} at near-ties)", flush=True)
        json.dump(spread, open(spread_path, "w"), indent=1)
        np.savez_compressed(out_path, **o)
    torch.set_num_threads(8)


def gen_cfg3(alg, CP, o):
    large = np.load(os.path.join(HERE, "sum_large.npz"))
    h = torch.from_numpy(large["cfg3_h"]).float()
    d, fin, W, el, _ = run(alg, CP, 4096, 11008, 0, H=torch.diag_embed(h), **CFG2)
    assert G.sha(d.Q_idxs) == str(large["cfg3_Q_idxs_sha256"]), "cfg3 rerun differs from sum_large"
    record(o, "cfg3", d, fin, W, el, 4096, 11008, 2)


def gen_cfg4t(alg, CP, o):
    large = np.load(os.path.join(HERE, "sum_large.npz"))
    d, fin, W, el, _ = run(alg, CP, 11008, 4096, 4, **CFG2)
    assert G.sha(d.Q_idxs) == str(large["cfg4t_Q_idxs_sha256"]), "cfg4t rerun differs from sum_large"
    record(o, "cfg4t", d, fin, W, el, 11008, 4096, 2)


def gen_main(alg, CP, o):
    g = np.load(os.path.join(HERE, "main_caller.npz"))
    for tag, name, m, n, seed in G.MAIN_LAYERS:
        h = torch.from_numpy(g[tag + "_h"])
        d, fin, W, el, _ = run(alg, CP, m, n, seed, H=torch.diag_embed(h), scale_W=False, Q_bits=2, L_bits=16,
                               R_bits=16, rank=200, iters=5, lplr_iters=5)
        assert G.sha(d.Q_idxs) == str(g[tag + "_Q_idxs_sha256"]), tag + " rerun differs from main_caller"
        record(o, tag, d, fin, W, el, m, n, 2)


def gen_cfg5(alg, CP, o):
    kw = dict(Q_bits=2, L_bits=4, R_bits=4, rank=256, iters=5, lplr_iters=10)
    runs = []
    for threads in (8, 8, 4):
        d, fin, W, el, _ = run(alg, CP, 4096, 4096, 0, threads=threads, **kw)
        runs.append((d, fin, W, el))
    torch.set_num_threads(8)
    d, fin, W, el = runs[0]
    record(o, "cfg5r", d, fin, W, el, 4096, 4096, 2)
    o["cfg5r_sketch_QLR"] = sketch(d, 4096)
    for k, v in d.errors.items():
        o["cfg5r_errors_" + k] = np.array(v, dtype=np.float64)
    c0 = d.Q_idxs.numpy().reshape(-1)
    fl = [int((c0 != r[0].Q_idxs.numpy().reshape(-1)).sum()) for r in runs[1:]]
    o["cfg5r_ref_flips"] = np.array(fl, dtype=np.int64)            # vs a repeat (8 thr), vs 4 threads
    sk = o["cfg5r_sketch_QLR"]
    o["cfg5r_ref_rel_frob"] = np.array([float(np.linalg.norm(sketch(r[0], 4096) - sk) / np.linalg.norm(sk))
                                        for r in runs[1:]])
    print("cfg5r reference run-to-run final code flips", fl, "rel frob", o["cfg5r_ref_rel_frob"], flush=True)


if __name__ == "__main__":
    what = sys.argv[1:] or ["cfg2seeds", "cfg3", "cfg4t", "main", "cfg5"]
    alg, q, CP = G._import_ref()
    o = dict(np.load(OUT)) if os.path.exists(OUT) else {}
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp())
    try:
        for w, f in (("main", gen_main), ("cfg4t", gen_cfg4t), ("cfg3", gen_cfg3), ("cfg5", gen_cfg5),
                     ("cfg2seeds", gen_cfg2_seeds)):
            if w in what:
                f(alg, CP, o)
                np.savez_compressed(OUT, **o)
        if "cfg2holdout" in what:
            oh = dict(np.load(OUT_HOLDOUT)) if os.path.exists(OUT_HOLDOUT) else {}
            gen_cfg2_seeds(alg, CP, oh, seeds=HOLDOUT_SEEDS, spread_path=SPREAD_HOLDOUT, out_path=OUT_HOLDOUT)
    finally:
        os.chdir(cwd)
