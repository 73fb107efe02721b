"""Golden fixture for a batch of layers with DISTINCT diagonal Hessians (round 6).

Test infrastructure only: imports the unmodified reference (read-only) in the build container,
like gen_golden.py.  The reference's real workload (main.py:147, 163-196) calls caldera() once
per layer, each with its own H = diag_embed(Hall[name]).  This records four such calls: the
self_attn.o_proj layers 17, 18, 19 and 21 of diag_Hessians.pt (896 x 896; main.py's default
layer range is 17-23, layer 20 is already in main_caller.npz), at main.py's driver parameters
(rank 200, Q 2-bit, L/R 16-bit, iters 5, lplr_iters 5, sigma_reg 1e-8, scale_W=False), on
synthetic fp16 weights randn * 0.02 (seeds 31-34; the model's weights are not in the reference).

Per tag mh<i>: _h, _name, _W_sha256, _firstQ_scale, _firstQ_idxs_sha256, _errors_Q/_LR,
_sketch_QLR (16-column Gaussian sketch of Q + L R, fp32), and the final codes as in
final_codes.npz (_Q_idxs_sha256, _rowhash, _ties_idx/_code/_dist, _Q_scale), plus the
reference's own 4- vs 8-thread spread (_ref_flips, _ref_rel_frob).

Also (`hessians`): main_hessians.npz, the diag_Hessians.pt entries of every projection main.py
decomposes with its defaults (layers 17-23, q/o/gate/up/down: both dims > 500 in the 896-hidden
language model; k/v are 128 x 896) -- data for bench.py --workload main on the GPU box, where
the reference does not exist.

Usage:  python tests/golden/gen_golden_multi_h.py [hessians]   -> tests/golden/multi_h.npz
                                                               (main_hessians.npz)
"""
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402
import gen_golden_codes as C  # noqa: E402

OUT = os.path.join(HERE, "multi_h.npz")
LAYERS = (17, 18, 19, 21)
SEED0 = 31
KW = dict(Q_bits=2, L_bits=16, R_bits=16, rank=200, iters=5, lplr_iters=5)


def main():
    alg, q, CP = G._import_ref()
    Hall = torch.load(G.HESS, weights_only=True)
    o = {}
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp())
    try:
        for i, layer in enumerate(LAYERS):
            tag = f"mh{i}"
            name = f"language_model.model.layers.{layer}.self_attn.o_proj"
            h = Hall[name].to(torch.float32)
            m = n = h.numel()
            H = torch.diag_embed(h)
            d, fin, W, el, firstq = C.run(alg, CP, m, n, SEED0 + i, H=H, scale_W=False, **KW)
            o[tag + "_h"] = h.numpy()
            o[tag + "_name"] = np.array(name)
            C.record(o, tag, d, fin, W, el, m, n, 2)
            o[tag + "_firstQ_scale"] = firstq["scale"].numpy()
            o[tag + "_firstQ_idxs_sha256"] = np.array(G.sha(firstq["A_idxs"]))
            for k, v in d.errors.items():
                o[tag + "_errors_" + k] = np.array(v, dtype=np.float64)
            o[tag + "_sketch_QLR"] = C.sketch(d, n)
            d4, _, _, _, _ = C.run(alg, CP, m, n, SEED0 + i, H=H, scale_W=False, threads=4, **KW)
            sk4 = C.sketch(d4, n)
            o[tag + "_ref_flips"] = np.int64((d.Q_idxs.numpy() != d4.Q_idxs.numpy()).sum())
            o[tag + "_ref_rel_frob"] = np.float64(np.linalg.norm(sk4 - o[tag + "_sketch_QLR"])
                                                  / np.linalg.norm(o[tag + "_sketch_QLR"]))
            print(tag, name, "h in", float(h.min()), float(h.max()), "errors", d.errors,
                  "ref 4 vs 8 threads: flips", int(o[tag + "_ref_flips"]), "rel", float(o[tag + "_ref_rel_frob"]),
                  flush=True)
        torch.set_num_threads(8)
        np.savez_compressed(OUT, **o)
    finally:
        os.chdir(cwd)


MAIN_PROJS = ("self_attn.q_proj", "self_attn.o_proj", "mlp.gate_proj", "mlp.up_proj", "mlp.down_proj")


def main_hessians():
    Hall = torch.load(G.HESS, weights_only=True)
    o = {}
    for layer in range(17, 24):
        for proj in MAIN_PROJS:
            name = f"language_model.model.layers.{layer}.{proj}"
            o[name] = Hall[name].to(torch.float32).numpy()
    np.savez_compressed(os.path.join(HERE, "main_hessians.npz"), **o)
    print(len(o), "Hessian diagonals", sorted({v.size for v in o.values()}))


if __name__ == "__main__":
    if sys.argv[1:] == ["hessians"]:
        main_hessians()
    else:
        main()
