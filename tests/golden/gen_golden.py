"""Generate the golden fixtures under tests/golden/ from the REFERENCE implementation.

Test infrastructure only.  This script imports the unmodified reference
(`/root/reference/rank-constrained-regression-main`, read-only) and records
inputs/outputs of the hot path `caldera()` (RCR/src/caldera/decomposition/alg.py:24-112)
and of its quantiser (RCR/src/caldera/utils/quantization.py:244-307).  It runs
only in the build container: /root/reference does not exist on the GPU box, so
the committed .npz/.json files are the only pins there.

Fixtures:
  quant_kat.npz   KAT-Q / KAT-NF / KAT-BB: LowMemoryQuantizer on hand-built tie rows,
                  zeros, random and wide-range inputs, block 64 and whole-matrix.
  e2e_cfg1.npz    BASELINE config 1 (512x512 fp16, r=16, Q4, L/R 2-bit, iters 3).
  e2e_nb.npz      notebook recipe RCR/caldera_playbook.ipynb cells 3-5 (summaries).
  trace_s.npz     teacher-forcing trace: every quantize_matrix / LR_init / update_LR /
                  activation_aware_error call of a small diag-H run, in call order.
  lplr_mid.npz    teacher-forcing fixture of the quantised-factor LPLR loop (768x1280,
                  r=64, L/R 4-bit, 10 lplr iterations, real-Hessian diag H): LR_init (L, R),
                  per-iteration pre-quantisation inputs (sketches; full at iteration 0),
                  codes, scales, near-tie indices and LPLR errors.
  sum_large.npz   configs 2, 3, 5 at full size: hashes, scalars, error lists and
                  float64 sketches (Q+LR)@Omega and (L1 R1)@Omega of the first LR step.

  main_caller.npz the primary caller's configuration (main.py:163-196): rank 200, L/R 16,
                  scale_W=False, real layer-20 diag Hessians, 896x4864 / 4864x896 / 896x896.

Usage:  python tests/golden/gen_golden.py [kat] [cfg1] [nb] [trace] [lplr] [seeds] [main] [tall] [large]
"""
import hashlib
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

REF = "/root/reference/rank-constrained-regression-main"
HESS = "/root/reference/diag_Hessians.pt"
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_ref():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from src.caldera.decomposition import alg  # noqa: E402
    from src.caldera.utils import quantization as q  # noqa: E402
    from src.caldera.utils.dataclasses import CalderaParams  # noqa: E402
    return alg, q, CalderaParams


def sha(t):
    return hashlib.sha256(np.ascontiguousarray(t.detach().cpu().numpy()).tobytes()).hexdigest()


def sketch_omega(n, k=16, seed=1234):
    """Fixed Gaussian probe used for the (Q+LR)@Omega sketches (float64)."""
    return np.random.default_rng(seed).standard_normal((n, k))


# ---------------------------------------------------------------------------
def gen_kat(q):
    rng = np.random.default_rng(7)
    inputs = {}
    # tie rows: each 64-block has its max at +-M, the rest at fractions that hit
    # exact .5 ties for k in {1, 7, 127, 32767} and their neighbours.
    fr = []
    for k in (1, 7, 127, 32767):
        for j in (0, 1, 2, 3, k // 2, k - 1):
            fr += [(j + 0.5) / k, -(j + 0.5) / k, (j + 0.25) / k]
    fr += [0.0, -0.0, 1.0, -1.0, 0.5, -0.5, 1e-30, -1e-30]
    fr = np.array(fr, dtype=np.float64)
    rows = []
    for M in (1.0, 2.0, 0.75, 3.3, 1e-6, 5.296875):
        for s in (0, 37):
            v = np.resize(np.roll(fr, s), 64) * M
            v[5] = M if s == 0 else -M
            rows.append(v)
    inputs["ties"] = np.array(rows, dtype=np.float32)  # (12, 64)
    z = np.zeros((4, 64), dtype=np.float32)
    z[1] = -0.0
    inputs["zeros"] = z
    inputs["rand"] = rng.standard_normal((64, 64)).astype(np.float32)
    w = rng.standard_normal((64, 64)) * np.exp(4 * rng.standard_normal((64, 64)))
    w[3, :8] = 1e-41  # subnormals
    inputs["wide"] = w.astype(np.float32)
    o = rng.standard_normal((64, 64)).astype(np.float32)
    o[rng.integers(0, 64, 20), rng.integers(0, 64, 20)] = 50.0 * rng.choice([-1, 1], 20)
    inputs["outl"] = o
    # an odd shape: 48 x 40 (numel 1920 = 30 blocks of 64)
    inputs["odd"] = (rng.standard_normal((48, 40)) * 0.02).astype(np.float32)

    out = {}
    for name, x in inputs.items():
        out[f"in_{name}"] = x
        xt = torch.from_numpy(x.copy())
        for method, bitsl in (("uniform", (2, 4, 8, 16)), ("nf4", (4,)), ("nf2", (2,)),
                              ("bbint4", (4,)), ("bbint2", (2,))):
            for bits in bitsl:
                for bs in (64, x.size):
                    qz = q.LowMemoryQuantizer(num_bits=bits, method=method, block_size=bs)
                    codes, params, shape = qz.quantize_block(xt.clone())
                    deq = qz.dequantize_block(codes, params, shape)
                    key = f"{method}_b{bits}_bs{'all' if bs == x.size else bs}_{name}"
                    out[key + "_codes"] = codes.numpy()
                    out[key + "_deq"] = deq.numpy()
                    if method.startswith("bbint"):
                        mn, sc, ov, oi = params
                        out[key + "_min"] = mn.numpy()
                        out[key + "_scale"] = sc.numpy()
                        out[key + "_ovals"] = ov.numpy()
                        out[key + "_oidx"] = oi.numpy()
                    else:
                        out[key + "_scale"] = params.numpy()
    np.savez_compressed(os.path.join(OUT, "quant_kat.npz"), **out)
    print("quant_kat.npz", len(out), "arrays")


# ---------------------------------------------------------------------------
def _params(CalderaParams, q, **kw):
    base = dict(update_order=["Q", "LR"], sigma_reg=1e-8)
    base.update(kw)
    return CalderaParams(**base)


def _decomp_arrays(d, prefix=""):
    o = {}
    for f in ("L", "R", "Q_idxs", "L_idxs", "R_idxs"):
        v = getattr(d, f)
        if v is not None:
            o[prefix + f] = v.detach().cpu().numpy()
    for f in ("Q_scale", "L_scale", "R_scale"):
        v = getattr(d, f)
        o[prefix + f] = np.asarray(v.detach().cpu().numpy() if torch.is_tensor(v) else v, dtype=np.float32)
    o[prefix + "global_scale"] = np.float64(d.global_scale)
    for k, v in d.errors.items():
        o[prefix + "errors_" + k] = np.array(v, dtype=np.float64)
    return o


def gen_cfg1(alg, q, CalderaParams):
    torch.manual_seed(0)
    W = (torch.randn(512, 512) * 0.02).to(torch.float16)
    p = _params(CalderaParams, q, Q_bits=4, rank=16, iters=3)
    t = time.time()
    d = alg.caldera(p, W, None, device="cpu", use_tqdm=False)
    print("cfg1", time.time() - t, d.errors)
    o = _decomp_arrays(d)
    o["W"] = W.numpy()
    o["Q"] = d.Q.numpy()
    o["W_scaled"] = d.W.numpy()
    np.savez_compressed(os.path.join(OUT, "e2e_cfg1.npz"), **o)


def gen_nb(alg, q, CalderaParams):
    qfQ = q.QuantizerFactory(method="uniform", block_size=64)
    qfLR = q.QuantizerFactory(method="uniform", block_size=64)
    p = CalderaParams(compute_quantized_component=True, compute_low_rank_factors=True,
                      Q_bits=4, L_bits=4, R_bits=4, rank=16, iters=20, lplr_iters=5,
                      activation_aware_LR=True, update_order=["Q", "LR"],
                      quant_factory_Q=qfQ, quant_factory_LR=qfLR, rand_svd=False, sigma_reg=1e-8)
    torch.manual_seed(42)
    W = torch.randn(1024, 1024)
    X = torch.eye(1024, 128)
    H = torch.matmul(X, X.T)
    t = time.time()
    d = alg.caldera(quant_params=p, W=W, H=H, device="cpu", use_tqdm=False, scale_W=True)
    print("nb", time.time() - t)
    o = _decomp_arrays(d)
    for k in ("Q_idxs",):
        o.pop(k)
    o["W_sha256"] = np.array(sha(W))
    o["Q_idxs_sha256"] = np.array(sha(d.Q_idxs))
    om = sketch_omega(1024)
    o["sketch_QLR"] = (d.Q.double() + d.L.double() @ d.R.double()).numpy() @ om
    o["norm_QLR"] = np.float64(torch.linalg.matrix_norm((d.Q + d.L @ d.R).double()).item())
    np.savez_compressed(os.path.join(OUT, "e2e_nb.npz"), **o)


# ---------------------------------------------------------------------------
class Tracer:
    """Wraps the alg.* step functions and records each call's inputs/outputs."""

    def __init__(self, alg, keep_big=True):
        self.alg, self.rec, self.keep_big = alg, [], keep_big
        self.orig = {n: getattr(alg, n) for n in
                     ("quantize_matrix", "LR_init", "update_LR", "activation_aware_error")}

    def __enter__(self):
        a, o, rec = self.alg, self.orig, self.rec

        def quantize_matrix(A, qp, qi=None):
            r = o["quantize_matrix"](A, qp, qi)
            rec.append(("quantize", dict(A=A, bits=qi.quant.num_bits, A_hat=r.A_hat,
                                         A_idxs=r.A_idxs, scale=r.scale)))
            return r

        def LR_init(ci, qp, H_sqrt, eigH, residual):
            L, R = o["LR_init"](ci, qp, H_sqrt, eigH, residual)
            rec.append(("lr_init", dict(residual=residual, H_sqrt_diag=torch.diagonal(H_sqrt),
                                        L=L, R=R)))
            return L, R

        def update_LR(ci, qp, residual, H_sqrt, eigH, device):
            o["update_LR"](ci, qp, residual, H_sqrt, eigH, device)
            rec.append(("update_lr", dict(L=ci.L, R=ci.R, L_idxs=ci.L_idxs, R_idxs=ci.R_idxs,
                                          L_scale=ci.L_scale, R_scale=ci.R_scale)))

        def activation_aware_error(W, H, ci, device):
            e = o["activation_aware_error"](W, H, ci, device)
            rec.append(("error", dict(value=torch.tensor(e, dtype=torch.float64))))
            return e

        for n, f in (("quantize_matrix", quantize_matrix), ("LR_init", LR_init),
                     ("update_LR", update_LR), ("activation_aware_error", activation_aware_error)):
            setattr(a, n, f)
        return self

    def __exit__(self, *exc):
        for n, f in self.orig.items():
            setattr(self.alg, n, f)


def resampled_h(name, n, seed=1):
    Hall = torch.load(HESS, weights_only=True)
    src = Hall[name].float()
    idx = torch.randint(0, src.numel(), (n,), generator=torch.Generator().manual_seed(seed))
    return src[idx]


def gen_trace(alg, q, CalderaParams):
    torch.manual_seed(3)
    W = (torch.randn(256, 512) * 0.02).to(torch.float16)
    h = resampled_h("language_model.model.layers.20.self_attn.q_proj", 512)
    H = torch.diag_embed(h)
    p = _params(CalderaParams, q, Q_bits=2, L_bits=4, R_bits=4, rank=32, iters=2, lplr_iters=3)
    with Tracer(alg) as tr:
        d = alg.caldera(p, W, H, device="cpu", use_tqdm=False)
    o = _decomp_arrays(d, "final_")
    o["W"] = W.numpy()
    o["h"] = h.numpy()
    o["W_scaled"] = d.W.numpy()
    kinds = []
    for i, (kind, dd) in enumerate(tr.rec):
        kinds.append(kind)
        for k, v in dd.items():
            if torch.is_tensor(v):
                o[f"c{i}_{k}"] = v.detach().cpu().numpy()
            else:
                o[f"c{i}_{k}"] = np.asarray(v)
    o["kinds"] = np.array(kinds)
    np.savez_compressed(os.path.join(OUT, "trace_s.npz"), **o)
    print("trace", kinds)


# ---------------------------------------------------------------------------
def near_ties(A, bits, tol=1e-4):
    """Flat indices of A whose scaled value x / max|A| * k (quantization.py:95, 266) lies
    within `tol` code units of a rounding boundary: the only places where a code may flip
    between two lstsq solutions that agree to ~1e-6 relative."""
    a = A.detach().double().numpy().reshape(-1)
    mx = max(np.abs(a).max(), 1e-8)
    s = a / mx * (2 ** (bits - 1) - 1)
    return np.nonzero(np.abs(np.abs(s - np.floor(s)) - 0.5) < tol)[0].astype(np.int32)


def gen_lplr(alg, q, CalderaParams, tag="lplr_mid", m=768, n=1280, rank=64, lplr_iters=10):
    """Teacher-forcing fixture for the quantised-factor LPLR loop (alg.py:160-188): the first
    update_LR call of a diag-H run with 4-bit factors.  Recorded: the LR_init (L, R) and, per
    LPLR iteration, the pre-quantisation L^T / R (full for iteration 0, a 16-column sketch
    for all), their codes and scales, their near-tie indices, and ||(res - L R) H_sqrt||."""
    torch.manual_seed(5)
    W = (torch.randn(m, n) * 0.02).to(torch.float16)
    h = resampled_h("language_model.model.layers.20.self_attn.q_proj", n, seed=2)
    p = _params(CalderaParams, q, Q_bits=2, L_bits=4, R_bits=4, rank=rank, iters=2, lplr_iters=lplr_iters)
    with Tracer(alg) as tr:
        d = alg.caldera(p, W, torch.diag_embed(h), device="cpu", use_tqdm=False)
    o = {"W_sha256": np.array(sha(W)), "h": h.numpy(), "global_scale": np.float64(d.global_scale),
         "m": np.int64(m), "n": np.int64(n), "rank": np.int64(rank), "lplr_iters": np.int64(lplr_iters)}
    kinds = [k for k, _ in tr.rec]
    i0 = kinds.index("lr_init")
    q1 = tr.rec[0][1]
    o["firstQ_idxs_sha256"] = np.array(sha(q1["A_idxs"]))
    o["firstQ_scale"] = q1["scale"].numpy()
    ini = tr.rec[i0][1]
    res, hs = ini["residual"], ini["H_sqrt_diag"]
    o["residual_sha256"] = np.array(sha(res))
    o["H_sqrt_diag"], o["L0"], o["R0"] = hs.numpy(), ini["L"].numpy(), ini["R"].numpy()
    omL, omR = sketch_omega(m), sketch_omega(n)
    errs, errs64 = [], []
    for it in range(lplr_iters):
        for side, j, om in (("L", i0 + 1 + 2 * it, omL), ("R", i0 + 2 + 2 * it, omR)):
            kind, c = tr.rec[j]
            assert kind == "quantize" and c["A"].shape == ((rank, m) if side == "L" else (rank, n))
            A = c["A"]
            if it == 0:
                o[f"{side}{it}_A"] = A.numpy()
            o[f"{side}{it}_sketch"] = A.double().numpy() @ om
            o[f"{side}{it}_idxs"] = c["A_idxs"].numpy()
            o[f"{side}{it}_scale"] = c["scale"].numpy()
            o[f"{side}{it}_ties"] = near_ties(A, c["bits"])
        Lh = tr.rec[i0 + 1 + 2 * it][1]["A_hat"].T
        Rh = tr.rec[i0 + 2 + 2 * it][1]["A_hat"]
        errs.append(float(torch.linalg.matrix_norm((res - Lh @ Rh) * hs)))   # as alg.py:182 (fp32)
        errs64.append(float(torch.linalg.matrix_norm((res.double() - Lh.double() @ Rh.double()) * hs.double())))
    o["lplr_err"] = np.array(errs)
    o["lplr_err64"] = np.array(errs64)
    upd = tr.rec[i0 + 1 + 2 * lplr_iters]
    assert upd[0] == "update_lr"
    o["best_L_idxs_sha256"] = np.array(sha(upd[1]["L_idxs"]))
    o["best_R_idxs_sha256"] = np.array(sha(upd[1]["R_idxs"]))
    for k, v in d.errors.items():
        o["errors_" + k] = np.array(v, dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, tag + ".npz"), **o)
    print(tag, "lplr errors", errs, "caldera errors", d.errors)


# ---------------------------------------------------------------------------
def run_large(alg, q, CalderaParams, tag, m, n, H, seed=0, scale_W=True, **kw):
    torch.manual_seed(seed)
    W = (torch.randn(m, n) * 0.02).to(torch.float16)
    p = _params(CalderaParams, q, **kw)
    t = time.time()
    with Tracer(alg) as tr:
        d = alg.caldera(p, W, H, device="cpu", use_tqdm=False, scale_W=scale_W)
    el = time.time() - t
    om = sketch_omega(n)
    o = {}
    o[tag + "_seconds"] = np.float64(el)
    o[tag + "_W_sha256"] = np.array(sha(W))
    o[tag + "_global_scale"] = np.float64(d.global_scale)
    first_q = next(dd for k, dd in tr.rec if k == "quantize")
    o[tag + "_firstQ_scale"] = first_q["scale"].numpy()
    o[tag + "_firstQ_idxs_sha256"] = np.array(sha(first_q["A_idxs"]))
    first_lr = next(dd for k, dd in tr.rec if k == "lr_init")
    L1, R1 = first_lr["L"].double(), first_lr["R"].double()
    o[tag + "_firstLR_sketch"] = L1.numpy() @ (R1.numpy() @ om)
    o[tag + "_firstLR_rownormR"] = torch.linalg.vector_norm(R1, dim=1).numpy()
    o[tag + "_firstLR_norm"] = np.float64(torch.linalg.matrix_norm(L1 @ R1).item())
    QLR = d.Q.double() + d.L.double() @ d.R.double()
    o[tag + "_sketch_QLR"] = QLR.numpy() @ om
    o[tag + "_norm_QLR"] = np.float64(torch.linalg.matrix_norm(QLR).item())
    for k, v in d.errors.items():
        o[tag + "_errors_" + k] = np.array(v, dtype=np.float64)
    for f in ("Q_scale", "L_scale", "R_scale"):
        v = getattr(d, f)
        o[tag + "_" + f] = np.asarray(v.numpy() if torch.is_tensor(v) else v, dtype=np.float32)
    o[tag + "_Q_idxs_sha256"] = np.array(sha(d.Q_idxs))
    print(tag, el, d.errors)
    return o


def gen_large(alg, q, CalderaParams, which=("cfg2", "cfg5", "cfg3")):
    path = os.path.join(OUT, "sum_large.npz")
    o = dict(np.load(path)) if os.path.exists(path) else {}
    if "cfg2" in which:
        o.update(run_large(alg, q, CalderaParams, "cfg2", 4096, 4096, None,
                           Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5))
    if "cfg5" in which:
        o.update(run_large(alg, q, CalderaParams, "cfg5", 4096, 4096, None,
                           Q_bits=2, L_bits=4, R_bits=4, rank=256, iters=5, lplr_iters=10))
    if "cfg3" in which:
        h = resampled_h("language_model.model.layers.20.mlp.down_proj", 11008)
        o["cfg3_h"] = h.numpy()
        o.update(run_large(alg, q, CalderaParams, "cfg3", 4096, 11008, torch.diag_embed(h),
                           Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5))
    np.savez_compressed(path, **o)


MAIN_LAYERS = (("main_down", "language_model.model.layers.20.mlp.down_proj", 896, 4864, 11),
               ("main_up", "language_model.model.layers.20.mlp.up_proj", 4864, 896, 12),
               ("main_o", "language_model.model.layers.20.self_attn.o_proj", 896, 896, 13))


def gen_main(alg, q, CalderaParams):
    """The primary caller's real configuration (main.py:163-196): rank 200, L/R 16, Q 2,
    iters 5, scale_W=False, H = diag_embed(Hall[name]) with the REAL diag_Hessians.pt entries
    of layer 20 (down_proj's h spans 2.7e-5 .. 24.6), on synthetic fp16 weights of the
    layers' shapes (the model's weights are not in the reference)."""
    path = os.path.join(OUT, "main_caller.npz")
    Hall = torch.load(HESS, weights_only=True)
    o = {}
    for tag, name, m, n, seed in MAIN_LAYERS:
        h = Hall[name].to(torch.float32)
        o[tag + "_h"] = h.numpy()
        o[tag + "_name"] = np.array(name)
        o.update(run_large(alg, q, CalderaParams, tag, m, n, torch.diag_embed(h), seed=seed, scale_W=False,
                           Q_bits=2, L_bits=16, R_bits=16, rank=200, iters=5, lplr_iters=5))
    np.savez_compressed(path, **o)


def gen_tall(alg, q, CalderaParams):
    """Config 4's tall gate/up projection shape 11008 x 4096 (H = I, r 128, Q2, iters 5)."""
    path = os.path.join(OUT, "sum_large.npz")
    o = dict(np.load(path))
    o.update(run_large(alg, q, CalderaParams, "cfg4t", 11008, 4096, None, seed=4,
                       Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5))
    np.savez_compressed(path, **o)


def gen_seeds(alg, q, CalderaParams, seeds=(1, 2, 3)):
    """Config 2 on the bench's other seeds (bench.py synth_batch: seed i -> matrix i): the
    Q+LR sketch, norm and error lists the bench and the B = 256 batch test pin."""
    path = os.path.join(OUT, "sum_large.npz")
    o = dict(np.load(path))
    for s in seeds:
        r = run_large(alg, q, CalderaParams, f"cfg2s{s}", 4096, 4096, None, seed=s,
                      Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5)
        keep = ("_W_sha256", "_global_scale", "_sketch_QLR", "_norm_QLR", "_errors_Q", "_errors_LR",
                "_firstQ_idxs_sha256", "_seconds")
        o.update({k: v for k, v in r.items() if k.endswith(keep)})
    np.savez_compressed(path, **o)


if __name__ == "__main__":
    what = sys.argv[1:] or ["kat", "cfg1", "nb", "trace", "lplr", "large", "seeds", "main", "tall"]
    alg, q, CP = _import_ref()
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp())  # bbint appends outlier_log.csv to CWD (quantization.py:126-136)
    try:
        if "kat" in what:
            gen_kat(q)
        if "cfg1" in what:
            gen_cfg1(alg, q, CP)
        if "nb" in what:
            gen_nb(alg, q, CP)
        if "trace" in what:
            gen_trace(alg, q, CP)
        if "lplr" in what:
            gen_lplr(alg, q, CP)
        if "seeds" in what:
            gen_seeds(alg, q, CP)
        if "main" in what:
            gen_main(alg, q, CP)
        if "tall" in what:
            gen_tall(alg, q, CP)
        large = [w for w in what if w in ("cfg2", "cfg3", "cfg5")]
        if "large" in what:
            large = ["cfg2", "cfg5", "cfg3"]
        if large:
            gen_large(alg, q, CP, large)
    finally:
        os.chdir(cwd)
