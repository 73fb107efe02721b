#!/usr/bin/env python3
"""Benchmark: CALDERA decompositions of synthetic 4096x4096 fp16 weight matrices
(BASELINE.json configs[1]: rank 128, Q 2-bit, L/R 16-bit, iters 5, update_order [Q, LR],
H = I) on MI355X.  One "step" = one batched pass of the hot path (caldera() of
alg.py:24-112) over B matrices resident in HBM.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--workload cfg2|cfg3|cfg5|model|main]
                  [--no-cpu-baseline] [--no-parity] [--no-api-path]

Multi-GPU: one process per GPU.  `python bench.py --gpus N` (N > 1, WORLD_SIZE unset) starts
`python -m torch.distributed.run --nproc-per-node N bench.py <same args>` as a child process
before anything touches the GPU and exits with its return code (rank 0's JSON line goes to the
shared stdout); launched by torch.distributed.run directly, WORLD_SIZE must equal --gpus.
--dry-run: the same launcher and gather over gloo on the CPU with a stub decomposer (tiny
matrices, no HIP device, no oracle): plumbing test of the N-rank path.  Every rank decomposes
its own batch (matrices are independent: weak scaling) and, inside each timed step, its
packed results (2-bit codes, L, R, scales) are gathered to rank 0 over RCCL -- the one
collective of the path; the timed region is bracketed by barrier + synchronize and the max
over ranks is reported.

Prints ONE JSON line (rank 0) with value = matrices/s over all ranks, the roofline of the
dominant kernel (timed with HIP events on its stream inside the timed region), parity of the
LAST TIMED STEP's own results (matrices 0-3 of rank 0's batch, seeds 0-3, against the
reference's golden sketches; matrix 0 also against the CPU baseline's output), the CPU
baseline (the reference's torch-CPU op sequence, oracle/caldera_torch_cpu.py, on this host),
and the drop-in API path (caldera_batch with the reference's output placement) timed on one
extra step of the same batch.

Workloads (BASELINE.json configs): cfg2 (default, the headline metric) 4096x4096, r 128, Q2,
L/R 16, iters 5, H = I; cfg3 4096x11008, diag H (the golden fixture's resampled
diag_Hessians.pt entry), r 128, Q2, L/R 16; cfg5 4096x4096, r 256, Q2, L/R 4, lplr 10;
model = BASELINE configs[3]: all 224 Llama-2-7B linear weights sharded round-robin over the
ranks (same-shape batches interleaved on HIP streams), packed on the device and gathered to
rank 0 over RCCL -- strong scaling (the model is fixed), timed end to end including the gather;
main = main.py's own layer set (35 projections of layers 17-23, rank 200) with each layer's real
diagonal Hessian, batched with per-matrix Hessians, beside the reference's one-call-per-layer loop.
"""
import argparse
import json
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

WORKLOADS = {
    "cfg2": dict(m=4096, n=4096, Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, lplr_iters=5, H=False,
                 batch=256, desc="BASELINE configs[1]: 4096x4096 fp16, rank 128, Q_bits 2, L/R_bits 16, "
                                 "iters 5, update_order [Q, LR], H = I"),
    "cfg3": dict(m=4096, n=11008, Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, lplr_iters=5, H=True,
                 batch=192, desc="BASELINE configs[2]: 4096x11008 fp16, activation-aware diag H (resampled "
                                "diag_Hessians.pt down_proj entry), rank 128, Q_bits 2, L/R_bits 16, iters 5"),
    "cfg4t": dict(m=11008, n=4096, Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, lplr_iters=5, H=False,
                  batch=64, seed0=4, desc="BASELINE configs[3]'s tall gate/up shape: 11008x4096 fp16, rank 128, "
                                          "Q_bits 2, L/R_bits 16, iters 5, H = I (matrix 0 = the golden run's "
                                          "seed 4)"),
    "cfg5": dict(m=4096, n=4096, Q_bits=2, L_bits=4, R_bits=4, rank=256, iters=5, lplr_iters=10, H=False,
                 batch=256, desc="BASELINE configs[4]: 4096x4096 fp16, rank 256, Q_bits 2, L/R_bits 4, "
                                "lplr_iters 10, iters 5, H = I"),
}
PEAK_FP32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
PEAK_F16_MFMA_TFLOPS = 2516.6  # 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz (dense fp16/bf16 MFMA)
PEAK_HBM_GBS = 8000.0
XGMI_LINK_GBS = 153.0  # one xGMI link, MI355X (SURVEY.md "Comm note for MI355X": 7 links x ~153 GB/s per GPU)


def golden():
    return np.load(os.path.join(ROOT, "tests", "golden", "sum_large.npz"), allow_pickle=False)


def make_params(wl):
    from src.caldera.utils.dataclasses import CalderaParams
    return CalderaParams(Q_bits=wl["Q_bits"], L_bits=wl["L_bits"], R_bits=wl["R_bits"], rank=wl["rank"],
                         iters=wl["iters"], lplr_iters=wl["lplr_iters"], update_order=["Q", "LR"], sigma_reg=1e-8)


def make_h(wl):
    """Diagonal of H (cfg3: the resampled real Hessian the golden run used) or None."""
    return torch.from_numpy(golden()["cfg3_h"]).float() if wl["H"] else None


def synth_W(wl, seed):
    """The survey's recipe: torch.manual_seed(seed); randn(m, n) * 0.02 -> fp16
    on the host generator (seeds 0-3 are the matrices the golden sketches pin)."""
    torch.manual_seed(seed)
    return (torch.randn(wl["m"], wl["n"]) * 0.02).to(torch.float16)


PINNED = 16  # batch positions whose matrices the golden runs pin (seeds 0-15, host RNG)
# config 2: positions 16-47 hold seeds 16-47 too -- the HELD-OUT goldens (tests/golden/
# final_codes_holdout.npz, exact_codes_cfg2_holdout.npz), matrices no schedule was tuned on
HOLDOUT = range(16, 48)


def synth_batch(wl, B, seed0, dev, host=PINNED):
    """B synthetic weights of the same recipe (randn * 0.02 -> fp16).  The first `host` come
    from the host generator (the survey's recipe: seeds seed0 + i, the matrices the golden runs
    pin), each moved to `dev` as soon as it is made; the rest from the device generator (seeded
    by seed0), so start-up does not grow with B or with the number of ranks sharing the host."""
    out = torch.empty((B, wl["m"], wl["n"]), dtype=torch.float16, device=dev)
    host = min(host, B)
    for i in range(host):
        out[i].copy_(synth_W(wl, seed0 + i))
    g = torch.Generator(device=dev)
    g.manual_seed(seed0 + 0x5EED)
    for i in range(host, B):
        out[i].copy_(torch.randn((wl["m"], wl["n"]), generator=g, device=dev) * 0.02)
    return out


def _sketch(Q, L, R, n):
    om = torch.from_numpy(np.random.default_rng(1234).standard_normal((n, 16))).to(Q.device)
    return (Q.double() @ om + L.double() @ (R.double() @ om)).cpu().numpy()


def parity_of_timed_step(name, decs, wl):
    """Relative Frobenius error (16-column Gaussian sketch) of Q + L R of the timed step's
    matrices against the reference's golden run of the same matrix, and their final integer
    codes against the reference's (tests/final_codes.py: bit-exact, or every flip at a
    reference near-tie).  cfg2: batch positions 0-15 = seeds 0-15 (tests/golden/final_codes.npz,
    with the reference's own 4- vs 8-thread spread per seed); cfg3 / cfg4t / cfg5: matrix 0."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from final_codes import compare, fixture
    fx = fixture()
    g = golden()
    if name == "cfg2":
        tags = ["cfg2"] + [f"cfg2s{s}" for s in range(1, 16)]
        tags = [t for t in tags if f"{t}_sketch_QLR" in fx.files]
        code_tags = tags
    else:
        tags = {"cfg3": ["cfg3"], "cfg4t": ["cfg4t"], "cfg5": ["cfg5"]}[name]
        code_tags = {"cfg3": ["cfg3"], "cfg4t": ["cfg4t"], "cfg5": ["cfg5r"]}[name]
    out, codes = {}, {}
    for i, tag in enumerate(tags[:len(decs)]):
        d = decs[i]
        sk = _sketch(d["Q"], d["L"], d["R"], wl["n"])
        ref = fx[f"{tag}_sketch_QLR"] if f"{tag}_sketch_QLR" in fx.files else g[f"{tag}_sketch_QLR"]
        out[f"seed{i}"] = float(np.linalg.norm(sk - ref) / np.linalg.norm(ref))
        ct = code_tags[i]
        if f"{ct}_rowhash" in fx.files and d.get("Q_idxs") is not None:
            codes[f"seed{i}"] = compare(ct, d["Q_idxs"], wl["m"], wl["n"])
    if codes:
        out["final_codes"] = codes
        out["final_codes_summary"] = {
            "matrices": len(codes), "bit_exact": sum(c["sha_equal"] for c in codes.values()),
            "flips_at_near_ties": sum(c["flips"] for c in codes.values()),
            "rows_unexplained": sum(c["rows_unexplained"] for c in codes.values())}
    if name == "cfg2" and os.path.exists(os.path.join(ROOT, "tests", "golden", "exact_codes_cfg2.npz")):
        # the same final codes against an EXACT rank-r step (fp64 top-128 eigenpairs, the
        # reference's fp32 Q step: tests/golden/gen_exact_codes.py) -- what a perfectly accurate
        # solver gives; the reference itself differs from it on 5 of these 16 seeds
        from final_codes import exact_fixture
        ex = exact_fixture()
        vs = {f"seed{i}": compare(f"s{i}", decs[i]["Q_idxs"], wl["m"], wl["n"], fx=ex)
              for i in range(min(16, len(decs))) if decs[i].get("Q_idxs") is not None}
        out["final_codes_vs_exact_lr"] = {
            "matrices": len(vs), "bit_exact": sum(c["sha_equal"] for c in vs.values()),
            "differing": {k: c for k, c in vs.items() if not c["sha_equal"]}}
    if name == "cfg2" and len(decs) >= HOLDOUT[-1] + 1 and os.path.exists(
            os.path.join(ROOT, "tests", "golden", "final_codes_holdout.npz")):
        out["holdout"] = holdout_parity(decs, wl)
    if name == "cfg2":  # the reference's own spread on the same matrices (4 vs 8 CPU threads)
        sp = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_spread_cfg2_seeds16.json")))["seeds"]
        out["reference_4_vs_8_threads"] = {f"seed{k}": v["rel_frob_QLR_ref4_vs_ref8"] for k, v in sp.items()}
        over = {k: v for k, v in out.items() if k.startswith("seed") and v > 1e-4}
        out["seeds_over_1e-4"] = {k: {"ours": v, "reference_spread": out["reference_4_vs_8_threads"].get(k)}
                                  for k, v in over.items()}
    return out


def holdout_parity(decs, wl):
    """Config 2's held-out seeds 16-47 (batch positions 16-47, host RNG): final codes against the
    reference's runs and against an exact rank-r step, Q + L R against the reference's sketch, with
    the reference's own 4- vs 8-thread spread.  No solver schedule or tolerance was chosen on these
    matrices (tests/golden/gen_golden_codes.py cfg2holdout, gen_exact_codes.py holdout)."""
    from final_codes import classify, compare
    gd = os.path.join(ROOT, "tests", "golden")
    fx = np.load(os.path.join(gd, "final_codes_holdout.npz"), allow_pickle=False)
    ex = np.load(os.path.join(gd, "exact_codes_cfg2_holdout.npz"), allow_pickle=False)
    sp = json.load(open(os.path.join(gd, "ref_spread_cfg2_holdout.json")))["seeds"]
    m, n = wl["m"], wl["n"]
    per, vs_ref, vs_ex, over, classes = {}, [], [], {}, {}
    for s in HOLDOUT:
        tag = f"cfg2s{s}"
        if f"{tag}_rowhash" not in fx.files or f"s{s}_rowhash" not in ex.files:
            continue
        d = decs[s]
        c = compare(tag, d["Q_idxs"], m, n, fx=fx)
        e = compare(f"s{s}", d["Q_idxs"], m, n, fx=ex)
        sk = _sketch(d["Q"], d["L"], d["R"], n)
        ref = fx[f"{tag}_sketch_QLR"].astype(np.float64)
        rel = float(np.linalg.norm(sk - ref) / np.linalg.norm(ref))
        spr = sp.get(str(s), {})
        cls = classify(c, e["sha_equal"], spr)
        classes.setdefault(cls, []).append(s)
        per[f"seed{s}"] = {"rel_frob_QLR": rel, "ref_spread": spr.get("rel_frob_QLR_ref4_vs_ref8"),
                           "codes_vs_ref": c, "codes_vs_exact_lr_bit_exact": e["sha_equal"], "class": cls}
        vs_ref.append(c)
        vs_ex.append(e)
        if rel > 1e-4:
            over[f"seed{s}"] = {"ours": rel, "reference_spread": spr.get("rel_frob_QLR_ref4_vs_ref8")}
    k = len(vs_ref)
    return {"matrices": k,
            "bit_exact_vs_reference": sum(c["sha_equal"] for c in vs_ref),
            "bit_exact_vs_exact_lr": sum(c["sha_equal"] for c in vs_ex),
            "reference_reproduces_itself": sum(1 for s in HOLDOUT if sp.get(str(s), {}).get(
                "final_code_flips_ref4_vs_ref8", 1) == 0),
            "rows_unexplained_vs_reference": sum(c["rows_unexplained"] for c in vs_ref),
            "flips_at_near_ties_vs_reference": sum(c["flips"] for c in vs_ref),
            "classes": {k: classes.get(k, []) for k in ("reference", "ref_spread", "exact_lr", "miss")},
            "classes_note": "final_codes.classify: the reference's codes / within its own 4- vs 8-thread spread / "
                            "bit-exact with an exact rank-r step where the reference's fp32 LAPACK lands elsewhere / "
                            "none of these",
            "seeds_over_1e-4": over, "per_seed": per}


def cpu_baseline(name, wl, dec0):
    """The reference's torch-CPU op sequence (oracle/caldera_torch_cpu.py) on the seed-0 matrix,
    on this host's threads; a bounded sample (all `iters` outer iterations for cfg2/cfg3, one
    outer iteration of cfg5's five, value scaled accordingly)."""
    from oracle import caldera_torch_cpu as T  # CPU baseline leg only
    W0 = synth_W(wl, wl.get("seed0", 0))
    h = make_h(wl)
    iters = 1 if name == "cfg5" else wl["iters"]
    t0 = time.perf_counter()
    d = T.caldera(W0, None if h is None else torch.diag_embed(h), Q_bits=wl["Q_bits"], L_bits=wl["L_bits"],
                  R_bits=wl["R_bits"], rank=wl["rank"], iters=iters, lplr_iters=wl["lplr_iters"],
                  sigma_reg=1e-8)
    el = time.perf_counter() - t0
    per = el * wl["iters"] / iters
    cpu = {"value": 1.0 / per, "unit": "matrices/s", "cores": torch.get_num_threads(), "kind": "port",
           "host": host_cpu_info(),
           "sample": (f"seed-0 {wl['m']}x{wl['n']} matrix, {iters} of {wl['iters']} outer iterations of the "
                      f"reference's torch-CPU op sequence (torch.linalg svd/lstsq on MKL, fp32), {el:.1f} s on "
                      f"{torch.get_num_threads()} host threads" + ("" if iters == wl["iters"] else
                                                                  f"; value = 1 / ({el:.1f} s x {wl['iters']})"))}
    par = {}
    if iters == wl["iters"] and dec0 is not None:
        exp = d["Q"].double() + d["L"].double() @ d["R"].double()
        got = (dec0["Q"].double() + dec0["L"].double() @ dec0["R"].double()).cpu()
        par["frob_err_vs_cpu_baseline"] = float(torch.linalg.norm(got - exp) / torch.linalg.norm(exp))
    return cpu, par


def host_cpu_info():
    """the CPU model (/proc/cpuinfo 'model name', as lscpu reports it), the
    host's logical CPUs, and torch's BLAS/LAPACK build (the MKL line of torch.__config__.show())
    the CPU baseline runs on."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    cfg = torch.__config__.show()
    mkl = next((ln.strip(" -") for ln in cfg.splitlines() if "Math Kernel Library" in ln), None)
    cap = next((ln.strip(" -") for ln in cfg.splitlines() if "CPU capability" in ln), None)
    blas = re.findall(r"\b(BLAS_INFO=[^,]*|LAPACK_INFO=[^,]*)", cfg)
    return {"cpu_model": model, "logical_cpus": os.cpu_count(), "torch_threads": torch.get_num_threads(),
            "torch": torch.__version__, "mkl": mkl, "cpu_capability": cap, "blas_lapack": blas,
            "mkl_available": bool(torch.backends.mkl.is_available())}


def single_call_latency(qp, W0, h, dev, calls=3):
    """The reference's own calling pattern (main.py:189-196: one caldera() call per layer): the
    drop-in caldera() on one resident matrix (B = 1), after one warm-up call; median of `calls`."""
    from src.caldera.decomposition.alg import caldera
    H = None if h is None else torch.diag_embed(h)
    caldera(qp, W0, H, device=dev, use_tqdm=False)
    ts = []
    for _ in range(calls):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        d = caldera(qp, W0, H, device=dev, use_tqdm=False)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        del d
    ms = 1000.0 * sorted(ts)[len(ts) // 2]
    return {"ms_per_call": ms, "matrices_per_s": 1000.0 / ms, "calls": calls,
            "note": "one drop-in caldera() call (B = 1) on the seed-0 matrix, resident in HBM, median"}


def model_parity(out, dev):
    """The whole-model results that golden reference runs pin (after the gather, on rank 0):
    layer 0/1 q, k, v, o_proj = config-2 seeds 0-3 / 7-10 (tests/golden/final_codes.npz) and
    layer-0 gate_proj = the cfg4t run (seed 4, 11008 x 4096): relative Frobenius error of
    Q + L R (sketch) and the final integer codes (tests/final_codes.py)."""
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from final_codes import compare, fixture
    fx, g = fixture(), golden()
    pins = {f"model.layers.{l}.self_attn.{p}_proj": (f"cfg2s{7 * l + i}" if 7 * l + i else "cfg2")
            for l in (0, 1) for i, p in enumerate("qkvo")}
    pins["model.layers.0.mlp.gate_proj"] = "cfg4t"
    res = {}
    for r in out:
        tag = pins.get(r.name)
        if tag is None or f"{tag}_rowhash" not in fx.files:
            continue
        m, n = r.m, r.n
        codes = K.unpack_codes(r.codes.to(dev).view(1, -1), m * n, r.Q_bits)
        Q = K.dequantize_uniform(codes.view(1, -1), torch.tensor([r.Q_scale], device=dev), r.Q_bits).view(m, n)
        sk = _sketch(Q, r.L.to(dev), r.R.to(dev), n)
        ref = fx[f"{tag}_sketch_QLR"] if f"{tag}_sketch_QLR" in fx.files else g[f"{tag}_sketch_QLR"]
        res[r.name] = {"golden": tag, "rel_frob_QLR": float(np.linalg.norm(sk - ref) / np.linalg.norm(ref)),
                       "final_codes": compare(tag, codes, m, n)}
    return res


def run_model(args):
    """BASELINE configs[3]: the 224 Llama-2-7B linear weights (random-init fp16, one host RNG
    seed per matrix, resident in HBM before the timed region), rank i % world decomposing
    matrix i (sharding.decompose_sharded: same-shape batches of <= 16 (8 GPUs) / 64 interleaved on
    their own HIP streams), results packed in HBM and gathered to rank 0 over RCCL.  One step = the
    whole model."""
    from ee274_convexcaldera_llm_quantization_amd import sharding as S
    from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams
    from ee274_convexcaldera_llm_quantization_amd.overlap import run_interleaved
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    K.load()
    wl = WORKLOADS["cfg2"]
    qp = make_params(wl)
    items = S.llama2_7b_matrices(32)
    mine = [items[i] for i in S.shard_indices(len(items), world, rank)]
    Wd = {}
    for name, m, n, seed in mine:
        # the survey's recipe on the HOST generator (torch.manual_seed(seed); randn * 0.02 ->
        # fp16), as sharding.engine_decompose_batch and the golden runs: layer-0/1 q,k,v,o
        # (seeds 0-3, 7-10) are tests/golden/final_codes.npz's cfg2 seeds, layer-0 gate_proj
        # (seed 4) is sum_large.npz's cfg4t run
        torch.manual_seed(seed)
        Wd[name] = (torch.randn(m, n) * 0.02).to(torch.float16).to(dev)
    ep = EngineParams.from_caldera_params(qp)

    # a rank's share at 8 GPUs is 28 matrices (3 shape batches, interleaved on their own HIP
    # streams); on fewer GPUs the same-shape batches grow (up to 64) so the one-CU-per-matrix
    # solver kernels fill the chip, and two of them are interleaved at a time (HBM: ~1.2 GB of
    # scratch per 11008x4096 matrix)
    max_batch = args.model_batch or (16 if world >= 8 else 64)
    group = args.model_group or (4 if max_batch <= 16 else 2)

    def make_run_all(grp_size):
        def run_all(batches, on_batch_done=None):
            """groups of grp_size same-shape batches interleaved on HIP streams, one group after
            another; on_batch_done(j, results) as batch j's last part finishes (the overlapped
            gather issues batch j's transfer then, sharding.decompose_sharded)"""
            res = []
            for g0 in range(0, len(batches), grp_size):
                gb = batches[g0:g0 + grp_size]
                parts, owner = [], []
                for j, b in enumerate(gb):
                    k = max(1, min(args.model_parts, len(b)))
                    for i in range(k):
                        parts.append(b[len(b) * i // k:len(b) * (i + 1) // k])
                        owner.append(g0 + j)
                engines = [CalderaEngine(ep) for _ in parts]
                left = {}
                for o in owner:
                    left[o] = left.get(o, 0) + 1

                def results_of(j):
                    return [S.MatrixResult(name, m, n, d["L"].shape[1], qp.Q_bits, d["codes"], d["Q_scale"], d["L"],
                                           d["R"], d["global_scale"], d["errors"])
                            for b, e, o in zip(parts, engines, owner) if o == j
                            for (name, m, n, _), d in zip(b, e.last_packed)]

                def part_done(i, _):
                    left[owner[i]] -= 1
                    if left[owner[i]] == 0 and on_batch_done is not None:
                        on_batch_done(owner[i], results_of(owner[i]))

                run_interleaved([e.run_iter(torch.stack([Wd[it[0]] for it in b])) for e, b in zip(engines, parts)],
                                dev, on_done=part_done)
                res += [r for j in range(g0, g0 + len(gb)) for r in results_of(j)]
            return res
        return run_all

    run_all = make_run_all(group)

    def decompose(batch_items):
        return run_all([batch_items])
    decompose.run_all = run_all
    decompose.blob_bound = lambda m, n: S.blob_bound(m, n, qp.Q_bits, qp.rank)

    def step():
        return S.decompose_sharded(items, decompose, rank=rank, world=world, max_batch=max_batch, device=dev)

    emu = None
    if args.emulate_world:
        # strong-scaling projection on ONE GPU ("scaling 1->8 GPUs (cfg4) >= 6x"):
        # time exactly rank r's round-robin share of the model at world W (shard_indices(224, W, r),
        # the batch sizes a W-GPU run uses) plus the packing of its results for the gather, for
        # every r (or --emulate-rank); the RCCL transfer itself is not included
        assert world == 1, "--emulate-world runs on one GPU"
        W_ = args.emulate_world
        mb_e = args.model_batch or (16 if W_ >= 8 else 64)
        grp_e = args.model_group or (4 if mb_e <= 16 else 2)

        run_all_e = make_run_all(grp_e)

        def dec_e(batch_items):
            return run_all_e([batch_items])
        dec_e.run_all = run_all_e
        ranks = [args.emulate_rank] if args.emulate_rank is not None else list(range(W_))
        share_t, tails = {}, {}
        for r_ in ranks:
            events = []

            def share_step(rec=None):
                t0 = time.perf_counter()

                def done(j, res_j):  # batch j of this share finished: its transfer could start now
                    if rec is not None:
                        rec.append((time.perf_counter() - t0, sum(r.codes.numel() * r.codes.element_size()
                                                                  + 4 * r.L.numel() + 4 * r.R.numel() for r in res_j)))
                S.decompose_sharded(items, dec_e, rank=r_, world=W_, max_batch=mb_e, gather=False, device=dev,
                                    on_batch_done=done)
            for _ in range(max(1, args.warmup)):
                share_step()
            torch.cuda.synchronize()
            ts, recs = [], []
            for _ in range(args.steps):
                rec = []
                t0 = time.perf_counter()
                share_step(rec)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
                recs.append(rec)
            k = sorted(range(len(ts)), key=lambda i: ts[i])[len(ts) // 2]
            share_t[r_] = ts[k]
            tails[r_] = recs[k]
        # the overlapped gather (sharding.decompose_sharded): batch j's packed arrays leave as it
        # finishes; a rank's transfers queue on its own xGMI link to rank 0 (fully connected, 7 x
        # ~153 GB/s per GPU: SURVEY.md "Comm note for MI355X"), so only what is still in flight when
        # the share's compute ends is exposed.  Rank 0's own share is local (no link)
        link = XGMI_LINK_GBS * 1e9

        def exposed(rec, t_end):
            busy = 0.0
            for t, nb in sorted(rec):
                busy = max(busy, t) + nb / link
            return max(0.0, busy - t_end)

        exp_s = {r_: (0.0 if r_ == 0 else exposed(tails[r_], share_t[r_])) for r_ in ranks}
        nov_s = {r_: (0.0 if r_ == 0 else sum(nb for _, nb in tails[r_]) / link) for r_ in ranks}
        # worst case: rank 0's ingress serialised onto one link, every peer's batches in one queue
        allrec = [(t, nb) for r_ in ranks if r_ != 0 for t, nb in tails[r_]]
        ser = exposed(allrec, max(share_t.values())) if allrec else 0.0
        emu = {"world": W_, "ranks_timed": ranks, "max_batch": mb_e, "interleaved_batches": grp_e,
               "matrices_per_share": len(S.shard_indices(len(items), W_, ranks[0])),
               "share_s": {str(k): v for k, v in share_t.items()}, "max_share_s": max(share_t.values()),
               "gather_model": {"xgmi_link_gbs": XGMI_LINK_GBS,
                                "source": "SURVEY.md comm note: 8 GPUs fully connected, 7 links x ~153 GB/s per GPU",
                                "share_payload_bytes": {str(k): int(sum(nb for _, nb in v)) for k, v in tails.items()},
                                "exposed_overlapped_s": {str(k): v for k, v in exp_s.items()},
                                "exposed_unoverlapped_s": {str(k): v for k, v in nov_s.items()},
                                "exposed_serialised_ingress_s": ser},
               "note": "rank r's round-robin share decomposed on one GPU (median of --steps); the gather's exposed "
                       "tail is modelled from each batch's measured finish time and packed bytes"}

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    for _ in range(args.steps):
        out = None
        out = step()
    # (decompose_sharded gathers inside step(): its last batch's transfer is inside the region)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        assert out is not None and [r.name for r in out] == [it[0] for it in items], "gather incomplete"
        result = {
            "metric": "weight matrices/sec (Llama-2-7B linear weights, rank-128, Q=2-bit, whole model)",
            "value": len(items) * args.steps / el, "unit": "matrices/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * el / args.steps, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None,
            "dtype": "f32 (fp16 W in; fp32-grade split-fp16 MFMA products, fp64 small solves; int2 codes)",
            "data": "synthetic: 224 random-init fp16 Llama-2-7B-shaped weights (randn*0.02, host RNG, seed = layer*7+proj)",
            "config": {"workload": "BASELINE configs[3]: 224 Llama-2-7B linear weights (32 x q,k,v,o 4096x4096, "
                                   "gate,up 11008x4096, down 4096x11008), r 128, Q2, L/R 16, iters 5, H = I; "
                                   "round-robin matrix sharding, RCCL gather of the packed (Q, L, R) to rank 0",
                       "name": "model", "matrices_per_step": len(items), "matrices_on_rank0": len(mine),
                       "max_batch": max_batch, "interleaved_batches": group,
                       "parallelism": f"dp{world} (matrix-sharded)"},
            "gathered_bytes": int(sum(r.codes.numel() * r.codes.element_size() + r.L.numel() * 4 + r.R.numel() * 4
                                      for r in out)),
            "gather": dict(S.LAST_GATHER),
        }
        if emu is not None:
            t1 = el / args.steps
            emu["t_model_1gpu_s"] = t1
            W_ = emu["world"]
            sh = {int(k): v for k, v in emu["share_s"].items()}
            gm = emu["gather_model"]
            emu[f"projected_speedup_{W_}"] = t1 / emu["max_share_s"]
            emu[f"projected_speedup_{W_}_incl_gather"] = t1 / max(
                sh[r_] + gm["exposed_overlapped_s"][str(r_)] for r_ in sh)
            emu[f"projected_speedup_{W_}_incl_gather_unoverlapped"] = t1 / max(
                sh[r_] + gm["exposed_unoverlapped_s"][str(r_)] for r_ in sh)
            emu[f"projected_speedup_{W_}_incl_gather_serialised_ingress"] = t1 / (emu["max_share_s"]
                                                                               + gm["exposed_serialised_ingress_s"])
            result["strong_scaling_projection"] = emu
        if not args.no_parity:
            result["parity_pinned"] = model_parity(out, dev)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


MAIN_PROJS = (("self_attn.q_proj", 896, 896), ("self_attn.o_proj", 896, 896), ("mlp.gate_proj", 4864, 896),
              ("mlp.up_proj", 4864, 896), ("mlp.down_proj", 896, 4864))


def run_main(args):
    """main.py's own workload (main.py:135-251 with its defaults): the projections of language-model
    layers 17-23 whose both dims exceed 500 (q, o 896x896; gate, up 4864x896; down 896x4864 -- 35
    matrices), each with ITS OWN diagonal Hessian (the real diag_Hessians.pt entries,
    tests/golden/main_hessians.npz), at the driver's parameters (rank 200, Q2, L/R 16, iters 5,
    lplr_iters 5, sigma_reg 1e-8, scale_W=False), on synthetic fp16 weights (randn * 0.02, seed =
    100 + layer-major index).  One step = every layer decomposed through the drop-in API as the
    layer-replacement caller runs it (model.py: api.caldera_groups -- same-shape layers batched with
    per-matrix Hessians, the three shape batches interleaved on HIP streams).  Beside it, the
    reference's calling pattern: one drop-in caldera() per layer (B = 1, main.py:189-196), timed
    over the same 35 layers."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != 1:
        raise SystemExit("bench.py --workload main runs on one GPU (the reference's caller is single-device)")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from ee274_convexcaldera_llm_quantization_amd import api, model
    from src.caldera.decomposition.alg import caldera
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    K.load()
    hz = np.load(os.path.join(ROOT, "tests", "golden", "main_hessians.npz"), allow_pickle=False)
    qp = model.driver_params(rank=200)
    jobs = []
    for layer in range(17, 24):
        for proj, m, n in MAIN_PROJS:
            name = f"language_model.model.layers.{layer}.{proj}"
            torch.manual_seed(100 + len(jobs))
            W = (torch.randn(m, n) * 0.02).to(torch.float16).to(dev)
            h = torch.from_numpy(hz[name]).to(dev)
            assert h.numel() == n
            jobs.append((name, W, h))
    shapes = {}
    for j in jobs:
        shapes.setdefault(tuple(j[1].shape), []).append(j)
    groups = list(shapes.values())

    def step():
        return api.caldera_groups(qp, [([j[1] for j in g], [j[2] for j in g]) for g in groups], device=dev,
                                  scale_W=False)

    def loop():
        return [caldera(qp, W, torch.diag_embed(h), device=dev, use_tqdm=False, scale_W=False) for _, W, h in jobs]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    for _ in range(args.steps):
        out = None
        out = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    loop()  # warm-up of the B = 1 path
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ref = loop()
    torch.cuda.synchronize()
    el1 = time.perf_counter() - t1
    # the batched results against the per-layer calls on the same matrices (another batch size:
    # split-K and lockstep scheduling differ, so agreement is to the solver tolerance, not bits)
    flat = [d for g in out for d in g]
    order = [j[0] for g in groups for j in g]
    by_name = dict(zip(order, flat))
    rel, flips = [], 0
    for (name, W, h), d1 in zip(jobs, ref):
        d = by_name[name]
        n = W.shape[1]
        a, b = _sketch(d.Q.to(dev), d.L.to(dev), d.R.to(dev), n), _sketch(d1.Q.to(dev), d1.L.to(dev), d1.R.to(dev), n)
        rel.append(float(np.linalg.norm(a - b) / np.linalg.norm(b)))
        flips += int((d.Q_idxs.cpu() != d1.Q_idxs.cpu()).sum())
    n_mat = len(jobs)
    print(json.dumps({
        "metric": "weight matrices/sec (main.py layer set: 35 projections of layers 17-23, rank-200, Q=2-bit, "
                  "per-layer real diag Hessians)",
        "value": n_mat * args.steps / el, "unit": "matrices/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1000.0 * el / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None,
        "dtype": "f32 (fp16 W in; fp32-grade split-fp16 MFMA products, fp64 small solves; int2 codes)",
        "data": "synthetic fp16 weights randn*0.02 (seed 100 + index) with the REAL diag_Hessians.pt entries "
                "of each layer (tests/golden/main_hessians.npz)",
        "config": {"workload": "main.py:135-251 defaults: language-model layers 17-23, q/o 896x896, gate/up "
                               "4864x896, down 896x4864; rank 200, Q2, L/R 16, iters 5, lplr 5, sigma_reg 1e-8, "
                               "scale_W=False; H = diag_embed(Hall[name]) per layer",
                   "name": "main", "matrices_per_step": n_mat,
                   "shape_batches": {f"{k[0]}x{k[1]}": len(v) for k, v in shapes.items()},
                   "parallelism": "dp1 (same-shape layers batched with per-matrix Hessians; shape batches "
                                  "interleaved on HIP streams)"},
        "b1_loop": {"matrices_per_s": n_mat / el1, "ms_per_layer": 1000.0 * el1 / n_mat,
                    "note": "the reference's calling pattern: one drop-in caldera() per layer (B = 1, "
                            "main.py:189-196), same 35 layers, resident in HBM"},
        "speedup_vs_b1_loop": (n_mat * args.steps / el) / (n_mat / el1),
        "batched_vs_b1": {"max_rel_frob_QLR": max(rel), "median_rel_frob_QLR": float(np.median(rel)),
                          "final_code_flips_total": flips},
    }), flush=True)


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` without WORLD_SIZE: run `python -m torch.distributed.run
    --nproc-per-node N bench.py <argv>` as a fresh child process (this process has not touched
    the GPU: importing torch does not) and return its exit code.  The ranks inherit stdout, so
    rank 0's one JSON line is this command's output."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # RCCL over dmabuf IPC (the box's only mode)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    sys.stdout.flush()
    return subprocess.run(cmd, env=env).returncode


def run_dry(args):
    """--dry-run: the N-rank step of main() without the GPU -- gloo process group on the CPU,
    every rank 'decomposes' its batch with a deterministic stub (tiny matrices: packed 2-bit
    codes, L, R of the result shapes; no arithmetic, no oracle), packs the results and gathers
    them to rank 0 inside the timed step, barrier + max over ranks; rank 0 prints one JSON line."""
    import torch.distributed as dist
    from ee274_convexcaldera_llm_quantization_amd import sharding as S
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    B, m, n, r = args.batch or 4, 32, 64, 4

    def step():
        g = torch.Generator().manual_seed(rank)
        res = [S.MatrixResult(f"rank{rank}.m{j}", m, n, r, 2, torch.randint(0, 256, (m * n // 4,), generator=g,
                                                                               dtype=torch.uint8),
                              1.0, torch.zeros(m, r), torch.zeros(r, n), 1.0, {"Q": [1.0], "LR": [1.0]})
               for j in range(B)]
        if world > 1:
            pl = S.gather_to_rank0(S.pack_results(res), device=torch.device("cpu"))
            return None if pl is None else [x for p in pl for x in S.unpack_results(p)]
        return res

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    out = None
    for _ in range(args.steps):
        out = step()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        assert out is not None and len(out) == B * world, "gather incomplete"
        print(json.dumps({
            "metric": "dry run (stub decomposer, gloo): N-rank launch + gather plumbing, not a measurement",
            "value": B * world * args.steps / el, "unit": "matrices/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * el / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "none (stub)", "data": "synthetic stub results",
            "dry_run": True, "gathered_matrices": len(out),
            "config": {"workload": "dry-run", "batch_per_gpu": B, "parallelism": f"dp{world} (matrix-sharded)"}}),
            flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=None, help="matrices per GPU (default: per workload)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS) + ["model", "main"], default="cfg2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-api-path", action="store_true")
    ap.add_argument("--model-parts", type=int, default=1,
                    help="model workload: each same-shape batch as this many interleaved parts")
    ap.add_argument("--model-group", type=int, default=None,
                    help="model workload: same-shape batches interleaved at a time (default 4 for batches <= 16, "
                         "else 2)")
    ap.add_argument("--model-batch", type=int, default=None,
                    help="--workload model: same-shape batch size (default 64 below 8 GPUs, 16 at 8)")
    ap.add_argument("--emulate-world", type=int, default=None,
                    help="--workload model on one GPU: also time each rank's share at this world size "
                         "(projected strong scaling)")
    ap.add_argument("--emulate-rank", type=int, default=None, help="with --emulate-world: only this rank")
    ap.add_argument("--solver-tol-steps", type=str, default=None,
                    help="comma-separated solver tolerances of the first LR updates (then the default)")
    ap.add_argument("--solver-refine-steps", type=str, default=None,
                    help="per LR update, '+'-separated filter degrees of extra outer iterations after "
                         "convergence, updates separated by ',' (e.g. '6' or '6+4,4')")
    ap.add_argument("--deg-cold", type=str, default=None,
                    help="comma-separated Chebyshev degrees of a cold solve's outer iterations (the last repeats; "
                         "default solver.RankRSolver's)")
    ap.add_argument("--no-l-split", action="store_true", help="sparse Gram without the l-split ELL (A/B)")
    ap.add_argument("--no-transposed-output", action="store_true",
                    help="solver products without the C^T epilogue output (transpose passes instead; A/B)")
    ap.add_argument("--streams", type=int, default=None,
                    help="batch parts interleaved on separate HIP streams (default: overlap.default_parts, "
                         "2 from 16 matrices on)")
    ap.add_argument("--dry-run", action="store_true",
                    help="plumbing test of the N-rank path: gloo on the CPU, a stub decomposer on tiny "
                         "matrices (no HIP device); the JSON line says dry_run")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the driver's form `python bench.py --gpus N`: one process per GPU, started here
        return launch_ranks(args.gpus, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one process per GPU "
                         f"(python bench.py --gpus N, or torch.distributed.run --nproc-per-node N ... --gpus N)")
    if args.dry_run:
        return run_dry(args)
    if args.workload == "model":
        return run_model(args)
    if args.workload == "main":
        return run_main(args)
    wl = WORKLOADS[args.workload]

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from ee274_convexcaldera_llm_quantization_amd import api, solver
    from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams
    from ee274_convexcaldera_llm_quantization_amd.overlap import default_parts, run_interleaved
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    K.load()
    if args.no_l_split:
        from ee274_convexcaldera_llm_quantization_amd import sgram
        sgram.L_SPLIT = False
    if args.no_transposed_output:
        solver.TRANSPOSED_OUT = False
    qp = make_params(wl)
    ep = EngineParams.from_caldera_params(qp)
    B = args.batch or wl["batch"]
    # rank 0 holds the pinned seeds (parity_timed_step); other ranks' batches come from the
    # device generator only, and each rank's host threads are capped at its share of the cores
    if world > 1:
        torch.set_num_threads(max(1, torch.get_num_threads() // world))
    pinned = (HOLDOUT[-1] + 1 if args.workload == "cfg2" else PINNED) if rank == 0 else 0
    Wb = synth_batch(wl, B, wl.get("seed0", 0) + 1000 * rank, dev, host=pinned)
    h = make_h(wl)
    h = None if h is None else h.to(dev)
    parts = max(1, args.streams or default_parts(B))
    tol_steps = tuple(float(x) for x in args.solver_tol_steps.split(",")) if args.solver_tol_steps else None
    refine_steps = (tuple(tuple(int(d) for d in x.split("+") if d) for x in args.solver_refine_steps.split(","))
                    if args.solver_refine_steps else None)

    skw = {"deg_cold": tuple(int(x) for x in args.deg_cold.split(","))} if args.deg_cold else None

    def step(nparts=None):
        nparts = parts if nparts is None else nparts
        # the hot path: caldera() (alg.py:24-112) on B matrices resident in HBM, results
        # (packed Q codes + scale, L, R, dequantised Q, error history) left in HBM.  The
        # drop-in API layer adds only output placement (alg.py:81 copies W to the host); it is
        # timed separately below ("api_path").
        engines = [CalderaEngine(ep, solver_kwargs=skw) for _ in range(nparts)]
        for e in engines:
            e.solver_tol_steps = tol_steps
            if refine_steps is not None:
                e.solver_refine_steps = refine_steps
        bnd = [B * i // nparts for i in range(nparts + 1)]
        outs = run_interleaved([e.run_iter(Wb[bnd[i]:bnd[i + 1]], h, True) for i, e in enumerate(engines)], dev)
        # no reference cycles: the previous step's buffers must be freed as soon as the
        # next step drops them, or the caching allocator grows and stalls on hipMalloc
        if world > 1:
            # N > 1: the one collective north_star names -- every rank's packed results
            # (2-bit codes, L, R, scales, errors) gathered to rank 0 over RCCL (HBM -> HBM).
            # Issued asynchronously: step i's transfer runs on the collective's stream under step
            # i + 1's compute and is waited for before step i + 1 issues its own (the last one
            # at the end of the timed region, inside it)
            from ee274_convexcaldera_llm_quantization_amd import sharding as S
            res = [S.MatrixResult(f"rank{rank}.m{j}", wl["m"], wl["n"], wl["rank"], wl["Q_bits"], d["codes"],
                                  d["Q_scale"], d["L"], d["R"], d["global_scale"], d["errors"])
                   for j, d in enumerate(pd for e in engines for pd in e.last_packed)]
            payload = S.pack_results(res, device=dev)
            finish_gather()   # stream-ordered: the host does not block here
            gather_stats["pending"] = S.gather_to_rank0_async(payload, device=dev,
                                                              sizes=[payload.numel()] * world)
            gather_stats["calls"] += 1
        return [d for o in outs for d in o], engines[0]

    gather_stats = {"ms": 0.0, "calls": 0, "bytes": 0, "ranks": 0, "pending": None}

    def finish_gather(tail=False):
        """Retire the previous step's gather: its completion is stream-ordered before what the
        current stream issues next (no host block).  tail (the end of the timed region): the
        compute is drained first, then the time to the gather's completion is its exposed part
        (gather_ms_per_step, per timed step)."""
        pg = gather_stats["pending"]
        if pg is None:
            return
        if tail:
            torch.cuda.synchronize()
            tg = time.perf_counter()
        pl = pg.wait()
        if tail:
            torch.cuda.synchronize()
            gather_stats["ms"] += 1000.0 * (time.perf_counter() - tg)
        gather_stats["bytes"] = 0 if pl is None else int(sum(x.numel() for x in pl))
        gather_stats["ranks"] = 0 if pl is None else len(pl)
        gather_stats["pending"] = None

    for _ in range(args.warmup):
        step()
    finish_gather(tail=True)
    torch.cuda.synchronize()
    if os.environ.get("CQ_BENCH_VERBOSE"):
        print(f"warmup done; reserved {torch.cuda.memory_reserved() / 2**30:.1f} GiB", file=sys.stderr, flush=True)
    # time the dominant kernel (the G X filter GEMMs) with HIP events on its stream
    solver.EVENT_PROBE.enable(True, max_pairs=400)
    solver.QUANT_PROBE.enable(True, max_pairs=8 * args.steps * parts)
    solver.LPLR_PROBE.enable(wl["L_bits"] < 16, max_pairs=64)
    solver.GRAM_PROBE.enable(True, max_pairs=16 * args.steps * parts)
    gather_stats.update(ms=0.0, calls=0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    decs = eng = None
    verbose = bool(os.environ.get("CQ_BENCH_VERBOSE"))
    for i in range(args.steps):
        decs = eng = None  # release the previous step's results before the next allocates
        decs, eng = step()
        if verbose:
            torch.cuda.synchronize()
            print(f"step {i}: {time.perf_counter() - t0:.3f} s (cumulative); reserved "
                  f"{torch.cuda.memory_reserved() / 2**30:.1f} GiB", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    solver.EVENT_PROBE.enable(False)
    probe = solver.EVENT_PROBE.summary()
    qprobe = solver.QUANT_PROBE.summary()
    solver.QUANT_PROBE.enable(False)
    lprobe = solver.LPLR_PROBE.summary()
    solver.LPLR_PROBE.enable(False)
    gprobe = solver.GRAM_PROBE.summary()
    solver.GRAM_PROBE.enable(False)
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total = args.steps * B * world
    value = total / el
    metric = ("weight matrices/sec (4096x4096, rank-128, Q=2-bit) + Frob err vs ref" if args.workload == "cfg2"
              else f"weight matrices/sec ({wl['m']}x{wl['n']}, rank-{wl['rank']}, Q={wl['Q_bits']}-bit, "
                   f"L/R={wl['L_bits']}-bit) + Frob err vs ref")
    result = {
        "metric": metric,
        "value": value, "unit": "matrices/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1000.0 * el / args.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32 (fp16 W in; fp32-grade split-fp16 MFMA products, fp64 small solves; int2 codes)",
        "data": f"synthetic: W = randn({wl['m']},{wl['n']})*0.02 -> fp16, seed per matrix",
        "config": {"workload": wl["desc"], "name": args.workload,
                   "batch_per_gpu": B, "matrices_per_step": B * world, "parallelism": f"dp{world} (matrix-sharded)"},
    }
    solver_p = eng.solver.p if eng.solver is not None else None

    def roofline_of(probe, launch_batch):
        """The dominant kernel's roofline from a probe summary (HIP events on its stream)."""
        t = probe["avg_ms"] * 1e-3
        flops, nbytes = probe["flops_per_launch"], probe["bytes_per_launch"]
        x3 = probe["kernel"].startswith("gemm_x3")
        # MFMA ceiling: split-fp16 products issue 3 fp16 MFMAs per fp32-equivalent product
        mfma_peak = PEAK_F16_MFMA_TFLOPS / 3.0 if x3 else PEAK_FP32_MFMA_TFLOPS
        t_mfma = flops / (mfma_peak * 1e12)
        t_hbm = nbytes / (PEAK_HBM_GBS * 1e9)
        traffic = None  # HBM bytes per launch from the committed PMC pass of this same config
        pmc_path = os.path.join(ROOT, "bench_pmc_traffic.json")  # travels to the GPU box (profiles/ does not)
        if os.path.exists(pmc_path):
            pms = json.load(open(pmc_path))
            for pm in (pms if isinstance(pms, list) else [pms]):
                if (pm["config"]["batch"] == launch_batch and pm["config"]["p"] == solver_p
                        and pm["config"].get("workload", "cfg2") == args.workload and pm["kernel"] == probe["kernel"]):
                    traffic = pm["hbm_bytes_per_launch"]
        ach_tf = flops / t / 1e12
        ach_gb = nbytes / t / 1e9
        if t_hbm >= t_mfma:
            roof = {"bound": "hbm", "achieved": ach_gb, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": ach_gb / PEAK_HBM_GBS}
        else:
            roof = {"bound": "mfma", "achieved": ach_tf, "peak": mfma_peak, "unit": "TFLOP/s",
                    "frac": ach_tf / mfma_peak}
        roof.update({"traffic": traffic, "kernel": probe["kernel"], "launches_timed": probe["count"],
                     "avg_launch_ms": probe["avg_ms"], "bytes_per_launch": nbytes,
                     "flops_per_launch_fp32_equiv": flops, "achieved_tflops_fp32_equiv": ach_tf,
                     "mfma_frac": ach_tf / mfma_peak, "solver_block_p": solver_p,
                     "matrices_per_launch": launch_batch})
        return roof

    def probe_of(summ, key):
        """the summary restricted to one probed kernel (the split-fp16 filter step <0> is the
        headline kernel; <1> the single-product steps)"""
        for kn, g in summ.get("kernels", {}).items():
            if kn.startswith(key):
                return {"count": g["count"], "avg_ms": g["avg_ms"], "flops_per_launch": g["flops_per_launch"],
                        "bytes_per_launch": g["bytes_per_launch"], "kernel": kn}
        return None

    p0 = probe_of(probe, "gemm_x3v_kernel<0>") if probe["count"] else None
    if p0 is None and probe["count"]:
        p0 = probe
    if p0 is not None:
        result["roofline"] = roofline_of(p0, B // parts)
        p1 = probe_of(probe, "gemm_x3v_kernel<1>")
        if p1 is not None:
            r1 = roofline_of(p1, B // parts)
            result["roofline_single_product"] = {k: r1[k] for k in ("bound", "achieved", "peak", "unit", "frac",
                                                                   "kernel", "launches_timed", "avg_launch_ms",
                                                                   "bytes_per_launch")}
        ag = probe.get("aggregate")
        if ag and ag["busy_ms"] > 0:
            gbs = ag["bytes"] / (ag["busy_ms"] * 1e-3) / 1e9
            result["roofline_aggregate"] = {
                "bound": "hbm", "achieved": gbs, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS,
                "launches": ag["launches"], "bytes": ag["bytes"], "busy_ms": ag["busy_ms"],
                "window_ms": ag["window_ms"],
                "note": (f"all probed filter launches (split <0> and single-product <1>) of the {parts} interleaved "
                         "parts' streams: their algorithmic bytes over the UNION of their launch windows (one clock "
                         "for all streams) -- the chip-level filter rate while the parts share it; the per-launch "
                         "frac above is one launch's rate under that sharing")}
        if parts > 1:
            result["roofline"]["concurrency"] = (
                f"{parts} interleaved batch parts on separate HIP streams: each launch shares the chip with the "
                "other part's kernels (the one-CU-per-matrix eigensolves and whitening run beside it), so its "
                "duration and this frac are per launch under that sharing; roofline_solo times the same kernel "
                "with one part")
    # the quantise kernel (fused Q update, every pass of a call; SURVEY.md 8(d) bytes_Q per call):
    # "w" = first Q step (quantise W itself, pure HBM), "lr" = Q steps recomputing W - L R on
    # split-fp16 MFMAs (3 fp16 products per fp32-equivalent flop; one recompute on the 2-bit list path)
    qroof = {}
    for kind, g in qprobe.items():
        t = g["avg_ms"] * 1e-3
        gbs = g["bytes_per_launch"] / t / 1e9
        # one recompute of L R per call, three fp16 products each: the 2-bit
        # list path (cq_q_update_x3 scale_hint) recomputes once; other widths take two passes
        f16 = 3 * g["flops_per_launch"]
        t_mfma = f16 / (PEAK_F16_MFMA_TFLOPS * 1e12)
        t_hbm = g["bytes_per_launch"] / (PEAK_HBM_GBS * 1e9)
        qroof["first_Q" if kind == "w" else "Q_with_LR"] = {
            "bound": "hbm" if t_hbm >= t_mfma else "mfma", "achieved_gbs": gbs, "frac_hbm": gbs / PEAK_HBM_GBS,
            "achieved_tflops_f16": f16 / t / 1e12, "frac_mfma": (f16 / t / 1e12) / PEAK_F16_MFMA_TFLOPS,
            "frac_of_bound": max(t_hbm, t_mfma) / t, "launches_timed": g["count"], "avg_call_ms": g["avg_ms"],
            "bytes_per_call": g["bytes_per_launch"],
            "kernel": ("quant_w_stream_kernel (cq_q_update_x3, r = 0, max|W| known)" if kind == "w"
                       else "q_update_p_kernel<2> + qp_codes_kernel (2-bit: one L R recompute, candidate lists; "
                            "q_update_p_kernel<0|1> two passes otherwise or on fallback)")}
        if kind != "w":
            qroof["Q_with_LR"]["second_recomputes_last_step"] = eng.q_fallbacks
    if qroof:
        result["roofline_quantise"] = qroof
    if lprobe:
        # the quantised-factor LPLR loop's m x n x r products (alg.py:162-177): split-fp16
        # (3 fp16 MFMA products per fp32-grade product) when Y is unweighted, else fp32 MFMA GEMMs.
        # achieved_tflops counts the algorithmic 2 m n r; frac_mfma prices the MFMA work actually
        # issued against its own dense peak (3 x fp16 products vs the fp16 peak for the split path)
        lx3 = eng.lplr_x3 and not wl["H"]
        result["roofline_lplr"] = {}
        for kind, g in lprobe.items():
            ach = g["flops_per_launch"] / (g["avg_ms"] * 1e-3) / 1e12
            result["roofline_lplr"][kind] = {
                "bound": "mfma", "achieved_tflops": ach,
                "peak_tflops": PEAK_F16_MFMA_TFLOPS / 3 if lx3 else PEAK_FP32_MFMA_TFLOPS,
                "frac_mfma": ach / (PEAK_F16_MFMA_TFLOPS / 3 if lx3 else PEAK_FP32_MFMA_TFLOPS),
                "frac_of_fp32_peak": ach / PEAK_FP32_MFMA_TFLOPS,
                "launches_timed": g["count"], "avg_call_ms": g["avg_ms"], "flops_per_call": g["flops_per_launch"],
                "kernel": ("x3 split-fp16 kernel (cq_gemm_x3, 3 x v_mfma_f32_16x16x32_f16)" if lx3
                           else "gemm_f32_kernel (v_mfma_f32_32x32x2_f32)")}
    if gprobe:
        # the LR update's MFMA-bound kernel (north_star: "MFMA utilisation on the LR update"):
        # the split-fp16 Gram (gemm_x3v_kernel<0>, sym_out), 3 fp16 MFMA products over the
        # upper half of the symmetric k x k output (fp32-equivalent flops k^2 n).  With sparse
        # 2-bit codes (sgram.py) it runs once per run on W's halves (A = W W^T, kind gram_A) and
        # every LR step forms G = A - s (P + P^T) from the codes (kind gram_sparse, HBM-bound)
        kind = "gram" if "gram" in gprobe else "gram_A" if "gram_A" in gprobe else None
        if kind is not None:
            gp = gprobe[kind]
            t = gp["avg_ms"] * 1e-3
            ach = gp["flops_per_launch"] / t / 1e12
            result["roofline_gram"] = {
                "bound": "mfma", "achieved": ach, "peak": PEAK_F16_MFMA_TFLOPS, "unit": "TFLOP/s (fp16 MFMA)",
                "frac": ach / PEAK_F16_MFMA_TFLOPS, "launches_timed": gp["count"], "avg_launch_ms": gp["avg_ms"],
                "f16_flops_per_launch": gp["flops_per_launch"], "fp32_equiv_tflops": ach / 3.0,
                "bytes_per_launch": gp["bytes_per_launch"],
                "operand": "Y = (W - Q) diag(ycol) per LR step" if kind == "gram" else
                           "W diag(ycol), once per decomposition (A of the sparse-code Gram)",
                "kernel": ("gemm_x3v_kernel<0> (split-fp16 Gram, sym_out: writes G's K-blocked halves)"
                           if kind == "gram" else "gemm_x3v_kernel<1|0> (Gram of W: one fp16 product when "
                           "H = I, W being exact in fp16; split-fp16 otherwise)")}
        if "gram_sparse" in gprobe:
            gp = gprobe["gram_sparse"]
            t = gp["avg_ms"] * 1e-3
            ach = gp["bytes_per_launch"] / t / 1e9
            result["roofline_gram_sparse"] = {
                "bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
                "launches_timed": gp["count"], "avg_launch_ms": gp["avg_ms"],
                "bytes_per_launch": gp["bytes_per_launch"],
                "kernels": "sgram_fill + sgram_spmm + sgram_combine (G = A - s (P + P^T) from the 2-bit codes)"}
    if world > 1:
        result["gather"] = {"collective": "torch.distributed.gather (RCCL) of packed (codes, L, R) to rank 0",
                            "gathered_bytes_per_step": gather_stats["bytes"], "ranks": gather_stats["ranks"],
                            "gather_ms_per_step": gather_stats["ms"] / max(1, gather_stats["calls"]),
                            "overlap": "step i's gather issued async on the collective's stream under step "
                                       "i + 1's compute (stream-ordered retire before step i + 1's own); "
                                       "gather_ms_per_step = the exposed tail after the last step's compute "
                                       "(inside the timed region) over the timed steps",
                            "included_in_value": True}
    st = eng.solver.stats.as_dict() if eng.solver is not None else {}
    result["solver"] = {"parts": parts, "deg_cold": list(eng.solver.deg_cold) if eng.solver is not None else None,
                        "matvecs_per_part": st.get("matvecs", 0),
                        "outer_iters": st.get("outer", 0), "stalled_matrices": st.get("stalls", 0),
                        "jacobi_unconverged": st.get("jacobi_unconverged", 0),
                        "block_jacobi_readbacks": st.get("bj_readbacks", 0),
                        "refine_iters": st.get("refines", 0)}
    if rank == 0 and not args.no_parity:
        # parity of the LAST TIMED STEP's own results (rank 0: batch positions 0-3 = seeds 0-3)
        par = parity_of_timed_step(args.workload, decs, wl)
        result["frob_err_vs_ref_sketch"] = par["seed0"]
        result["parity_timed_step"] = {"vs": "reference golden run of the same matrix (tests/golden/sum_large.npz, "
                                             "16-column Gaussian sketch of Q + L R)", **par}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, par = cpu_baseline(args.workload, wl, decs[0] if decs else None)
        result["cpu_baseline"] = cpu
        result.update(par)
    decs = eng = None
    if not args.no_api_path:
        # the drop-in API (caldera_batch: the reference's output placement, W copied to the host
        # as alg.py:81 does, dataclass assembly) on one extra step of the same resident batch
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = api.caldera_batch(qp, Wb, None if h is None else torch.diag_embed(h), device=dev)
        torch.cuda.synchronize()
        ta = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([ta], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ta = float(t.item())
        del out
        result["api_path"] = {"matrices_per_s": B * world / ta, "ms_per_step": 1000.0 * ta,
                              "note": "one step through api.caldera_batch (drop-in layout, W to host)"}
        if rank == 0 and world == 1:
            result["api_single"] = single_call_latency(qp, Wb[0], h, dev)
    if parts > 1 and world == 1 and probe["count"]:
        # the dominant kernel alone: one untimed step of the whole batch as one part (launches of
        # B matrices, nothing beside them), HIP events as in the timed region.  The parts' cached
        # scratch (scratch.py: per stream and shape) goes back to the device first: the one-part
        # buffers are twice as large, and at config 3 (B = 192) both sets do not fit 288 GB.
        # Last, after the API path, which reuses the parts' warm scratch (after a release its
        # step would time the re-allocation: 7.1 s instead of 0.85 s)
        from ee274_convexcaldera_llm_quantization_amd import scratch
        scratch.release()
        torch.cuda.empty_cache()
        solver.EVENT_PROBE.enable(True, max_pairs=400)
        solver.QUANT_PROBE.enable(True, max_pairs=16)
        step(1)
        torch.cuda.synchronize()
        solver.EVENT_PROBE.enable(False)
        psolo = solver.EVENT_PROBE.summary()
        qsolo = solver.QUANT_PROBE.summary()
        solver.QUANT_PROBE.enable(False)
        if psolo["count"]:
            result["roofline_solo"] = roofline_of(probe_of(psolo, "gemm_x3v_kernel<0>") or psolo, B)
            result["roofline_solo"]["note"] = ("one untimed step of the same batch as one part (no concurrent "
                                               "kernels): the kernel's own efficiency")
            p1 = probe_of(psolo, "gemm_x3v_kernel<1>")
            if p1 is not None:
                result["roofline_solo"]["single_product_frac"] = roofline_of(p1, B)["frac"]
        for kind, g in qsolo.items():
            gbs = g["bytes_per_launch"] / (g["avg_ms"] * 1e-3) / 1e9
            result.setdefault("roofline_quantise_solo", {})["first_Q" if kind == "w" else "Q_with_LR"] = {
                "achieved_gbs": gbs, "frac_hbm": gbs / PEAK_HBM_GBS, "avg_call_ms": g["avg_ms"],
                "launches_timed": g["count"], "bytes_per_call": g["bytes_per_launch"],
                "note": "the same untimed one-part step: the quantise kernel without a concurrent stream"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
