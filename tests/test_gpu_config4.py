"""BASELINE configs[3] (the reference's main.py:135-251 per-layer loop over a whole model) as a
-m gpu workload: the first two Llama-2-7B layers (14 matrices, all three shapes) through
sharding.decompose_sharded + engine_decompose_batch at world 1 -- the same code every rank
runs at N GPUs (the RCCL gather itself is covered by the world-2 gloo test and by bench.py
at N > 1).  Weights are the survey's host-RNG recipe, seed = layer * 7 + proj index, so the
matrices the reference's golden runs cover are pinned: layer 0/1 q, k, v, o_proj = config-2
seeds 0-3 / 7-10 (tests/golden/final_codes.npz), layer-0 gate_proj = the cfg4t run (seed 4,
11008 x 4096)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from final_codes import assert_codes_within_reference_spread, compare, fixture, frob_bar

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _omega(n, k=16, seed=1234):
    return np.random.default_rng(seed).standard_normal((n, k))


def test_config4_first_two_layers_sharded():
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    from ee274_convexcaldera_llm_quantization_amd import sharding as S
    from src.caldera.utils.dataclasses import CalderaParams
    fx = fixture()
    spread = json.load(open(os.path.join(GOLDEN, "ref_spread_cfg2_seeds16.json")))["seeds"]
    qp = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, update_order=["Q", "LR"], sigma_reg=1e-8)
    items = S.llama2_7b_matrices(2)
    assert len(items) == 14 and {(m, n) for _, m, n, _ in items} == {(4096, 4096), (11008, 4096), (4096, 11008)}
    res = S.decompose_sharded(items, S.engine_decompose_batch(qp, DEV), rank=0, world=1, max_batch=16)
    assert [r.name for r in res] == [it[0] for it in items]

    # the payload every rank gathers to rank 0 (packed in HBM), and back
    buf = S.pack_results(res, device=DEV)
    back = S.unpack_results(buf)
    nbytes = 0
    for r, b in zip(res, back):
        assert b.name == r.name and b.Q_scale == r.Q_scale and b.errors == r.errors
        assert torch.equal(b.codes, r.codes) and torch.equal(b.L, r.L) and torch.equal(b.R, r.R)
        assert b.codes.numel() == r.m * r.n // 4 and b.L.shape == (r.m, 128) and b.R.shape == (128, r.n)
        nbytes += r.m * r.n // 4 + 4 * 128 * (r.m + r.n)
    assert buf.numel() >= nbytes and buf.numel() - nbytes < 64 * 1024   # arrays + small JSON header
    print(f"config 4 (2 layers): {len(res)} matrices, payload {buf.numel() / 2**20:.1f} MiB")

    pins = {f"model.layers.{l}.self_attn.{p}_proj": (7 * l + i) for l in (0, 1) for i, p in enumerate("qkvo")}
    pins["model.layers.0.mlp.gate_proj"] = "cfg4t"
    checked = 0
    for r in res:
        pin = pins.get(r.name)
        if pin is None:
            continue
        tag = pin if isinstance(pin, str) else ("cfg2" if pin == 0 else f"cfg2s{pin}")
        m, n = r.m, r.n
        codes = K.unpack_codes(r.codes.view(1, -1), m * n, 2)
        Q = K.dequantize_uniform(codes.view(1, -1), torch.tensor([r.Q_scale], device=DEV), 2).view(m, n)
        om = torch.from_numpy(_omega(n)).to(DEV)
        sk = (Q.double() @ om + r.L.double() @ (r.R.double() @ om)).cpu().numpy()
        ref = fx[f"{tag}_sketch_QLR"] if f"{tag}_sketch_QLR" in fx.files else np.load(
            os.path.join(GOLDEN, "sum_large.npz"))[f"{tag}_sketch_QLR"]
        rel = float(np.linalg.norm(sk - ref) / np.linalg.norm(ref))
        c = compare(tag, codes, m, n)
        sp = spread.get(str(pin), {}) if not isinstance(pin, str) else {}
        print(f"  {r.name} vs golden {tag}: rel Frobenius {rel:.2e}, final codes {c}")
        qn = float(torch.linalg.norm(Q.double() + r.L.double() @ r.R.double()))
        bar = frob_bar(tag, c, qn, sp.get("rel_frob_QLR_ref4_vs_ref8", 0.0))
        assert rel <= bar, (r.name, rel, bar, sp)
        assert_codes_within_reference_spread(c, sp, r.name)
        checked += 1
    assert checked == 9
