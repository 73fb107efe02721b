"""The fused Q update's opt-in pass-0 variants give the default path's results bit for bit.

Pass 0 of cq_q_update_x3 (the absmax of W - L R, alg.py:262 + quantization.py:260-268) has
three implementations chosen once per process by environment switches read in the library:
the default (split-fp16 products, one 32-column chunk of W per load), CQ_QP0_PAIRW=1 (two
chunks per W load) and CQ_QP0_APPROX=1 (hi x hi product with an exact fix-up of the candidate
chunks).  Each runs in its own child process on the same seeded inputs; packed codes, scales
and error sums must equal the default's (also a child process) exactly: the max decides every code."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import hashlib, json, sys
sys.path.insert(0, sys.argv[1])
import torch
import ee274_convexcaldera_llm_quantization_amd._lib as K
out = {}
for bits in (2, 4):
    g = torch.Generator(device="cuda:0").manual_seed(1234 + bits)
    B, m, n, r = 4, 512, 1024, 64
    W = torch.randn(B, m, n, device="cuda:0", generator=g).half()
    L = torch.randn(B, m, r, device="cuda:0", generator=g) * 0.3
    R = torch.randn(B, r, n, device="cuda:0", generator=g) * 0.3
    packed = torch.empty(B, m * n * bits // 8, dtype=torch.uint8, device="cuda:0")
    sc = torch.empty(B, device="cuda:0")
    err = torch.empty(B, dtype=torch.float64, device="cuda:0")
    K.q_update_x3(W, L, R, bits, packed=packed, scale=sc, err_out=err)
    torch.cuda.synchronize()
    out[bits] = [hashlib.sha256(packed.cpu().numpy().tobytes()).hexdigest(),
                 sc.cpu().tolist(), err.cpu().tolist()]
print("RESULT " + json.dumps(out))
"""


def _run(env_extra):
    env = dict(os.environ)
    env.pop("CQ_QP0_APPROX", None)
    env.pop("CQ_QP0_PAIRW", None)
    env.update(env_extra)
    p = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def test_pass0_variants_bit_identical():
    base = _run({})
    for env in ({"CQ_QP0_PAIRW": "1"}, {"CQ_QP0_APPROX": "1"}):
        got = _run(env)
        assert got == base, (env, got, base)
    # four matrices, four different positive scales (the inputs are not degenerate)
    assert len(set(base["2"][1])) == 4 and all(s > 0 for s in base["2"][1])
