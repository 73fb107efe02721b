"""The fused Q update (cq_q_update_x3: res = W - L R, alg.py:262, quantised whole-matrix,
quantization.py:260-268) reproduces the round-2 kernel bit for bit after round 3's changes to
it: pass 1 now gathers a row's 2-bit code bytes across four 32-column chunks and stores 32
contiguous bytes per row (instead of one 2-byte store per lane and chunk), and the opt-in pass-0
variants were removed from the library.

tests/golden/qupdate_r02_fingerprints.json holds the round-2 library's packed codes (SHA-256),
scales and error sums on the host-seeded inputs of tests/qupdate_cases.py (full config-2 shape,
a partial last code group, 4-bit packing, K = 256, fp32 W), recorded on an MI355X by
tools/ab_qupdate_r02.py, which runs both libraries in one process."""
import json
import os

import pytest
import torch

from conftest import GOLDEN
import qupdate_cases as C

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", C.CASES, ids=[c[0] for c in C.CASES])
def test_q_update_matches_round2_kernel(case):
    import ee274_convexcaldera_llm_quantization_amd._lib as K
    ref = json.load(open(os.path.join(GOLDEN, "qupdate_r02_fingerprints.json")))["cases"][case[0]]
    got = C.run(K, case, torch.device("cuda:0"))
    assert got["packed_sha256"] == ref["packed_sha256"]
    assert got["scale"] == ref["scale"]
    assert got["err"] == ref["err"]
