"""Census of the large device copies (torch copy_/clone/contiguous) one config-2 engine run
makes at B = 256: count, bytes and the engine/solver line that issued them.
  python tools/diag/copy_census.py [B]"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
import torch  # noqa: E402

from ee274_convexcaldera_llm_quantization_amd.engine import CalderaEngine, EngineParams  # noqa: E402
from src.caldera.utils.dataclasses import CalderaParams  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dev = "cuda:0"
census = collections.Counter()
nbytes = collections.Counter()


def where():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "ee274" in fr.filename:
            return f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.line.strip()[:70]}"
    return "?"


def wrap(name):
    orig = getattr(torch.Tensor, name)

    def f(self, *a, **k):
        out = orig(self, *a, **k)
        if self.is_cuda and self.numel() * self.element_size() >= (1 << 24):
            key = (name, where())
            census[key] += 1
            nbytes[key] += self.numel() * self.element_size()
        return out
    setattr(torch.Tensor, name, f)


for nm in ("copy_", "clone", "contiguous", "index_copy_"):
    wrap(nm)
g = torch.Generator(device=dev).manual_seed(0)
Wb = (torch.randn(B, 4096, 4096, device=dev, generator=g) * 0.02).half()
qp = CalderaParams(Q_bits=2, L_bits=16, R_bits=16, rank=128, iters=5, update_order=["Q", "LR"], sigma_reg=1e-8)
CalderaEngine(EngineParams.from_caldera_params(qp)).run(Wb)
torch.cuda.synchronize()
for key, c in census.most_common():
    print(f"{c:4d} x {nbytes[key] / c / 2**20:9.1f} MiB  {key[0]:12s} {key[1]}")
