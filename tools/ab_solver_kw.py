"""GPU tool: bench.py's default workload (config 2, parity fields included) under RankRSolver
keyword overrides, one JSON line: value, parity summary, exact-LR and held-out rates.
    python tools/ab_solver_kw.py cheap_one_pass=True
    python tools/ab_solver_kw.py BJ_SMALL_SUBPROBLEMS=512      (upper case: a solver module constant)"""
import contextlib
import io
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]

import bench  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd import solver  # noqa: E402


def main():
    kw = {}
    for spec in sys.argv[1:]:
        k, v = spec.split("=")
        if k.isupper():   # a solver module constant (e.g. BJ_SMALL_SUBPROBLEMS=512)
            setattr(solver, k, type(getattr(solver, k))(eval(v)))
            kw[k] = eval(v)
            continue
        kw[k] = eval(v)
    consts = {k: kw.pop(k) for k in list(kw) if k.isupper()}
    init = solver.RankRSolver.__init__

    def patched(self, *a, **k):
        k.update(kw)
        init(self, *a, **k)

    solver.RankRSolver.__init__ = patched
    sys.argv = ["bench.py", "--no-cpu-baseline", "--no-api-path"]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main()
    d = json.loads(buf.getvalue().strip().splitlines()[-1])
    p = d.get("parity_timed_step", {})
    print(json.dumps({"kw": {k: str(v) for k, v in {**kw, **consts}.items()}, "value": round(d["value"], 1),
                      "pinned": p.get("final_codes_summary"),
                      "exact_lr": (p.get("final_codes_vs_exact_lr") or {}).get("bit_exact"),
                      "holdout": (p.get("holdout") or {}).get("bit_exact_vs_reference")}), flush=True)


if __name__ == "__main__":
    main()
