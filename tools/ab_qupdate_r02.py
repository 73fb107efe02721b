"""GPU tool: fused Q update of the current tree vs the round-2 library (tools/ab/libcaldera_hip_r02.so,
built from commit d81e5f2 before the gathered code stores and the variant clean-up).  Both run the
cases of tests/qupdate_cases.py in one process; the round-2 outputs are written to
tests/golden/qupdate_r02_fingerprints.json and must equal the current ones bit for bit.

  python tools/ab_qupdate_r02.py [--write]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]
import torch  # noqa: E402

import ee274_convexcaldera_llm_quantization_amd._lib as K  # noqa: E402
import qupdate_cases as C  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    K.load()
    new = {c[0]: C.run(K, c, dev) for c in C.CASES}
    cur = K._lib
    old = ctypes.CDLL(os.path.join(ROOT, "tools", "ab", "libcaldera_hip_r02.so"))
    for name, (res, args) in K._SIGS.items():
        if hasattr(old, name):
            fn = getattr(old, name)
            fn.restype, fn.argtypes = res, args
    K._lib = old
    try:
        ref = {c[0]: C.run(K, c, dev) for c in C.CASES}
    finally:
        K._lib = cur
    same = {t: new[t] == ref[t] for t in ref}
    print(json.dumps({"identical": same, "r02": ref, "current": new}, indent=1))
    if "--write" in sys.argv:
        json.dump({"generated_by": "tools/ab_qupdate_r02.py --write (round-2 library, commit d81e5f2)",
                   "cases": ref}, open(os.path.join(ROOT, "tests", "golden", "qupdate_r02_fingerprints.json"), "w"),
                  indent=1)
    sys.exit(0 if all(same.values()) else 1)


if __name__ == "__main__":
    main()
