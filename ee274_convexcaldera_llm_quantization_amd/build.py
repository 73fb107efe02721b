"""Build libcaldera_hip.so in-tree with hipcc for gfx950 (no JIT cache, no pip install: the
.so travels with the repo snapshot to the GPU box)."""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libcaldera_hip.so")
SOURCES = ["cq_quant.hip", "cq_gemm.hip", "cq_small.hip", "cq_x3.hip", "cq_qupdate.hip", "cq_codebook.hip",
           "cq_calib.hip", "cq_bjacobi.hip", "cq_sgram.hip"]
# per-source extra flags: the row-panel Q update keeps its per-element epilogue in scalar fp32
# (packed fp32 VALU beside MFMAs costs more issue cycles than the scalar pair it replaces)
EXTRA = {"cq_qupdate.hip": ["-fno-slp-vectorize"]}
FLAGS = ["-O3", "--offload-arch=gfx950", "-fPIC", "-shared", "-std=c++17",
         # bit-exact quantiser: no FMA contraction, IEEE-correct fp32 division/sqrt
         "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


STAMP = OUT + ".srchash"  # content hash of the sources the .so was built from


def _deps():
    return ([os.path.join(CSRC, s) for s in SOURCES + ["cq_common.h", "cq_x3.h"]]
            + [os.path.join(HERE, "..", "include", "caldera_hip.h")])


def source_hash() -> str:
    """SHA-256 over the kernel sources, the public header and the compile flags."""
    h = hashlib.sha256((" ".join(FLAGS) + repr(sorted(EXTRA.items()))).encode())
    for d in _deps():
        if os.path.exists(d):
            with open(d, "rb") as f:
                h.update(os.path.basename(d).encode() + b"\0" + f.read())
    return h.hexdigest()


def built_hash() -> str | None:
    try:
        with open(STAMP) as f:
            return f.read().strip()
    except OSError:
        return None


def needs_build() -> bool:
    """Content-based (mtimes do not survive every copy): the .so is current iff the hash
    stamped next to it at build time equals the hash of the sources now in the tree."""
    return not os.path.exists(OUT) or built_hash() != source_hash()


def build(force: bool = False, verbose: bool = True) -> str:
    """Each source compiles to its own object in parallel (no relocatable device code: every
    kernel is launched from its own translation unit), then one link."""
    if not force and not needs_build():
        return OUT
    objdir = os.path.join(HERE, "_build")
    os.makedirs(objdir, exist_ok=True)
    procs, objs = [], []
    for src in SOURCES:
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        objs.append(obj)
        cmd = [hipcc(), *[f for f in FLAGS if f != "-shared"], *EXTRA.get(src, []), "-c", "-o", obj,
               os.path.join(CSRC, src)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), src))
    failed = [src for p, src in procs if p.wait() != 0]
    if failed:
        raise RuntimeError(f"hipcc failed on {failed}")
    digest = source_hash()
    tmp = OUT + ".tmp"
    subprocess.run([hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", tmp, *objs], check=True)
    os.replace(tmp, OUT)
    with open(STAMP, "w") as f:
        f.write(digest + "\n")
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
