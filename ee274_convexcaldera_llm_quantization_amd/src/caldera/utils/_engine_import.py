"""Locate the engine package whether the drop-in is imported as `src.caldera...` (reference
style: sys.path.append('<package dir>'), as main.py:20-23 does) or as
`ee274_convexcaldera_llm_quantization_amd.src.caldera...`."""
import importlib
import os
import sys

_PKG = "ee274_convexcaldera_llm_quantization_amd"
try:
    _pkg = importlib.import_module(_PKG)
except ImportError:  # imported through the reference-style path: add the repo root
    sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), *[".."] * 4)))
    _pkg = importlib.import_module(_PKG)

kernels = importlib.import_module(_PKG + "._lib")
api = importlib.import_module(_PKG + ".api")
qlog = importlib.import_module(_PKG + ".qlog")
