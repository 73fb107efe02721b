#!/bin/bash
# Jacobi sweeps per Rayleigh-Ritz eigensolve in a config-2 decomposition (B = 256)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 300 python -u tools/jacobi_sweeps_engine.py 256 > $O/jacobi_sweeps.log 2>&1 || exit 1
