#!/bin/bash
# solver schedule sweep at config 2, B = 256 (warm solves: cheap / split degrees)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 900 python -u tools/tune_solver.py cfg2 256 "tol=1e-5" "deg_warm=(10,6,6,6,6,6)" "deg_warm=(8,7,6,6,6,6)" "deg_warm=(12,6,6,6,6,6)" "cheap_warm=0, deg_warm=(10,6,6,6,6,6)" "cheap_warm=0, deg_warm=(12,6,6,6,6,6)" "cheap_warm=0, deg_warm=(8,6,6,6,6,6)" "cheap_cold=2" "deg_cold=(6,12,10,12,12,12,12)" "deg_warm=(10,5,5,5,5,5)" > $O/tune.log 2>&1 || exit 1
