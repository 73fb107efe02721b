#!/bin/bash
# solver schedule at config 2 under the two-part default
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ak; mkdir -p $O
timeout -k 10 900 python -u tools/tune_solver.py cfg2 256 --parts 2 "tol=1e-5" "cheap_cold=2" "deg_warm=(10,6,6,6,6,6)" "deg_warm=(8,7,6,6,6,6)" "cheap_cold=4, deg_cold=(6,8,12,12,12,12,12)" "tol=1e-5" > $O/tune_p2.log 2>&1 || exit 1
