# GPU box, round 4 (x): warm-degree neighbours of (9, 7) on config 2 at B = 256.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04x}; mkdir -p $O
timeout -k 10 1000 python3 -u tools/tune_solver.py cfg2 256 "" "deg_warm=(9,7,6)" "deg_warm=(8,7,6)" "deg_warm=(9,8,6)" \
    "deg_warm=(8,8,6)" "deg_warm=(7,8,6)" "deg_warm=(9,7,6), deg_cold=(6,13,13,13)" "deg_warm=(9,7,6)" > $O/tune.log 2>&1 || exit $?
cut -c1-200 $O/tune.log
