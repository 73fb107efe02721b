# GPU box, round 4 (v): solver degree sweep on config 2 at B = 256 (tools/tune_solver.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04v}; mkdir -p $O
timeout -k 10 1000 python3 -u tools/tune_solver.py cfg2 256 ${SPECS:-"" "deg_warm=(12,6,6)" "deg_warm=(11,6,6)" "deg_warm=(9,7,6)" \
    "deg_warm=(10,6,6)" "deg_cold=(6,13,13,13)" "deg_cold=(6,11,11,11)" "deg_cold=(8,12,12,12)"} > $O/tune.log 2>&1 || exit $?
cut -c1-200 $O/tune.log
