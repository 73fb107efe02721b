# GPU box: full GPU test suite, then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_all.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_all.log
[ $rc -eq 0 ] || exit $rc
[ -n "$NO_BENCH" ] && exit 0
if [ "$1" = full ]; then BA=""; else BA="--no-cpu-baseline"; fi
timeout -k 10 600 python3 bench.py $BA > gpurun_out/bench.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/bench.log | tail -3
exit $rc
