# GPU box, round 4 first call: GPU suite, default bench, MFMA counter passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
bash tools/pmc_mfma.sh $O/pmc_mfma > $O/pmc_mfma.log 2>&1; rc=$?; tail -60 $O/pmc_mfma.log; exit $rc
