# GPU box, round 4: new-kernel tests first, then the GPU suite (no -x: every failure listed),
# the default bench, and the MFMA counter passes.  Each step has its own limit; a crash ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04a}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codes.py tests/test_gpu_qupdate_variants.py -q -x --timeout 120 \
    --timeout-method thread > $O/new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -4 $O/new_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 $O/gpu_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-400
[ -n "$NOPMC" ] && exit 0
bash tools/pmc_mfma.sh $O/pmc_mfma > $O/pmc_mfma.log 2>&1; rc=$?; tail -60 $O/pmc_mfma.log; exit $rc
