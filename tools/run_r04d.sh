# GPU box, round 4 (d): kernels/solver tests first, suite, default bench, single-call trace,
# first-LR tolerance sweep near the products' precision floor.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04d}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_caldera.py -q -x \
    --timeout 120 --timeout-method thread > $O/new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -4 $O/new_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/gpu_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-300
mkdir -p $O/kt_single
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_single/t -o run --output-format csv -- python3 tools/bench_single.py 3 > $O/kt_single/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_single > $O/kt_single/summary.txt; head -24 $O/kt_single/summary.txt; grep median $O/kt_single/s.log
[ -n "$NOSWEEP" ] || TAG=${TAG:-r04d}_tol SCHEDS="${SCHEDS:-8e-6 6e-6}" bash tools/sweep_first_tol.sh
