# GPU box, round 4 (e): fp16-slab sparse-Gram SpMM: sgram tests, suite, cfg2 / cfg4t benches,
# kernel traces of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04e}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sgram.py tests/test_gpu_codes.py -q -x --timeout 120 \
    --timeout-method thread > $O/new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -4 $O/new_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/gpu_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-200
for w in ${WORKLOADS:-cfg4t}; do
  timeout -k 10 400 python3 -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-api-path > $O/bench_$w.log 2>&1 || exit $?
  tail -1 $O/bench_$w.log | cut -c1-200
done
for w in cfg2 cfg4t; do
  mkdir -p $O/kt_$w
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_$w/t -o run --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_$w/s.log 2>&1 || exit $?
  python3 tools/ktrace_summary.py $O/kt_$w > $O/kt_$w/summary.txt; head -22 $O/kt_$w/summary.txt | cut -c1-150
done
