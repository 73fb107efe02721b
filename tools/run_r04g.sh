# GPU box, round 4 (g): codes tests, suite, benches (cfg2 with the CPU baseline, cfg4t, cfg3,
# model, cfg5), kernel trace of cfg2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04g}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codes.py tests/test_gpu_sgram.py -q -x --timeout 120 \
    --timeout-method thread > $O/new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -4 $O/new_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/gpu_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in ${WORKLOADS:-model cfg4t cfg2}; do
  timeout -k 10 500 python3 -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-api-path > $O/bench_$w.log 2>&1 || exit $?
  tail -1 $O/bench_$w.log | cut -c1-200
done
