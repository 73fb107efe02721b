# GPU box, round 4 (f): codes tests, suite, benches (cfg2 with the CPU baseline, cfg4t, cfg3,
# model, cfg5), kernel trace of cfg2.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04f}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codes.py tests/test_gpu_sgram.py -q -x --timeout 120 \
    --timeout-method thread > $O/new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -4 $O/new_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/gpu_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python3 -u bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | cut -c1-200
for w in ${WORKLOADS:-cfg4t cfg3 model cfg5}; do
  timeout -k 10 500 python3 -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-api-path > $O/bench_$w.log 2>&1 || exit $?
  tail -1 $O/bench_$w.log | cut -c1-200
done
mkdir -p $O/kt_cfg2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_cfg2/t -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_cfg2/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_cfg2 > $O/kt_cfg2/summary.txt; head -30 $O/kt_cfg2/summary.txt | cut -c1-150
mkdir -p $O/kt_single
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_single/t -o run --output-format csv -- python3 tools/bench_single.py 3 > $O/kt_single/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_single > $O/kt_single/summary.txt; head -16 $O/kt_single/summary.txt | cut -c1-150; grep median $O/kt_single/s.log
