# GPU box, round 4 (an): weighted R = (U^T W) diag(ycol) on exact W halves (colw epilogue) -- sgram
# tests, GPU suite, config 3 / model / config 2 benches, config 3 kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04an}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sgram.py tests/test_gpu_kernels.py -k "sgram or residual_split or gram" -q -x --timeout 120 --timeout-method thread > $O/sgram_tests.log 2>&1
rc=$?; echo "sgram tests rc=$rc"; tail -1 $O/sgram_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for w in cfg3 model; do
  timeout -k 10 500 python3 -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-api-path > $O/bench_$w.log 2>&1 || exit $?
  echo "$w $(tail -1 $O/bench_$w.log | cut -c1-150)"
done
mkdir -p $O/kt_cfg3
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/kt_cfg3/t -o run --output-format csv -- python3 bench.py --workload cfg3 --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_cfg3/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_cfg3 > $O/kt_cfg3/summary.txt; grep "x3v\|residual_split\|total" $O/kt_cfg3/summary.txt | head -8 | cut -c1-150
