# GPU box, round 4 (ai): fp64 Gram LDS pitch -- Gram tests, suite, config 2 bench + kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04ai}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -k "gram" -q -x --timeout 120 --timeout-method thread > $O/new_tests.log 2>&1
rc=$?; echo "gram tests rc=$rc"; tail -2 $O/new_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
mkdir -p $O/kt_cfg2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_cfg2/t -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_cfg2/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_cfg2 > $O/kt_cfg2/summary.txt; grep -i "gram_f64\|total" $O/kt_cfg2/summary.txt | head -6 | cut -c1-150
tail -1 $O/kt_cfg2/s.log | cut -c1-120
