# GPU box, round 4 (ap): NT as a template argument (no policy branch in the default loops) --
# x3 tests, config 5 and config 2 kernel traces, config 2 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04ap}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
mkdir -p $O/kt_cfg5 $O/kt_cfg2
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt_cfg5/t -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_cfg5/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_cfg5 > $O/kt_cfg5/summary.txt; head -4 $O/kt_cfg5/summary.txt | cut -c1-150
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_cfg2/t -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_cfg2/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_cfg2 > $O/kt_cfg2/summary.txt; head -4 $O/kt_cfg2/summary.txt | cut -c1-150
