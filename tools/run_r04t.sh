# GPU box, round 4 (t): Jacobi seat arrays double-buffered -- eigen tests, Jacobi micro-bench,
# config 2 bench and kernel trace, single call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04t}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/bench_jacobi.py 256 192 > $O/jacobi.log 2>&1 || exit $?
grep ms/call $O/jacobi.log
timeout -k 10 500 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("api_single"))'
mkdir -p $O/kt_cfg2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_cfg2/t -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_cfg2/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_cfg2 > $O/kt_cfg2/summary.txt; grep -i "jacobi\|total" $O/kt_cfg2/summary.txt | head -4 | cut -c1-150
