# GPU box, round 4 (q): round-state check -- smoke, the GPU suite, the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04q}; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $O/gpu_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python3 -u bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["cpu_baseline"]["value"], d.get("api_single"), d["parity_timed_step"].get("final_codes", "")[:300] if isinstance(d["parity_timed_step"].get("final_codes"), str) else "")'
timeout -k 10 200 python3 -u tools/bench_jacobi.py 256 192 > $O/jacobi.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/bench_single.py 3 > $O/single.log 2>&1 || exit $?
grep median $O/single.log
cat $O/jacobi.log | grep ms/call
timeout -k 10 200 python3 -u tools/bench_qupdate_list.py 256 10 > $O/qlist.log 2>&1 || exit $?
cat $O/qlist.log
mkdir -p $O/kt_cfg2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_cfg2/t -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_cfg2/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_cfg2 > $O/kt_cfg2/summary.txt; head -12 $O/kt_cfg2/summary.txt | cut -c1-150
