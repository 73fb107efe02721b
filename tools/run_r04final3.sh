# GPU box, round 4 (final 3): smoke, GPU suite, default bench line (CPU baseline included), its
# rocprofv3 --kernel-trace --stats summary, and the other workloads' bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04final3}; mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["cpu_baseline"]["value"], d["api_single"]["ms_per_call"])'
mkdir -p $O/stats
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/stats/t -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/stats/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/stats > $O/stats/summary.txt; head -3 $O/stats/summary.txt | cut -c1-150
for w in cfg4t cfg3 model cfg5; do
  timeout -k 10 500 python3 -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-api-path > $O/bench_$w.log 2>&1 || exit $?
  echo "$w $(tail -1 $O/bench_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
