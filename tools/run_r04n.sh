# GPU box, round 4 (n): counted end-of-chunk wait in the Q-update ring with candidate stores in
# flight; four-wave slice placement.  Q-update / sgram tests, list micro-bench, config 2 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04n}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_qupdate_variants.py tests/test_gpu_sgram.py tests/test_gpu_kernels.py -q -x --timeout 120 \
    --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/bench_qupdate_list.py 256 10 > $O/qlist.log 2>&1 || exit $?
timeout -k 10 240 python3 -u tools/probe_spmm_conflicts.py 64 5 > $O/probe.log 2>&1 || exit $?
tail -2 $O/probe.log
cat $O/qlist.log
timeout -k 10 500 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], json.dumps(d["roofline_quantise"]["Q_with_LR"])[:300], d.get("api_single"))'
