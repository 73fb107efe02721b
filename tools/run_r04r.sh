# GPU box, round 4 (r): Q-update variants after the list-path geometry change.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04r}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_qupdate_variants.py tests/test_gpu_kernels.py tests/test_gpu_caldera.py tests/test_gpu_configs.py -q --timeout 200 \
    --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log; [ $rc -eq 0 ] || [ -n "$CONT" ] || exit $rc
timeout -k 10 200 python3 -u tools/bench_qupdate_list.py 256 10 > $O/qlist.log 2>&1 || exit $?
cat $O/qlist.log
for w in ${WORKLOADS:-cfg2 cfg3}; do
  timeout -k 10 500 python3 -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-api-path > $O/bench_$w.log 2>&1 || exit $?
  tail -1 $O/bench_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["name"], d["value"], d["ms_per_step"], json.dumps(d["roofline_quantise"]["Q_with_LR"])[:200])'
done
