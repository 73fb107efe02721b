# GPU box, round 4 (h): streaming first-Q kernel with per-thread fixed error weights: its tests, config 3 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04h}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_qupdate_variants.py -q -x --timeout 120 \
    --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in ${WORKLOADS:-cfg3}; do
  timeout -k 10 500 python3 -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-api-path > $O/bench_$w.log 2>&1 || exit $?
  tail -1 $O/bench_$w.log | cut -c1-200
done
if [ -n "$CONFIGS" ]; then
  timeout -k 10 800 python3 -u tools/cpu_gpu_configs.py > $O/cpu_gpu_configs.json 2> $O/cpu_gpu_configs.err || exit $?
  cat $O/cpu_gpu_configs.json | cut -c1-220
fi
