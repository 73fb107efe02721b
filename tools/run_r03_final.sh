# GPU box (repo root): the round-3 record -- GPU suite, default bench (with the CPU baseline),
# the other workloads, and a kernel trace of the default config.  Each step has its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log | cut -c1-200
for w in ${WORKLOADS:-cfg3 cfg5 model}; do
  timeout -k 10 400 python3 -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$w.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$w.log | cut -c1-160
done
if [ -n "$KTRACE" ]; then bash tools/ktrace.sh $KTRACE --steps 2 --warmup 1 --no-cpu-baseline --no-parity > /dev/null 2>&1 || exit $?; head -24 gpurun_out/kt_$KTRACE/summary.txt; fi
