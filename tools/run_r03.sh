# GPU box runner (round 3): optional A/B of the Q update vs the round-2 library, the GPU test
# suite (PYTEST_K filter), then the default bench line.  Every GPU step has its own time limit;
# a fault, abort or time-out ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
if [ -n "$AB" ]; then
  timeout -k 10 300 python3 -u tools/ab_qupdate_r02.py ${AB_WRITE:+--write} > gpurun_out/ab_qupdate.log 2>&1; rc=$?
  echo "ab_qupdate rc=$rc"; grep -A8 '"identical"' gpurun_out/ab_qupdate.log | head -10
  ok $rc || exit $rc
fi
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1500 python3 -u -m pytest tests -m gpu -v -rf --timeout 400 --timeout-method thread ${PYTEST_X:+-x} \
      ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -25 gpurun_out/gpu_tests.log
  ok $rc || exit $rc
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 900 python3 -u bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; grep -v amdgpu.ids gpurun_out/bench.log | tail -4
  exit $rc
fi
