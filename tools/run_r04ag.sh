# GPU box, round 4 (ag): L2 prefetch of the split filter's B two K steps ahead (CQ_X3_PF A/B):
# x3 tests under the prefetch, bound probe, config 2 bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04ag}; mkdir -p $O
CQ_X3_PF=1 timeout -k 10 300 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests_pf.log 2>&1
rc=$?; echo "tests (pf) rc=$rc"; tail -2 $O/tests_pf.log; [ $rc -eq 0 ] || exit $rc
for pf in 0 1; do
  CQ_X3_PF=$pf timeout -k 10 300 python3 -u tools/probe_x3_shared.py 256 > $O/probe_pf$pf.log 2>&1 || exit $?
  echo "pf=$pf"; grep "split\|exact\|single" $O/probe_pf$pf.log | grep "shared_G=0"
done
for pf in 0 1 0 1; do
  CQ_X3_PF=$pf timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-api-path > $O/bench_pf$pf.log 2>&1 || exit $?
  echo "pf=$pf $(tail -1 $O/bench_pf$pf.log | cut -c1-160)"
done
