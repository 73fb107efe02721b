# GPU box, round 4 (aj): ELL prefetch depth of the sparse-Gram SpMM (CQ_SG_PF = 6 / 8 / 12 A/B):
# sgram tests under each depth, micro-bench, config 2 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04aj}; mkdir -p $O
CQ_SG_PF=12 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sgram.py -q -x --timeout 120 --timeout-method thread > $O/tests_pf12.log 2>&1
rc=$?; echo "sgram tests (pf 12) rc=$rc"; tail -1 $O/tests_pf12.log; [ $rc -eq 0 ] || exit $rc
for pf in 6 8 12 6 12; do
  CQ_SG_PF=$pf timeout -k 10 300 python3 -u tools/bench_sgram.py 256 3 > $O/micro_pf$pf.log 2>&1 || exit $?
  echo "pf=$pf $(grep "^count" $O/micro_pf$pf.log | head -1 | tr '\n' ' ')"
done
for pf in 6 12; do
  CQ_SG_PF=$pf timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-api-path --no-parity > $O/bench_pf$pf.log 2>&1 || exit $?
  echo "pf=$pf $(tail -1 $O/bench_pf$pf.log | cut -c1-140)"
done
