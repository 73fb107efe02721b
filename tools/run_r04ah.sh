# GPU box, round 4 (ah): s_setprio around the split products' MFMA clusters (CQ_X3_PRIO A/B).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04ah}; mkdir -p $O
for pr in 0 1 0 1; do
  CQ_X3_PRIO=$pr timeout -k 10 300 python3 -u tools/probe_x3_shared.py 256 > $O/probe_prio$pr.log 2>&1 || exit $?
  echo "prio=$pr"; grep "shared_G=0" $O/probe_prio$pr.log
done
for pr in 0 1; do
  CQ_X3_PRIO=$pr timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-api-path --no-parity > $O/bench_prio$pr.log 2>&1 || exit $?
  echo "prio=$pr $(tail -1 $O/bench_prio$pr.log | cut -c1-140)"
done
