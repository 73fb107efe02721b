# GPU box, round 4 (ab): non-temporal LDS-DMA loads of the streamed B operand (CQ_X3_NT A/B),
# config 2 bench and kernel trace under each policy.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04ab}; mkdir -p $O
for nt in 0 1 0 1; do
  CQ_X3_NT=$nt timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/bench_nt$nt.log 2>&1 || exit $?
  echo "nt=$nt $(tail -1 $O/bench_nt$nt.log | cut -c1-200)"
done
for nt in 0 1; do
  mkdir -p $O/kt_nt$nt
  CQ_X3_NT=$nt timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_nt$nt/t -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_nt$nt/s.log 2>&1 || exit $?
  python3 tools/ktrace_summary.py $O/kt_nt$nt > $O/kt_nt$nt/summary.txt; echo "== nt=$nt"; grep -i "x3v\|total" $O/kt_nt$nt/summary.txt | head -6 | cut -c1-150
done
