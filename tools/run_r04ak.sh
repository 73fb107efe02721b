# GPU box, round 4 (ak): kernel traces of config 4t and config 3 on the current tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04ak}; mkdir -p $O
for w in cfg4t cfg3; do
  mkdir -p $O/kt_$w
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/kt_$w/t -o run --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_$w/s.log 2>&1 || exit $?
  python3 tools/ktrace_summary.py $O/kt_$w > $O/kt_$w/summary.txt; echo "== $w"; head -14 $O/kt_$w/summary.txt | cut -c1-150
  tail -1 $O/kt_$w/s.log | cut -c1-150
done
