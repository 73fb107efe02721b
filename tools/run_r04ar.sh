# GPU box, round 4 (ar): kernel traces of config 4t, config 3 and the whole model at the final state.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04ar}; mkdir -p $O
for w in cfg4t cfg3 model; do
  mkdir -p $O/kt_$w
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/kt_$w/t -o run --output-format csv -- python3 bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_$w/s.log 2>&1 || exit $?
  python3 tools/ktrace_summary.py $O/kt_$w > $O/kt_$w/summary.txt; echo "== $w"; head -6 $O/kt_$w/summary.txt | cut -c1-140
done
