# GPU box, round 4 (ao): config 5 kernel trace on the current tree (compare r04l).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04ao}; mkdir -p $O/kt_cfg5
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt_cfg5/t -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_cfg5/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_cfg5 > $O/kt_cfg5/summary.txt; head -16 $O/kt_cfg5/summary.txt | cut -c1-150
