# GPU box, round 4 (l): kernel traces of config 5 (B = 256, 1 timed step) and of one caldera() call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04l}; mkdir -p $O/kt_cfg5 $O/kt_single
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_cfg5/t -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 1 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_cfg5/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_cfg5 > $O/kt_cfg5/summary.txt; head -30 $O/kt_cfg5/summary.txt | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_single/t -o run --output-format csv -- python3 tools/bench_single.py 3 > $O/kt_single/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_single > $O/kt_single/summary.txt; head -24 $O/kt_single/summary.txt | cut -c1-160; grep median $O/kt_single/s.log
