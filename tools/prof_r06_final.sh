# Round-6 final evidence: smoke, the default bench under the kernel tracer (its by-grid summary:
# the filter launch average the bench line's HIP-event probe must agree with), one-part stats.
set -e
export TMPDIR=/tmp
O=${1:-gpurun_out/r06z}
mkdir -p $O/kt $O/kt1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py > $O/bench_default_ktrace.log 2>&1
python3 tools/ktrace_summary.py $O/kt > $O/bench_default_ktrace_by_grid.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt1 -o run --output-format csv -- python3 bench.py --streams 1 --steps 1 --warmup 1 --no-parity --no-cpu-baseline --no-api-path > $O/kt1.log 2>&1
python3 tools/ktrace_summary.py $O/kt1 > $O/kt1_by_grid.txt
