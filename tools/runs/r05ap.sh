#!/bin/bash
# round-5 final head: smoke, default bench, its kernel trace (same command), one-part kernel
# stats at B = 256, GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ap; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py > $O/bench_default_ktrace.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt1 -o run --output-format csv -- \
    python3 bench.py --streams 1 --steps 1 --warmup 1 --no-parity --no-cpu-baseline --no-api-path > $O/kt1.log 2>&1 || exit 4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 5
