#!/bin/bash
# default bench with the concurrent and solo rooflines; its kernel trace (same command); GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ae; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py > $O/bench_default_ktrace.log 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 3
