#!/bin/bash
# static priority in the Q update: GPU suite, list micro-bench kernel trace, default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktq -o run -- python3 tools/bench_qupdate_list.py 256 5 > $O/ktq.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-path --steps 3 > $O/bench.log 2>&1 || exit 3
