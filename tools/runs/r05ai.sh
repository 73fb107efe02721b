#!/bin/bash
# head after the parts threshold change: GPU suite, default bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ai; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 2
