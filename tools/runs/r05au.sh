#!/bin/bash
# dequantised Q from the packed codes: default bench (parity fields must equal r05at's),
# one-part kernel stats, GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05au; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt1 -o run --output-format csv -- \
    python3 bench.py --streams 1 --steps 1 --warmup 1 --no-parity --no-cpu-baseline --no-api-path > $O/kt1.log 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 3
