#!/bin/bash
# vectorised transpose-split stores, balanced triangular CholQR multiply, symmetric Gram's
# idle diagonal wave block: kernel tests, default bench, one-part kernel stats, GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05am; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
    -k "transpose_split or gram_f64 or b_triu or blocked_operand" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
    python3 bench.py --streams 1 --steps 1 --warmup 1 --no-parity --no-cpu-baseline --no-api-path > $O/kt.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 4
