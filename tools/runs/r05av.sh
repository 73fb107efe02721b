#!/bin/bash
# Ritz rotation writing the filter's first operands (cq_gemm_rot_split): kernel tests, default
# bench (parity fields must equal r05au's), one-part kernel stats, GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05av; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "rot_split or triu" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt1 -o run --output-format csv -- \
    python3 bench.py --streams 1 --steps 1 --warmup 1 --no-parity --no-cpu-baseline --no-api-path > $O/kt1.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 4
