#!/bin/bash
# CholQR product writing the Rayleigh-Ritz operand (cq_gemm_triu_split): its kernel test,
# default bench (parity fields must equal r05ap's bit for bit), one-part kernel stats, GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05at; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
    -k "triu or transpose_split" > $O/kernel_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt1 -o run --output-format csv -- \
    python3 bench.py --streams 1 --steps 1 --warmup 1 --no-parity --no-cpu-baseline --no-api-path > $O/kt1.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 4
