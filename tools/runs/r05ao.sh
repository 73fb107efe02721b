#!/bin/bash
# gram: diagonal tiles rotate the wave -> block map, the idle block skips its MFMAs; A/B vs HEAD
# (working tree vs HEAD build); default bench; GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ao; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread \
    -k "transpose_split or gram_f64 or b_triu or blocked_operand" > $O/kernel_tests.log 2>&1 || exit 1
for r in 1 2; do
  for L in "" "--lib tools/probes/lib_head.so"; do
    timeout -k 10 120 python -u tools/bench_small_kernels.py 128 $L >> $O/small_kernels.log 2>&1 || exit 2
  done
done
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 4
