#!/bin/bash
# round-5 first GPU pass: new gate / small-p Jacobi tests, default bench, model + 8-GPU share projection
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_kernels.py -k "small_p" tests/test_gpu_sgram.py -k "small_p or gates" > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-path > $O/bench.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --workload model --no-parity --steps 3 --emulate-world 8 > $O/model.log 2>&1 || exit 3
