#!/bin/bash
# streaming first-Q quantise (no-weights instantiation, FMA packing, W two groups ahead) + whitening without the fp64 copy (ABI 4): GPU suite, default bench, kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-api-path --steps 3 > $O/bench.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --no-cpu-baseline --no-api-path --no-parity --steps 1 --warmup 1 > $O/kt.log 2>&1 || exit 3
