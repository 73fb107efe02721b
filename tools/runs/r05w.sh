#!/bin/bash
# C^T epilogue output (filter / Rayleigh-Ritz / tall L without transpose passes), NaN-residual list test: GPU suite, bench, kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-api-path --steps 3 > $O/bench.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --no-cpu-baseline --no-api-path --no-parity --steps 1 --warmup 1 > $O/kt.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --workload model --emulate-world 8 --no-cpu-baseline --no-api-path --steps 2 > $O/model8.log 2>&1 || exit 4
