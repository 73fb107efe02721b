#!/bin/bash
# two interleaved parts by default (B >= 32): GPU suite, default bench (CPU baseline + API path) and its kernel trace, PMC traffic passes at 128 matrices per launch, cfg3/cfg4t/cfg5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ad; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 2
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py > $O/bench_default_ktrace.log 2>&1 || exit 3
timeout -k 10 1000 bash tools/profile_round.sh r05ad 256 128 > $O/profile_round.log 2>&1 || exit 4
timeout -k 10 400 python -u bench.py --workload cfg3 --no-cpu-baseline --no-api-path --steps 3 > $O/bench_cfg3.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --workload cfg4t --no-cpu-baseline --no-api-path --steps 3 > $O/bench_cfg4t.log 2>&1 || exit 6
timeout -k 10 400 python -u bench.py --workload cfg5 --no-cpu-baseline --no-api-path --steps 2 > $O/bench_cfg5.log 2>&1 || exit 7
