#!/bin/bash
# v1 two-class lists at the 1 GB capacities: GPU suite, benches (cfg2 default line incl. CPU baseline, cfg5, cfg3, cfg4t, model)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --workload cfg5 --no-cpu-baseline --no-api-path --steps 2 > $O/bench_cfg5.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --workload cfg3 --no-cpu-baseline --no-api-path --steps 2 > $O/bench_cfg3.log 2>&1 || exit 4
timeout -k 10 400 python -u bench.py --workload cfg4t --no-cpu-baseline --no-api-path --steps 2 > $O/bench_cfg4t.log 2>&1 || exit 5
