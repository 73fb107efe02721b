#!/bin/bash
# round-5 final head: the other workloads (config 3, config 4's tall shape, config 5) and the
# whole model with its projected 8-GPU rank shares
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aq; mkdir -p $O
timeout -k 10 400 python -u bench.py --workload cfg3 --no-cpu-baseline --no-api-path --steps 3 > $O/bench_cfg3.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload cfg4t --no-cpu-baseline --no-api-path --steps 3 > $O/bench_cfg4t.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --workload cfg5 --no-cpu-baseline --no-api-path --steps 2 > $O/bench_cfg5.log 2>&1 || exit 3
timeout -k 10 500 python -u bench.py --workload model --emulate-world 8 --no-cpu-baseline --no-api-path --steps 2 > $O/bench_model.log 2>&1 || exit 4
