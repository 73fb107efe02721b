#!/bin/bash
# default bench and config 3 with the solo-roofline step moved after the API path
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ar; mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload cfg3 --no-cpu-baseline --steps 3 > $O/bench_cfg3.log 2>&1 || exit 2
