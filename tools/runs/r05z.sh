#!/bin/bash
# round-5 final validation at the head: smoke, GPU suite, default bench (CPU baseline + API path), cfg3 / cfg4t / cfg5 / model benches
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py > $O/bench_default.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --workload cfg3 --no-cpu-baseline --no-api-path --steps 3 > $O/bench_cfg3.log 2>&1 || exit 4
timeout -k 10 400 python -u bench.py --workload cfg4t --no-cpu-baseline --no-api-path --steps 3 > $O/bench_cfg4t.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --workload cfg5 --no-cpu-baseline --no-api-path --steps 2 > $O/bench_cfg5.log 2>&1 || exit 6
timeout -k 10 400 python -u bench.py --workload model --emulate-world 8 --no-cpu-baseline --no-api-path --steps 2 > $O/bench_model8.log 2>&1 || exit 7
