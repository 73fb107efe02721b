#!/bin/bash
# share with split-K off under interleaving; model projection; cfg3 l-split A/B; full GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 200 python -u tools/bench_share.py --steps 3 > $O/share.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --workload model --no-parity --steps 3 --emulate-world 8 > $O/model_emulate8.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py --workload cfg3 --no-cpu-baseline --no-api-path --no-parity --steps 2 > $O/cfg3_split.log 2>&1 || exit 3
timeout -k 10 400 python -u bench.py --workload cfg3 --no-cpu-baseline --no-api-path --no-parity --steps 2 --no-l-split > $O/cfg3_nosplit.log 2>&1 || exit 4
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 5
