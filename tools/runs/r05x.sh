#!/bin/bash
# C^T epilogue output vs transpose passes, same box: bench x2 each, kernel traces
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-api-path --no-parity --steps 3 > $O/bench_ct_$rep.log 2>&1 || exit 1
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-api-path --no-parity --steps 3 --no-transposed-output > $O/bench_noct_$rep.log 2>&1 || exit 2
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_ct -o run -- python3 bench.py --no-cpu-baseline --no-api-path --no-parity --steps 1 --warmup 1 > $O/kt_ct.log 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_noct -o run -- python3 bench.py --no-cpu-baseline --no-api-path --no-parity --steps 1 --warmup 1 --no-transposed-output > $O/kt_noct.log 2>&1 || exit 4
