#!/bin/bash
# r05i from the PMC step: Q update traffic, bench, cfg3 traces, cfg5 bench + trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_f -o run -- python3 tools/bench_qupdate_list.py 256 2 > $O/pmc_f.log 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_w -o run -- python3 tools/bench_qupdate_list.py 256 2 > $O/pmc_w.log 2>&1 || exit 7
python3 tools/pmc_sum.py $O/pmc_f $O/pmc_w q_update qp_codes qp_finalize > $O/pmc_quant.json 2>&1 || exit 8
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-path --steps 2 > $O/bench.log 2>&1 || exit 9
timeout -k 10 400 python -u bench.py --workload cfg5 --no-cpu-baseline --no-api-path --steps 2 > $O/bench_cfg5.log 2>&1 || exit 12
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt5 -o run -- python3 bench.py --workload cfg5 --no-cpu-baseline --no-api-path --no-parity --steps 1 --warmup 1 > $O/kt5.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt3 -o run -- python3 bench.py --workload cfg3 --no-cpu-baseline --no-api-path --no-parity --steps 1 --warmup 1 > $O/kt3.log 2>&1 || exit 10
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt3n -o run -- python3 bench.py --workload cfg3 --no-cpu-baseline --no-api-path --no-parity --steps 1 --warmup 1 --no-l-split > $O/kt3n.log 2>&1 || exit 11
