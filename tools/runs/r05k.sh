#!/bin/bash
# fused |C| max for the LPLR split scales; bool two-class lists: GPU suite, Q update A/B, cfg5, cfg2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 --lib tools/probes/lib_base.so > $O/qu_base.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 > $O/qu_new.log 2>&1 || exit 3
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 --lib tools/probes/lib_base.so > $O/qu_base2.log 2>&1 || exit 4
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 > $O/qu_new2.log 2>&1 || exit 5
timeout -k 10 400 python -u bench.py --workload cfg5 --no-cpu-baseline --no-api-path --steps 2 > $O/bench_cfg5.log 2>&1 || exit 6
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-path --steps 2 > $O/bench.log 2>&1 || exit 7
