#!/bin/bash
# pass-2 epilogue on lane masks (fma-mix residual, max3 |.|, scalar classification): GPU suite, list micro-bench A/B vs HEAD, kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 --lib tools/probes/lib_base.so > $O/qu_base.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 > $O/qu_new.log 2>&1 || exit 3
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 --lib tools/probes/lib_base.so > $O/qu_base2.log 2>&1 || exit 4
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 > $O/qu_new2.log 2>&1 || exit 5
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktq -o run -- python3 tools/bench_qupdate_list.py 256 5 > $O/ktq.log 2>&1 || exit 6
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktqb -o run -- python3 tools/bench_qupdate_list.py 256 5 --lib tools/probes/lib_base.so > $O/ktqb.log 2>&1 || exit 7
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-path --steps 3 > $O/bench.log 2>&1 || exit 8
