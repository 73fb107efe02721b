#!/bin/bash
# software-pipelined pass 2: Q-update tests, list micro-bench A/B (kernel traces), GPU suite, bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aj; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_qupdate_variants.py -x -v --timeout 120 --timeout-method thread > $O/qu_tests.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_pipe -o run -- python3 tools/bench_qupdate_list.py 256 5 > $O/kt_pipe.log 2>&1 || exit 2
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_nopipe -o run -- python3 tools/bench_qupdate_list.py 256 5 --lib tools/probes/lib_qu_nopipe.so > $O/kt_nopipe.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 4
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-api-path --steps 3 > $O/bench.log 2>&1 || exit 5
