#!/bin/bash
# Q update with staggered (deferred-epilogue) late waves: bit-identity tests, A/B vs the HEAD build, bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_qupdate_variants.py > $O/tests_qupdate.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 --lib tools/probes/lib_base.so > $O/qu_base.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 > $O/qu_new.log 2>&1 || exit 3
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 --lib tools/probes/lib_base.so > $O/qu_base2.log 2>&1 || exit 4
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 > $O/qu_new2.log 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-path --steps 2 > $O/bench.log 2>&1 || exit 6
