#!/bin/bash
# l-split sparse Gram + staggered Q update: tests, probe, A/B, share, benches
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 120 tools/probes/probe_filter_intake 256 > $O/probe_intake.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_sgram.py tests/test_gpu_qupdate_variants.py tests/test_gpu_codes.py > $O/tests.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 --lib tools/probes/lib_base.so > $O/qu_base.log 2>&1 || exit 3
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 > $O/qu_new.log 2>&1 || exit 4
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 --lib tools/probes/lib_base.so > $O/qu_base2.log 2>&1 || exit 5
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 > $O/qu_new2.log 2>&1 || exit 6
timeout -k 10 200 python -u tools/bench_share.py --steps 3 > $O/share.log 2>&1 || exit 7
timeout -k 10 200 python -u tools/bench_share.py --steps 3 --no-splitk > $O/share_nosplitk.log 2>&1 || exit 8
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/bench_share.py --steps 1 > $O/share_kt.log 2>&1 || exit 9
python3 tools/timeline.py $O/kt > $O/timeline.txt 2>&1 || exit 10
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-path --steps 2 > $O/bench.log 2>&1 || exit 11
timeout -k 10 400 python -u bench.py --workload cfg3 --no-cpu-baseline --no-api-path --steps 2 > $O/bench_cfg3.log 2>&1 || exit 12
