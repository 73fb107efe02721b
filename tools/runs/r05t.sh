#!/bin/bash
# round-5 final profiles: kernel trace + stats of the default bench command, PMC traffic passes (profile_round.sh), Q pass-2 no-epilogue probe
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py > $O/bench_default_ktrace.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktq_noepi -o run -- python3 tools/bench_qupdate_list.py 256 5 --lib tools/probes/lib_qu_no_epi.so > $O/ktq_noepi.log 2>&1 || exit 2
timeout -k 10 1000 bash tools/profile_round.sh r05 256 > $O/profile_round.log 2>&1 || exit 3
