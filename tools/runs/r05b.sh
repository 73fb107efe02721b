#!/bin/bash
# config-4 share (rank 0 of 8) timeline: kernel trace + step times
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 200 python -u tools/bench_share.py --steps 3 > $O/share.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/bench_share.py --steps 1 > $O/share_kt.log 2>&1 || exit 2
python3 tools/timeline.py $O/kt > $O/timeline.txt 2>&1 || exit 3
timeout -k 10 200 python -u tools/bench_share.py --steps 3 --group 1 > $O/share_seq.log 2>&1 || exit 4
