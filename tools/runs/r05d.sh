#!/bin/bash
# filter intake probe; config-4 share timeline (ready-first) and batch-size variants; B = 256 seeds test
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 120 tools/probes/probe_filter_intake 256 > $O/probe_intake.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/bench_share.py --steps 1 > $O/share_kt.log 2>&1 || exit 2
python3 tools/timeline.py $O/kt > $O/timeline.txt 2>&1 || exit 3
timeout -k 10 200 python -u tools/bench_share.py --steps 3 --max-batch 8 > $O/share_mb8.log 2>&1 || exit 4
timeout -k 10 200 python -u tools/bench_share.py --steps 3 --max-batch 8 --group 8 > $O/share_mb8_g8.log 2>&1 || exit 5
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_configs.py -k full_batch > $O/test_full_batch.log 2>&1 || exit 6
