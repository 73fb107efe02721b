set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "q_update or quant or cfg1 or Q" > gpurun_out/qt.log 2>&1 || { tail -30 gpurun_out/qt.log; exit 1; }
tail -2 gpurun_out/qt.log
CQ_QU_KERNEL=1 timeout -k 10 240 python3 tools/bench_filter.py 128 2>&1 | grep "q_update\|q checksum"
timeout -k 10 240 python3 tools/bench_filter.py 128 2>&1 | grep "q_update\|q checksum"
