# GPU box: Q-update tests, then the Q-update micro-bench with pass 0's W loads in pairs of
# chunks (CQ_QP0_PAIRW=1) and one chunk at a time (default); checksums must agree
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "q_update or quant or cfg or Q or caldera or variants" > gpurun_out/qt.log 2>&1 || { tail -30 gpurun_out/qt.log; exit 1; }
tail -2 gpurun_out/qt.log
CQ_QP0_PAIRW=1 timeout -k 10 240 python3 tools/bench_filter.py 256 > gpurun_out/qu_pairw.log 2>&1 || { tail -5 gpurun_out/qu_pairw.log; exit 1; }
grep "q_update\|q checksum" gpurun_out/qu_pairw.log
timeout -k 10 240 python3 tools/bench_filter.py 256 > gpurun_out/qu_default.log 2>&1 || { tail -5 gpurun_out/qu_default.log; exit 1; }
grep "q_update\|q checksum" gpurun_out/qu_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof3 -o run --output-format csv -- python3 tools/bench_filter.py 256 > gpurun_out/qprof3.log 2>&1 || { tail -5 gpurun_out/qprof3.log; exit 1; }
grep -h "q_update_p" gpurun_out/qprof3/run_kernel_stats.csv | cut -c1-40,150-260
