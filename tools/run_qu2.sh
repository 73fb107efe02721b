# GPU box: Q-update tests, then the Q-update micro-bench with the exact and the approximate
# absmax pass (checksums must agree), then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "q_update or quant or cfg or Q or caldera" > gpurun_out/qt.log 2>&1 || { tail -30 gpurun_out/qt.log; exit 1; }
tail -2 gpurun_out/qt.log
CQ_QP0_APPROX=1 timeout -k 10 240 python3 tools/bench_filter.py 256 > gpurun_out/qu_approx.log 2>&1 || { tail -5 gpurun_out/qu_approx.log; exit 1; }
grep "q_update\|q checksum" gpurun_out/qu_approx.log
timeout -k 10 240 python3 tools/bench_filter.py 256 > gpurun_out/qu_default.log 2>&1 || { tail -5 gpurun_out/qu_default.log; exit 1; }
grep "q_update\|q checksum" gpurun_out/qu_default.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof -o run --output-format csv -- python3 tools/bench_filter.py 256 > gpurun_out/qprof.log 2>&1 || { tail -5 gpurun_out/qprof.log; exit 1; }
grep -h "q_update_p\|qp_norms" gpurun_out/qprof/*/run_kernel_stats.csv gpurun_out/qprof/run_kernel_stats.csv 2>/dev/null | cut -c1-200 || true
