# GPU box: Q-update A/B (approximate vs default absmax pass, checksums must agree), the full
# GPU suite, the default bench line, then the round's profile (kernel stats + PMC traffic)
set -o pipefail
cd $GRAFT_REPO_ROOT
CQ_QP0_APPROX=1 timeout -k 10 240 python3 tools/bench_filter.py 256 > gpurun_out/qu_approx.log 2>&1 || { tail -5 gpurun_out/qu_approx.log; exit 1; }
grep "q_update\|q checksum" gpurun_out/qu_approx.log
timeout -k 10 240 python3 tools/bench_filter.py 256 > gpurun_out/qu_default.log 2>&1 || { tail -5 gpurun_out/qu_default.log; exit 1; }
grep "q_update\|q checksum" gpurun_out/qu_default.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { tail -30 gpurun_out/gpu_all.log; exit 1; }
tail -2 gpurun_out/gpu_all.log
timeout -k 10 600 python3 bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.log | tail -1 | cut -c1-400
bash tools/profile_round.sh ${TAG:-r02l} 256 && cat gpurun_out/prof_${TAG:-r02l}/summary.txt | head -20
