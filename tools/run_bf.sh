# GPU box: filter/Gram/Q-update micro-bench for kernel variants given as arguments
set -o pipefail
cd $GRAFT_REPO_ROOT
B=$1; shift
for v in "$@"; do
  timeout -k 10 240 env CQ_X3_KERNEL=$v python3 tools/bench_filter.py $B > gpurun_out/bf_$v.log 2>&1 || { cat gpurun_out/bf_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/bf_$v.log
done
