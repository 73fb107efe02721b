set -o pipefail
cd $GRAFT_REPO_ROOT
export CQ_X3_KERNEL=$1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kt_$1.log 2>&1 || { tail -30 gpurun_out/kt_$1.log; exit 1; }
tail -2 gpurun_out/kt_$1.log
CQ_X3_CLOCK=1 timeout -k 10 240 python3 tools/bench_filter.py 128 2>&1 | grep -v amdgpu.ids | grep -v "q_update\|q checksum"
