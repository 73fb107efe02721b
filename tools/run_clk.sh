# GPU box: average shader clock of the x3 filter kernel per ablation variant, from
# GRBM_GUI_ACTIVE (GPU-clock cycles) over the kernel-trace duration
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex gemm_x3w -d gpurun_out/clk_$v -o run \
    --output-format csv -- /usr/bin/env CQ_X3_KERNEL=$v python3 tools/bench_filter.py 64 > gpurun_out/clk_$v.log 2>&1 || { tail -5 gpurun_out/clk_$v.log; exit 1; }
  grep "^\[" gpurun_out/clk_$v.log | head -3
done
