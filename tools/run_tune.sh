# GPU box: solver tuning sweep (tools/tune_solver.py) at batch $1 over the remaining specs
cd $GRAFT_REPO_ROOT
B=$1; shift
timeout -k 10 900 python3 -u tools/tune_solver.py $B "$@" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/tune.log
