# GPU box, round 4 (ad): filter-product bound probe (distinct vs shared G), nt on / off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04ad}; mkdir -p $O
timeout -k 10 300 python3 -u tools/probe_x3_shared.py 256 > $O/probe.log 2>&1 || exit $?
cat $O/probe.log | grep -v amdgpu.ids
CQ_X3_NT=0 timeout -k 10 300 python3 -u tools/probe_x3_shared.py 256 > $O/probe_nt0.log 2>&1 || exit $?
cat $O/probe_nt0.log | grep -v amdgpu.ids
