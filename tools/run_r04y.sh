# GPU box, round 4 (y): warm degrees (9, 7) vs (10, 7) on configs 3, 4t and 5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04y}; mkdir -p $O
for wl in "cfg3 192" "cfg4t 64" "cfg5 256"; do
  timeout -k 10 500 python3 -u tools/tune_solver.py $wl "" "deg_warm=(9,7,6)" "" "deg_warm=(9,7,6)" > $O/tune_${wl%% *}.log 2>&1 || exit $?
  echo "== $wl"; cut -c1-190 $O/tune_${wl%% *}.log | grep -v amdgpu.ids
done
