# GPU box, round 4 (zb): all workloads on the current tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04zb}; mkdir -p $O
for w in ${WORKLOADS:-cfg3 cfg4t model cfg5}; do
  timeout -k 10 500 python3 -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-api-path > $O/bench_$w.log 2>&1 || exit $?
  tail -1 $O/bench_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["name"], round(d["value"],1), round(d["ms_per_step"],1))'
done
