# GPU box: the non-default bench workloads (config 5, config 3, config 4 tall, whole model),
# one bench.py process each with its own time limit; stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in cfg5 cfg3 cfg4t model; do
  timeout -k 10 500 python3 -u bench.py --workload $w --no-cpu-baseline --no-api-path > gpurun_out/bench_$w.log 2>&1
  rc=$?; echo "$w rc=$rc"; grep '^{' gpurun_out/bench_$w.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['unit'], d['ms_per_step'], d.get('solver'))" || true
  [ $rc -eq 0 ] || exit $rc
done
