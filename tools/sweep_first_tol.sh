# GPU box: the first LR steps' solver tolerance vs final-code parity and throughput (config 2,
# B = 256, 16 pinned seeds): one bench run per schedule, the relevant fields per line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_tolsweep}; mkdir -p $O
for sched in ${SCHEDS:-none 3e-6 1e-6 1e-6,3e-6}; do
  arg=""; [ "$sched" = none ] || arg="--solver-tol-steps $sched"
  timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-api-path $arg > $O/b_$sched.log 2>&1 || exit $?
  python3 - "$sched" $O/b_$sched.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
p = d["parity_timed_step"]
print(json.dumps({"first_lr_tol": sys.argv[1], "matrices_per_s": round(d["value"], 2), "ms_per_step": round(d["ms_per_step"], 1),
                  "matvecs": d["solver"]["matvecs_per_part"], "bit_exact_vs_reference": p["final_codes_summary"]["bit_exact"],
                  "bit_exact_vs_exact_lr": p.get("final_codes_vs_exact_lr", {}).get("bit_exact"),
                  "differing_vs_exact_lr": sorted(p.get("final_codes_vs_exact_lr", {}).get("differing", {})),
                  "seed15": p["seed15"], "seed8": p["seed8"]}))
PY
done
