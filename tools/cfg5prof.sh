# kernel-time breakdown of one cfg5 step (B = 64): rocprofv3 --kernel-trace --stats
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg5prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg5prof/stats -o run --output-format csv -- python3 bench.py --workload cfg5 --steps 1 --warmup 1 --no-cpu-baseline --no-api-path --no-parity > gpurun_out/cfg5prof/s.log 2>&1
python3 - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob('gpurun_out/cfg5prof/stats/**/run_kernel_stats.csv', recursive=True)[0])))
tot = sum(float(r['TotalDurationNs']) for r in rows)
with open('gpurun_out/cfg5prof/summary.txt', 'w') as f:
    f.write(f"total kernel time {tot/1e6:.1f} ms (warmup + 1 timed step)\n")
    for r in rows[:25]:
        f.write(f"{float(r['Percentage']):6.2f}% {float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):6d} calls "
                f"avg {float(r['AverageNs'])/1e6:8.3f} ms  {r['Name'][:110]}\n")
print(open('gpurun_out/cfg5prof/summary.txt').read())
PY
