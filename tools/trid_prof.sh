# kernel breakdown of the tridiagonal eigensolver (tools/bench_jacobi.py, B = 256, p = 192)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/tridprof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tridprof/s -o run --output-format csv -- python3 tools/bench_jacobi.py 256 192 > gpurun_out/tridprof/log 2>&1
python3 - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob('gpurun_out/tridprof/s/**/run_kernel_stats.csv', recursive=True)[0])))
for r in rows[:8]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {int(r['Calls']):5d} calls avg {float(r['AverageNs'])/1e6:7.3f} ms  {r['Name'][:90]}")
PY
