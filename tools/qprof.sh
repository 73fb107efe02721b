set -e
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof/stats -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api-path --no-parity > gpurun_out/qprof/s.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex q_update -d gpurun_out/qprof/f -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-api-path --no-parity > gpurun_out/qprof/f.log 2>&1
grep -h "q_update\|quant_w" gpurun_out/qprof/stats/run_kernel_stats.csv | cut -c1-200
python3 - <<'PY'
import csv, glob, collections
rows = list(csv.DictReader(open(glob.glob('gpurun_out/qprof/f/*counter_collection.csv')[0])))
agg = collections.defaultdict(list)
for r in rows:
    agg[r['Kernel_Name'][:60]].append(float(r['Counter_Value']))
for k, v in agg.items(): print(k, len(v), sum(v)/len(v))
PY
