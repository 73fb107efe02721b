# LDS counters of the sparse-code Gram kernels (GPU box): one rocprofv3 --pmc pass per group.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sgram; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
    -d $OUT/a -o run --output-format csv -- python3 tools/bench_sgram.py 64 1 > $OUT/a.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_sgram/a/**/run_counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0][:60]
    if "sgram" in k:
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"   {c:24s} {x:.4g}")
PY
