# GPU box, round 4 (j): LDS swizzle of the split-fp16 product images for gfx950's ds_read_b128
# lane groups -- GPU suite, config 2 / 4t benches, config 2 kernel trace, PMC (bank conflicts).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04j}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for w in ${WORKLOADS:-cfg2 cfg4t}; do
  timeout -k 10 500 python3 -u bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-api-path > $O/bench_$w.log 2>&1 || exit $?
  tail -1 $O/bench_$w.log | cut -c1-200
done
mkdir -p $O/kt_cfg2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt_cfg2/t -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-api-path > $O/kt_cfg2/s.log 2>&1 || exit $?
python3 tools/ktrace_summary.py $O/kt_cfg2 > $O/kt_cfg2/summary.txt; head -16 $O/kt_cfg2/summary.txt | cut -c1-150
bash tools/pmc_mfma.sh $O/pmc > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
tail -3 $O/pmc.log
