# GPU box: MFMA / issue counters of the split-fp16 products (filter gemm_x3v_kernel<false|true>,
# the Gram A) and the 2-bit Q update (q_update_p_kernel<2>, qp_codes_kernel) on the default
# workload at a smaller batch.  One rocprofv3 --pmc pass per counter group (SQ <= 8, GRBM <= 2);
# counters this rocprofv3 does not list are dropped before the pass.
#   bash tools/pmc_mfma.sh OUTDIR [bench args...]
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_mfma}; shift
ARGS=${*:---steps 1 --warmup 0 --batch 64 --no-cpu-baseline --no-api-path --no-parity}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
pick() {  # the counters of "$@" that rocprofv3 -L lists
  for c in "$@"; do grep -qw "$c" $OUT/counters.txt && printf '%s ' "$c"; done
}
A=$(pick SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
         SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE GRBM_COUNT)
B=$(pick SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS \
         SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT)
echo "pass A: $A"; echo "pass B: $B"
REGEX=${REGEX:-'gemm_x3v|q_update_p|qp_codes|sgram'}
i=0
for grp in "$A" "$B"; do
  i=$((i + 1))
  [ -n "$grp" ] || continue
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "$REGEX" -d $OUT/p$i -o run --output-format csv \
      -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_mfma_summary.py $OUT
