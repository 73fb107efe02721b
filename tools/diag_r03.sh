#!/bin/bash
# Round-3 diagnostics (GPU box, repo root): available counters, SQ counter passes over the
# fused Q-update micro-benchmark, and the Gram's HBM traffic in one bench step.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/diag_r03
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex q_update_p -d $OUT/q$i -o run --output-format csv -- \
      python3 tools/bench_qupdate_lr.py 64 2 > $OUT/q$i.log 2>&1 || echo "pass $i rc=$?"
done
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm_x3v -d $OUT/gram_fetch -o run --output-format csv -- \
    python3 bench.py --batch 256 --steps 1 --warmup 0 --no-parity --no-cpu-baseline --no-api-path > $OUT/gram_fetch.log 2>&1 || echo "fetch rc=$?"
python3 tools/profile_summary_pmc.py $OUT/q1 $OUT/q2 $OUT/gram_fetch > $OUT/summary.txt 2>&1
cat $OUT/summary.txt | head -60
