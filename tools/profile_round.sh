#!/bin/bash
# Profiling recipe for one round (run on the GPU box from the repo root):
#   bash tools/profile_round.sh <round-tag> <batch>
# 1) kernel stats of the default bench config, 2) two separate PMC passes (FETCH_SIZE,
# WRITE_SIZE) restricted to the split-fp16 filter GEMM; summaries land in gpurun_out/.
set -eo pipefail
TAG=${1:-r01}; B=${2:-64}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 bench.py --batch $B --steps 1 --warmup 1 --no-parity > $OUT/stats.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm_x3 -d $OUT/pmc_fetch -o run \
    --output-format csv -- python3 bench.py --batch $B --steps 1 --warmup 0 --no-parity > $OUT/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex gemm_x3 -d $OUT/pmc_write -o run \
    --output-format csv -- python3 bench.py --batch $B --steps 1 --warmup 0 --no-parity > $OUT/pmc_write.log 2>&1
python3 tools/profile_summary.py $OUT/stats $OUT/pmc_fetch $OUT/pmc_write > $OUT/summary.txt
python3 tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write $B 192 4096 > $OUT/pmc_traffic.json
