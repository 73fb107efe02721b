#!/bin/bash
# Profiling recipe for one round (run on the GPU box from the repo root):
#   bash tools/profile_round.sh <round-tag> <batch> [<matrices per launch>]
# (the bench splits a batch of >= 32 into two interleaved parts: launches of batch / 2)
# 1) kernel stats of the default bench config, 2) two separate PMC passes (FETCH_SIZE,
# WRITE_SIZE) restricted to the split-fp16 filter GEMM, 3) the same two passes restricted to
# the quantise kernels; summaries land in gpurun_out/.
set -eo pipefail
TAG=${1:-r01}; B=${2:-64}; LB=${3:-$B}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 bench.py --batch $B --steps 1 --warmup 1 --no-parity --no-cpu-baseline --no-api-path > $OUT/stats.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-include-regex gemm_x3 -d $OUT/pmc_$c -o run \
      --output-format csv -- python3 bench.py --batch $B --steps 1 --warmup 0 --no-parity --no-cpu-baseline --no-api-path > $OUT/pmc_$c.log 2>&1
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-include-regex 'quant_w_stream|q_update_p|q_update_v' -d $OUT/qpmc_$c -o run \
      --output-format csv -- python3 bench.py --batch $B --steps 1 --warmup 0 --no-parity --no-cpu-baseline --no-api-path > $OUT/qpmc_$c.log 2>&1
done
python3 tools/profile_summary.py $OUT/stats $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE > $OUT/summary.txt
python3 tools/pmc_traffic.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE $LB 192 4096 > $OUT/pmc_traffic.json
python3 tools/pmc_traffic_quant.py $OUT/qpmc_FETCH_SIZE $OUT/qpmc_WRITE_SIZE $LB 4096 4096 2 > $OUT/pmc_traffic_quant.json
