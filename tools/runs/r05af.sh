#!/bin/bash
# whole-model (config 4) batching: batch size x batches interleaved at a time, one GPU
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05af; mkdir -p $O
for cfg in "64 2" "64 3" "32 4" "32 6" "64 2"; do
  set -- $cfg
  timeout -k 10 400 python -u bench.py --workload model --no-cpu-baseline --no-api-path --steps 2 --model-batch $1 --model-group $2 > $O/model_b$1_g$2_$RANDOM.log 2>&1 || exit 1
done
