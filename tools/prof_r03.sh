#!/bin/bash
# Round-3 profiling recipe (GPU box, repo root): kernel-trace stats of the default bench
# config, then separate PMC passes (FETCH_SIZE, WRITE_SIZE) over every kernel of one step.
#   bash tools/prof_r03.sh <tag> [batch]
set -o pipefail
TAG=${1:-r03}; B=${2:-256}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BA="--batch $B --steps 1 --warmup 1 --no-parity --no-cpu-baseline --no-api-path"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 bench.py $BA > $OUT/stats.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c -d $OUT/pmc_$c -o run --output-format csv -- \
      python3 bench.py $BA > $OUT/pmc_$c.log 2>&1 || exit $?
done
python3 tools/profile_summary.py $OUT/stats $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE > $OUT/summary.txt
python3 tools/pmc_traffic.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE $B 192 4096 > $OUT/pmc_traffic.json || true
python3 tools/pmc_traffic_quant.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE $B 4096 4096 2 > $OUT/pmc_traffic_quant.json || true
head -50 $OUT/summary.txt
