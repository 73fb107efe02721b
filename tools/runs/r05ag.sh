#!/bin/bash
# parts at config 2 (2 vs 3) and the default_parts threshold at small batches (B = 32, 16: 1 vs 2 parts), same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ag; mkdir -p $O
for s in 2 3 2 3; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-api-path --no-parity --steps 3 --streams $s > $O/cfg2_s${s}_$RANDOM.log 2>&1 || exit 1
done
for b in 32 16; do for s in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-api-path --no-parity --steps 3 --batch $b --streams $s > $O/cfg2_b${b}_s$s.log 2>&1 || exit 2
done; done
