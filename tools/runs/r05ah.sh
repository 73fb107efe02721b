#!/bin/bash
# default_parts threshold at B = 8 / 4; the config-4 rank share and whole model with each same-shape batch as 2 parts
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ah; mkdir -p $O
for b in 8 4; do for s in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-api-path --no-parity --steps 3 --batch $b --streams $s > $O/cfg2_b${b}_s$s.log 2>&1 || exit 1
done; done
for mp in 1 2; do
  timeout -k 10 400 python -u bench.py --workload model --emulate-world 8 --no-cpu-baseline --no-api-path --steps 2 --model-parts $mp > $O/model8_p$mp.log 2>&1 || exit 2
done
