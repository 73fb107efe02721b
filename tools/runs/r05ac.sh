#!/bin/bash
# two HIP streams per batch (ready-first interleaving) on the other workloads, same box; cfg2 with parity at 2 streams
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ac; mkdir -p $O
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-api-path --steps 3 --streams 2 > $O/bench_cfg2_s2_parity.log 2>&1 || exit 1
for w in cfg3 cfg5 cfg4t; do
  for s in 1 2; do
    timeout -k 10 400 python -u bench.py --workload $w --no-cpu-baseline --no-api-path --no-parity --steps 2 --streams $s > $O/bench_${w}_s$s.log 2>&1 || exit 2
  done
done
