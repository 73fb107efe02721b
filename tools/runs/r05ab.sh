#!/bin/bash
# config 2 with the batch interleaved on 1 / 2 / 4 HIP streams (ready-first), same box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ab; mkdir -p $O
for s in 1 2 4 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-api-path --no-parity --steps 3 --streams $s > $O/bench_s${s}_$RANDOM.log 2>&1 || exit 1
done
timeout -k 10 600 python -u tools/tune_solver.py cfg2 256 "tol=1e-5" "jacobi_values_sweeps=2" "jacobi_values_sweeps=3" "tol=1e-5" > $O/tune_jv.log 2>&1 || exit 2
