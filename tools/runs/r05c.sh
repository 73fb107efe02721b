#!/bin/bash
# config-4 share: ready-first vs round-robin interleaving; first-LR-step refinement A/B (cfg2, B = 256)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 200 python -u tools/bench_share.py --steps 3 > $O/share_ready.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_share.py --steps 3 --rr > $O/share_rr.log 2>&1 || exit 2
for v in none 4 8 6+6; do
  a=""; [ $v != none ] && a="--solver-refine-steps $v"
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-api-path --steps 2 $a > $O/bench_refine_$v.log 2>&1 || exit 3
done
