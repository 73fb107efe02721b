#!/bin/bash
# l-split ELL A/B where it applies (config 4's tall shape, the whole-model rank share, config 3), kernel traces of cfg4t
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
for v in split nosplit; do
  a=""; [ $v = nosplit ] && a="--no-l-split"
  timeout -k 10 400 python -u bench.py --workload cfg4t --no-cpu-baseline --no-api-path --steps 3 $a > $O/bench_cfg4t_$v.log 2>&1 || exit 1
  timeout -k 10 400 python -u bench.py --workload model --emulate-world 8 --no-cpu-baseline --no-api-path --steps 2 $a > $O/model8_$v.log 2>&1 || exit 2
  timeout -k 10 400 python -u bench.py --workload cfg3 --no-cpu-baseline --no-api-path --steps 3 $a > $O/bench_cfg3_$v.log 2>&1 || exit 3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt4t_$v -o run -- python3 bench.py --workload cfg4t --no-cpu-baseline --no-api-path --no-parity --steps 1 --warmup 1 $a > $O/kt4t_$v.log 2>&1 || exit 4
done
timeout -k 10 300 python -u tools/list_density.py > $O/list_density_cfg2.log 2>&1 || exit 5
timeout -k 10 300 python -u tools/list_density.py --workload cfg3 > $O/list_density_cfg3.log 2>&1 || exit 6
timeout -k 10 300 python -u tools/list_density.py --workload cfg4t > $O/list_density_cfg4t.log 2>&1 || exit 7
