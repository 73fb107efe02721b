#!/bin/bash
# static wave priority A/B: Q update pass 2 (waves >= 4 / 6 / 8 of 12) and the split-fp16 products (filter micro-bench); filter intake probe modes 0-7
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 300 tools/probes/probe_filter_intake 256 > $O/probe_intake.log 2>&1 || exit 1
for v in base prio4 prio prio8; do
  lib=tools/probes/lib_qu_$v.so; [ $v = base ] && lib=ee274_convexcaldera_llm_quantization_amd/libcaldera_hip.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 tools/bench_qupdate_list.py 256 5 --lib $lib > $O/kt_$v.log 2>&1 || exit 2
done
for v in base xprio6 xprio8 xprio4 base; do
  lib=tools/probes/lib_qu_$v.so; [ $v = base ] && lib=ee274_convexcaldera_llm_quantization_amd/libcaldera_hip.so
  timeout -k 10 300 python3 -u tools/bench_filter.py 256 --lib $lib >> $O/filter.log 2>&1 || exit 3
done
