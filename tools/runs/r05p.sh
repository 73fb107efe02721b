#!/bin/bash
# pass-2 probes on the mask epilogue: full drain vs counted wait, list stores, static priority (kernel traces)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
for v in base drain nostore prio; do
  lib=tools/probes/lib_qu_$v.so; [ $v = base ] && lib=ee274_convexcaldera_llm_quantization_amd/libcaldera_hip.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 tools/bench_qupdate_list.py 256 5 --lib $lib > $O/kt_$v.log 2>&1 || exit 1
done
