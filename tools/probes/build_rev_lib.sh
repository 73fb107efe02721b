#!/bin/bash
# Build the HIP library from the sources of a git revision into tools/probes/lib_<name>.so
# (test infrastructure for same-box A/Bs against the working tree, e.g.
# tools/bench_small_kernels.py --lib tools/probes/lib_head.so):
#   bash tools/probes/build_rev_lib.sh <rev> <name>
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
REV=${1:-HEAD}; NAME=${2:-head}
T=$(mktemp -d)
git -C $ROOT archive $REV ee274_convexcaldera_llm_quantization_amd/csrc include | tar -x -C $T
F="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt"
objs=""
for s in $T/ee274_convexcaldera_llm_quantization_amd/csrc/*.hip; do
  extra=""; [ "$(basename $s)" = cq_qupdate.hip ] && extra="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc $F $extra -I$T/include -c -o ${s%.hip}.o $s &
  objs="$objs ${s%.hip}.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/probes/lib_$NAME.so $objs
rm -rf $T
echo built tools/probes/lib_$NAME.so
