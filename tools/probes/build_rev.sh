#!/bin/bash
# Build libcaldera_hip.so from the kernel sources of git revision $1 into tools/probes/lib_$2.so
# (A/B timing of a kernel change on one box: tools/bench_qupdate_list.py --lib ...)
set -e
rev=$1; name=$2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
T=$(mktemp -d)
mkdir -p $T/a/csrc $T/include
for f in $(git -C $ROOT ls-tree --name-only $rev ee274_convexcaldera_llm_quantization_amd/csrc/); do
  git -C $ROOT show $rev:$f > $T/a/csrc/$(basename $f)
done
git -C $ROOT show $rev:include/caldera_hip.h > $T/include/caldera_hip.h
F="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt"
objs=""
for s in $T/a/csrc/*.hip; do
  extra=""; [ "$(basename $s)" = cq_qupdate.hip ] && extra="-fno-slp-vectorize"
  /opt/rocm/bin/hipcc $F $extra -c -o ${s%.hip}.o $s &
  objs="$objs ${s%.hip}.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/probes/lib_$name.so $objs
rm -rf $T
echo built tools/probes/lib_$name.so
