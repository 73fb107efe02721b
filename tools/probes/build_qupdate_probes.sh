#!/bin/bash
# Probe builds of the 2-bit list-path Q update (test infrastructure, never the product library):
# each variant removes one part of pass 2's work from a temporary copy of the sources and builds
# tools/probes/lib_qu_<variant>.so, for tools/bench_qupdate_list.py --lib (codes are wrong on purpose)
#   no_r    the R^T stage loaded for the first chunk only (later chunks reuse it)
#   no_w    the W ring filled in the prologue only
#   no_epi  no pass-2 epilogue (residual, max, error, lists): the products are folded into the max
#   mfma1   one MFMA per block and K step instead of three
#   drain   the counted end-of-chunk wait even after list stores (timing only: with stores in
#           flight the count does not prove the next stage landed)
#   nostore the candidate lists classified but not stored
#   prio    s_setprio 1 for the second half of the waves (static priority); prio4 / prio8:
#           for waves 4-11 / 8-11 of the 12
#   xprio6 / xprio8 / xprio4: the same for the split-fp16 products' K loops (cq_x3.hip: waves >= 6 / 8 / 4
#           of 12; the 8-wave 256 x 256 tile's waves >= 4)
# (variants to build: the arguments, default all)
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
for v in ${@:-no_r no_w no_epi mfma1 drain nostore prio}; do
  T=$(mktemp -d); mkdir -p $T/a/csrc $T/include
  cp $ROOT/ee274_convexcaldera_llm_quantization_amd/csrc/* $T/a/csrc/; cp $ROOT/include/caldera_hip.h $T/include/
  f=$T/a/csrc/cq_qupdate.hip
  case $v in
    no_r)  sed -i 's/^\(\s*\)qp_issue_r<NW, RROW>(Rhb, Rlb, (ch + 1) \* QP_BN/\1if (false) qp_issue_r<NW, RROW>(Rhb, Rlb, (ch + 1) * QP_BN/' $f ;;
    no_w)  sed -i 's/^\(\s*\)if (wlive) issue_w(ch + QP_WD - 1/\1if (false) issue_w(ch + QP_WD - 1/' $f ;;
    no_epi) sed -i 's/^\(\s*\)if constexpr (PASS == 2) {$/\1if constexpr (PASS == 2) { mx = max(mx, __float_as_uint(v[0] + v[1] + v[2] + v[3] + v[4] + v[5] + v[6] + v[7]) \& 0x7fffffffu); continue;/' $f ;;
    mfma1) sed -i 's/^\(\s*\)acc\[rb\]\[c\] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fl\[ks\]\[c\], lh\[rb\]\[ks\], acc\[rb\]\[c\], 0, 0, 0);/\1(void)0;/; s/^\(\s*\)acc\[rb\]\[c\] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fh\[ks\]\[c\], ll\[rb\]\[ks\], acc\[rb\]\[c\], 0, 0, 0);/\1(void)0;/' $f ;;
    drain) sed -i 's/^\(\s*\)if (!stored \&\& wlive) wait_vm(/\1if (wlive) wait_vm(/' $f ;;
    nostore) sed -i 's/^\(\s*\)laR\[pos\] = make_uint2/\1if (q.m < 0) laR[pos] = make_uint2/; s/^\(\s*\)gvR\[2 \* pos\] = /\1if (q.m < 0) gvR[2 * pos] = /; s/^\(\s*\)gvR\[2 \* pos + 1\] = /\1if (q.m < 0) gvR[2 * pos + 1] = /; s/^\(\s*\)gidR\[pos\] = /\1if (q.m < 0) gidR[pos] = /' $f ;;
    prio4) sed -i 's/^\(\s*\)int sw = 0;   \/\/ slot of chunk ch/\1if (wid >= 4) __builtin_amdgcn_s_setprio(1);\n\1int sw = 0;/' $f ;;
    prio8) sed -i 's/^\(\s*\)int sw = 0;   \/\/ slot of chunk ch/\1if (wid >= 8) __builtin_amdgcn_s_setprio(1);\n\1int sw = 0;/' $f ;;
    xprio*) th=${v#xprio}; g=$T/a/csrc/cq_x3.hip
       python3 - "$g" "$th" <<'PYEOF'
import sys
p, th = sys.argv[1], sys.argv[2]
s = open(p).read().split("\n")
loops = [i for i, l in enumerate(s) if l == "    for (int64_t t = 0; t < nt; ++t) {"]
assert len(loops) == 5, loops
for n, i in enumerate(reversed(loops)):   # the last loop is the 8-wave 256 x 256 tile's
    s.insert(i, f"    if (wid >= {4 if n == 0 else th}) __builtin_amdgcn_s_setprio(1);")
open(p, "w").write("\n".join(s))
PYEOF
       f=$g ;;
    prio) sed -i 's/^\(\s*\)int sw = 0;   \/\/ slot of chunk ch/\1if (wid >= NW \/ 2) __builtin_amdgcn_s_setprio(1);\n\1int sw = 0;/' $f ;;
  esac
  if cmp -s $f $ROOT/ee274_convexcaldera_llm_quantization_amd/csrc/cq_qupdate.hip; then echo "probe $v: patch did not apply"; exit 1; fi
  F="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt"
  objs=""
  for s in $T/a/csrc/*.hip; do
    extra=""; [ "$(basename $s)" = cq_qupdate.hip ] && extra="-fno-slp-vectorize"
    /opt/rocm/bin/hipcc $F $extra -c -o ${s%.hip}.o $s &
    objs="$objs ${s%.hip}.o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/tools/probes/lib_qu_$v.so $objs
  rm -rf $T
  echo built tools/probes/lib_qu_$v.so
done
