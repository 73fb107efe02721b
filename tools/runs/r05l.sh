#!/bin/bash
# what bounds the list-path Q update: probe builds (tools/probes/build_qupdate_probes.sh) vs the library
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 --lib tools/probes/lib_qu_bool.so > $O/qu_lib.log 2>&1 || exit 1
for v in no_r no_w no_epi mfma1; do
  timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 --lib tools/probes/lib_qu_$v.so > $O/qu_$v.log 2>&1 || exit 2
done
timeout -k 10 120 python -u tools/bench_qupdate_list.py 256 10 --lib tools/probes/lib_qu_bool.so > $O/qu_lib2.log 2>&1 || exit 3
