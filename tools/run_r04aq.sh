# GPU box, round 4 (aq): non-temporal B loads on / off with NT as a template argument (probe A/B).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04aq}; mkdir -p $O
for nt in 1 0 1 0; do
  CQ_X3_NT=$nt timeout -k 10 300 python3 -u tools/probe_x3_shared.py 256 > $O/probe_nt$nt.log 2>&1 || exit $?
  echo "nt=$nt"; grep "shared_G=0" $O/probe_nt$nt.log
done
