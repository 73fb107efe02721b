# GPU box, round 4 (r): Q-update variants after the list-path geometry change.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04r}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_qupdate_variants.py tests/test_gpu_kernels.py tests/test_gpu_caldera.py tests/test_gpu_configs.py -q --timeout 200 \
    --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
