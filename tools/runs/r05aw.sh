#!/bin/bash
# round-end tree (clean rebuild): smoke, GPU suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aw; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 2
