#!/bin/bash
# filter intake probe, modes 0-7 (X^T via LDS-DMA vs registers), config-2 B = 256 shapes
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 300 tools/probes/probe_filter_intake 256 > $O/probe_intake.log 2>&1 || exit 1
