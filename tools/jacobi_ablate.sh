#!/bin/bash
# Diagnostic: time the p=192 Jacobi with phases removed (outputs are wrong in ablated builds).
set -e
mkdir -p "$(dirname "$0")/../build_diag"
cd "$(dirname "$0")/.."
for A in 0 1 2 4 7; do
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -fPIC -shared -std=c++17 -ffp-contract=off -DCQ_JAC_ABL=$A \
    -o build_diag/libcq_abl$A.so ee274_convexcaldera_llm_quantization_amd/csrc/cq_quant.hip \
    ee274_convexcaldera_llm_quantization_amd/csrc/cq_gemm.hip ee274_convexcaldera_llm_quantization_amd/csrc/cq_small.hip \
    ee274_convexcaldera_llm_quantization_amd/csrc/cq_x3.hip
done
