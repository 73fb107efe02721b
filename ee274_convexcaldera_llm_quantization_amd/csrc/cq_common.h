// Shared helpers for the gfx950 CALDERA kernels: status/error plumbing for the C-ABI,
// wave64 reductions, and launch-geometry constants.  No compatibility layers: CDNA4 only.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/caldera_hip.h"

namespace cq {

constexpr int kWave = 64;        // CDNA wavefront width (hard-coded: warpSize folds to 64 on gfx950)
constexpr int kCUs = 256;        // MI355X: 8 XCDs x 32 CUs
constexpr int kMaxGrid = 2048;   // memory-bound grid cap (Guideline 11)

int set_error(int code, const char* fmt, ...);
int check_launch(const char* what);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- wave64 reductions (DPP/shuffle via __shfl_xor over 64 lanes) ----
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        uint32_t o = __shfl_xor(v, off, 64);
        v = v > o ? v : o;
    }
    return v;
}

// |x| as order-preserving uint bits (NaN sorts above +inf, matching torch max NaN propagation).
__device__ __forceinline__ uint32_t abs_bits(float x) { return __float_as_uint(x) & 0x7fffffffu; }

// Block-wide fp64 sum of one value per thread; result valid in thread 0.  blockDim multiple of 64.
__device__ __forceinline__ double block_sum_f64(double v, double* lds /* >= 16 */) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) lds[wid] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) {
        const int nw = blockDim.x >> 6;
        for (int i = 0; i < nw; ++i) s += lds[i];
    }
    __syncthreads();
    return s;
}

// ---- uniform quantiser arithmetic (quantization.py:93-105, :244-269), shared by the
// standalone quantiser and the fused Q update
__device__ __forceinline__ float quant_scale(uint32_t bits, float eps) {
    const float m = __uint_as_float(bits);
    return (m != m) ? m : fmaxf(m, eps);  // torch.maximum propagates NaN; fmaxf would not
}

// code = rint((x / s) * k): two IEEE roundings then round-half-even (quantization.py:95-96,266)
__device__ __forceinline__ float quant_code(float x, float s, float k) {
    const float norm = x / s;
    const float scaled = norm * k;
    return rintf(scaled);
}
__device__ __forceinline__ float dequant(float c, float k, float s) { return (c / k) * s; }

}  // namespace cq

#define CQ_REQUIRE(cond, ...)                                  \
    do {                                                       \
        if (!(cond)) return ::cq::set_error(CQ_EINVAL, __VA_ARGS__); \
    } while (0)
