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

// Correctly rounded a / b for many quotients with one divisor (Markstein): y = RN(1/b) from
// one IEEE division, q = RN(a y), r = a - q b (exact by FMA), q' = RN(q + r y) = RN(a / b)
// (Muller et al., Handbook of Floating-Point Arithmetic, Thm 5.8) whenever the quotient is a
// normal number; zero, tiny, huge and non-finite cases take the IEEE division.  Three VALU
// ops instead of the ~10 of the correctly rounded division sequence.
__device__ __forceinline__ float div_rn(float a, float b, float y) {
    const float q = a * y;
    const float aq = fabsf(q);
    if (!(aq >= 0x1p-100f && aq <= 0x1p100f)) return a / b;
    const float r = __builtin_fmaf(-q, b, a);
    return __builtin_fmaf(r, y, q);
}
// Branch-free form for kernels that checked once that the divisor is a finite normal number
// and that |a| <= |b| (a quantiser's scale is the max |x|): quotients then never overflow,
// and a tiny quotient only needs |result| << 1/2, which the FMA path gives.
__device__ __forceinline__ float div_fast(float a, float b, float y) {
    const float q = a * y;
    const float r = __builtin_fmaf(-q, b, a);
    return __builtin_fmaf(r, y, q);
}
__device__ __forceinline__ bool div_fast_ok(float b) { return b >= 0x1p-126f && b <= 0x1p126f; }
// quant_code / dequant with the divisor reciprocals precomputed (ys = RN(1/s), yk = RN(1/k))
__device__ __forceinline__ float quant_code_r(float x, float s, float ys, float k) {
    return rintf(div_rn(x, s, ys) * k);
}
__device__ __forceinline__ float dequant_r(float c, float k, float yk, float s) { return div_rn(c, k, yk) * s; }

// block-Jacobi eigensolver (cq_bjacobi.hip) behind cq_jacobi_eigh for p > kBlockJacobiMinP
constexpr int64_t kBlockJacobiMinP = 192;
size_t bj_workspace(int64_t p, int64_t batch);
int bj_eigh(double* A, int64_t p, int64_t batch, int max_sweeps, double tol, double* evals, float* V32,
            double* V64, int* sweeps_out, void* ws, size_t ws_bytes, hipStream_t s);
constexpr int BJ_BEGIN = 1, BJ_SWEEPS = 2, BJ_END = 4;
int bj_stage(double* A, int64_t p, int64_t batch, int phase, int nsweeps, double tol, bool want_v, double* evals,
             float* V32, double* V64, int* sweeps_out, int* pending_out, void* ws, size_t ws_bytes, hipStream_t s);

}  // namespace cq

#define CQ_REQUIRE(cond, ...)                                  \
    do {                                                       \
        if (!(cond)) return ::cq::set_error(CQ_EINVAL, __VA_ARGS__); \
    } while (0)
