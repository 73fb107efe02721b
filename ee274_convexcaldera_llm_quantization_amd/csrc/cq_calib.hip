// Hessian calibration kernels: the per-channel diagonal of the activation
// second moment that main.py:296-308 accumulates (a_aT = A A^T in float64) and that
// diag_Hessians.pt ships (Hall[name], main.py:163).  HBM-bound streaming reductions: every
// activation element is read once (coalesced, 16-byte loads on the vector path), squared in
// fp64 (exact for fp32/fp16/bf16 inputs) and summed in a fixed order, so results are
// run-to-run deterministic.  The full-Hessian variant is the fp64-MFMA Gram (cq_gram_f64).
#include "cq_common.h"

#include <hip/hip_bf16.h>

namespace cq {

template <int DT>
__device__ __forceinline__ float load_act(const void* x, int64_t i) {
    if constexpr (DT == CQ_F32) return reinterpret_cast<const float*>(x)[i];
    else if constexpr (DT == CQ_F16) return __half2float(reinterpret_cast<const __half*>(x)[i]);
    else return __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(x)[i] << 16);
}

// four consecutive elements from a 4-aligned index (16 bytes fp32, 8 bytes fp16/bf16)
template <int DT>
__device__ __forceinline__ void load_act4(const void* x, int64_t i, float v[4]) {
    if constexpr (DT == CQ_F32) {
        const float4 f = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(x) + i);
        v[0] = f.x; v[1] = f.y; v[2] = f.z; v[3] = f.w;
    } else {
        const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(x) + i);
        const uint32_t w[2] = {u.x, u.y};
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const uint32_t lo = w[t] & 0xffffu, hi = w[t] >> 16;
            if constexpr (DT == CQ_F16) {
                v[2 * t] = __half2float(__ushort_as_half((unsigned short)lo));
                v[2 * t + 1] = __half2float(__ushort_as_half((unsigned short)hi));
            } else {
                v[2 * t] = __uint_as_float(lo << 16);
                v[2 * t + 1] = __uint_as_float(hi << 16);
            }
        }
    }
}

constexpr int kColWaves = 4;  // waves per block, each striding the block's row chunk

// Block (64 * kColWaves threads) = 64 lanes x VEC columns of one row chunk; wave w takes rows
// r0 + w, r0 + w + kColWaves, ...  Partials of the 4 waves are combined through LDS in wave
// order and written to part[chunk][col].
template <int DT, int VEC>
__global__ __launch_bounds__(64 * kColWaves) void act_colsq_partial_kernel(
    const void* __restrict__ x, int64_t rows, int64_t cols, int64_t ld, int64_t rows_per_chunk,
    double* __restrict__ part) {
    __shared__ double lds[kColWaves][64 * VEC];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t c0 = ((int64_t)blockIdx.x * 64 + lane) * VEC;
    const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
    const int64_t r1 = r0 + rows_per_chunk < rows ? r0 + rows_per_chunk : rows;
    double acc[VEC];
#pragma unroll
    for (int t = 0; t < VEC; ++t) acc[t] = 0.0;
    if (c0 < cols) {
        for (int64_t i = r0 + wid; i < r1; i += kColWaves) {
            float v[VEC];
            if constexpr (VEC == 4) {
                load_act4<DT>(x, i * ld + c0, v);
            } else {
                v[0] = load_act<DT>(x, i * ld + c0);
            }
#pragma unroll
            for (int t = 0; t < VEC; ++t) {
                const double d = (double)v[t];
                acc[t] = __builtin_fma(d, d, acc[t]);  // d*d exact in fp64: one rounding, as the sum
            }
        }
    }
#pragma unroll
    for (int t = 0; t < VEC; ++t) lds[wid][lane * VEC + t] = acc[t];
    __syncthreads();
    if (wid == 0 && c0 < cols) {
#pragma unroll
        for (int t = 0; t < VEC; ++t) {
            double s = lds[0][lane * VEC + t];
#pragma unroll
            for (int w = 1; w < kColWaves; ++w) s += lds[w][lane * VEC + t];
            if (c0 + t < cols) part[(int64_t)blockIdx.y * cols + c0 + t] = s;
        }
    }
}

__global__ __launch_bounds__(256) void act_colsq_finalize_kernel(const double* __restrict__ part, int64_t chunks,
                                                                 int64_t cols, double* __restrict__ out,
                                                                 int accumulate, double post) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= cols) return;
    double s = 0.0;
    for (int64_t k = 0; k < chunks; ++k) s += part[k * cols + j];
    out[j] = ((accumulate ? out[j] : 0.0) + s) * post;
}

// One wave per row: lanes stride the row (coalesced), wave_sum in a fixed butterfly order.
template <int DT>
__global__ __launch_bounds__(256) void act_rowsq_kernel(const void* __restrict__ x, int64_t rows, int64_t len,
                                                        int64_t ld, double* __restrict__ out, int accumulate,
                                                        double post) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= rows) return;
    double acc = 0.0;
    for (int64_t j = lane; j < len; j += 64) {
        const double d = (double)load_act<DT>(x, i * ld + j);
        acc = __builtin_fma(d, d, acc);
    }
    acc = wave_sum(acc);
    if (lane == 0) out[i] = ((accumulate ? out[i] : 0.0) + acc) * post;
}

// chunks of >= 16 rows, enough (column blocks x chunks) to cover the CUs several times over
static int64_t colsq_chunks(int64_t rows, int64_t cols) {
    const int64_t cblocks = ceil_div(cols, 256);
    int64_t chunks = ceil_div(4 * kCUs, cblocks);
    const int64_t maxc = ceil_div(rows, 16);
    if (chunks > maxc) chunks = maxc;
    return chunks < 1 ? 1 : chunks;
}

}  // namespace cq

using namespace cq;

extern "C" {

size_t cq_act_sqsum_workspace(int64_t rows, int64_t cols) {
    if (rows <= 0 || cols <= 0) return 0;
    return (size_t)colsq_chunks(rows, cols) * cols * sizeof(double);
}

int cq_act_sqsum_cols(int dtype, const void* x, int64_t rows, int64_t cols, int64_t ld, double* out,
                      int accumulate, double post, void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(out && cols > 0 && rows >= 0 && ld >= cols, "cq_act_sqsum_cols: bad args");
    CQ_REQUIRE(dtype == CQ_F32 || dtype == CQ_F16 || dtype == CQ_BF16, "cq_act_sqsum_cols: dtype");
    CQ_REQUIRE(rows == 0 || x, "cq_act_sqsum_cols: null x");
    hipStream_t s = as_stream(stream);
    if (rows == 0) {  // no tokens: out = (accumulate ? out : 0) * post
        act_colsq_finalize_kernel<<<(int)ceil_div(cols, 256), 256, 0, s>>>(nullptr, 0, cols, out, accumulate, post);
        return check_launch("cq_act_sqsum_cols");
    }
    const int64_t chunks = colsq_chunks(rows, cols);
    if (!ws || ws_bytes < (size_t)chunks * cols * sizeof(double))
        return set_error(CQ_EWORKSPACE, "cq_act_sqsum_cols: workspace too small");
    double* part = reinterpret_cast<double*>(ws);
    const int64_t rpc = ceil_div(rows, chunks);
    const int esz = dtype == CQ_F32 ? 4 : 2;
    const bool vec = cols % 4 == 0 && ld % 4 == 0 && (reinterpret_cast<uintptr_t>(x) % (4 * esz)) == 0;
    const int64_t cpb = vec ? 256 : 64;  // columns per block
    dim3 grid((unsigned)ceil_div(cols, cpb), (unsigned)chunks);
#define CQ_CS(DT)                                                                                        \
    if (vec) act_colsq_partial_kernel<DT, 4><<<grid, 64 * kColWaves, 0, s>>>(x, rows, cols, ld, rpc, part); \
    else act_colsq_partial_kernel<DT, 1><<<grid, 64 * kColWaves, 0, s>>>(x, rows, cols, ld, rpc, part)
    if (dtype == CQ_F32) { CQ_CS(CQ_F32); }
    else if (dtype == CQ_F16) { CQ_CS(CQ_F16); }
    else { CQ_CS(CQ_BF16); }
#undef CQ_CS
    act_colsq_finalize_kernel<<<(int)ceil_div(cols, 256), 256, 0, s>>>(part, chunks, cols, out, accumulate, post);
    return check_launch("cq_act_sqsum_cols");
}

int cq_act_sqsum_rows(int dtype, const void* x, int64_t rows, int64_t len, int64_t ld, double* out,
                      int accumulate, double post, void* stream) {
    CQ_REQUIRE(out && rows > 0 && len >= 0 && ld >= len, "cq_act_sqsum_rows: bad args");
    CQ_REQUIRE(dtype == CQ_F32 || dtype == CQ_F16 || dtype == CQ_BF16, "cq_act_sqsum_rows: dtype");
    CQ_REQUIRE(len == 0 || x, "cq_act_sqsum_rows: null x");
    hipStream_t s = as_stream(stream);
    const unsigned g = (unsigned)ceil_div(rows, 4);
    if (dtype == CQ_F32) act_rowsq_kernel<CQ_F32><<<g, 256, 0, s>>>(x, rows, len, ld, out, accumulate, post);
    else if (dtype == CQ_F16) act_rowsq_kernel<CQ_F16><<<g, 256, 0, s>>>(x, rows, len, ld, out, accumulate, post);
    else act_rowsq_kernel<CQ_BF16><<<g, 256, 0, s>>>(x, rows, len, ld, out, accumulate, post);
    return check_launch("cq_act_sqsum_rows");
}

}  // extern "C"
