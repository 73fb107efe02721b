// Byte/integer-exact kernels of the CALDERA hot path on gfx950:
//   * global RMS scaling of W           (RCR/src/caldera/decomposition/alg.py:38-42)
//   * uniform absmax quantise / dequant  (RCR/src/caldera/utils/quantization.py:93-105,244-307)
//   * offset-binary int2/int4 packing    (engine storage of Q codes; unpacked to the
//                                          reference int8 layout at the API boundary)
//   * residual builder W - Q, column-weighted (alg.py:124 + diagonal-H form of alg.py:211)
//   * fp64 weighted square sums           (denominator of alg.py:298 for diagonal H)
//
// All of these are HBM-bound streaming kernels: 16-byte vector loads where the layout
// allows, a grid capped at ~2048 workgroups with grid-stride loops, and deterministic
// two-stage fp64 reductions (per-workgroup partials in caller workspace, then one
// finalisation workgroup per matrix) so results are bitwise reproducible run to run.
//
// Numerics follow the reference op by op: IEEE fp32 division x/max (this file is built
// with -ffp-contract=off and correctly-rounded division), rintf (round-half-even, as
// torch.round), multiply by k as a separate rounding, dequant (float(c)/k)*max.
#include "cq_common.h"

#include <mutex>
#include <string>

namespace cq {

static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(CQ_EHIP, "%s: %s", what, hipGetErrorString(e));
    return CQ_OK;
}

constexpr int kThreads = 256;

// ------------------------------------------------------------------ RMS scale (alg.py:38-42)
template <int DT>
__global__ __launch_bounds__(kThreads) void rms_partial_kernel(const void* __restrict__ W,
                                                                int64_t numel, double* part) {
    __shared__ double lds[16];
    const int64_t b = blockIdx.y;
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    if (DT == CQ_F16) {
        const __half* w = reinterpret_cast<const __half*>(W) + b * numel;
        for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < numel; i += stride) {
            const float f = __half2float(w[i]);
            // W.square() in fp16: the square is rounded to fp16 (exact sum of those below)
            acc += (double)__half2float(__float2half_rn(f * f));
        }
    } else {
        const float* w = reinterpret_cast<const float*>(W) + b * numel;
        for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < numel; i += stride) {
            const float f = w[i];
            acc += (double)(f * f);
        }
    }
    const double s = block_sum_f64(acc, lds);
    if (threadIdx.x == 0) part[b * gridDim.x + blockIdx.x] = s;
}

// 8 consecutive elements per thread and step (one 16-byte fp16 load, two fp32 ones): the same
// per-element terms, summed in fp64 (the sum of the fp16 squares is exact at any order)
template <int DT>
__device__ __forceinline__ void load8(const void* __restrict__ X, int64_t e, float (&v)[8]) {
    if (DT == CQ_F16) {
        const uint4 r = *reinterpret_cast<const uint4*>(reinterpret_cast<const __half*>(X) + e);
        const __half* h = reinterpret_cast<const __half*>(&r);
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __half2float(h[u]);
    } else {
        const float4 a = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(X) + e);
        const float4 c = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(X) + e + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
    }
}

template <int DT>
__global__ __launch_bounds__(kThreads) void rms_partial8_kernel(const void* __restrict__ W, int64_t numel,
                                                                 double* part) {
    __shared__ double lds[16];
    const int64_t b = blockIdx.y;
    double acc0 = 0.0, acc1 = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kThreads * 8;
    for (int64_t e = ((int64_t)blockIdx.x * kThreads + threadIdx.x) * 8; e < numel; e += stride) {
        float v[8];
        load8<DT>(W, b * numel + e, v);
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            if (DT == CQ_F16) {  // W.square() in fp16 (see rms_partial_kernel)
                acc0 += (double)__half2float(__float2half_rn(v[u] * v[u]));
                acc1 += (double)__half2float(__float2half_rn(v[u + 1] * v[u + 1]));
            } else {
                acc0 += (double)(v[u] * v[u]);
                acc1 += (double)(v[u + 1] * v[u + 1]);
            }
        }
    }
    const double s = block_sum_f64(acc0 + acc1, lds);
    if (threadIdx.x == 0) part[b * gridDim.x + blockIdx.x] = s;
}

template <int DT>
__global__ void rms_finalize_kernel(const double* part, int nparts, int64_t numel, int do_scale,
                                    float* gs_out) {
    const int64_t b = blockIdx.x;
    if (threadIdx.x != 0) return;
    if (!do_scale) {
        gs_out[b] = 1.0f;
        return;
    }
    double s = 0.0;
    for (int i = 0; i < nparts; ++i) s += part[b * nparts + i];
    // mean: fp32 accumulate type, divided in fp32, then rounded to W's dtype; sqrt in dtype.
    const float mean = (float)s / (float)numel;
    if (DT == CQ_F16) {
        const float mh = __half2float(__float2half_rn(mean));
        gs_out[b] = __half2float(__float2half_rn(sqrtf(mh)));
    } else {
        gs_out[b] = sqrtf(mean);
    }
}

template <int DT>
__global__ __launch_bounds__(kThreads) void scale_apply_kernel(const void* __restrict__ W,
                                                                int64_t numel, const float* gs,
                                                                void* __restrict__ Ws) {
    const int64_t b = blockIdx.y;
    const float g = gs[b];
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    if (DT == CQ_F16) {
        const __half* w = reinterpret_cast<const __half*>(W) + b * numel;
        __half* o = reinterpret_cast<__half*>(Ws) + b * numel;
        for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < numel; i += stride)
            o[i] = __float2half_rn(__half2float(w[i]) / g);
    } else {
        const float* w = reinterpret_cast<const float*>(W) + b * numel;
        float* o = reinterpret_cast<float*>(Ws) + b * numel;
        for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < numel; i += stride)
            o[i] = w[i] / g;
    }
}

static int grid_for(int64_t work, int64_t batch) {
    int64_t g = ceil_div(work, kThreads * 4);
    int64_t cap = std::max<int64_t>(1, kMaxGrid / std::max<int64_t>(1, batch));
    cap = std::max<int64_t>(cap, 64);
    return (int)std::max<int64_t>(1, std::min(g, cap));
}

// ------------------------------------------------------------------ weighted square sum
template <int DT>
__global__ __launch_bounds__(kThreads) void wsq_partial_kernel(const void* __restrict__ X,
                                                                int64_t numel,
                                                                const float* __restrict__ w,
                                                                int64_t ncols, double* part, int64_t wst) {
    __shared__ double lds[16];
    const int64_t b = blockIdx.y;
    if (w) w += b * wst;  // per-matrix weights (stride 0: shared)
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < numel; i += stride) {
        const float f = DT == CQ_F16 ? __half2float(reinterpret_cast<const __half*>(X)[b * numel + i])
                                     : reinterpret_cast<const float*>(X)[b * numel + i];
        const double wf = w ? (double)w[i % ncols] : 1.0;
        acc += (double)f * (double)f * wf;
    }
    const double s = block_sum_f64(acc, lds);
    if (threadIdx.x == 0) part[b * gridDim.x + blockIdx.x] = s;
}

template <int DT>
__global__ __launch_bounds__(kThreads) void wsq_partial8_kernel(const void* __restrict__ X, int64_t numel,
                                                                 const float* __restrict__ w, int64_t ncols,
                                                                 double* part, int64_t wst) {
    __shared__ double lds[16];
    const int64_t b = blockIdx.y;
    if (w) w += b * wst;  // per-matrix weights (stride 0: shared)
    double acc0 = 0.0, acc1 = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kThreads * 8;
    for (int64_t e = ((int64_t)blockIdx.x * kThreads + threadIdx.x) * 8; e < numel; e += stride) {
        float v[8];
        load8<DT>(X, b * numel + e, v);
        float wv[8] = {1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f};
        if (w) load8<CQ_F32>(w, e % ncols, wv);   // ncols % 8 == 0: the 8 columns are contiguous
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            acc0 += (double)v[u] * (double)v[u] * (double)wv[u];
            acc1 += (double)v[u + 1] * (double)v[u + 1] * (double)wv[u + 1];
        }
    }
    const double s = block_sum_f64(acc0 + acc1, lds);
    if (threadIdx.x == 0) part[b * gridDim.x + blockIdx.x] = s;
}

// out[b] = sum_i x[b][i] y[b][i] (fp32 or fp64 inputs, fp64 accumulation), per-block partials
template <typename T>
__global__ __launch_bounds__(kThreads) void dot_partial_kernel(const T* __restrict__ X, const T* __restrict__ Y,
                                                                int64_t numel, double* part) {
    __shared__ double lds[16];
    const int64_t b = blockIdx.y;
    const T* x = X + b * numel;
    const T* y = Y + b * numel;
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < numel; i += stride)
        acc += (double)x[i] * (double)y[i];
    const double s = block_sum_f64(acc, lds);
    if (threadIdx.x == 0) part[b * gridDim.x + blockIdx.x] = s;
}

__global__ void sum_parts_kernel(const double* part, int nparts, double* out, int accumulate) {
    const int64_t b = blockIdx.x;
    if (threadIdx.x != 0) return;
    double s = 0.0;
    for (int i = 0; i < nparts; ++i) s += part[b * nparts + i];
    out[b] = accumulate ? out[b] + s : s;
}

// ------------------------------------------------------------------ uniform quantiser
// Per-block kernel (block_size <= 4096): one wave per block, two passes over the block
// (max, then quantise) — the second pass hits L1/L2.
template <int BITS>
__global__ __launch_bounds__(kThreads) void quant_block_kernel(
    const float* __restrict__ x, int64_t nblocks_total, int64_t bs, float eps,
    void* __restrict__ codes, uint8_t* __restrict__ packed, float* __restrict__ deq,
    float* __restrict__ scale) {
    constexpr float k = (float)((1 << (BITS - 1)) - 1);
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * kThreads) >> 6;
    for (int64_t blk = wave; blk < nblocks_total; blk += nwaves) {
        const float* xb = x + blk * bs;
        uint32_t mb = 0;
        for (int64_t i = lane; i < bs; i += 64) {
            const uint32_t a = abs_bits(xb[i]);
            mb = a > mb ? a : mb;
        }
        mb = wave_max_u32(mb);
        const float s = quant_scale(mb, eps);
        if (lane == 0) scale[blk] = s;
        for (int64_t i = lane; i < bs; i += 64) {
            const float c = quant_code(xb[i], s, k);
            const int64_t e = blk * bs + i;
            if (codes) {
                if (BITS <= 8) reinterpret_cast<int8_t*>(codes)[e] = (int8_t)(int)c;
                else reinterpret_cast<int16_t*>(codes)[e] = (int16_t)(int)c;
            }
            if (deq) deq[e] = dequant(c, k, s);
        }
        if constexpr (BITS <= 4) if (packed) {
            // pack after codes are known: recompute per byte group (cheap, L1-resident)
            constexpr int per = 8 / BITS;
            for (int64_t g = lane; g < bs / per; g += 64) {
                uint32_t byte = 0;
#pragma unroll
                for (int t = 0; t < per; ++t) {
                    const float c = quant_code(xb[g * per + t], s, k);
                    byte = (byte << BITS) | (uint32_t)((int)c + (int)k);
                }
                packed[(blk * bs) / per + g] = (uint8_t)byte;
            }
        }
    }
}

// Whole-matrix / large-block absmax (atomicMax on |x| bits per block id).
__global__ __launch_bounds__(kThreads) void absmax_atomic_kernel(const float* __restrict__ x,
                                                                  int64_t numel, int64_t bs,
                                                                  uint32_t* __restrict__ mx) {
    const int64_t b = blockIdx.y;
    const float* xb = x + b * numel;
    const int64_t nb = numel / bs;
    uint32_t m = 0;
    int64_t cur = -1;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < numel; i += stride) {
        const int64_t blk = i / bs;
        if (blk != cur) {
            if (cur >= 0 && m) atomicMax(&mx[b * nb + cur], m);
            cur = blk;
            m = 0;
        }
        const uint32_t a = abs_bits(xb[i]);
        m = a > m ? a : m;
    }
    if (nb == 1) {  // common whole-matrix case: one atomic per wave
        m = wave_max_u32(m);
        if ((threadIdx.x & 63) == 0 && m) atomicMax(&mx[b], m);
    } else if (cur >= 0 && m) {
        atomicMax(&mx[b * nb + cur], m);
    }
}

// Elementwise quantise with a known per-block max; 4 elements per thread when possible.
template <int BITS, bool PACK, bool ERR>
__global__ __launch_bounds__(kThreads) void quant_known_kernel(
    const float* __restrict__ x, int64_t numel, int64_t bs, float eps,
    const uint32_t* __restrict__ mx, void* __restrict__ codes, uint8_t* __restrict__ packed,
    float* __restrict__ deq, const float* __restrict__ ew, int64_t encols, double* part, int64_t ews) {
    constexpr float k = (float)((1 << (BITS - 1)) - 1);
    __shared__ double lds[16];
    const int64_t b = blockIdx.y;
    if (ew) ew += b * ews;  // per-matrix error weights (stride 0: shared)
    const int64_t nb = numel / bs;
    const float* xb = x + b * numel;
    double acc = 0.0;
    const int64_t ngroups = numel / 4;  // caller guarantees numel % 4 == 0
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    const bool single = (nb == 1);
    const float s_single = single ? quant_scale(mx[b], eps) : 0.f;
    for (int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x; g < ngroups; g += stride) {
        const float4 v = reinterpret_cast<const float4*>(xb)[g];
        const float xs[4] = {v.x, v.y, v.z, v.w};
        float cs[4], ds[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int64_t e = g * 4 + t;
            const float s = single ? s_single : quant_scale(mx[b * nb + e / bs], eps);
            cs[t] = quant_code(xs[t], s, k);
            ds[t] = dequant(cs[t], k, s);
            if (ERR) {
                const float d = ds[t] - xs[t];
                const double wv = ew ? (double)ew[e % encols] : 1.0;
                acc += (double)(d * d) * wv;
            }
        }
        const int64_t eb = b * numel + g * 4;
        if (codes) {
            if (BITS <= 8) {
                char4 c4 = make_char4((signed char)(int)cs[0], (signed char)(int)cs[1],
                                      (signed char)(int)cs[2], (signed char)(int)cs[3]);
                reinterpret_cast<char4*>(reinterpret_cast<int8_t*>(codes) + eb)[0] = c4;
            } else {
                short4 c4 = make_short4((short)(int)cs[0], (short)(int)cs[1], (short)(int)cs[2],
                                        (short)(int)cs[3]);
                reinterpret_cast<short4*>(reinterpret_cast<int16_t*>(codes) + eb)[0] = c4;
            }
        }
        if (deq) reinterpret_cast<float4*>(deq + eb)[0] = make_float4(ds[0], ds[1], ds[2], ds[3]);
        if (PACK) {
            const uint32_t q0 = (uint32_t)((int)cs[0] + (int)k), q1 = (uint32_t)((int)cs[1] + (int)k);
            const uint32_t q2 = (uint32_t)((int)cs[2] + (int)k), q3 = (uint32_t)((int)cs[3] + (int)k);
            if (BITS == 2) {
                packed[eb / 4] = (uint8_t)((q0 << 6) | (q1 << 4) | (q2 << 2) | q3);
            } else {
                reinterpret_cast<uchar2*>(packed + eb / 2)[0] =
                    make_uchar2((uint8_t)((q0 << 4) | q1), (uint8_t)((q2 << 4) | q3));
            }
        }
    }
    if (ERR) {
        const double s = block_sum_f64(acc, lds);
        if (threadIdx.x == 0) part[b * gridDim.x + blockIdx.x] = s;
    }
}

__global__ void finalize_scale_kernel(const uint32_t* mx, int64_t n, float eps, float* scale) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) scale[i] = quant_scale(mx[i], eps);
}

// ------------------------------------------------------------------ dequantise codes
// quantization.py:103-105 + :292-295: out = (float(c) / k) * scale[blk]; codes int8/int16 or
// offset-binary packed (bits 2/4).
template <int BITS, int FMT>  // FMT 0: int8, 1: int16, 2: packed
__global__ __launch_bounds__(kThreads) void dequant_kernel(const void* __restrict__ codes,
                                                           const float* __restrict__ scale,
                                                           int64_t total, int64_t bs,
                                                           float* __restrict__ out) {
    constexpr float k = (float)((1 << (BITS - 1)) - 1);
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < total; e += stride) {
        float c;
        if (FMT == 0) c = (float)reinterpret_cast<const int8_t*>(codes)[e];
        else if (FMT == 1) c = (float)reinterpret_cast<const int16_t*>(codes)[e];
        else {
            constexpr int per = 8 / BITS;
            const uint32_t byte = reinterpret_cast<const uint8_t*>(codes)[e / per];
            const int sh = BITS * (per - 1 - (int)(e % per));
            c = (float)((int)((byte >> sh) & ((1u << BITS) - 1u)) - (int)k);
        }
        out[e] = dequant(c, k, scale[e / bs]);
    }
}

// A wave per 1024-element chunk (one scale: block_size % 1024 == 0): lane l takes elements
// 256 u + 4 l .. + 3 of sub-block u = 0..3, so each of the four 16-byte stores covers 1 KB of
// consecutive outputs; the same per-element arithmetic as dequant_kernel.  Codes as int8
// bytes (FMT 0, one 4-byte load per sub-block) or packed fields (FMT 2)
template <int BITS, int FMT>
__global__ __launch_bounds__(kThreads) void dequant16_kernel(const void* __restrict__ codes,
                                                             const float* __restrict__ scale,
                                                             int64_t total, int64_t bs,
                                                             float* __restrict__ out) {
    static_assert(FMT == 0 || FMT == 2, "int8 or packed codes");
    constexpr float k = (float)((1 << (BITS - 1)) - 1);
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (kThreads / 64);
    for (int64_t ch = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); ch * 1024 < total; ch += nwaves) {
        const int64_t c0 = ch * 1024;
        const float sc = scale[c0 / bs];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t e = c0 + 256 * u + 4 * lane;
            float c[4];
            if (FMT == 0) {
                const uint32_t r = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const int8_t*>(codes) + e);
#pragma unroll
                for (int t = 0; t < 4; ++t) c[t] = (float)(int8_t)(uint8_t)(r >> (8 * t));
            } else {
                constexpr int per = 8 / BITS;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int64_t x = e + t;
                    const uint32_t byte = reinterpret_cast<const uint8_t*>(codes)[x / per];
                    const int sh = BITS * (per - 1 - (int)(x % per));
                    c[t] = (float)((int)((byte >> sh) & ((1u << BITS) - 1u)) - (int)k);
                }
            }
            *reinterpret_cast<float4*>(out + e) =
                make_float4(dequant(c[0], k, sc), dequant(c[1], k, sc), dequant(c[2], k, sc), dequant(c[3], k, sc));
        }
    }
}

// 16 codes per thread and step: 4 (2-bit) or 8 (4-bit) packed bytes in, one 16-byte store out
template <int BITS>
__global__ __launch_bounds__(256) void unpack16_kernel(const uint8_t* __restrict__ packed, int64_t ncodes,
                                                       int8_t* __restrict__ codes) {
    constexpr int per = 8 / BITS;
    constexpr int k = (1 << (BITS - 1)) - 1;
    constexpr uint32_t mask = (1u << BITS) - 1u;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x * 16;
    for (int64_t e = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; e < ncodes; e += stride) {
        uint8_t by[16 / per];
        if (BITS == 2) {
            const uint32_t r = *reinterpret_cast<const uint32_t*>(packed + e / per);
#pragma unroll
            for (int t = 0; t < 4; ++t) by[t] = (uint8_t)(r >> (8 * t));
        } else {
            const uint2 r = *reinterpret_cast<const uint2*>(packed + e / per);
#pragma unroll
            for (int t = 0; t < 8; ++t) by[t] = (uint8_t)((t < 4 ? r.x : r.y) >> (8 * (t & 3)));
        }
        uint4 o;
        uint8_t* ob = reinterpret_cast<uint8_t*>(&o);
#pragma unroll
        for (int u = 0; u < 16; ++u)
            ob[u] = (uint8_t)(int8_t)((int)((by[u / per] >> (BITS * (per - 1 - (u % per)))) & mask) - k);
        *reinterpret_cast<uint4*>(codes + e) = o;
    }
}

// ------------------------------------------------------------------ unpack
template <int BITS>
__global__ void unpack_kernel(const uint8_t* __restrict__ packed, int64_t nbytes_total,
                              int8_t* __restrict__ codes) {
    constexpr int per = 8 / BITS;
    constexpr int k = (1 << (BITS - 1)) - 1;
    constexpr uint32_t mask = (1u << BITS) - 1u;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes_total; i += stride) {
        const uint32_t byte = packed[i];
#pragma unroll
        for (int t = 0; t < per; ++t)
            codes[i * per + t] = (int8_t)((int)((byte >> (BITS * (per - 1 - t))) & mask) - k);
    }
}

// ------------------------------------------------------------------ residual builder
template <int DT, int BITS>
__global__ __launch_bounds__(kThreads) void build_residual_kernel(
    const void* __restrict__ Ws, const uint8_t* __restrict__ qc, const float* __restrict__ qscale,
    const float* __restrict__ ycol, int64_t m, int64_t n, float* __restrict__ Y,
    float* __restrict__ res, int64_t ycs) {
    constexpr float k = BITS == 32 ? 1.f : (float)((1 << (BITS - 1)) - 1);
    const int64_t b = blockIdx.y;
    if (ycol) ycol += b * ycs;  // per-matrix column weights (stride 0: shared)
    const int64_t numel = m * n;
    const float s = (qc && qscale) ? qscale[b] : 0.f;
    const int64_t ngroups = numel / 4;  // n % 4 == 0 guaranteed by caller
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x; g < ngroups; g += stride) {
        const int64_t e = g * 4;
        float w[4];
        if (DT == CQ_F16) {
            const ushort4 h = reinterpret_cast<const ushort4*>(reinterpret_cast<const __half*>(Ws) + b * numel)[g];
            w[0] = __half2float(__ushort_as_half(h.x));
            w[1] = __half2float(__ushort_as_half(h.y));
            w[2] = __half2float(__ushort_as_half(h.z));
            w[3] = __half2float(__ushort_as_half(h.w));
        } else {
            const float4 f = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(Ws) + b * numel)[g];
            w[0] = f.x; w[1] = f.y; w[2] = f.z; w[3] = f.w;
        }
        float q[4] = {0.f, 0.f, 0.f, 0.f};
        if (qc) {
            if (BITS == 2) {
                const uint32_t byte = qc[b * (numel / 4) + g];
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    q[t] = dequant((float)((int)((byte >> (6 - 2 * t)) & 3u) - 1), k, s);
            } else if (BITS == 4) {
                const uchar2 by = reinterpret_cast<const uchar2*>(qc + b * (numel / 2))[g];
                const uint32_t v0 = by.x, v1 = by.y;
                q[0] = dequant((float)((int)(v0 >> 4) - 7), k, s);
                q[1] = dequant((float)((int)(v0 & 15u) - 7), k, s);
                q[2] = dequant((float)((int)(v1 >> 4) - 7), k, s);
                q[3] = dequant((float)((int)(v1 & 15u) - 7), k, s);
            } else if (BITS == 32) {  // dense fp32 Q (codebook methods)
                const float4 f = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(qc) + b * numel)[g];
                q[0] = f.x; q[1] = f.y; q[2] = f.z; q[3] = f.w;
            } else if (BITS == 8) {
                const char4 c = reinterpret_cast<const char4*>(qc + b * numel)[g];
                q[0] = dequant((float)c.x, k, s); q[1] = dequant((float)c.y, k, s);
                q[2] = dequant((float)c.z, k, s); q[3] = dequant((float)c.w, k, s);
            } else {
                const short4 c = reinterpret_cast<const short4*>(reinterpret_cast<const int16_t*>(qc) + b * numel)[g];
                q[0] = dequant((float)c.x, k, s); q[1] = dequant((float)c.y, k, s);
                q[2] = dequant((float)c.z, k, s); q[3] = dequant((float)c.w, k, s);
            }
        }
        float r[4], y[4];
        const int64_t j0 = e % n;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            r[t] = w[t] - q[t];
            y[t] = ycol ? r[t] * ycol[j0 + t] : r[t];
        }
        if (res) reinterpret_cast<float4*>(res + b * numel)[g] = make_float4(r[0], r[1], r[2], r[3]);
        if (Y) reinterpret_cast<float4*>(Y + b * numel)[g] = make_float4(y[0], y[1], y[2], y[3]);
    }
}

// ------------------------------------------------------------------ row/col scaling
__global__ __launch_bounds__(kThreads) void scale_rc_kernel(
    const float* __restrict__ X, int64_t ldx, int64_t sx, int tx, float* __restrict__ Y, int64_t ldy,
    int64_t sy, int64_t rows, int64_t cols, const float* __restrict__ rs, int64_t rss,
    const float* __restrict__ cs, int64_t css) {
    const int64_t b = blockIdx.z;
    const int64_t total = rows * cols;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t e = (int64_t)blockIdx.x * kThreads + threadIdx.x; e < total; e += stride) {
        const int64_t i = e / cols, j = e % cols;
        float v = tx ? X[b * sx + j * ldx + i] : X[b * sx + i * ldx + j];
        if (rs) v *= rs[b * rss + i];
        if (cs) v *= cs[b * css + j];
        Y[b * sy + i * ldy + j] = v;
    }
}

}  // namespace cq

namespace cq {

template <int BITS>
static void launch_known(bool pack, bool err, dim3 grid, hipStream_t s, const float* x,
                         int64_t numel, int64_t bs, float eps, const uint32_t* mx, void* codes,
                         uint8_t* packed, float* deq, const float* ew, int64_t encols,
                         double* part, int64_t ews) {
#define CQ_LK(P, E) quant_known_kernel<BITS, P, E><<<grid, kThreads, 0, s>>>(x, numel, bs, eps, mx, codes, packed, deq, ew, encols, part, ews)
    if (pack && err) CQ_LK(true, true);
    else if (pack) CQ_LK(true, false);
    else if (err) CQ_LK(false, true);
    else CQ_LK(false, false);
#undef CQ_LK
}

static int quant_known_dispatch(const float* x, int64_t batch, int64_t numel, int64_t bs,
                                int bits, float eps, const uint32_t* mx, void* codes,
                                uint8_t* packed, float* deq, float* scale, const float* ew,
                                int64_t encols, int64_t ews, double* err_out, double* part, hipStream_t s) {
    const int g = grid_for(numel, batch);
    dim3 grid(g, batch);
    const bool err = ew != nullptr || err_out != nullptr;
    const bool pack = packed != nullptr && bits <= 4;
    switch (bits) {
        case 2: launch_known<2>(pack, err, grid, s, x, numel, bs, eps, mx, codes, packed, deq, ew, encols, part, ews); break;
        case 4: launch_known<4>(pack, err, grid, s, x, numel, bs, eps, mx, codes, packed, deq, ew, encols, part, ews); break;
        case 8: launch_known<8>(false, err, grid, s, x, numel, bs, eps, mx, codes, nullptr, deq, ew, encols, part, ews); break;
        default: launch_known<16>(false, err, grid, s, x, numel, bs, eps, mx, codes, nullptr, deq, ew, encols, part, ews); break;
    }
    const int64_t nsc = batch * (numel / bs);
    if (scale) finalize_scale_kernel<<<(int)ceil_div(nsc, 256), 256, 0, s>>>(mx, nsc, eps, scale);
    if (err) sum_parts_kernel<<<batch, 64, 0, s>>>(part, g, err_out, 0);
    return check_launch("cq_quantize_uniform");
}

}  // namespace cq

using namespace cq;

extern "C" {

int cq_abi_version(void) { return CQ_ABI_VERSION; }
const char* cq_last_error(void) { return g_err; }

size_t cq_rms_scale_workspace(int64_t batch, int64_t numel) {
    return (size_t)batch * grid_for(numel, batch) * sizeof(double);
}

int cq_rms_scale(int dtype, const void* W, int64_t batch, int64_t numel, int do_scale,
                 float* gs_out, void* Ws_out, void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(W && gs_out && Ws_out && batch > 0 && numel > 0, "cq_rms_scale: bad args");
    CQ_REQUIRE(dtype == CQ_F16 || dtype == CQ_F32, "cq_rms_scale: dtype must be f16/f32");
    const int g = grid_for(numel, batch);
    if (ws_bytes < (size_t)batch * g * sizeof(double) || !ws)
        return set_error(CQ_EWORKSPACE, "cq_rms_scale: workspace too small");
    hipStream_t s = as_stream(stream);
    double* part = reinterpret_cast<double*>(ws);
    dim3 grid(g, batch);
    // 16-byte loads where every matrix starts 16-byte aligned (the scaling pass stays scalar:
    // a vector form measured no faster)
    const bool v8 = numel % 8 == 0 && (reinterpret_cast<uintptr_t>(W) & 15) == 0;
    if (dtype == CQ_F16) {
        if (v8) rms_partial8_kernel<CQ_F16><<<grid, kThreads, 0, s>>>(W, numel, part);
        else rms_partial_kernel<CQ_F16><<<grid, kThreads, 0, s>>>(W, numel, part);
        rms_finalize_kernel<CQ_F16><<<batch, 64, 0, s>>>(part, g, numel, do_scale, gs_out);
        scale_apply_kernel<CQ_F16><<<grid, kThreads, 0, s>>>(W, numel, gs_out, Ws_out);
    } else {
        if (v8) rms_partial8_kernel<CQ_F32><<<grid, kThreads, 0, s>>>(W, numel, part);
        else rms_partial_kernel<CQ_F32><<<grid, kThreads, 0, s>>>(W, numel, part);
        rms_finalize_kernel<CQ_F32><<<batch, 64, 0, s>>>(part, g, numel, do_scale, gs_out);
        scale_apply_kernel<CQ_F32><<<grid, kThreads, 0, s>>>(W, numel, gs_out, Ws_out);
    }
    return check_launch("cq_rms_scale");
}

int cq_weighted_sqsum(int dtype, const void* x, int64_t batch, int64_t numel, const float* w,
                      int64_t ncols, int64_t w_stride, double* out, void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(x && out && batch > 0 && numel > 0, "cq_weighted_sqsum: bad args");
    CQ_REQUIRE(!w || ncols > 0, "cq_weighted_sqsum: ncols");
    const int g = grid_for(numel, batch);
    if (ws_bytes < (size_t)batch * g * sizeof(double) || !ws)
        return set_error(CQ_EWORKSPACE, "cq_weighted_sqsum: workspace too small");
    hipStream_t s = as_stream(stream);
    double* part = reinterpret_cast<double*>(ws);
    dim3 grid(g, batch);
    const bool v8 = numel % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                    (!w || (ncols % 8 == 0 && w_stride % 4 == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0));
    if (v8) {
        if (dtype == CQ_F16) wsq_partial8_kernel<CQ_F16><<<grid, kThreads, 0, s>>>(x, numel, w, ncols, part, w_stride);
        else wsq_partial8_kernel<CQ_F32><<<grid, kThreads, 0, s>>>(x, numel, w, ncols, part, w_stride);
    } else if (dtype == CQ_F16) {
        wsq_partial_kernel<CQ_F16><<<grid, kThreads, 0, s>>>(x, numel, w, ncols, part, w_stride);
    } else {
        wsq_partial_kernel<CQ_F32><<<grid, kThreads, 0, s>>>(x, numel, w, ncols, part, w_stride);
    }
    sum_parts_kernel<<<batch, 64, 0, s>>>(part, g, out, 0);
    return check_launch("cq_weighted_sqsum");
}

int cq_batched_dot(int dtype, const void* x, const void* y, int64_t batch, int64_t numel, double* out, void* ws,
                   size_t ws_bytes, void* stream) {
    CQ_REQUIRE(x && y && out && batch > 0 && numel > 0, "cq_batched_dot: bad args");
    CQ_REQUIRE(dtype == CQ_F32 || dtype == CQ_F64, "cq_batched_dot: dtype must be CQ_F32 or CQ_F64");
    const int g = grid_for(numel, batch);
    if (ws_bytes < (size_t)batch * g * sizeof(double) || !ws)
        return set_error(CQ_EWORKSPACE, "cq_batched_dot: workspace too small");
    hipStream_t s = as_stream(stream);
    double* part = reinterpret_cast<double*>(ws);
    dim3 grid(g, batch);
    if (dtype == CQ_F64)
        dot_partial_kernel<double><<<grid, kThreads, 0, s>>>(reinterpret_cast<const double*>(x),
                                                             reinterpret_cast<const double*>(y), numel, part);
    else
        dot_partial_kernel<float><<<grid, kThreads, 0, s>>>(reinterpret_cast<const float*>(x),
                                                            reinterpret_cast<const float*>(y), numel, part);
    sum_parts_kernel<<<batch, 64, 0, s>>>(part, g, out, 0);
    return check_launch("cq_batched_dot");
}

size_t cq_quantize_workspace(int64_t batch, int64_t numel, int64_t block_size) {
    const int64_t nb = block_size > 0 ? numel / block_size : 1;
    return align_up((size_t)batch * nb * sizeof(uint32_t), 256) +
           (size_t)batch * grid_for(numel, batch) * sizeof(double);
}

int cq_quantize_uniform(const float* x, int64_t batch, int64_t numel, int64_t block_size,
                        int bits, float eps, void* codes, uint8_t* packed, float* deq,
                        float* scale, const float* err_w, int64_t err_ncols, int64_t err_w_stride,
                        double* err_out, void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(x && scale && batch > 0 && numel > 0 && block_size > 0, "cq_quantize_uniform: bad args");
    CQ_REQUIRE(bits == 2 || bits == 4 || bits == 8 || bits == 16, "Bit-width not supported!");
    CQ_REQUIRE(numel % block_size == 0, "cq_quantize_uniform: numel %% block_size != 0");
    CQ_REQUIRE(!packed || bits > 4 || (numel % 4 == 0 && block_size % 4 == 0),
               "cq_quantize_uniform: packing needs numel, block_size multiples of 4");
    CQ_REQUIRE(!err_w || err_ncols > 0, "cq_quantize_uniform: err_ncols");
    hipStream_t s = as_stream(stream);
    const bool err = err_out != nullptr;
    const bool small_blocks = block_size <= 4096 && !err;
    if (small_blocks) {
        const int64_t nbt = batch * (numel / block_size);
        const int g = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(nbt, kThreads / 64), 4096));
        switch (bits) {
#define CQ_QB(B) quant_block_kernel<B><<<g, kThreads, 0, s>>>(x, nbt, block_size, eps, codes, packed, deq, scale)
            case 2: CQ_QB(2); break;
            case 4: CQ_QB(4); break;
            case 8: CQ_QB(8); break;
            default: CQ_QB(16); break;
#undef CQ_QB
        }
        return check_launch("cq_quantize_uniform(block)");
    }
    CQ_REQUIRE(numel % 4 == 0 && block_size % 4 == 0,
               "cq_quantize_uniform: large-block path needs numel, block_size multiples of 4");
    if (ws_bytes < cq_quantize_workspace(batch, numel, block_size) || !ws)
        return set_error(CQ_EWORKSPACE, "cq_quantize_uniform: workspace too small");
    const int64_t nb = numel / block_size;
    uint32_t* mx = reinterpret_cast<uint32_t*>(ws);
    double* part = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) +
                                             align_up((size_t)batch * nb * sizeof(uint32_t), 256));
    if (hipMemsetAsync(mx, 0, (size_t)batch * nb * sizeof(uint32_t), s) != hipSuccess)
        return set_error(CQ_EHIP, "cq_quantize_uniform: memset failed");
    absmax_atomic_kernel<<<dim3(grid_for(numel, batch), batch), kThreads, 0, s>>>(x, numel, block_size, mx);
    return quant_known_dispatch(x, batch, numel, block_size, bits, eps, mx, codes, packed, deq,
                                scale, err_w, err_ncols, err_w_stride, err_out, part, s);
}

int cq_quantize_uniform_known_max(const float* x, int64_t batch, int64_t numel, int bits,
                                  float eps, const uint32_t* absmax_bits, void* codes,
                                  uint8_t* packed, float* deq, float* scale,
                                  const float* err_w, int64_t err_ncols, int64_t err_w_stride,
                                  double* err_out, void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(x && absmax_bits && batch > 0 && numel > 0, "cq_quantize_uniform_known_max: bad args");
    CQ_REQUIRE(bits == 2 || bits == 4 || bits == 8 || bits == 16, "Bit-width not supported!");
    CQ_REQUIRE(numel % 4 == 0, "cq_quantize_uniform_known_max: numel %% 4 != 0");
    const bool err = err_out != nullptr;
    if (err && (ws_bytes < (size_t)batch * grid_for(numel, batch) * sizeof(double) || !ws))
        return set_error(CQ_EWORKSPACE, "cq_quantize_uniform_known_max: workspace too small");
    return quant_known_dispatch(x, batch, numel, numel, bits, eps, absmax_bits, codes, packed,
                                deq, scale, err_w, err_ncols, err_w_stride, err_out,
                                reinterpret_cast<double*>(ws), as_stream(stream));
}

int cq_dequant_uniform(const void* codes, int packed, const float* scale, int64_t total,
                       int64_t block_size, int bits, float* out, void* stream) {
    CQ_REQUIRE(codes && scale && out && total > 0 && block_size > 0, "cq_dequant_uniform: bad args");
    CQ_REQUIRE(bits == 2 || bits == 4 || bits == 8 || bits == 16, "Bit-width not supported!");
    CQ_REQUIRE(!packed || bits <= 4, "cq_dequant_uniform: packed needs bits 2/4");
    const int g = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, kThreads), kMaxGrid));
    hipStream_t s = as_stream(stream);
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool v16 = total % 1024 == 0 && block_size % 1024 == 0 && al16(out) && bits <= 8 &&
                     (packed || (reinterpret_cast<uintptr_t>(codes) & 3) == 0);
    if (v16) {
        const int g16 = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, 1024 * (kThreads / 64)), kMaxGrid));
#define CQ_DQ16(B, F) dequant16_kernel<B, F><<<g16, kThreads, 0, s>>>(codes, scale, total, block_size, out)
        if (packed) { if (bits == 2) CQ_DQ16(2, 2); else CQ_DQ16(4, 2); }
        else if (bits == 8) CQ_DQ16(8, 0);
        else if (bits == 4) CQ_DQ16(4, 0);
        else CQ_DQ16(2, 0);
#undef CQ_DQ16
        return check_launch("cq_dequant_uniform");
    }
#define CQ_DQ(B, F) dequant_kernel<B, F><<<g, kThreads, 0, s>>>(codes, scale, total, block_size, out)
    if (packed) { if (bits == 2) CQ_DQ(2, 2); else CQ_DQ(4, 2); }
    else if (bits == 16) CQ_DQ(16, 1);
    else if (bits == 8) CQ_DQ(8, 0);
    else if (bits == 4) CQ_DQ(4, 0);
    else CQ_DQ(2, 0);
#undef CQ_DQ
    return check_launch("cq_dequant_uniform");
}

int cq_unpack_codes(const uint8_t* packed, int64_t batch, int64_t numel, int bits, int8_t* codes,
                    void* stream) {
    CQ_REQUIRE(packed && codes && (bits == 2 || bits == 4) && numel % 4 == 0, "cq_unpack_codes: bad args");
    const int64_t nbytes = batch * numel * bits / 8;
    const int g = (int)std::min<int64_t>(ceil_div(nbytes, 256), kMaxGrid);
    hipStream_t s = as_stream(stream);
    const int64_t ncodes = batch * numel;
    if (ncodes % 16 == 0 && (reinterpret_cast<uintptr_t>(codes) & 15) == 0 &&
        (reinterpret_cast<uintptr_t>(packed) & (bits == 2 ? 3 : 7)) == 0) {
        const int g16 = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(ncodes, 16 * 256), kMaxGrid));
        if (bits == 2) unpack16_kernel<2><<<g16, 256, 0, s>>>(packed, ncodes, codes);
        else unpack16_kernel<4><<<g16, 256, 0, s>>>(packed, ncodes, codes);
        return check_launch("cq_unpack_codes");
    }
    if (bits == 2) unpack_kernel<2><<<g, 256, 0, s>>>(packed, nbytes, codes);
    else unpack_kernel<4><<<g, 256, 0, s>>>(packed, nbytes, codes);
    return check_launch("cq_unpack_codes");
}

int cq_build_residual(int dtype, const void* Ws, const uint8_t* packed, const float* scale,
                      int bits, const float* ycol, int64_t ycol_stride, int64_t batch, int64_t m, int64_t n,
                      float* Y, float* res_out, void* stream) {
    CQ_REQUIRE(Ws && batch > 0 && m > 0 && n > 0 && (Y || res_out), "cq_build_residual: bad args");
    CQ_REQUIRE(n % 4 == 0, "cq_build_residual: n %% 4 != 0");
    CQ_REQUIRE(!packed || scale || bits == 32, "cq_build_residual: scale required with codes");
    CQ_REQUIRE(!packed || bits == 2 || bits == 4 || bits == 8 || bits == 16 || bits == 32, "Bit-width not supported!");
    const int g = grid_for(m * n, batch);
    dim3 grid(g, batch);
    hipStream_t s = as_stream(stream);
#define CQ_BR(DT, B) build_residual_kernel<DT, B><<<grid, kThreads, 0, s>>>(Ws, packed, scale, ycol, m, n, Y, res_out, ycol_stride)
    const int bsel = packed ? bits : 2;
    if (dtype == CQ_F16) {
        switch (bsel) { case 2: CQ_BR(CQ_F16, 2); break; case 4: CQ_BR(CQ_F16, 4); break;
                        case 8: CQ_BR(CQ_F16, 8); break; case 32: CQ_BR(CQ_F16, 32); break; default: CQ_BR(CQ_F16, 16); }
    } else {
        switch (bsel) { case 2: CQ_BR(CQ_F32, 2); break; case 4: CQ_BR(CQ_F32, 4); break;
                        case 8: CQ_BR(CQ_F32, 8); break; case 32: CQ_BR(CQ_F32, 32); break; default: CQ_BR(CQ_F32, 16); }
    }
#undef CQ_BR
    return check_launch("cq_build_residual");
}

int cq_scale_rc(const float* X, int64_t ldx, int64_t stride_x, int trans_x, float* Y, int64_t ldy,
                int64_t stride_y, int64_t rows, int64_t cols, int64_t batch, const float* rowscale,
                int64_t rowscale_stride, const float* colscale, int64_t colscale_stride,
                void* stream) {
    CQ_REQUIRE(X && Y && rows > 0 && cols > 0 && batch > 0, "cq_scale_rc: bad args");
    const int g = grid_for(rows * cols, batch);
    scale_rc_kernel<<<dim3(g, 1, batch), kThreads, 0, as_stream(stream)>>>(
        X, ldx, stride_x, trans_x, Y, ldy, stride_y, rows, cols, rowscale, rowscale_stride, colscale,
        colscale_stride);
    return check_launch("cq_scale_rc");
}

}  // extern "C"
