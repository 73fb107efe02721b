// Codebook / affine quantisers of the reference on gfx950 (quantization.py methods other
// than "uniform"):
//   * NF4 / NF2  — absmax scale, index = number of level midpoints below x / scale
//                  (quantization.py:39-91 levels/thresholds/_quantize_nf/_dequantize_nf,
//                  dispatch :270-279 and :296-298);
//   * bbint4 / bbint2 — per block: mean, unbiased std, |x - mean| > 6 std outliers replaced
//                  by the mean and kept aside, min/max affine codes packed MSB-first
//                  (quantization.py:107-243, dispatch :280-283 and :299-302).
//
// Both are HBM-bound streaming kernels.  Numerics follow the reference op by op (this file
// is built with -ffp-contract=off and IEEE division): x / scale in fp32, the thresholds
// (l_i + l_{i+1}) / 2 in fp32, bbint's (x - min) / scale, rint (half-even) and the two
// roundings of the dequant u * scale + min.  bbint's mean is the reference's fp32 mean: for
// blocks of <= 256 elements in torch's CPU reduction order (4 interleaved 8-lane fp32
// accumulators, as oracle/caldera_oracle.py:torch_row_sum_f32 restates), for longer blocks
// the fp64 sum rounded to fp32 (torch's multi-threaded cascade order is not reproducible);
// the std is the fp64 two-pass value rounded to fp32.
//
// bbint geometry: a block is split into chunks of <= 4096 elements, one 256-thread
// workgroup per chunk; all reductions are per-chunk partials combined in a fixed order, so
// every output (including the order of the outlier list, torch.nonzero's row-major order)
// is deterministic.  The outlier list is compacted with an exclusive scan over the chunk
// counts of ALL matrices in the batch: matrix b's outliers follow matrix b-1's.
#include "cq_common.h"

namespace cq {

constexpr int kCbThreads = 256;
constexpr int64_t kChunk = 4096;  // bbint chunk: 256 threads x 16 elements

__device__ __forceinline__ float nanmax_f(float a, float b) {  // torch.maximum: NaN propagates
    return (a != a) ? a : ((b != b) ? b : fmaxf(a, b));
}

// NF levels (quantization.py:45-57), exactly the fp32 roundings torch.tensor(..., float32)
// makes of the decimal literals.
__constant__ float kNF4[16] = {-1.334f, -1.0f, -0.784f, -0.617f, -0.476f, -0.347f, -0.226f, -0.112f,
                               0.0f,    0.112f, 0.226f, 0.347f,  0.476f,  0.617f,  0.784f,  1.0f};
__constant__ float kNF2[4] = {-0.8165f, -0.3333f, 0.3333f, 0.8165f};

template <int BITS>
__device__ __forceinline__ float nf_level(int i) { return BITS == 4 ? kNF4[i] : kNF2[i]; }

// index = sum_t (x/s > thr_t), thr_t = (l_t + l_{t+1}) / 2 in fp32 (quantization.py:61,80-83)
template <int BITS>
__device__ __forceinline__ int nf_index(float ws) {
    constexpr int NL = 1 << BITS;
    int idx = 0;
#pragma unroll
    for (int t = 0; t < NL - 1; ++t) {
        const float thr = (nf_level<BITS>(t) + nf_level<BITS>(t + 1)) / 2.0f;
        idx += (ws > thr) ? 1 : 0;
    }
    return idx;
}

// ------------------------------------------------------------------ NF, small blocks
// One wave per block: absmax, then index / dequant / error in a second pass (L1/L2 hits).
template <int BITS>
__global__ __launch_bounds__(kCbThreads) void nf_block_kernel(
    const float* __restrict__ x, int64_t nbt, int64_t bs, int64_t nblk_per, float eps,
    uint8_t* __restrict__ idx, float* __restrict__ deq, float* __restrict__ scale,
    const float* __restrict__ ew, int64_t encols, double* __restrict__ perr, int64_t ews) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * kCbThreads + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * kCbThreads) >> 6;
    for (int64_t blk = wave; blk < nbt; blk += nwaves) {
        const float* xb = x + blk * bs;
        uint32_t mb = 0;
        for (int64_t i = lane; i < bs; i += 64) {
            const uint32_t a = abs_bits(xb[i]);
            mb = a > mb ? a : mb;
        }
        mb = wave_max_u32(mb);
        const float s = quant_scale(mb, eps);  // max(absmax, eps), NaN-propagating
        if (lane == 0) scale[blk] = s;
        double acc = 0.0;
        const int64_t e_in_mat0 = (blk % nblk_per) * bs;
        for (int64_t i = lane; i < bs; i += 64) {
            const float xv = xb[i];
            const int q = nf_index<BITS>(xv / s);
            const float d = nf_level<BITS>(q) * s;
            if (idx) idx[blk * bs + i] = (uint8_t)q;
            if (deq) deq[blk * bs + i] = d;
            if (perr) {
                const float df = d - xv;
                acc += (double)(df * df) * (ew ? (double)ew[(blk / nblk_per) * ews + (e_in_mat0 + i) % encols] : 1.0);
            }
        }
        if (perr) {
            acc = wave_sum(acc);
            if (lane == 0) perr[blk] = acc;
        }
    }
}

// ------------------------------------------------------------------ NF, large blocks
__global__ __launch_bounds__(kCbThreads) void cb_absmax_kernel(const float* __restrict__ x, int64_t numel,
                                                               int64_t bs, uint32_t* __restrict__ mx) {
    const int64_t b = blockIdx.y;
    const float* xb = x + b * numel;
    const int64_t nb = numel / bs;
    uint32_t m = 0;
    int64_t cur = -1;
    const int64_t stride = (int64_t)gridDim.x * kCbThreads;
    for (int64_t i = (int64_t)blockIdx.x * kCbThreads + threadIdx.x; i < numel; i += stride) {
        const int64_t blk = i / bs;
        if (blk != cur) {
            if (cur >= 0 && m) atomicMax(&mx[b * nb + cur], m);
            cur = blk;
            m = 0;
        }
        const uint32_t a = abs_bits(xb[i]);
        m = a > m ? a : m;
    }
    if (cur >= 0 && m) atomicMax(&mx[b * nb + cur], m);
}

template <int BITS>
__global__ __launch_bounds__(kCbThreads) void nf_known_kernel(
    const float* __restrict__ x, int64_t numel, int64_t bs, float eps, const uint32_t* __restrict__ mx,
    uint8_t* __restrict__ idx, float* __restrict__ deq, float* __restrict__ scale,
    const float* __restrict__ ew, int64_t encols, double* __restrict__ part, int64_t ews) {
    __shared__ double lds[16];
    const int64_t b = blockIdx.y;
    if (ew) ew += b * ews;  // per-matrix error weights (stride 0: shared)
    const int64_t nb = numel / bs;
    const float* xb = x + b * numel;
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kCbThreads;
    for (int64_t e = (int64_t)blockIdx.x * kCbThreads + threadIdx.x; e < numel; e += stride) {
        const float s = quant_scale(mx[b * nb + e / bs], eps);
        if (e % bs == 0 && scale) scale[b * nb + e / bs] = s;
        const float xv = xb[e];
        const int q = nf_index<BITS>(xv / s);
        const float d = nf_level<BITS>(q) * s;
        if (idx) idx[b * numel + e] = (uint8_t)q;
        if (deq) deq[b * numel + e] = d;
        if (part) {
            const float df = d - xv;
            acc += (double)(df * df) * (ew ? (double)ew[e % encols] : 1.0);
        }
    }
    if (part) {
        const double s = block_sum_f64(acc, lds);
        if (threadIdx.x == 0) part[b * gridDim.x + blockIdx.x] = s;
    }
}

// per-matrix sum of per-unit partials in a fixed order: out[b] = sum_t part[b * n + t]
__global__ void cb_sum_parts_kernel(const double* __restrict__ part, int64_t n, double* __restrict__ out) {
    const int64_t b = blockIdx.x;
    double s = 0.0;
    for (int64_t t = threadIdx.x; t < n; t += 64) s += part[b * n + t];
    s = wave_sum(s);
    if (threadIdx.x == 0) out[b] = s;
}

template <int BITS>
__global__ void nf_dequant_kernel(const uint8_t* __restrict__ idx, const float* __restrict__ scale, int64_t total,
                                  int64_t bs, float* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride)
        out[e] = nf_level<BITS>(idx[e] & ((1 << BITS) - 1)) * scale[e / bs];
}

// ------------------------------------------------------------------ bbint
// Chunk c of block blk covers elements [c*kChunk, min(bs, (c+1)*kChunk)) of the block; the
// chunk id is blk * nch + c with blk the global block (matrix-major) index.
struct BBGeom {
    int64_t bs, nch, nbt, nblk_per;
    __device__ __forceinline__ int64_t len(int64_t c) const {
        const int64_t lo = c * kChunk;
        return (bs - lo) < kChunk ? (bs - lo) : kChunk;
    }
};

// fp32 sum in torch's CPU order for short rows (oracle/caldera_oracle.py:torch_row_sum_f32)
__device__ float torch_order_sum(const float* v, int64_t n, float* sacc /* 32 */) {
    const int64_t nfull = (n / 32) * 32;
    const int t = threadIdx.x;
    if (t < 32) {
        float a = 0.f;
        for (int64_t j = 0; j < nfull; j += 32) a = a + v[j + t];
        sacc[t] = a;
    }
    __syncthreads();
    float s = 0.f;
    if (t == 0) {
        float acc[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) acc[l] = sacc[l];
        for (int k = 1; k < 4; ++k)
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[l] = acc[l] + sacc[8 * k + l];
        const int64_t rest = n - nfull;
        int64_t j = 0;
        for (; j + 8 <= rest; j += 8)
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[l] = acc[l] + v[nfull + j + l];
#pragma unroll
        for (int l = 0; l < 8; ++l) s = s + acc[l];
        for (; j < rest; ++j) s = s + v[nfull + j];
    }
    return s;
}

// pass 1: per-chunk fp64 sum (+ torch-order fp32 sum of a one-chunk block of <= 256)
__global__ __launch_bounds__(kCbThreads) void bb_sum_kernel(const float* __restrict__ x, BBGeom g,
                                                            double* __restrict__ psum, float* __restrict__ tsum) {
    __shared__ double lds[16];
    __shared__ float sacc[32];
    const int64_t ch = blockIdx.x;
    const int64_t blk = ch / g.nch, c = ch % g.nch;
    const float* xc = x + blk * g.bs + c * kChunk;
    const int64_t n = g.len(c);
    double acc = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += kCbThreads) acc += (double)xc[i];
    const double s = block_sum_f64(acc, lds);
    if (threadIdx.x == 0) psum[ch] = s;
    if (g.bs <= 256) {  // block == chunk
        const float ts = torch_order_sum(xc, n, sacc);
        if (threadIdx.x == 0) tsum[blk] = ts;
    }
}

// per block: mean64 (for the variance) and the reference's fp32 mean
__global__ void bb_mean_kernel(BBGeom g, const double* __restrict__ psum, const float* __restrict__ tsum,
                               double* __restrict__ mean64, float* __restrict__ mean32) {
    const int64_t blk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (blk >= g.nbt) return;
    double s = 0.0;
    for (int64_t c = 0; c < g.nch; ++c) s += psum[blk * g.nch + c];
    const double m = s / (double)g.bs;
    mean64[blk] = m;
    mean32[blk] = g.bs <= 256 ? tsum[blk] / (float)g.bs : (float)m;  // weight_blocks.mean(dim=1)
}

// pass 2: per-chunk sum of (x - mean64)^2
__global__ __launch_bounds__(kCbThreads) void bb_var_kernel(const float* __restrict__ x, BBGeom g,
                                                            const double* __restrict__ mean64,
                                                            double* __restrict__ psq) {
    __shared__ double lds[16];
    const int64_t ch = blockIdx.x;
    const int64_t blk = ch / g.nch, c = ch % g.nch;
    const float* xc = x + blk * g.bs + c * kChunk;
    const int64_t n = g.len(c);
    const double m = mean64[blk];
    double acc = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += kCbThreads) {
        const double d = (double)xc[i] - m;
        acc += d * d;
    }
    const double s = block_sum_f64(acc, lds);
    if (threadIdx.x == 0) psq[ch] = s;
}

// per block: std = max(std_unbiased, eps) (quantization.py:113-114), thr = 6 * std in fp32
__global__ void bb_thr_kernel(BBGeom g, float eps, const double* __restrict__ psq, float* __restrict__ thr) {
    const int64_t blk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (blk >= g.nbt) return;
    double s = 0.0;
    for (int64_t c = 0; c < g.nch; ++c) s += psq[blk * g.nch + c];
    const float sd = g.bs > 1 ? (float)sqrt(s / (double)(g.bs - 1)) : __int_as_float(0x7fc00000);
    thr[blk] = 6.0f * nanmax_f(sd, eps);
}

__device__ __forceinline__ bool bb_outlier(float xv, float mean, float thr) { return fabsf(xv - mean) > thr; }

// pass 3: per-chunk outlier count and min / max of the outlier-replaced values
__global__ __launch_bounds__(kCbThreads) void bb_mask_kernel(const float* __restrict__ x, BBGeom g,
                                                             const float* __restrict__ mean32,
                                                             const float* __restrict__ thr,
                                                             int64_t* __restrict__ pcnt, float* __restrict__ pmin,
                                                             float* __restrict__ pmax) {
    __shared__ float smn[4], smx[4];
    __shared__ int scnt[4];
    const int64_t ch = blockIdx.x;
    const int64_t blk = ch / g.nch, c = ch % g.nch;
    const float* xc = x + blk * g.bs + c * kChunk;
    const int64_t n = g.len(c);
    const float mu = mean32[blk], th = thr[blk];
    float mn = __int_as_float(0x7f800000), mx = -__int_as_float(0x7f800000);
    int cnt = 0;
    for (int64_t i = threadIdx.x; i < n; i += kCbThreads) {
        const float xv = xc[i];
        const bool o = bb_outlier(xv, mu, th);
        const float v = o ? mu : xv;
        cnt += o;
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, off, 64));
        mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        cnt += __shfl_xor(cnt, off, 64);
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { smn[w] = mn; smx[w] = mx; scnt[w] = cnt; }
    __syncthreads();
    if (threadIdx.x == 0) {
        float a = smn[0], z = smx[0];
        int64_t k = scnt[0];
        for (int i = 1; i < kCbThreads / 64; ++i) {
            a = fminf(a, smn[i]);
            z = fmaxf(z, smx[i]);
            k += scnt[i];
        }
        pcnt[ch] = k;
        pmin[ch] = a;
        pmax[ch] = z;
    }
}

// per block: min, max -> scale = max((max - min) / levels, eps)  (quantization.py:139-142)
__global__ void bb_scale_kernel(BBGeom g, float eps, float levels, const float* __restrict__ pmin,
                                const float* __restrict__ pmax, float* __restrict__ bmin, float* __restrict__ bscale) {
    const int64_t blk = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (blk >= g.nbt) return;
    float mn = pmin[blk * g.nch], mx = pmax[blk * g.nch];
    for (int64_t c = 1; c < g.nch; ++c) {
        mn = fminf(mn, pmin[blk * g.nch + c]);
        mx = fmaxf(mx, pmax[blk * g.nch + c]);
    }
    bmin[blk] = mn;
    bscale[blk] = nanmax_f((mx - mn) / levels, eps);
}

// exclusive scan of the chunk outlier counts over the whole batch (one workgroup), and the
// per-matrix totals (n_out[b]).
__global__ __launch_bounds__(kCbThreads) void bb_scan_kernel(const int64_t* __restrict__ pcnt, int64_t nchunks,
                                                             int64_t chunks_per_mat, int64_t* __restrict__ poff,
                                                             int64_t* __restrict__ n_out) {
    __shared__ int64_t sh[kCbThreads];
    const int t = threadIdx.x;
    const int64_t per = ceil_div(nchunks, kCbThreads);
    const int64_t lo = t * per, hi = (lo + per) < nchunks ? (lo + per) : nchunks;
    int64_t s = 0;
    for (int64_t i = lo; i < hi; ++i) s += pcnt[i];
    sh[t] = s;
    __syncthreads();
    if (t == 0) {
        int64_t run = 0;
        for (int i = 0; i < kCbThreads; ++i) {
            const int64_t v = sh[i];
            sh[i] = run;
            run += v;
        }
    }
    __syncthreads();
    int64_t run = sh[t];
    for (int64_t i = lo; i < hi; ++i) {
        poff[i] = run;
        run += pcnt[i];
    }
    __syncthreads();
    // per-matrix totals from the offsets
    const int64_t nmat = nchunks / chunks_per_mat;
    for (int64_t b = t; b < nmat; b += kCbThreads) {
        const int64_t first = b * chunks_per_mat, last = first + chunks_per_mat - 1;
        n_out[b] = poff[last] + pcnt[last] - poff[first];
    }
}

// pass 4: codes (packed MSB-first), dequant with outliers restored, error partials, and the
// outlier list (values, (row, col) in the reference's (nblocks, bs) view) at the scanned
// offsets, in row-major order (ballot prefix within each 256-element step).
template <int LB>  // log2 of the bits per code: 1 -> 2-bit (bbint2), 2 -> 4-bit (bbint4)
__global__ __launch_bounds__(kCbThreads) void bb_emit_kernel(
    const float* __restrict__ x, BBGeom g, const float* __restrict__ mean32, const float* __restrict__ thr,
    const float* __restrict__ bmin, const float* __restrict__ bscale, const int64_t* __restrict__ poff,
    uint8_t* __restrict__ packed, float* __restrict__ deq, float* __restrict__ out_vals, int64_t* __restrict__ out_idx,
    const float* __restrict__ ew, int64_t encols, double* __restrict__ perr, int64_t ews) {
    constexpr int BITS = 1 << LB;
    constexpr int PER = 8 / BITS;
    constexpr float LEVELS = (float)((1 << BITS) - 1);
    __shared__ int wcnt[kCbThreads / 64];
    __shared__ double lds[16];
    const int64_t ch = blockIdx.x;
    const int64_t blk = ch / g.nch, c = ch % g.nch;
    const int64_t c0 = c * kChunk;
    const float* xc = x + blk * g.bs + c0;
    const int64_t n = g.len(c);
    const float mu = mean32[blk], th = thr[blk], mn = bmin[blk], sc = bscale[blk];
    const int64_t row = blk % g.nblk_per;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t base = poff ? poff[ch] : 0;
    double acc = 0.0;
    // element i of the chunk is handled by thread i % 256 at step i / 256 (row-major order)
    for (int64_t s0 = 0; s0 < n; s0 += kCbThreads) {
        const int64_t i = s0 + threadIdx.x;
        const bool in = i < n;
        const float xv = in ? xc[i] : 0.f;
        const bool o = in && bb_outlier(xv, mu, th);
        const float v = o ? mu : xv;
        float q = rintf((v - mn) / sc);
        q = fminf(fmaxf(q, 0.f), LEVELS);
        float d = q * sc + mn;  // two roundings (no contraction in this file)
        d = o ? xv : d;
        const int64_t e = blk * g.bs + c0 + i;
        if (in && deq) deq[e] = d;
        if (in && perr) {
            const float df = d - xv;
            acc += (double)(df * df) * (ew ? (double)ew[(blk / g.nblk_per) * ews + ((row * g.bs) + c0 + i) % encols] : 1.0);
        }
        if (packed) {  // PER consecutive codes per byte, first code in the high bits
            uint32_t code = in ? (uint32_t)q : 0u;
            uint32_t byte = code;
#pragma unroll
            for (int t = 1; t < PER; ++t) byte = (byte << BITS) | (uint32_t)__shfl_down((int)code, t, 64);
            if (in && (i % PER) == 0) packed[e / PER] = (uint8_t)byte;
        }
        if (out_vals) {
            const uint64_t bal = __ballot(o);
            if (lane == 0) wcnt[w] = __popcll(bal);
            __syncthreads();
            int64_t pre = base;
            for (int k = 0; k < w; ++k) pre += wcnt[k];
            const uint64_t below = lane ? (bal & ((~0ull) >> (64 - lane))) : 0ull;
            if (o) {
                const int64_t slot = pre + __popcll(below);
                out_vals[slot] = xv;
                out_idx[2 * slot] = row;
                out_idx[2 * slot + 1] = c0 + i;
            }
            for (int k = 0; k < kCbThreads / 64; ++k) base += wcnt[k];
            __syncthreads();
        }
    }
    if (perr) {
        const double s = block_sum_f64(acc, lds);
        if (threadIdx.x == 0) perr[ch] = s;
    }
}

// dequantise packed bbint codes: u * scale + min per block, then the outliers scattered back
// (quantization.py:157-172 / :224-243)
template <int LB>
__global__ void bb_dequant_kernel(const uint8_t* __restrict__ packed, const float* __restrict__ bmin,
                                  const float* __restrict__ bscale, int64_t total, int64_t bs,
                                  float* __restrict__ out) {
    constexpr int BITS = 1 << LB;
    constexpr int PER = 8 / BITS;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
        const uint32_t byte = packed[e / PER];
        const int sh = BITS * (PER - 1 - (int)(e % PER));
        const float u = (float)((byte >> sh) & ((1u << BITS) - 1u));
        const int64_t blk = e / bs;
        out[e] = u * bscale[blk] + bmin[blk];
    }
}

__global__ void bb_scatter_kernel(const float* __restrict__ vals, const int64_t* __restrict__ idx, int64_t k,
                                  int64_t bs, float* __restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < k) out[idx[2 * t] * bs + idx[2 * t + 1]] = vals[t];
}

struct BBWs {  // workspace carve-up shared by cq_bbint_stats and cq_bbint_emit
    double *psum, *psq, *mean64, *perr;
    float *tsum, *mean32, *thr, *pmin, *pmax;
    int64_t *pcnt, *poff;
    size_t bytes;
};

static BBWs bb_carve(void* ws, int64_t nbt, int64_t nchunks) {
    BBWs w{};
    char* p = reinterpret_cast<char*>(ws);
    size_t o = 0;
    auto take = [&](size_t n) { char* r = p ? p + o : nullptr; o = align_up(o + n, 256); return r; };
    w.psum = reinterpret_cast<double*>(take(nchunks * 8));
    w.psq = reinterpret_cast<double*>(take(nchunks * 8));
    w.perr = reinterpret_cast<double*>(take(nchunks * 8));
    w.pcnt = reinterpret_cast<int64_t*>(take(nchunks * 8));
    w.poff = reinterpret_cast<int64_t*>(take(nchunks * 8));
    w.pmin = reinterpret_cast<float*>(take(nchunks * 4));
    w.pmax = reinterpret_cast<float*>(take(nchunks * 4));
    w.mean64 = reinterpret_cast<double*>(take(nbt * 8));
    w.tsum = reinterpret_cast<float*>(take(nbt * 4));
    w.mean32 = reinterpret_cast<float*>(take(nbt * 4));
    w.thr = reinterpret_cast<float*>(take(nbt * 4));
    w.bytes = o;
    return w;
}

static BBGeom bb_geom(int64_t batch, int64_t numel, int64_t bs) {
    BBGeom g;
    g.bs = bs;
    g.nch = ceil_div(bs, kChunk);
    g.nblk_per = numel / bs;
    g.nbt = batch * g.nblk_per;
    return g;
}

}  // namespace cq

using namespace cq;

extern "C" {

size_t cq_quantize_nf_workspace(int64_t batch, int64_t numel, int64_t block_size) {
    const int64_t nb = block_size > 0 ? numel / block_size : 1;
    return align_up((size_t)batch * nb * sizeof(uint32_t), 256) + align_up((size_t)batch * nb * sizeof(double), 256) +
           (size_t)batch * kMaxGrid * sizeof(double);
}

int cq_quantize_nf(const float* x, int64_t batch, int64_t numel, int64_t block_size, int bits, float eps,
                   uint8_t* idx, float* deq, float* scale, const float* err_w, int64_t err_ncols, int64_t err_w_stride,
                   double* err_out, void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(x && scale && batch > 0 && numel > 0 && block_size > 0, "cq_quantize_nf: bad args");
    CQ_REQUIRE(bits == 2 || bits == 4, "cq_quantize_nf: bits must be 2 (nf2) or 4 (nf4)");
    CQ_REQUIRE(numel % block_size == 0, "cq_quantize_nf: numel %% block_size != 0");
    CQ_REQUIRE(!err_w || err_ncols > 0, "cq_quantize_nf: err_ncols");
    if (!ws || ws_bytes < cq_quantize_nf_workspace(batch, numel, block_size))
        return set_error(CQ_EWORKSPACE, "cq_quantize_nf: workspace too small");
    hipStream_t s = as_stream(stream);
    const int64_t nblk = numel / block_size, nbt = batch * nblk;
    char* w = reinterpret_cast<char*>(ws);
    uint32_t* mx = reinterpret_cast<uint32_t*>(w);
    double* pblk = reinterpret_cast<double*>(w + align_up((size_t)nbt * sizeof(uint32_t), 256));
    double* part = reinterpret_cast<double*>(reinterpret_cast<char*>(pblk) + align_up((size_t)nbt * sizeof(double), 256));
    if (block_size <= 4096) {
        const int g = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(nbt, kCbThreads / 64), 8192));
        double* pe = err_out ? pblk : nullptr;
        if (bits == 4) nf_block_kernel<4><<<g, kCbThreads, 0, s>>>(x, nbt, block_size, nblk, eps, idx, deq, scale, err_w, err_ncols, pe, err_w_stride);
        else nf_block_kernel<2><<<g, kCbThreads, 0, s>>>(x, nbt, block_size, nblk, eps, idx, deq, scale, err_w, err_ncols, pe, err_w_stride);
        if (err_out) cb_sum_parts_kernel<<<batch, 64, 0, s>>>(pblk, nblk, err_out);
        return check_launch("cq_quantize_nf(block)");
    }
    if (hipMemsetAsync(mx, 0, (size_t)nbt * sizeof(uint32_t), s) != hipSuccess) return check_launch("cq_quantize_nf(memset)");
    const int g = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(numel, kCbThreads * 4), std::max<int64_t>(64, kMaxGrid / batch)));
    cb_absmax_kernel<<<dim3(g, batch), kCbThreads, 0, s>>>(x, numel, block_size, mx);
    double* pe = err_out ? part : nullptr;
    if (bits == 4) nf_known_kernel<4><<<dim3(g, batch), kCbThreads, 0, s>>>(x, numel, block_size, eps, mx, idx, deq, scale, err_w, err_ncols, pe, err_w_stride);
    else nf_known_kernel<2><<<dim3(g, batch), kCbThreads, 0, s>>>(x, numel, block_size, eps, mx, idx, deq, scale, err_w, err_ncols, pe, err_w_stride);
    if (err_out) cb_sum_parts_kernel<<<batch, 64, 0, s>>>(part, g, err_out);
    return check_launch("cq_quantize_nf");
}

int cq_dequant_nf(const uint8_t* idx, const float* scale, int64_t total, int64_t block_size, int bits, float* out,
                  void* stream) {
    CQ_REQUIRE(idx && scale && out && total > 0 && block_size > 0, "cq_dequant_nf: bad args");
    CQ_REQUIRE(bits == 2 || bits == 4, "cq_dequant_nf: bits must be 2 or 4");
    const int g = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, 256), 8192));
    if (bits == 4) nf_dequant_kernel<4><<<g, 256, 0, as_stream(stream)>>>(idx, scale, total, block_size, out);
    else nf_dequant_kernel<2><<<g, 256, 0, as_stream(stream)>>>(idx, scale, total, block_size, out);
    return check_launch("cq_dequant_nf");
}

size_t cq_bbint_workspace(int64_t batch, int64_t numel, int64_t block_size) {
    if (block_size <= 0 || numel % block_size) return 0;
    const BBGeom g = bb_geom(batch, numel, block_size);
    return bb_carve(nullptr, g.nbt, g.nbt * g.nch).bytes;
}

int cq_bbint_stats(const float* x, int64_t batch, int64_t numel, int64_t block_size, int bits, float eps,
                   float* bmin, float* bscale, int64_t* n_outliers, void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(x && bmin && bscale && n_outliers && batch > 0 && numel > 0 && block_size > 0, "cq_bbint_stats: bad args");
    CQ_REQUIRE(bits == 2 || bits == 4, "cq_bbint_stats: bits must be 2 (bbint2) or 4 (bbint4)");
    CQ_REQUIRE(numel % block_size == 0, "cq_bbint_stats: numel %% block_size != 0");
    if (!ws || ws_bytes < cq_bbint_workspace(batch, numel, block_size))
        return set_error(CQ_EWORKSPACE, "cq_bbint_stats: workspace too small");
    const BBGeom g = bb_geom(batch, numel, block_size);
    const int64_t nchunks = g.nbt * g.nch;
    BBWs w = bb_carve(ws, g.nbt, nchunks);
    hipStream_t s = as_stream(stream);
    const int gb = (int)ceil_div(g.nbt, 256);
    bb_sum_kernel<<<nchunks, kCbThreads, 0, s>>>(x, g, w.psum, w.tsum);
    bb_mean_kernel<<<gb, 256, 0, s>>>(g, w.psum, w.tsum, w.mean64, w.mean32);
    bb_var_kernel<<<nchunks, kCbThreads, 0, s>>>(x, g, w.mean64, w.psq);
    bb_thr_kernel<<<gb, 256, 0, s>>>(g, eps, w.psq, w.thr);
    bb_mask_kernel<<<nchunks, kCbThreads, 0, s>>>(x, g, w.mean32, w.thr, w.pcnt, w.pmin, w.pmax);
    bb_scale_kernel<<<gb, 256, 0, s>>>(g, eps, bits == 4 ? 15.f : 3.f, w.pmin, w.pmax, bmin, bscale);
    bb_scan_kernel<<<1, kCbThreads, 0, s>>>(w.pcnt, nchunks, g.nblk_per * g.nch, w.poff, n_outliers);
    return check_launch("cq_bbint_stats");
}

int cq_bbint_emit(const float* x, int64_t batch, int64_t numel, int64_t block_size, int bits, const float* bmin,
                  const float* bscale, uint8_t* packed, float* deq, float* out_vals, int64_t* out_idx,
                  const float* err_w, int64_t err_ncols, int64_t err_w_stride, double* err_out, void* ws, size_t ws_bytes,
                  void* stream) {
    CQ_REQUIRE(x && bmin && bscale && batch > 0 && numel > 0 && block_size > 0, "cq_bbint_emit: bad args");
    CQ_REQUIRE(bits == 2 || bits == 4, "cq_bbint_emit: bits must be 2 or 4");
    CQ_REQUIRE(!packed || block_size % (8 / bits) == 0, "cq_bbint_emit: block_size must be a multiple of %d", 8 / bits);
    CQ_REQUIRE(!out_vals == !out_idx, "cq_bbint_emit: out_vals and out_idx go together");
    CQ_REQUIRE(!err_w || err_ncols > 0, "cq_bbint_emit: err_ncols");
    if (!ws || ws_bytes < cq_bbint_workspace(batch, numel, block_size))
        return set_error(CQ_EWORKSPACE, "cq_bbint_emit: workspace too small");
    const BBGeom g = bb_geom(batch, numel, block_size);
    const int64_t nchunks = g.nbt * g.nch;
    BBWs w = bb_carve(ws, g.nbt, nchunks);
    hipStream_t s = as_stream(stream);
    double* pe = err_out ? w.perr : nullptr;
    if (bits == 4)
        bb_emit_kernel<2><<<nchunks, kCbThreads, 0, s>>>(x, g, w.mean32, w.thr, bmin, bscale, w.poff, packed, deq,
                                                         out_vals, out_idx, err_w, err_ncols, pe, err_w_stride);
    else
        bb_emit_kernel<1><<<nchunks, kCbThreads, 0, s>>>(x, g, w.mean32, w.thr, bmin, bscale, w.poff, packed, deq,
                                                         out_vals, out_idx, err_w, err_ncols, pe, err_w_stride);
    if (err_out) cb_sum_parts_kernel<<<batch, 64, 0, s>>>(w.perr, g.nblk_per * g.nch, err_out);
    return check_launch("cq_bbint_emit");
}

int cq_dequant_bbint(const uint8_t* packed, int bits, const float* bmin, const float* bscale, int64_t total,
                     int64_t block_size, const float* out_vals, const int64_t* out_idx, int64_t n_outliers,
                     float* out, void* stream) {
    CQ_REQUIRE(packed && bmin && bscale && out && total > 0 && block_size > 0, "cq_dequant_bbint: bad args");
    CQ_REQUIRE(bits == 2 || bits == 4, "cq_dequant_bbint: bits must be 2 or 4");
    CQ_REQUIRE(n_outliers == 0 || (out_vals && out_idx), "cq_dequant_bbint: outliers missing");
    hipStream_t s = as_stream(stream);
    const int g = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(total, 256), 8192));
    if (bits == 4) bb_dequant_kernel<2><<<g, 256, 0, s>>>(packed, bmin, bscale, total, block_size, out);
    else bb_dequant_kernel<1><<<g, 256, 0, s>>>(packed, bmin, bscale, total, block_size, out);
    if (n_outliers > 0)
        bb_scatter_kernel<<<(int)ceil_div(n_outliers, 256), 256, 0, s>>>(out_vals, out_idx, n_outliers, block_size, out);
    return check_launch("cq_dequant_bbint");
}

}  // extern "C"
