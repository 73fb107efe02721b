// Batched FP32 GEMM for the rank-r solver on gfx950 matrix cores.
//
// Every dense product of the CALDERA hot path runs here (RCR/src/caldera/decomposition/
// alg.py): the Gram Y Y^T feeding the truncated SVD (replaces torch.linalg.svd, :217),
// the Chebyshev-filtered subspace iteration G X, Ritz rotations, R = U^T Y (:219-225),
// the LPLR normal-equation products (:162-182), the residual W - L R (:262) fused with
// the whole-matrix absmax the quantiser needs (quantization.py:262), and the
// diagonal-H activation-aware error (:286-302) fused as a weighted square-sum epilogue.
//
// Parity needs fp32 inputs, so the instruction is
// v_mfma_f32_32x32x2_f32: exact f32 products, one rounding per product (a k-ordered fmaf
// chain), 64 FLOP/clk/SIMD.  Geometry: 256 threads = 4 waves; a 128x128 output tile per
// workgroup, 64x64 per wave as 2x2 MFMA blocks of 32x32; K staged through LDS in
// 16-deep slices, double-buffered (global loads of slice t+1 are in flight while slice t
// feeds the MFMAs; one barrier per slice).  LDS images are K-major ([k][m], [k][n]) so
// each MFMA operand fetch is one conflict-free ds_read_b32 of 32 consecutive floats per
// half-wave.  Grid: (N tiles, M tiles, batch); tall-skinny products get their
// parallelism from the batch of matrices processed in lockstep.
#include "cq_common.h"

namespace cq {

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int BM = 128, BN = 128, BK = 16, PAD = 4;
constexpr int LDA_S = BM + PAD, LDB_S = BN + PAD;
constexpr int kGemmThreads = 256;

struct KArgs {
    int64_t M, N, K;
    const float* A; int64_t lda, sa;
    const float* B; int64_t ldb, sb;
    float* C; int64_t ldc, sc;
    const void* D; int64_t ldd, sd;
    float alpha, beta, gamma;
    const float *alpha_v, *beta_v, *gamma_v;
    uint32_t* absmax;
    const float* w; int64_t sw;
    double* part;
    int vec_a, vec_b;
};

// Stage one BM x BK slice of op(A) into registers (4 floats x 2 per thread).
template <bool TA>
__device__ __forceinline__ void load_a(const KArgs& a, const float* A, int64_t m0, int64_t k0,
                                       float4 (&r)[2]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int idx = t + it * kGemmThreads;
        if (!TA) {  // A row-major M x K: rows of BK contiguous floats
            const int row = idx >> 2, kq = (idx & 3) * 4;
            const int64_t gi = m0 + row, gk = k0 + kq;
            if (a.vec_a && gi < a.M && gk + 3 < a.K) {
                r[it] = *reinterpret_cast<const float4*>(A + gi * a.lda + gk);
            } else {
                float v[4];
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    v[c] = (gi < a.M && gk + c < a.K) ? A[gi * a.lda + gk + c] : 0.f;
                r[it] = make_float4(v[0], v[1], v[2], v[3]);
            }
        } else {    // A stored K x M: rows of BM contiguous floats
            const int kr = idx >> 5, iq = (idx & 31) * 4;
            const int64_t gk = k0 + kr, gi = m0 + iq;
            if (a.vec_a && gk < a.K && gi + 3 < a.M) {
                r[it] = *reinterpret_cast<const float4*>(A + gk * a.lda + gi);
            } else {
                float v[4];
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    v[c] = (gk < a.K && gi + c < a.M) ? A[gk * a.lda + gi + c] : 0.f;
                r[it] = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
    }
}

template <bool TA>
__device__ __forceinline__ void store_a(float* As, const float4 (&r)[2]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int idx = t + it * kGemmThreads;
        if (!TA) {
            const int row = idx >> 2, kq = (idx & 3) * 4;
            As[(kq + 0) * LDA_S + row] = r[it].x;
            As[(kq + 1) * LDA_S + row] = r[it].y;
            As[(kq + 2) * LDA_S + row] = r[it].z;
            As[(kq + 3) * LDA_S + row] = r[it].w;
        } else {
            const int kr = idx >> 5, iq = (idx & 31) * 4;
            *reinterpret_cast<float4*>(As + kr * LDA_S + iq) = r[it];
        }
    }
}

// op(B) is K x N.  TB: B stored N x K.
template <bool TB>
__device__ __forceinline__ void load_b(const KArgs& a, const float* B, int64_t n0, int64_t k0,
                                       float4 (&r)[2]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int idx = t + it * kGemmThreads;
        if (!TB) {  // K x N row-major: rows of BN contiguous
            const int kr = idx >> 5, jq = (idx & 31) * 4;
            const int64_t gk = k0 + kr, gj = n0 + jq;
            if (a.vec_b && gk < a.K && gj + 3 < a.N) {
                r[it] = *reinterpret_cast<const float4*>(B + gk * a.ldb + gj);
            } else {
                float v[4];
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    v[c] = (gk < a.K && gj + c < a.N) ? B[gk * a.ldb + gj + c] : 0.f;
                r[it] = make_float4(v[0], v[1], v[2], v[3]);
            }
        } else {    // N x K: rows of BK contiguous
            const int row = idx >> 2, kq = (idx & 3) * 4;
            const int64_t gj = n0 + row, gk = k0 + kq;
            if (a.vec_b && gj < a.N && gk + 3 < a.K) {
                r[it] = *reinterpret_cast<const float4*>(B + gj * a.ldb + gk);
            } else {
                float v[4];
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    v[c] = (gj < a.N && gk + c < a.K) ? B[gj * a.ldb + gk + c] : 0.f;
                r[it] = make_float4(v[0], v[1], v[2], v[3]);
            }
        }
    }
}

template <bool TB>
__device__ __forceinline__ void store_b(float* Bs, const float4 (&r)[2]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const int idx = t + it * kGemmThreads;
        if (!TB) {
            const int kr = idx >> 5, jq = (idx & 31) * 4;
            *reinterpret_cast<float4*>(Bs + kr * LDB_S + jq) = r[it];
        } else {
            const int row = idx >> 2, kq = (idx & 3) * 4;
            Bs[(kq + 0) * LDB_S + row] = r[it].x;
            Bs[(kq + 1) * LDB_S + row] = r[it].y;
            Bs[(kq + 2) * LDB_S + row] = r[it].z;
            Bs[(kq + 3) * LDB_S + row] = r[it].w;
        }
    }
}

template <bool TA, bool TB, int EPI, bool DF16>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_f32_kernel(KArgs a) {
    __shared__ __attribute__((aligned(16))) float smem[2 * BK * LDA_S + 2 * BK * LDB_S];
    float* As0 = smem;
    float* Bs0 = smem + 2 * BK * LDA_S;

    const int64_t b = blockIdx.z;
    const int64_t m0 = (int64_t)blockIdx.y * BM, n0 = (int64_t)blockIdx.x * BN;
    const float* A = a.A + b * a.sa;
    const float* B = a.B + b * a.sb;

    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int li = lane & 31, lk = lane >> 5;

    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int64_t nt = ceil_div(a.K, BK);
    float4 ra[2], rb[2];
    if (nt > 0) {
        load_a<TA>(a, A, m0, 0, ra);
        load_b<TB>(a, B, n0, 0, rb);
        store_a<TA>(As0, ra);
        store_b<TB>(Bs0, rb);
    }
    __syncthreads();
    for (int64_t t = 0; t < nt; ++t) {
        const int cur = (int)(t & 1);
        if (t + 1 < nt) {
            load_a<TA>(a, A, m0, (t + 1) * BK, ra);
            load_b<TB>(a, B, n0, (t + 1) * BK, rb);
        }
        const float* As = As0 + cur * BK * LDA_S;
        const float* Bs = Bs0 + cur * BK * LDB_S;
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2) {
            const float* ar = As + (kk + lk) * LDA_S + wm * 64 + li;
            const float* br = Bs + (kk + lk) * LDB_S + wn * 64 + li;
            const float a0 = ar[0], a1 = ar[32];
            const float b0 = br[0], b1 = br[32];
            acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (t + 1 < nt) {
            store_a<TA>(As0 + (1 - cur) * BK * LDA_S, ra);
            store_b<TB>(Bs0 + (1 - cur) * BK * LDB_S, rb);
        }
        __syncthreads();
    }

    // ---------------- epilogue
    float* C = a.C ? a.C + b * a.sc : nullptr;
    const float* Df = (!DF16 && a.D) ? reinterpret_cast<const float*>(a.D) + b * a.sd : nullptr;
    const __half* Dh = (DF16 && a.D) ? reinterpret_cast<const __half*>(a.D) + b * a.sd : nullptr;
    const float* w = a.w ? a.w + b * a.sw : nullptr;
    uint32_t mx = 0;
    double esum = 0.0;
    const float alpha = a.alpha_v ? a.alpha_v[b] : a.alpha;
    const float beta = a.beta_v ? a.beta_v[b] : a.beta;
    const float gamma = a.gamma_v ? a.gamma_v[b] : a.gamma;
#pragma unroll
    for (int bi = 0; bi < 2; ++bi) {
#pragma unroll
        for (int bj = 0; bj < 2; ++bj) {
            const int64_t j = n0 + wn * 64 + bj * 32 + li;
            if (j >= a.N) continue;
            const float wj = (EPI == CQ_EPI_WERR && w) ? w[j] : 1.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t i = m0 + wm * 64 + bi * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
                if (i >= a.M) continue;
                const float v = acc[bi][bj][r];
                if (EPI == CQ_EPI_LINEAR) {
                    float o = alpha * v;
                    if (beta != 0.f) o += beta * C[i * a.ldc + j];
                    if (gamma != 0.f) o += gamma * Df[i * a.ldd + j];
                    C[i * a.ldc + j] = o;
                } else {
                    const float d = DF16 ? __half2float(Dh[i * a.ldd + j]) : Df[i * a.ldd + j];
                    const float e = d - v;
                    if (EPI == CQ_EPI_RESID) {
                        if (C) C[i * a.ldc + j] = e;
                        const uint32_t ab = abs_bits(e);
                        mx = ab > mx ? ab : mx;
                    } else {
                        esum += (double)(e * e) * (double)wj;
                    }
                }
            }
        }
    }
    if (EPI == CQ_EPI_RESID) {
        mx = wave_max_u32(mx);
        if (lane == 0 && mx) atomicMax(&a.absmax[b], mx);
    } else if (EPI == CQ_EPI_WERR) {
        __shared__ double red[16];
        const double s = block_sum_f64(esum, red);
        if (threadIdx.x == 0)
            a.part[(b * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = s;
    }
}

__global__ void werr_finalize_kernel(const double* part, int64_t ntiles, double* out) {
    const int64_t b = blockIdx.x;
    if (threadIdx.x != 0) return;
    double s = 0.0;
    for (int64_t t = 0; t < ntiles; ++t) s += part[b * ntiles + t];
    out[b] = s;
}

}  // namespace cq

using namespace cq;

template <int EPI, bool DF16>
static void launch_gemm(bool ta, bool tb, dim3 grid, hipStream_t s, const KArgs& k) {
    if (!ta && !tb) gemm_f32_kernel<false, false, EPI, DF16><<<grid, kGemmThreads, 0, s>>>(k);
    else if (!ta && tb) gemm_f32_kernel<false, true, EPI, DF16><<<grid, kGemmThreads, 0, s>>>(k);
    else if (ta && !tb) gemm_f32_kernel<true, false, EPI, DF16><<<grid, kGemmThreads, 0, s>>>(k);
    else gemm_f32_kernel<true, true, EPI, DF16><<<grid, kGemmThreads, 0, s>>>(k);
}

extern "C" {

size_t cq_gemm_workspace(const cq_gemm_args* a) {
    if (!a || a->epi != CQ_EPI_WERR) return 0;
    return (size_t)a->batch * ceil_div(a->M, BM) * ceil_div(a->N, BN) * sizeof(double);
}

int cq_gemm_f32(const cq_gemm_args* g, void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(g, "cq_gemm_f32: null args");
    CQ_REQUIRE(g->M > 0 && g->N > 0 && g->K >= 0 && g->batch > 0, "cq_gemm_f32: bad shape");
    CQ_REQUIRE((g->A && g->B) || g->K == 0, "cq_gemm_f32: null A/B");
    CQ_REQUIRE(g->epi >= CQ_EPI_LINEAR && g->epi <= CQ_EPI_WERR, "cq_gemm_f32: bad epi");
    CQ_REQUIRE(g->batch <= 65535 && ceil_div(g->M, BM) <= 65535, "cq_gemm_f32: grid too large");
    if (g->epi == CQ_EPI_LINEAR) {
        CQ_REQUIRE(g->C, "cq_gemm_f32: null C");
        CQ_REQUIRE((g->gamma == 0.f && !g->gamma_v) || (g->D && !g->d_f16), "cq_gemm_f32: gamma needs fp32 D");
        CQ_REQUIRE((g->beta == 0.f && !g->beta_v) || g->C, "cq_gemm_f32: beta needs C");
    } else {
        CQ_REQUIRE(g->D, "cq_gemm_f32: epilogue needs D");
    }
    if (g->epi == CQ_EPI_RESID) CQ_REQUIRE(g->absmax_bits, "cq_gemm_f32: RESID needs absmax_bits");
    if (g->epi == CQ_EPI_WERR) {
        CQ_REQUIRE(g->err_out, "cq_gemm_f32: WERR needs err_out");
        if (!ws || ws_bytes < cq_gemm_workspace(g))
            return set_error(CQ_EWORKSPACE, "cq_gemm_f32: workspace too small");
    }
    KArgs k;
    k.M = g->M; k.N = g->N; k.K = g->K;
    k.A = g->A; k.lda = g->lda; k.sa = g->stride_a;
    k.B = g->B; k.ldb = g->ldb; k.sb = g->stride_b;
    k.C = g->C; k.ldc = g->ldc; k.sc = g->stride_c;
    k.D = g->D; k.ldd = g->ldd; k.sd = g->stride_d;
    k.alpha = g->alpha; k.beta = g->beta; k.gamma = g->gamma;
    k.alpha_v = g->alpha_v; k.beta_v = g->beta_v; k.gamma_v = g->gamma_v;
    k.absmax = g->absmax_bits;
    k.w = g->w; k.sw = g->stride_w;
    k.part = reinterpret_cast<double*>(ws);
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    k.vec_a = al16(g->A) && g->lda % 4 == 0 && g->stride_a % 4 == 0;
    k.vec_b = al16(g->B) && g->ldb % 4 == 0 && g->stride_b % 4 == 0;
    dim3 grid((unsigned)ceil_div(g->N, BN), (unsigned)ceil_div(g->M, BM), (unsigned)g->batch);
    hipStream_t s = as_stream(stream);
    const bool ta = g->trans_a != 0, tb = g->trans_b != 0;
    switch (g->epi) {
        case CQ_EPI_LINEAR: launch_gemm<CQ_EPI_LINEAR, false>(ta, tb, grid, s, k); break;
        case CQ_EPI_RESID:
            if (g->d_f16) launch_gemm<CQ_EPI_RESID, true>(ta, tb, grid, s, k);
            else launch_gemm<CQ_EPI_RESID, false>(ta, tb, grid, s, k);
            break;
        default:
            if (g->d_f16) launch_gemm<CQ_EPI_WERR, true>(ta, tb, grid, s, k);
            else launch_gemm<CQ_EPI_WERR, false>(ta, tb, grid, s, k);
            werr_finalize_kernel<<<(unsigned)g->batch, 64, 0, s>>>(
                k.part, (int64_t)grid.x * grid.y, g->err_out);
            break;
    }
    return check_launch("cq_gemm_f32");
}

}  // extern "C"
