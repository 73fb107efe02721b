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

constexpr int BM = 128, BN = 192, BK = 16, PAD = 4;
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
    int64_t tri;
    int b_triu;  // op(B) upper triangular (op(B)[k][n] = 0 for k > n): zero K slices skipped
    _Float16 *th, *tl;  // gemm_triu_kernel<., true>: K-blocked split halves of C^T
    float tscale;       // ... at this scale
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

// op(B) is K x N.  TB: B stored N x K.  BNT = tile width (64 or 128): BNT/64 float4 per thread.
template <bool TB, int BNT>
__device__ __forceinline__ void load_b(const KArgs& a, const float* B, int64_t n0, int64_t k0,
                                       float4 (&r)[3]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int it = 0; it < BNT / 64; ++it) {
        const int idx = t + it * kGemmThreads;
        if (!TB) {  // K x N row-major: rows of BNT contiguous
            const int kr = idx / (BNT / 4), jq = (idx % (BNT / 4)) * 4;
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

template <bool TB, int BNT>
__device__ __forceinline__ void store_b(float* Bs, const float4 (&r)[3]) {
    const int t = threadIdx.x;
#pragma unroll
    for (int it = 0; it < BNT / 64; ++it) {
        const int idx = t + it * kGemmThreads;
        if (!TB) {
            const int kr = idx / (BNT / 4), jq = (idx % (BNT / 4)) * 4;
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

// Shared epilogue: acc[bi][bj] holds the 32x32 C blocks of this wave (C/D layout of the
// f32 MFMA: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)).
template <int EPI, bool DF16, int NB>
__device__ __forceinline__ void gemm_epilogue(const KArgs& a, f32x16 (&acc)[2][NB], int64_t b,
                                              int64_t m0, int64_t n0, int wm, int wn, int li,
                                              int lk, int lane) {
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
        for (int bj = 0; bj < NB; ++bj) {
            const int64_t j = n0 + wn * (32 * NB) + bj * 32 + li;
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

// NB = 32-wide MFMA column blocks per wave (2: 128x128 tile, 1: 128x64 tile for narrow N).
// a.tri != 0: SYRK mode — grid.x enumerates the upper-triangular 128x128 tiles only.
// TRIU: a.b_triu (own instantiation: the slice test costs the plain kernel its third wave per SIMD)
template <bool TA, bool TB, int EPI, bool DF16, int NB, bool TRIU = false>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_f32_kernel(KArgs a) {
    constexpr int BNT = 64 * NB;
    __shared__ __attribute__((aligned(16))) float smem[2 * BK * LDA_S + 2 * BK * LDB_S];
    float* As0 = smem;
    float* Bs0 = smem + 2 * BK * LDA_S;

    const int64_t b = blockIdx.z;
    int64_t tm = blockIdx.y, tn = blockIdx.x;
    if (a.tri) {  // decode upper-triangular tile index (tm <= tn)
        const int64_t T = a.tri;
        int64_t e = blockIdx.x, row = 0;
        while (e >= T - row) { e -= T - row; ++row; }
        tm = row;
        tn = row + e;
    }
    const int64_t m0 = tm * BM, n0 = tn * BNT;
    const float* A = a.A + b * a.sa;
    const float* B = a.B + b * a.sb;

    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int li = lane & 31, lk = lane >> 5;

    f32x16 acc[2][NB];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int64_t nt = ceil_div(a.K, BK);
    float4 ra[2], rb[3];
    if (nt > 0) {
        load_a<TA>(a, A, m0, 0, ra);
        load_b<TB, BNT>(a, B, n0, 0, rb);
        store_a<TA>(As0, ra);
        store_b<TB, BNT>(Bs0, rb);
    }
    __syncthreads();
    for (int64_t t = 0; t < nt; ++t) {
        const int cur = (int)(t & 1);
        if (t + 1 < nt) {
            load_a<TA>(a, A, m0, (t + 1) * BK, ra);
            load_b<TB, BNT>(a, B, n0, (t + 1) * BK, rb);
        }
        const float* As = As0 + cur * BK * LDA_S;
        const float* Bs = Bs0 + cur * BK * LDB_S;
        // TRIU (op(B) upper triangular): a wave whose last column n0 + 32 NB (wn + 1) - 1 lies
        // before this slice sees only zeros of op(B) and skips the slice's MFMAs (exact zero
        // products: the same bits).  A per-32-column-block skip cost the allocator a wave per SIMD.
        bool live = true;
        if constexpr (TRIU) live = t * BK <= n0 + 32 * NB * (wn + 1) - 1;
        if (live) {
#pragma unroll
            for (int kk = 0; kk < BK; kk += 2) {
                const float* ar = As + (kk + lk) * LDA_S + wm * 64 + li;
                const float* br = Bs + (kk + lk) * LDB_S + wn * (32 * NB) + li;
                const float a0 = ar[0], a1 = ar[32];
                float bv[NB];
#pragma unroll
                for (int j = 0; j < NB; ++j) bv[j] = br[32 * j];
#pragma unroll
                for (int j = 0; j < NB; ++j) {
                    acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bv[j], acc[0][j], 0, 0, 0);
                    acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bv[j], acc[1][j], 0, 0, 0);
                }
            }
        }
        if (t + 1 < nt) {
            store_a<TA>(As0 + (1 - cur) * BK * LDA_S, ra);
            store_b<TB, BNT>(Bs0 + (1 - cur) * BK * LDB_S, rb);
        }
        __syncthreads();
    }

    gemm_epilogue<EPI, DF16, NB>(a, acc, b, m0, n0, wm, wn, li, lk, lane);
}

// CholQR's X Wt (Wt upper triangular, K = N = 32 NBLK <= 192; solver._cholqr).  In
// gemm_f32_kernel<TRIU> the waves of columns 0-95 skip half the K slices, but those of columns
// 96-191 run all of them, and the SIMDs holding the latter set the time.  The measured
// difference from the full product is 6 % (0.86 vs 0.915 ms per B = 256 call,
// profiles/r05u_kt_kernel_stats.csv).  Here every wave owns 32 rows x all N columns (NBLK
// blocks of 32 x 32).  A 16-deep slice t feeds only the blocks it reaches (block c: t <= 2c + 1),
// unrolled at compile time, so the four waves carry equal work: 42 block-slices each at
// N = 192 instead of 36 and 72.  Per output element it uses the same instruction, operands and
// k order as gemm_f32_kernel, and the skipped terms are exact zeros, so the bits are the same
// (test_gemm_b_triu_matches_plain).  LINEAR epilogue with alpha only.  SPLIT: the epilogue
// also writes the K-blocked split halves of C^T at a.tscale -- the operand of the Rayleigh-Ritz
// product that follows CholQR (cq_gemm_triu_split), the same bits cq_transpose_split gives
// from C, without its pass over C.
template <int NBLK, bool SPLIT = false>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_triu_kernel(KArgs a) {
    static_assert(NBLK >= 1 && 32 * NBLK <= BN, "one 192-wide tile");
    constexpr int NT = 2 * NBLK;   // 16-deep K slices (K = 32 NBLK)
    __shared__ __attribute__((aligned(16))) float smem[2 * BK * LDA_S + 2 * BK * LDB_S];
    float* As0 = smem;
    float* Bs0 = smem + 2 * BK * LDA_S;
    const int64_t b = blockIdx.z;
    const int64_t m0 = (int64_t)blockIdx.y * BM;
    const float* A = a.A + b * a.sa;
    const float* B = a.B + b * a.sb;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int li = lane & 31, lk = lane >> 5;
    f32x16 acc[NBLK];
#pragma unroll
    for (int c = 0; c < NBLK; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
    float4 ra[2], rb[3];
    load_a<false>(a, A, m0, 0, ra);
    load_b<false, BN>(a, B, 0, 0, rb);
    store_a<false>(As0, ra);
    store_b<false, BN>(Bs0, rb);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int cur = t & 1;
        if (t + 1 < NT) {
            load_a<false>(a, A, m0, (t + 1) * BK, ra);
            load_b<false, BN>(a, B, 0, (t + 1) * BK, rb);
        }
        const float* As = As0 + cur * BK * LDA_S;
        const float* Bs = Bs0 + cur * BK * LDB_S;
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2) {
            const float a0 = As[(kk + lk) * LDA_S + 32 * wid + li];
#pragma unroll
            for (int c = t / 2; c < NBLK; ++c)
                acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, Bs[(kk + lk) * LDB_S + 32 * c + li], acc[c], 0, 0, 0);
        }
        if (t + 1 < NT) {
            store_a<false>(As0 + (1 - cur) * BK * LDA_S, ra);
            store_b<false, BN>(Bs0 + (1 - cur) * BK * LDB_S, rb);
        }
        __syncthreads();
    }
    float* C = a.C + b * a.sc;
    const float alpha = a.alpha_v ? a.alpha_v[b] : a.alpha;
#pragma unroll
    for (int c = 0; c < NBLK; ++c) {
        const int64_t j = 32 * c + li;
#pragma unroll
        for (int q = 0; q < 4; ++q) {   // registers 4q .. 4q + 3: rows i0 .. i0 + 3
            const int64_t i0 = m0 + 32 * wid + 8 * q + 4 * lk;
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] = alpha * acc[c][4 * q + e];
                if (i0 + e < a.M) C[(i0 + e) * a.ldc + j] = v[e];
            }
            if constexpr (SPLIT) {
                if (i0 < a.M) {   // M % 32 == 0 (host check): the four rows are live together
                    _Float16 h[4], l[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float xs = v[e] * a.tscale;
                        h[e] = (_Float16)xs;
                        l[e] = (_Float16)(xs - (float)h[e]);
                    }
                    // C^T (N x M) K-blocked over its columns (C's rows): (j, i) at
                    // (i / 32) N 32 + j 32 + i % 32, four consecutive i in 8 bytes
                    const int64_t o = b * a.M * a.N + (i0 >> 5) * a.N * 32 + j * 32 + (i0 & 31);
                    *reinterpret_cast<uint2*>(a.th + o) = *reinterpret_cast<const uint2*>(h);
                    *reinterpret_cast<uint2*>(a.tl + o) = *reinterpret_cast<const uint2*>(l);
                }
            }
        }
    }
}

// ------------------------------------------------------------------ K-contiguous ("NT") GEMM
// Both operands arrive with K contiguous: A row-major M x K, B stored N x K (op(B) = B^T).
// LDS images [row][k] (row stride BK2 + 4 floats: 16 consecutive rows hit 16 distinct
// 16-byte bank slots), filled by 16-byte ds_write_b128 straight from 16-byte global loads.
// K is permuted inside each 32-deep slice so every lane's MFMA operands for 16 consecutive
// MFMA steps are 16 contiguous floats: lane half h owns k = 16h .. 16h+15 of the slice and
// step s contracts k = s (h = 0) with k = 16 + s (h = 1).  Fragments load with 4
// ds_read_b128 per 32-row block, 64 v_mfma_f32_32x32x2_f32 per wave per slice.
constexpr int BK2 = 32, BKP = BK2 + 4;

template <int BNT>
__device__ __forceinline__ void nt_load(const KArgs& a, const float* P, int64_t rows, int64_t ld,
                                        int64_t r0, int64_t k0, bool vec, float4* r, int nvec) {
    const int t = threadIdx.x;
    for (int it = 0; it < nvec; ++it) {
        const int idx = t + it * kGemmThreads;
        const int row = idx >> 3, kq = (idx & 7) * 4;
        const int64_t gr = r0 + row, gk = k0 + kq;
        if (vec && gr < rows && gk + 3 < a.K) {
            r[it] = *reinterpret_cast<const float4*>(P + gr * ld + gk);
        } else {
            float v[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = (gr < rows && gk + c < a.K) ? P[gr * ld + gk + c] : 0.f;
            r[it] = make_float4(v[0], v[1], v[2], v[3]);
        }
    }
}

__device__ __forceinline__ void nt_store(float* S, const float4* r, int nvec) {
    const int t = threadIdx.x;
    for (int it = 0; it < nvec; ++it) {
        const int idx = t + it * kGemmThreads;
        const int row = idx >> 3, kq = (idx & 7) * 4;
        *reinterpret_cast<float4*>(S + row * BKP + kq) = r[it];
    }
}

template <int EPI, bool DF16, int NB>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_nt_kernel(KArgs a) {
    constexpr int BNT = 64 * NB;
    constexpr int NVA = BM * BK2 / 4 / kGemmThreads;   // float4 per thread, A slice
    constexpr int NVB = BNT * BK2 / 4 / kGemmThreads;  // float4 per thread, B slice
    __shared__ __attribute__((aligned(16))) float smem[2 * BM * BKP + 2 * BNT * BKP];
    float* As0 = smem;
    float* Bs0 = smem + 2 * BM * BKP;

    const int64_t b = blockIdx.z;
    int64_t tm = blockIdx.y, tn = blockIdx.x;
    if (a.tri) {
        const int64_t T = a.tri;
        int64_t e = blockIdx.x, row = 0;
        while (e >= T - row) { e -= T - row; ++row; }
        tm = row;
        tn = row + e;
    }
    const int64_t m0 = tm * BM, n0 = tn * BNT;
    const float* A = a.A + b * a.sa;
    const float* B = a.B + b * a.sb;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid >> 1, wn = wid & 1;
    const int li = lane & 31, lk = lane >> 5;

    f32x16 acc[2][NB];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int64_t nt = ceil_div(a.K, BK2);
    float4 ra[NVA], rb[NVB];
    if (nt > 0) {
        nt_load<BNT>(a, A, a.M, a.lda, m0, 0, a.vec_a, ra, NVA);
        nt_load<BNT>(a, B, a.N, a.ldb, n0, 0, a.vec_b, rb, NVB);
        nt_store(As0, ra, NVA);
        nt_store(Bs0, rb, NVB);
    }
    __syncthreads();
    for (int64_t t = 0; t < nt; ++t) {
        const int cur = (int)(t & 1);
        if (t + 1 < nt) {
            nt_load<BNT>(a, A, a.M, a.lda, m0, (t + 1) * BK2, a.vec_a, ra, NVA);
            nt_load<BNT>(a, B, a.N, a.ldb, n0, (t + 1) * BK2, a.vec_b, rb, NVB);
        }
        const float* As = As0 + cur * BM * BKP;
        const float* Bs = Bs0 + cur * BNT * BKP;
#pragma unroll
        for (int half = 0; half < 2; ++half) {  // k = 16 lk + 8 half + (0..7)
            float af[2][8], bf[NB][8];
#pragma unroll
            for (int bi = 0; bi < 2; ++bi) {
                const float* ap = As + (wm * 64 + bi * 32 + li) * BKP + 16 * lk + 8 * half;
                const float4 x0 = *reinterpret_cast<const float4*>(ap);
                const float4 x1 = *reinterpret_cast<const float4*>(ap + 4);
                af[bi][0] = x0.x; af[bi][1] = x0.y; af[bi][2] = x0.z; af[bi][3] = x0.w;
                af[bi][4] = x1.x; af[bi][5] = x1.y; af[bi][6] = x1.z; af[bi][7] = x1.w;
            }
#pragma unroll
            for (int bj = 0; bj < NB; ++bj) {
                const float* bp = Bs + (wn * (32 * NB) + bj * 32 + li) * BKP + 16 * lk + 8 * half;
                const float4 y0 = *reinterpret_cast<const float4*>(bp);
                const float4 y1 = *reinterpret_cast<const float4*>(bp + 4);
                bf[bj][0] = y0.x; bf[bj][1] = y0.y; bf[bj][2] = y0.z; bf[bj][3] = y0.w;
                bf[bj][4] = y1.x; bf[bj][5] = y1.y; bf[bj][6] = y1.z; bf[bj][7] = y1.w;
            }
#pragma unroll
            for (int s2 = 0; s2 < 8; ++s2)
#pragma unroll
                for (int bi = 0; bi < 2; ++bi)
#pragma unroll
                    for (int bj = 0; bj < NB; ++bj)
                        acc[bi][bj] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[bi][s2], bf[bj][s2],
                                                                           acc[bi][bj], 0, 0, 0);
        }
        if (t + 1 < nt) {
            nt_store(As0 + (1 - cur) * BM * BKP, ra, NVA);
            nt_store(Bs0 + (1 - cur) * BNT * BKP, rb, NVB);
        }
        __syncthreads();
    }
    gemm_epilogue<EPI, DF16, NB>(a, acc, b, m0, n0, wm, wn, li, lk, lane);
}

__global__ void werr_finalize_kernel(const double* part, int64_t ntiles, double* out) {
    const int64_t b = blockIdx.x;
    if (threadIdx.x != 0) return;
    double s = 0.0;
    for (int64_t t = 0; t < ntiles; ++t) s += part[b * ntiles + t];
    out[b] = s;
}

// Copy the upper triangle of square C onto its lower triangle (SYRK completion), 64x64 tiles
// through LDS so both the read and the transposed write are coalesced.
__global__ __launch_bounds__(256) void mirror_upper_kernel(float* __restrict__ C, int64_t n, int64_t ldc,
                                                            int64_t sc) {
    __shared__ float tile[64][65];
    const int64_t b = blockIdx.z;
    const int64_t ti = blockIdx.y, tj = blockIdx.x;  // destination tile (ti > tj: lower)
    if (ti <= tj) return;
    float* Cb = C + b * sc;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    // source: upper tile (tj, ti)
    for (int r = ty; r < 64; r += 4) {
        const int64_t i = tj * 64 + r, j = ti * 64 + tx;
        tile[r][tx] = (i < n && j < n) ? Cb[i * ldc + j] : 0.f;
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int64_t i = ti * 64 + r, j = tj * 64 + tx;
        if (i < n && j < n) Cb[i * ldc + j] = tile[tx][r];
    }
}

}  // namespace cq

using namespace cq;

template <int EPI, bool DF16, int NB>
static void launch_gemm_nb(bool ta, bool tb, dim3 grid, hipStream_t s, const KArgs& k) {
    if constexpr (EPI == CQ_EPI_LINEAR && !DF16) {
        if (!ta && !tb && k.b_triu) {
            gemm_f32_kernel<false, false, EPI, DF16, NB, true><<<grid, kGemmThreads, 0, s>>>(k);
            return;
        }
    }
    if (!ta && !tb) gemm_f32_kernel<false, false, EPI, DF16, NB><<<grid, kGemmThreads, 0, s>>>(k);
    else if (!ta && tb) gemm_f32_kernel<false, true, EPI, DF16, NB><<<grid, kGemmThreads, 0, s>>>(k);
    else if (ta && !tb) gemm_f32_kernel<true, false, EPI, DF16, NB><<<grid, kGemmThreads, 0, s>>>(k);
    else gemm_f32_kernel<true, true, EPI, DF16, NB><<<grid, kGemmThreads, 0, s>>>(k);
}

template <int EPI, bool DF16>
static void launch_gemm(bool ta, bool tb, int nb, dim3 grid, hipStream_t s, const KArgs& k) {
    if (nb == 1) launch_gemm_nb<EPI, DF16, 1>(ta, tb, grid, s, k);
    else if (nb == 3) launch_gemm_nb<EPI, DF16, 3>(ta, tb, grid, s, k);
    else launch_gemm_nb<EPI, DF16, 2>(ta, tb, grid, s, k);
}

// tile width 64 * nb: a single 192-wide tile for 128 < N <= 192 (the solver block p), else
// 128-wide tiles unless the last one would be at most half full
static int pick_nb(int64_t N) {
    if (N > 128 && N <= 192) return 3;
    const int64_t r = N % 128;
    return (N <= 64 || (r != 0 && r <= 64)) ? 1 : 2;
}

extern "C" {

size_t cq_gemm_workspace(const cq_gemm_args* a) {
    if (!a || a->epi != CQ_EPI_WERR) return 0;
    return (size_t)a->batch * ceil_div(a->M, BM) * ceil_div(a->N, 64 * pick_nb(a->N)) * sizeof(double);
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
    if (g->syrk) {
        CQ_REQUIRE(g->epi == CQ_EPI_LINEAR && g->M == g->N && g->beta == 0.f && !g->beta_v &&
                       g->gamma == 0.f && !g->gamma_v && !g->alpha_v,
                   "cq_gemm_f32: syrk needs square C, LINEAR epilogue, alpha only");
    }
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
    const int nb = g->syrk ? 2 : pick_nb(g->N);
    dim3 grid((unsigned)ceil_div(g->N, 64 * nb), (unsigned)ceil_div(g->M, BM), (unsigned)g->batch);
    k.tri = 0;
    k.b_triu = g->b_triu;
    k.th = k.tl = nullptr;
    k.tscale = 1.f;
    CQ_REQUIRE(!g->b_triu || (!g->trans_a && !g->trans_b && !g->syrk && g->epi == CQ_EPI_LINEAR),
               "cq_gemm_f32: b_triu needs a plain product (no transposes, LINEAR epilogue)");
    if (g->syrk) {
        const int64_t T = ceil_div(g->N, BM);
        k.tri = T;
        grid = dim3((unsigned)(T * (T + 1) / 2), 1, (unsigned)g->batch);
    }
    hipStream_t s = as_stream(stream);
    const bool ta = g->trans_a != 0, tb = g->trans_b != 0;
    if (g->b_triu && g->N == g->K && g->N % 32 == 0 && g->N <= BN && g->beta == 0.f && !g->beta_v &&
        g->gamma == 0.f && !g->gamma_v) {
        // the solver's square triangular factor: balanced waves (gemm_triu_kernel)
        const dim3 tg(1, (unsigned)ceil_div(g->M, BM), (unsigned)g->batch);
        switch (g->N / 32) {
            case 1: gemm_triu_kernel<1><<<tg, kGemmThreads, 0, s>>>(k); break;
            case 2: gemm_triu_kernel<2><<<tg, kGemmThreads, 0, s>>>(k); break;
            case 3: gemm_triu_kernel<3><<<tg, kGemmThreads, 0, s>>>(k); break;
            case 4: gemm_triu_kernel<4><<<tg, kGemmThreads, 0, s>>>(k); break;
            case 5: gemm_triu_kernel<5><<<tg, kGemmThreads, 0, s>>>(k); break;
            default: gemm_triu_kernel<6><<<tg, kGemmThreads, 0, s>>>(k); break;
        }
        return check_launch("cq_gemm_f32");
    }
    switch (g->epi) {
        case CQ_EPI_LINEAR:
            launch_gemm<CQ_EPI_LINEAR, false>(ta, tb, nb, grid, s, k);
            if (g->syrk) {
                const unsigned t64 = (unsigned)ceil_div(g->N, 64);
                mirror_upper_kernel<<<dim3(t64, t64, (unsigned)g->batch), 256, 0, s>>>(
                    g->C, g->N, g->ldc, g->stride_c);
            }
            break;
        case CQ_EPI_RESID:
            if (g->d_f16) launch_gemm<CQ_EPI_RESID, true>(ta, tb, nb, grid, s, k);
            else launch_gemm<CQ_EPI_RESID, false>(ta, tb, nb, grid, s, k);
            break;
        default:
            if (g->d_f16) launch_gemm<CQ_EPI_WERR, true>(ta, tb, nb, grid, s, k);
            else launch_gemm<CQ_EPI_WERR, false>(ta, tb, nb, grid, s, k);
            werr_finalize_kernel<<<(unsigned)g->batch, 64, 0, s>>>(
                k.part, (int64_t)grid.x * grid.y, g->err_out);
            break;
    }
    return check_launch("cq_gemm_f32");
}

int cq_gemm_triu_split(const float* X, const float* Wt, int64_t M, int64_t p, int64_t batch, float* C,
                       uint16_t* hi, uint16_t* lo, float scale, void* stream) {
    CQ_REQUIRE(X && Wt && C && hi && lo, "cq_gemm_triu_split: null pointer");
    CQ_REQUIRE(p > 0 && p % 32 == 0 && p <= BN, "cq_gemm_triu_split: p must be a multiple of 32, <= 192");
    CQ_REQUIRE(M > 0 && M % 32 == 0 && batch > 0 && batch <= 65535 && ceil_div(M, BM) <= 65535,
               "cq_gemm_triu_split: bad shape (M % 32 == 0)");
    KArgs k{};
    k.M = M; k.N = p; k.K = p;
    k.A = X; k.lda = p; k.sa = M * p;
    k.B = Wt; k.ldb = p; k.sb = p * p;
    k.C = C; k.ldc = p; k.sc = M * p;
    k.alpha = 1.f; k.beta = 0.f; k.gamma = 0.f;
    auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    k.vec_a = al16(X);
    k.vec_b = al16(Wt);
    k.b_triu = 1;
    k.th = reinterpret_cast<_Float16*>(hi);
    k.tl = reinterpret_cast<_Float16*>(lo);
    k.tscale = scale;
    CQ_REQUIRE((reinterpret_cast<uintptr_t>(hi) & 7) == 0 && (reinterpret_cast<uintptr_t>(lo) & 7) == 0,
               "cq_gemm_triu_split: halves must be 8-byte aligned");
    const dim3 tg(1, (unsigned)ceil_div(M, BM), (unsigned)batch);
    hipStream_t s = as_stream(stream);
    switch (p / 32) {
        case 1: gemm_triu_kernel<1, true><<<tg, kGemmThreads, 0, s>>>(k); break;
        case 2: gemm_triu_kernel<2, true><<<tg, kGemmThreads, 0, s>>>(k); break;
        case 3: gemm_triu_kernel<3, true><<<tg, kGemmThreads, 0, s>>>(k); break;
        case 4: gemm_triu_kernel<4, true><<<tg, kGemmThreads, 0, s>>>(k); break;
        case 5: gemm_triu_kernel<5, true><<<tg, kGemmThreads, 0, s>>>(k); break;
        default: gemm_triu_kernel<6, true><<<tg, kGemmThreads, 0, s>>>(k); break;
    }
    return check_launch("cq_gemm_triu_split");
}

}  // extern "C"
