// Small dense kernels of the rank-r solver that replaces the full LAPACK SVD of
// RCR/src/caldera/decomposition/alg.py:217 (and lstsq at :163,175, eigh at :23):
//
//   cq_gram_f64      C = A^T B, fp32 inputs, fp64 accumulation, split-K.  CholQR Grams
//                    (X^T X), Rayleigh-Ritz matrices (X^T G X) and LPLR normal matrices.
//   cq_spd_whiten    symmetric Gaussian elimination S = L D L^T -> Wt = L^{-T} D^{-1/2}
//                    (Wt^T S Wt = I): the triangular factor of CholQR / normal equations.
//   cq_jacobi_eigh   parallel cyclic Jacobi (round-robin pairing, p/2 disjoint rotations
//                    per round, one workgroup per matrix), fp64, sorted descending.
//   cq_ritz_residual max_i ||G x_i - theta_i x_i|| / theta_0 convergence test.
//
// These are latency-bound p x p problems (p <= 512).  Throughput comes from the batch:
// one workgroup per matrix, B matrices decomposed in lockstep, so a 1-CU kernel costs
// 1/256 of the chip while the other CUs run the batch's GEMMs.
#include "cq_common.h"

namespace cq {

// ------------------------------------------------------------------ fp64-accumulated Gram
constexpr int GT = 64;   // output tile
constexpr int GK = 32;   // K slice
constexpr int kGramThreads = 256;

__global__ __launch_bounds__(kGramThreads) void gram_f64_kernel(
    int64_t M, int64_t N, int64_t K, int64_t kchunk, int splits, const float* __restrict__ A,
    int ta, int64_t lda, int64_t sa, const float* __restrict__ B, int tb, int64_t ldb, int64_t sb,
    double* __restrict__ part) {
    __shared__ float As[GK][GT + 1];
    __shared__ float Bs[GK][GT + 1];
    const int64_t b = blockIdx.z / splits;
    const int split = blockIdx.z % splits;
    const int64_t i0 = (int64_t)blockIdx.y * GT, j0 = (int64_t)blockIdx.x * GT;
    const float* Ab = A + b * sa;
    const float* Bb = B + b * sb;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    double acc[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = 0.0;
    const int64_t kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
    for (int64_t k0 = kbeg; k0 < kend; k0 += GK) {
        // load GK x GT of A (element (k, i)) and B (element (k, j))
        for (int e = threadIdx.x; e < GK * GT; e += kGramThreads) {
            int kk, ii;
            if (!ta) { kk = e / GT; ii = e % GT; } else { ii = e / GK; kk = e % GK; }
            const int64_t gk = k0 + kk, gi = i0 + ii;
            float v = 0.f;
            if (gk < kend && gi < M) v = ta ? Ab[gi * lda + gk] : Ab[gk * lda + gi];
            As[kk][ii] = v;
            int jj;
            if (!tb) { kk = e / GT; jj = e % GT; } else { jj = e / GK; kk = e % GK; }
            const int64_t gk2 = k0 + kk, gj = j0 + jj;
            float w = 0.f;
            if (gk2 < kend && gj < N) w = tb ? Bb[gj * ldb + gk2] : Bb[gk2 * ldb + gj];
            Bs[kk][jj] = w;
        }
        __syncthreads();
#pragma unroll 4
        for (int kk = 0; kk < GK; ++kk) {
            double av[4], bv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) av[u] = (double)As[kk][ty * 4 + u];
#pragma unroll
            for (int v = 0; v < 4; ++v) bv[v] = (double)Bs[kk][tx * 4 + v];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int v = 0; v < 4; ++v) acc[u][v] = fma(av[u], bv[v], acc[u][v]);
        }
        __syncthreads();
    }
    double* P = part + ((int64_t)b * splits + split) * M * N;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int64_t i = i0 + ty * 4 + u, j = j0 + tx * 4 + v;
            if (i < M && j < N) P[i * N + j] = acc[u][v];
        }
}

__global__ void gram_reduce_kernel(const double* __restrict__ part, int64_t MN, int splits,
                                   int64_t batch, double* __restrict__ C) {
    const int64_t total = batch * MN;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = e / MN, o = e % MN;
        double s = 0.0;
        for (int t = 0; t < splits; ++t) s += part[(b * splits + t) * MN + o];
        C[e] = s;
    }
}

static int gram_splits(int64_t M, int64_t N, int64_t K, int64_t batch) {
    const int64_t tiles = ceil_div(M, GT) * ceil_div(N, GT) * batch;
    int64_t s = ceil_div(1024, tiles);
    s = std::min<int64_t>(s, std::max<int64_t>(1, K / 256));
    return (int)std::max<int64_t>(1, std::min<int64_t>(s, 64));
}

// ------------------------------------------------------------------ SPD whitening
// Symmetric Gaussian elimination S = L D L^T on the upper triangle (the trailing block stays
// symmetric), E = L^{-1} built alongside; Wt = E^T D^{-1/2}.  One workgroup per matrix,
// operands L2-resident; every thread batches UNR independent element updates so the
// loads of a step are in flight together (the step is latency-bound, not FLOP-bound).
constexpr int kSmallThreads = 1024;
constexpr int UNR = 8;

__global__ __launch_bounds__(kSmallThreads) void spd_whiten_kernel(double* __restrict__ S_all,
                                                                    int64_t p, double* __restrict__ E_all,
                                                                    float* __restrict__ W32,
                                                                    int* __restrict__ info) {
    extern __shared__ double fac[];  // row factors of the current step + pivots
    double* piv = fac + p;
    __shared__ int bad;
    __shared__ double dmax_s;
    const int64_t b = blockIdx.x;
    double* S = S_all + b * p * p;
    double* E = E_all + b * p * p;
    const int tid = threadIdx.x;
    for (int64_t e = tid; e < p * p; e += kSmallThreads) E[e] = (e / p == e % p) ? 1.0 : 0.0;
    if (tid == 0) {
        bad = 0;
        double dm = 0.0;
        for (int64_t j = 0; j < p; ++j) dm = fmax(dm, fabs(S[j * p + j]));
        dmax_s = dm;
    }
    __syncthreads();
    const double dmax = dmax_s;
    for (int64_t j = 0; j < p; ++j) {
        const double d = S[j * p + j];
        if (!(d > 1e-300 && d > dmax * 1e-30)) {  // not positive definite (or NaN)
            if (tid == 0) bad = (int)(j + 1);
            __syncthreads();
            break;
        }
        for (int64_t i = j + 1 + tid; i < p; i += kSmallThreads) fac[i] = S[j * p + i] / d;  // upper row j
        if (tid == 0) piv[j] = d;
        __syncthreads();
        // upper trailing: S[i][c] -= f_i S[j][c] for j < i <= c ;  E[i][c] -= f_i E[j][c], c <= j, i > j
        const int64_t t = p - j - 1;               // trailing size
        const int64_t nS = t * (t + 1) / 2;        // upper-triangular trailing elements
        const int64_t nE = t * (j + 1);
        const int64_t work = nS + nE;
        for (int64_t e0 = tid; e0 < work; e0 += (int64_t)kSmallThreads * UNR) {
            double* dst[UNR];
            double val[UNR];
            double src[UNR];
            double f[UNR];
#pragma unroll
            for (int u = 0; u < UNR; ++u) {
                const int64_t e = e0 + (int64_t)u * kSmallThreads;
                dst[u] = nullptr;
                if (e < nS) {
                    // e -> (ri, ci) in the upper triangle of the t x t trailing block, row-major
                    // rows of decreasing length: invert with a float sqrt then fix up
                    const double tt = (double)t;
                    int64_t ri = (int64_t)((2.0 * tt + 1.0 - sqrt((2.0 * tt + 1.0) * (2.0 * tt + 1.0) - 8.0 * (double)e)) * 0.5);
                    if (ri < 0) ri = 0;
                    while (ri > 0 && ri * t - ri * (ri - 1) / 2 > e) --ri;
                    while ((ri + 1) * t - (ri + 1) * ri / 2 <= e) ++ri;
                    const int64_t ci = ri + (e - (ri * t - ri * (ri - 1) / 2));
                    const int64_t i = j + 1 + ri, c = j + 1 + ci;
                    dst[u] = S + i * p + c;
                    src[u] = S[j * p + c];
                    f[u] = fac[i];
                } else if (e < work) {
                    const int64_t q = e - nS;
                    const int64_t i = j + 1 + q / (j + 1), c = q % (j + 1);
                    dst[u] = E + i * p + c;
                    src[u] = E[j * p + c];
                    f[u] = fac[i];
                }
                val[u] = dst[u] ? *dst[u] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < UNR; ++u)
                if (dst[u]) *dst[u] = val[u] - f[u] * src[u];
        }
        __syncthreads();
    }
    if (bad) {
        if (tid == 0) info[b] = bad;
        return;
    }
    if (tid == 0) info[b] = 0;
    // Wt[a][c] = E[c][a] / sqrt(piv[c])  (upper triangular); staged in S (fp64)
    for (int64_t e = tid; e < p * p; e += kSmallThreads) {
        const int64_t a = e / p, c = e % p;
        const double v = (c >= a) ? E[c * p + a] / sqrt(piv[c]) : 0.0;
        if (W32) W32[b * p * p + e] = (float)v;
        S[e] = v;
    }
}

// ------------------------------------------------------------------ Jacobi eigensolver
// Parallel cyclic Jacobi: round-robin pairing, p/2 disjoint rotations per round.  A is updated
// on 2x2 blocks (pair a, pair b), upper blocks only, mirrored; eigenvectors are accumulated
// TRANSPOSED (Vt rows = eigenvector components) so a rotation of columns i, j of V is a
// coalesced update of rows i, j of Vt.  Loads are batched UNR-deep per thread.
__device__ __forceinline__ void rr_pair(int64_t P, int64_t rd, int64_t q, int64_t& i, int64_t& j) {
    const int64_t n1 = P - 1;
    if (q == 0) { i = n1; j = rd % n1; }
    else { i = (rd + q) % n1; j = (rd - q + n1) % n1; }
    if (i > j) { const int64_t t = i; i = j; j = t; }
}

__global__ __launch_bounds__(kSmallThreads) void jacobi_kernel(double* __restrict__ A_all,
                                                                int64_t p, int max_sweeps, double tol,
                                                                double* __restrict__ Vt_all,
                                                                double* __restrict__ evals,
                                                                float* __restrict__ V32,
                                                                double* __restrict__ V64,
                                                                int* __restrict__ sweeps_out) {
    extern __shared__ double sm[];
    const int64_t P = p + (p & 1);
    const int64_t H = P / 2;
    double* cs = sm;          // H
    double* sn = sm + H;      // H
    int* pi = reinterpret_cast<int*>(sm + 2 * H);  // H
    int* pj = pi + H;                               // H
    __shared__ double red[16];
    __shared__ int stop, nact;
    const int64_t b = blockIdx.x;
    double* A = A_all + b * p * p;
    double* Vt = Vt_all + b * p * p;
    const int tid = threadIdx.x;
    for (int64_t e = tid; e < p * p; e += kSmallThreads) Vt[e] = (e / p == e % p) ? 1.0 : 0.0;
    // symmetrise in place (Rayleigh-Ritz matrices X^T G X carry rounding asymmetry)
    for (int64_t e = tid; e < p * p; e += kSmallThreads) {
        const int64_t i = e / p, j = e % p;
        if (i < j) {
            const double s = 0.5 * (A[i * p + j] + A[j * p + i]);
            A[i * p + j] = s;
            A[j * p + i] = s;
        }
    }
    __syncthreads();
    const int64_t nup = H * (H + 1) / 2;
    int sweep = 0;
    for (; sweep < max_sweeps; ++sweep) {
        double off = 0.0, dg = 0.0;
        for (int64_t e = tid; e < p * p; e += kSmallThreads) {
            const double v = A[e];
            if (e / p == e % p) dg += v * v; else off += v * v;
        }
        const double offs = block_sum_f64(off, red);
        const double dgs = block_sum_f64(dg, red);
        if (tid == 0) stop = (offs <= tol * tol * dgs) ? 1 : 0;
        __syncthreads();
        if (stop) break;
        for (int64_t rd = 0; rd < P - 1; ++rd) {
            if (tid == 0) nact = 0;
            __syncthreads();
            for (int64_t q = tid; q < H; q += kSmallThreads) {
                int64_t i, j;
                rr_pair(P, rd, q, i, j);
                double c = 1.0, s = 0.0;
                if (j < p) {
                    const double aij = A[i * p + j];
                    const double aii = A[i * p + i], ajj = A[j * p + j];
                    if (fabs(aij) > 1e-300 && fabs(aij) > 1e-17 * sqrt(fabs(aii * ajj))) {
                        const double th = (ajj - aii) / (2.0 * aij);
                        const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(1.0 + th * th));
                        c = 1.0 / sqrt(1.0 + t * t);
                        s = t * c;
                        atomicAdd(&nact, 1);
                    }
                }
                cs[q] = c; sn[q] = s; pi[q] = (int)i; pj[q] = (int)j;
            }
            __syncthreads();
            if (nact == 0) continue;
            // ---- A <- J^T A J on upper 2x2 pair blocks (qa <= qb), mirrored
            for (int64_t e0 = tid; e0 < nup; e0 += (int64_t)kSmallThreads * 4) {
                double x[4][4];
                int64_t off4[4][4];
                double ca[4], sa4[4], cb[4], sb4[4];
                bool live[4], diag[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int64_t e = e0 + (int64_t)u * kSmallThreads;
                    live[u] = false;
                    diag[u] = false;
                    if (e < nup) {
                        int64_t qb = (int64_t)((sqrt(8.0 * (double)e + 1.0) - 1.0) * 0.5);
                        while (qb * (qb + 1) / 2 > e) --qb;
                        while ((qb + 1) * (qb + 2) / 2 <= e) ++qb;
                        const int64_t qa = e - qb * (qb + 1) / 2;
                        ca[u] = cs[qa]; sa4[u] = sn[qa]; cb[u] = cs[qb]; sb4[u] = sn[qb];
                        if (sa4[u] != 0.0 || sb4[u] != 0.0) {
                            live[u] = true;
                            diag[u] = (qa == qb);
                            const int64_t ia = pi[qa], ja = pj[qa], ib = pi[qb], jb = pj[qb];
                            const bool va = ja < p, vb = jb < p;
                            off4[u][0] = ia * p + ib;
                            off4[u][1] = vb ? ia * p + jb : -1;
                            off4[u][2] = va ? ja * p + ib : -1;
                            off4[u][3] = (va && vb) ? ja * p + jb : -1;
#pragma unroll
                            for (int w = 0; w < 4; ++w) x[u][w] = off4[u][w] >= 0 ? A[off4[u][w]] : 0.0;
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (!live[u]) continue;
                    const double y00 = cb[u] * x[u][0] - sb4[u] * x[u][1], y01 = sb4[u] * x[u][0] + cb[u] * x[u][1];
                    const double y10 = cb[u] * x[u][2] - sb4[u] * x[u][3], y11 = sb4[u] * x[u][2] + cb[u] * x[u][3];
                    double z00 = ca[u] * y00 - sa4[u] * y10, z10 = sa4[u] * y00 + ca[u] * y10;
                    double z01 = ca[u] * y01 - sa4[u] * y11, z11 = sa4[u] * y01 + ca[u] * y11;
                    if (diag[u]) { z01 = 0.0; z10 = 0.0; }
                    const double z[4] = {z00, z01, z10, z11};
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const int64_t o = off4[u][w];
                        if (o < 0) continue;
                        A[o] = z[w];
                        if (!diag[u]) {  // mirror: (r, c) -> (c, r)
                            const int64_t rr = o / p, cc = o % p;
                            A[cc * p + rr] = z[w];
                        }
                    }
                }
            }
            // ---- Vt rows i, j <- rotation (coalesced along the row)
            const int64_t nv = H * p;
            for (int64_t e0 = tid; e0 < nv; e0 += (int64_t)kSmallThreads * UNR) {
                double vi[UNR], vj[UNR];
                int64_t oi[UNR], oj[UNR];
                double c[UNR], s[UNR];
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    const int64_t e = e0 + (int64_t)u * kSmallThreads;
                    oi[u] = -1;
                    if (e < nv) {
                        const int64_t q = e / p, xcol = e % p;
                        s[u] = sn[q];
                        if (s[u] != 0.0) {
                            c[u] = cs[q];
                            oi[u] = (int64_t)pi[q] * p + xcol;
                            oj[u] = (int64_t)pj[q] * p + xcol;
                            vi[u] = Vt[oi[u]];
                            vj[u] = Vt[oj[u]];
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < UNR; ++u) {
                    if (oi[u] < 0) continue;
                    Vt[oi[u]] = c[u] * vi[u] - s[u] * vj[u];
                    Vt[oj[u]] = s[u] * vi[u] + c[u] * vj[u];
                }
            }
            __syncthreads();
        }
    }
    if (tid == 0 && sweeps_out) sweeps_out[b] = sweep;
    // sort descending by rank counting (ties broken by index); eigenvector i = row i of Vt
    for (int64_t i = tid; i < p; i += kSmallThreads) {
        const double di = A[i * p + i];
        int64_t rank = 0;
        for (int64_t j = 0; j < p; ++j) {
            const double dj = A[j * p + j];
            rank += (dj > di) || (dj == di && j < i);
        }
        evals[b * p + rank] = di;
        pi[i] = (int)rank;
    }
    __syncthreads();
    for (int64_t e = tid; e < p * p; e += kSmallThreads) {
        const int64_t i = e / p, x = e % p;  // component x of eigenvector i
        const double v = Vt[e];
        const int64_t rk = pi[i];
        if (V32) V32[b * p * p + x * p + rk] = (float)v;
        if (V64) V64[b * p * p + x * p + rk] = v;
    }
}

// ------------------------------------------------------------------ Ritz residuals
__global__ __launch_bounds__(256) void ritz_partial_kernel(const float* __restrict__ X,
                                                            const float* __restrict__ Z,
                                                            const double* __restrict__ theta,
                                                            int64_t k, int64_t p, int64_t r,
                                                            int64_t rows_per, double* part) {
    const int64_t b = blockIdx.y, chunk = blockIdx.x;
    const int64_t r0 = chunk * rows_per, r1 = min(k, r0 + rows_per);
    for (int64_t c = threadIdx.x; c < r; c += blockDim.x) {
        const float th = (float)theta[b * p + c];
        double s = 0.0;
        for (int64_t i = r0; i < r1; ++i) {
            const float d = Z[b * k * p + i * p + c] - th * X[b * k * p + i * p + c];
            s += (double)d * d;
        }
        part[(b * gridDim.x + chunk) * r + c] = s;
    }
}

__global__ void ritz_final_kernel(const double* part, int nchunks, int64_t p, int64_t r,
                                  const double* theta, float* out) {
    __shared__ double red[16];
    const int64_t b = blockIdx.x;
    double mx = 0.0;
    for (int64_t c = threadIdx.x; c < r; c += blockDim.x) {
        double s = 0.0;
        for (int t = 0; t < nchunks; ++t) s += part[(b * nchunks + t) * r + c];
        mx = fmax(mx, sqrt(s));
    }
    // block max via shuffles
    for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = 0.0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) m = fmax(m, red[i]);
        const double t0 = fabs(theta[b * p]);
        out[b] = (float)(t0 > 0 ? m / t0 : m);
    }
}

}  // namespace cq

using namespace cq;

extern "C" {

size_t cq_gram_f64_workspace(int64_t M, int64_t N, int64_t K, int64_t batch) {
    return (size_t)batch * gram_splits(M, N, K, batch) * M * N * sizeof(double);
}

int cq_gram_f64(int64_t M, int64_t N, int64_t K, int64_t batch, const float* A, int trans_a,
                int64_t lda, int64_t stride_a, const float* B, int trans_b, int64_t ldb,
                int64_t stride_b, double* C, void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(A && B && C && M > 0 && N > 0 && K > 0 && batch > 0, "cq_gram_f64: bad args");
    const int splits = gram_splits(M, N, K, batch);
    if (!ws || ws_bytes < cq_gram_f64_workspace(M, N, K, batch))
        return set_error(CQ_EWORKSPACE, "cq_gram_f64: workspace too small");
    CQ_REQUIRE(batch * splits <= 65535, "cq_gram_f64: batch too large");
    const int64_t kchunk = ceil_div(ceil_div(K, splits), GK) * GK;
    hipStream_t s = as_stream(stream);
    dim3 grid((unsigned)ceil_div(N, GT), (unsigned)ceil_div(M, GT), (unsigned)(batch * splits));
    gram_f64_kernel<<<grid, kGramThreads, 0, s>>>(M, N, K, kchunk, splits, A, trans_a, lda,
                                                   stride_a, B, trans_b, ldb, stride_b,
                                                   reinterpret_cast<double*>(ws));
    const int64_t tot = batch * M * N;
    gram_reduce_kernel<<<(unsigned)std::min<int64_t>(ceil_div(tot, 256), 4096), 256, 0, s>>>(
        reinterpret_cast<double*>(ws), M * N, splits, batch, C);
    return check_launch("cq_gram_f64");
}

int cq_spd_whiten(double* S, int64_t p, int64_t batch, float* Wt32, double* Wt64, int* info,
                  void* stream) {
    CQ_REQUIRE(S && p > 0 && batch > 0 && info && Wt64, "cq_spd_whiten: bad args (Wt64 is required scratch)");
    hipStream_t s = as_stream(stream);
    // E is built in Wt64; the final fp64 Wt is staged in S and copied to Wt64.
    spd_whiten_kernel<<<(unsigned)batch, kSmallThreads, 2 * p * sizeof(double), s>>>(S, p, Wt64, Wt32, info);
    if (hipMemcpyAsync(Wt64, S, (size_t)batch * p * p * sizeof(double), hipMemcpyDeviceToDevice, s) != hipSuccess)
        return set_error(CQ_EHIP, "cq_spd_whiten: copy failed");
    return check_launch("cq_spd_whiten");
}

size_t cq_jacobi_workspace(int64_t p, int64_t batch) {
    return (size_t)batch * p * p * sizeof(double);
}

int cq_jacobi_eigh(double* A, int64_t p, int64_t batch, int max_sweeps, double tol, double* evals,
                   float* V32, double* V64, int* sweeps_out, void* ws, size_t ws_bytes,
                   void* stream) {
    CQ_REQUIRE(A && evals && p > 0 && batch > 0 && max_sweeps > 0, "cq_jacobi_eigh: bad args");
    CQ_REQUIRE(p <= 4096, "cq_jacobi_eigh: p too large");
    if (!ws || ws_bytes < cq_jacobi_workspace(p, batch))
        return set_error(CQ_EWORKSPACE, "cq_jacobi_eigh: workspace too small");
    const int64_t H = (p + (p & 1)) / 2;
    const size_t lds = 2 * H * sizeof(double) + 2 * (2 * H) * sizeof(int);
    jacobi_kernel<<<(unsigned)batch, kSmallThreads, lds, as_stream(stream)>>>(
        A, p, max_sweeps, tol, reinterpret_cast<double*>(ws), evals, V32, V64, sweeps_out);
    return check_launch("cq_jacobi_eigh");
}

size_t cq_ritz_workspace(int64_t k, int64_t r, int64_t batch) {
    const int64_t nch = std::min<int64_t>(64, std::max<int64_t>(1, k / 64));
    return (size_t)batch * nch * r * sizeof(double);
}

int cq_ritz_residual(const float* X, const float* Z, const double* theta, int64_t k, int64_t p,
                     int64_t r, int64_t batch, float* out, void* ws, size_t ws_bytes,
                     void* stream) {
    CQ_REQUIRE(X && Z && theta && out && k > 0 && p > 0 && r > 0 && r <= p, "cq_ritz_residual: bad args");
    if (!ws || ws_bytes < cq_ritz_workspace(k, r, batch))
        return set_error(CQ_EWORKSPACE, "cq_ritz_residual: workspace too small");
    hipStream_t s = as_stream(stream);
    const int64_t nch = std::min<int64_t>(64, std::max<int64_t>(1, k / 64));
    const int64_t rows_per = ceil_div(k, nch);
    double* part = reinterpret_cast<double*>(ws);
    ritz_partial_kernel<<<dim3((unsigned)nch, (unsigned)batch), 256, 0, s>>>(X, Z, theta, k, p, r, rows_per, part);
    ritz_final_kernel<<<(unsigned)batch, 256, 0, s>>>(part, (int)nch, p, r, theta, out);
    return check_launch("cq_ritz_residual");
}

}  // extern "C"
