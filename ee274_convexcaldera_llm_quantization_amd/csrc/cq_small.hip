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


// fp64-MFMA variant for the non-transposed case (C = A^T B, A: K x M, B: K x N, row-major):
// v_mfma_f64_16x16x4_f64 on fp32 operands converted exactly to fp64 (products exact, fp64
// accumulation: the same arithmetic contract as gram_f64_kernel).  64 x 64 tile per
// workgroup, 4 waves of 32 x 32 (2 x 2 blocks), GK-deep LDS slices filled by float4 loads
// with a one-slice register prefetch.  sym (A == B): tiles below the block diagonal are
// skipped and mirrored by the reduction.  TK: both operands transposed (C = A B^T with A: M x K,
// B: N x K row-major, K contiguous -- the LPLR loop's R H_sqrt (R H_sqrt)^T): float4 loads run
// along K and are transposed into the same LDS slice layout.
using f64x4v = __attribute__((ext_vector_type(4))) double;

template <bool TK>
__global__ __launch_bounds__(kGramThreads) void gram_f64_mfma_kernel(
    int64_t M, int64_t N, int64_t K, int64_t kchunk, int splits, const float* __restrict__ A,
    int64_t lda, int64_t sa, const float* __restrict__ B, int64_t ldb, int64_t sb, int sym,
    double* __restrict__ part) {
    // row pitch: GT + 16 floats puts the fragment reads' four K rows (lane >> 4) 16 banks apart
    // (conflict-free; GT + 4 overlapped them: 3.2 conflict cycles per LDS instruction in PMC);
    // the TK stash writes columns and keeps GT + 4
    constexpr int GP = TK ? GT + 4 : GT + 16;
    __shared__ float As[2][GK][GP];
    __shared__ float Bs[2][GK][GP];
    const int64_t b = blockIdx.z / splits;
    const int split = blockIdx.z % splits;
    if (sym && blockIdx.x < blockIdx.y) return;
    const int64_t i0 = (int64_t)blockIdx.y * GT, j0 = (int64_t)blockIdx.x * GT;
    const float* Ab = A + b * sa;
    const float* Bb = B + b * sb;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int wi = wid >> 1, wj = wid & 1;  // wave block: rows 32 wi, cols 32 wj
    // slice loader: GK rows x 64 columns of A and of B, 2 float4 per thread each
    const int lr = t >> 4, lc = (t & 15) * 4;  // rows lr and lr + 16, columns lc .. lc+3
    // TK: 64 operand rows x GK along K, 2 float4 per thread each: rows tr and tr + 32, K tk .. tk+3
    const int tr = t >> 3, tk = (t & 7) * 4;
    const int64_t kbeg = split * kchunk, kend = min(K, kbeg + kchunk);
    auto ld4 = [&](const float* base, int64_t ld, int64_t lim, int64_t k, int64_t c0) -> float4 {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (k < kend) {
            const float* src = base + k * ld + c0;
            if (c0 + 3 < lim) v = *reinterpret_cast<const float4*>(src);
            else {
                if (c0 < lim) v.x = src[0];
                if (c0 + 1 < lim) v.y = src[1];
                if (c0 + 2 < lim) v.z = src[2];
            }
        }
        return v;
    };
    f64x4v acc[2][2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v) acc[u][v] = f64x4v{0.0, 0.0, 0.0, 0.0};
    float4 ra[2], rb[2];
    // TK loads: row `row` of a K-contiguous operand, K elements k .. k+3 (zero past kend / lim)
    auto ld4t = [&](const float* base, int64_t ld, int64_t lim, int64_t row, int64_t k) -> float4 {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < lim && k < kend) {
            const float* src = base + row * ld + k;
            if (k + 3 < kend) v = *reinterpret_cast<const float4*>(src);
            else {
                v.x = src[0];
                if (k + 1 < kend) v.y = src[1];
                if (k + 2 < kend) v.z = src[2];
            }
        }
        return v;
    };
    auto fetch = [&](int64_t k0) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if constexpr (TK) {
                ra[h] = ld4t(Ab, lda, M, i0 + tr + 32 * h, k0 + tk);
                rb[h] = ld4t(Bb, ldb, N, j0 + tr + 32 * h, k0 + tk);
            } else {
                ra[h] = ld4(Ab, lda, M, k0 + lr + 16 * h, i0 + lc);
                rb[h] = ld4(Bb, ldb, N, k0 + lr + 16 * h, j0 + lc);
            }
        }
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if constexpr (TK) {
                const int c = tr + 32 * h;
                As[buf][tk + 0][c] = ra[h].x; As[buf][tk + 1][c] = ra[h].y;
                As[buf][tk + 2][c] = ra[h].z; As[buf][tk + 3][c] = ra[h].w;
                Bs[buf][tk + 0][c] = rb[h].x; Bs[buf][tk + 1][c] = rb[h].y;
                Bs[buf][tk + 2][c] = rb[h].z; Bs[buf][tk + 3][c] = rb[h].w;
            } else {
                *reinterpret_cast<float4*>(&As[buf][lr + 16 * h][lc]) = ra[h];
                *reinterpret_cast<float4*>(&Bs[buf][lr + 16 * h][lc]) = rb[h];
            }
        }
    };
    const int nsl = (int)ceil_div(kend - kbeg, GK);
    if (nsl > 0) { fetch(kbeg); stash(0); }
    __syncthreads();
    const int li = lane & 15, lk = lane >> 4;
    for (int sl = 0; sl < nsl; ++sl) {
        const int cur = sl & 1;
        if (sl + 1 < nsl) fetch(kbeg + (int64_t)(sl + 1) * GK);
#pragma unroll
        for (int kk = 0; kk < GK; kk += 4) {
            double a0 = (double)As[cur][kk + lk][32 * wi + li];
            double a1 = (double)As[cur][kk + lk][32 * wi + 16 + li];
            double b0 = (double)Bs[cur][kk + lk][32 * wj + li];
            double b1 = (double)Bs[cur][kk + lk][32 * wj + 16 + li];
            acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
        }
        if (sl + 1 < nsl) stash(1 - cur);
        __syncthreads();
    }
    double* P = part + ((int64_t)b * splits + split) * M * N;
    // C/D map of the f64 16x16x4 form: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int v = 0; v < 2; ++v)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t i = i0 + 32 * wi + 16 * u + lk + 4 * r;
                const int64_t j = j0 + 32 * wj + 16 * v + li;
                if (i < M && j < N) P[i * N + j] = acc[u][v][r];
            }
}

__global__ void gram_reduce_sym_kernel(const double* __restrict__ part, int64_t M, int splits,
                                       int64_t batch, double* __restrict__ C) {
    const int64_t MN = M * M, total = batch * MN;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = e / MN, o = e % MN, i = o / M, j = o % M;
        const int64_t src = (i / GT > j / GT) ? j * M + i : o;  // lower tiles were skipped
        double s = 0.0;
        for (int t2 = 0; t2 < splits; ++t2) s += part[(b * splits + t2) * MN + src];
        C[e] = s;
    }
}

static int gram_splits(int64_t M, int64_t N, int64_t K, int64_t batch) {
    const int64_t tiles = ceil_div(M, GT) * ceil_div(N, GT) * batch;
    int64_t s = ceil_div(1024, tiles);
    s = std::min<int64_t>(s, std::max<int64_t>(1, K / 256));
    return (int)std::max<int64_t>(1, std::min<int64_t>(s, 64));
}

// ------------------------------------------------------------------ Jacobi, V in registers
// A (fp64, packed upper triangle) lives in LDS in index space; the eigenvector matrix V
// (fp32) lives in REGISTERS in "seat" space.  The round-robin is the circle method with
// fixed adjacent seat pairs (2k, 2k+1): between rounds every player except seat 0 moves one
// seat (even seats +1 pair, odd seats -1 pair, with the two end turns), so a V column only
// ever moves to a neighbouring pair.  Thread (pair-group pg, row-group rg) holds PPT pairs x
// RPT rows of V; a round's rotations are register-local and the seat shift is register
// moves plus one lane shuffle up and one down per row.  V never touches memory until the
// end, which removes the per-round O(p^2) global traffic of accumulating V.  fp32 V keeps
// orthogonality to ~sqrt(rounds)*eps32 (~3e-6); the solver re-orthonormalises its final
// Ritz block (CholQR), and A stays fp64 so the rotations themselves are fp64-accurate.
template <int PPT, int RPT, int JBR, int NTH>
__global__ __launch_bounds__(NTH) void jacobi_reg_kernel(const double* __restrict__ A_all,
                                                                    int p, int max_sweeps, double tol,
                                                                    double* __restrict__ evals,
                                                                    float* __restrict__ V32,
                                                                    double* __restrict__ V64,
                                                                    int* __restrict__ sweeps_out) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int P = p + (p & 1);
    const int H = P / 2;
    double2* csn = reinterpret_cast<double2*>(smem_raw);  // H: (cos, sin) of pair k's rotation
    int4* lohi = reinterpret_cast<int4*>(csn + H);         // H: pair k's (smaller, larger) index and
                                                           // their packed-row offsets (pko)
    int* flp = reinterpret_cast<int*>(lohi + H);           // H  (seat 2k holds the larger index)
    int* seat = flp + H;                                // P
    int* seat2 = seat + P;                              // P
    int* rnk = seat2 + P;                               // P
    double* a = reinterpret_cast<double*>(rnk + P + ((9 * H + 3 * P) & 1));
    __shared__ double red[16];
    __shared__ int stop;
    const int64_t b = blockIdx.x;
    const double* Ag = A_all + b * (int64_t)p * p;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool wantv = V32 != nullptr || V64 != nullptr;  // else eigenvalues only: no V work
    const int pg = lane & 31;                 // pair group
    const int rg = 2 * wid + (lane >> 5);     // row group
    const int k0 = pg * PPT, x0 = rg * RPT;
    auto pk = [p](int i, int j) -> int {
        if (i > j) { const int t = i; i = j; j = t; }
        return i * p - ((i * (i - 1)) >> 1) + (j - i);
    };
    // packed offset of row i's diagonal minus i: element (i, j), i <= j, at pko(i) + j
    auto pko = [p](int i) -> int { return i * p - ((i * (i - 1)) >> 1) - i; };
    // element (x, y) from the two indices and their row offsets
    auto pkx = [](int x, int ox, int y, int oy) -> int { return x <= y ? ox + y : oy + x; };
    for (int i = wid; i < p; i += (NTH / 64))
        for (int c = lane; c < p; c += 64)
            if (c >= i) a[pk(i, c)] = 0.5 * (Ag[i * p + c] + Ag[c * p + i]);
    for (int s = tid; s < P; s += NTH) seat[s] = s;
    float ev[PPT][RPT], od[PPT][RPT];
#pragma unroll
    for (int u = 0; u < PPT; ++u)
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            const int k = k0 + u, x = x0 + r;
            ev[u][r] = (x == 2 * k) ? 1.f : 0.f;
            od[u][r] = (x == 2 * k + 1) ? 1.f : 0.f;
        }
    __syncthreads();
    const double skip_rel = fmax(1e-17, 0.01 * tol);
    const double skip_rel2 = skip_rel * skip_rel;   // the threshold test squared: no sqrt per pair
    // this thread's pair blocks (qa <= qb) of the JBR == 1 update, fixed for the whole solve
    // (only the indices the pairs hold change between rounds): H (H + 1) / 2 <= 4656 blocks
    // for p <= 192, at most JMB per thread
    constexpr int JMB = 5;
    const int nblk = H * (H + 1) / 2;
    int bqa[JMB], bqb[JMB];
#pragma unroll
    for (int u = 0; u < JMB; ++u) {
        const int e = tid + u * NTH;
        bqa[u] = -1;
        bqb[u] = 0;
        if (JBR == 1 && e < nblk) {
            int qb = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
            if (qb * (qb + 1) / 2 > e) --qb;
            if ((qb + 1) * (qb + 2) / 2 <= e) ++qb;
            bqa[u] = e - qb * (qb + 1) / 2;
            bqb[u] = qb;
        }
    }
    // seat and next-round seat arrays swap roles every round (one barrier fewer than a copy)
    int* scur = seat;
    int* snxt = seat2;
    int sweep = 0;
    for (; sweep < max_sweeps; ++sweep) {
        double off = 0.0, dg = 0.0;
        for (int i = wid; i < p; i += (NTH / 64))
            for (int c = i + lane; c < p; c += 64) {
                const double v = a[pk(i, c)];
                if (c == i) dg += v * v; else off += 2.0 * v * v;
            }
        const double offs = block_sum_f64(off, red);
        const double dgs = block_sum_f64(dg, red);
        if (tid == 0) stop = (offs <= tol * tol * dgs) ? 1 : 0;
        __syncthreads();
        if (stop) break;
        for (int rd = 0; rd < P - 1; ++rd) {
            int act = 0;
            for (int k = tid; k < H; k += NTH) {
                const int se = scur[2 * k], so = scur[2 * k + 1];
                const int i = min(se, so), j = max(se, so);
                double c = 1.0, s = 0.0;
                if (j < p) {
                    const double aij = a[pk(i, j)];
                    const double aii = a[pk(i, i)], ajj = a[pk(j, j)];
                    // threshold Jacobi: elements below tol/100 of their diagonal scale are left
                    // alone (their total stays under the off-norm tolerance), so the last sweeps
                    // skip most pair-block updates
                    if (fabs(aij) > 1e-300 && aij * aij > skip_rel2 * fabs(aii * ajj)) {
                        const double th = (ajj - aii) / (2.0 * aij);
                        const double t = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(1.0 + th * th));
                        c = 1.0 / sqrt(1.0 + t * t);
                        s = t * c;
                        act = 1;
                    }
                }
                csn[k] = make_double2(c, s); lohi[k] = make_int4(i, j, pko(i), pko(j)); flp[k] = se > so;
                // seats of the next round (circle shift with fixed adjacent pairs)
                snxt[2 * k] = (k == 0) ? se : (k == 1) ? scur[1] : scur[2 * k - 2];
                snxt[2 * k + 1] = (k == H - 1) ? se : scur[2 * k + 3];
            }
            const bool any = __syncthreads_or(act);
            if (any) {
                // ---- A <- J^T A J on pair blocks (qa <= qb) in LDS
                if constexpr (JBR == 1) {
                    // one pair block at a time, few live values (V stays in registers); a
                    // pair's rotation and its indices with their row offsets are two 16-byte reads
#pragma unroll
                    for (int u = 0; u < JMB; ++u) {
                        const int qa = bqa[u], qb = bqb[u];
                        if (qa < 0) continue;
                        const double2 rca = csn[qa], rcb = csn[qb];
                        const double sa = rca.y, sb = rcb.y;
                        if (sa == 0.0 && sb == 0.0) continue;
                        const double ca = rca.x, cb = rcb.x;
                        const int4 pa = lohi[qa], pb = lohi[qb];
                        const int ia = pa.x, ja = pa.y, ib = pb.x, jb = pb.y;
                        const int oia = pa.z, oja = pa.w, oib = pb.z, ojb = pb.w;
                        const bool va = ja < p, vb = jb < p;
                        if (qa == qb) {
                            if (!va) continue;
                            const int o0 = pkx(ia, oia, ia, oia), o1 = pkx(ia, oia, ja, oja), o3 = pkx(ja, oja, ja, oja);
                            const double x0 = a[o0], x1 = a[o1], x3 = a[o3];
                            const double y00 = cb * x0 - sb * x1, y01 = sb * x0 + cb * x1;
                            const double y10 = cb * x1 - sb * x3, y11 = sb * x1 + cb * x3;
                            a[o0] = ca * y00 - sa * y10;
                            a[o3] = sa * y01 + ca * y11;
                            a[o1] = 0.0;
                        } else {
                            const int o0 = pkx(ia, oia, ib, oib);
                            const int o1 = vb ? pkx(ia, oia, jb, ojb) : -1;
                            const int o2 = va ? pkx(ja, oja, ib, oib) : -1;
                            const int o3 = (va && vb) ? pkx(ja, oja, jb, ojb) : -1;
                            const double x0 = a[o0];
                            const double x1 = o1 >= 0 ? a[o1] : 0.0;
                            const double x2 = o2 >= 0 ? a[o2] : 0.0;
                            const double x3 = o3 >= 0 ? a[o3] : 0.0;
                            const double y00 = cb * x0 - sb * x1, y01 = sb * x0 + cb * x1;
                            const double y10 = cb * x2 - sb * x3, y11 = sb * x2 + cb * x3;
                            a[o0] = ca * y00 - sa * y10;
                            if (o1 >= 0) a[o1] = ca * y01 - sa * y11;
                            if (o2 >= 0) a[o2] = sa * y00 + ca * y10;
                            if (o3 >= 0) a[o3] = sa * y01 + ca * y11;
                        }
                    }
                } else
                for (int e0 = tid; e0 < nblk; e0 += NTH * JBR) {
                    int o[JBR][4];
                    double x[JBR][4], ca[JBR], sa[JBR], cb[JBR], sb[JBR];
                    bool live[JBR], dgn[JBR];
#pragma unroll
                    for (int u = 0; u < JBR; ++u) {
                        const int e = e0 + u * NTH;
                        live[u] = false;
                        dgn[u] = false;
                        if (e < nblk) {
                            int qb = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
                            if (qb * (qb + 1) / 2 > e) --qb;
                            if ((qb + 1) * (qb + 2) / 2 <= e) ++qb;
                            const int qa = e - qb * (qb + 1) / 2;
                            ca[u] = csn[qa].x; sa[u] = csn[qa].y; cb[u] = csn[qb].x; sb[u] = csn[qb].y;
                            const int ia = lohi[qa].x, ja = lohi[qa].y, ib = lohi[qb].x, jb = lohi[qb].y;
                            const bool va = ja < p, vb = jb < p;
                            if ((sa[u] != 0.0 || sb[u] != 0.0) && (qa != qb || va)) {
                                live[u] = true;
                                dgn[u] = (qa == qb);
                                if (dgn[u]) {
                                    o[u][0] = pk(ia, ia); o[u][1] = pk(ia, ja);
                                    o[u][2] = o[u][1]; o[u][3] = pk(ja, ja);
                                } else {
                                    o[u][0] = pk(ia, ib);
                                    o[u][1] = vb ? pk(ia, jb) : -1;
                                    o[u][2] = va ? pk(ja, ib) : -1;
                                    o[u][3] = (va && vb) ? pk(ja, jb) : -1;
                                }
#pragma unroll
                                for (int w4 = 0; w4 < 4; ++w4) x[u][w4] = o[u][w4] >= 0 ? a[o[u][w4]] : 0.0;
                            }
                        }
                    }
#pragma unroll
                    for (int u = 0; u < JBR; ++u) {
                        if (!live[u]) continue;
                        const double y00 = cb[u] * x[u][0] - sb[u] * x[u][1], y01 = sb[u] * x[u][0] + cb[u] * x[u][1];
                        const double y10 = cb[u] * x[u][2] - sb[u] * x[u][3], y11 = sb[u] * x[u][2] + cb[u] * x[u][3];
                        if (dgn[u]) {
                            a[o[u][0]] = ca[u] * y00 - sa[u] * y10;
                            a[o[u][3]] = sa[u] * y01 + ca[u] * y11;
                            a[o[u][1]] = 0.0;
                        } else {
                            a[o[u][0]] = ca[u] * y00 - sa[u] * y10;
                            if (o[u][1] >= 0) a[o[u][1]] = ca[u] * y01 - sa[u] * y11;
                            if (o[u][2] >= 0) a[o[u][2]] = sa[u] * y00 + ca[u] * y10;
                            if (o[u][3] >= 0) a[o[u][3]] = sa[u] * y01 + ca[u] * y11;
                        }
                    }
                }
                // ---- V rotations (registers; skipped when only eigenvalues are wanted)
#pragma unroll
                for (int u = 0; u < PPT; ++u) {
                    if (!wantv) break;
                    const int k = k0 + u;
                    if (k < H) {
                        const float c = (float)csn[k].x, s = (float)csn[k].y;
                        if (s != 0.f) {
                            const bool f = flp[k] != 0;
#pragma unroll
                            for (int r = 0; r < RPT; ++r) {
                                const float e = ev[u][r], o2 = od[u][r];
                                if (!f) { ev[u][r] = c * e - s * o2; od[u][r] = s * e + c * o2; }
                                else { od[u][r] = c * o2 - s * e; ev[u][r] = s * o2 + c * e; }
                            }
                        }
                    }
                }
            }
            // ---- seat shift of V (every round, rotations or not)
#pragma unroll
            for (int r = 0; r < RPT; ++r) {
                if (!wantv) break;
                const float from_left = __shfl_up(ev[PPT - 1][r], 1, 32);   // ev of pair k0-1
                const float from_right = __shfl_down(od[0][r], 1, 32);      // od of pair k0+PPT
                float ne[PPT], no[PPT];
#pragma unroll
                for (int u = 0; u < PPT; ++u) {
                    const int k = k0 + u;
                    const float evm1 = (u == 0) ? from_left : ev[u - 1][r];
                    const float odp1 = (u == PPT - 1) ? from_right : od[u + 1][r];
                    ne[u] = (k == 0) ? ev[u][r] : (k == 1) ? od[u - (u > 0 ? 1 : 0)][r] : evm1;
                    no[u] = (k == H - 1) ? ev[u][r] : odp1;
                    if (k >= H) { ne[u] = ev[u][r]; no[u] = od[u][r]; }
                }
                // k == 1 with u == 0 needs od of pair 0 from the left neighbour
                const float od0_left = __shfl_up(od[PPT - 1][r], 1, 32);
                if (PPT == 1 && k0 == 1) ne[0] = od0_left;
#pragma unroll
                for (int u = 0; u < PPT; ++u) { ev[u][r] = ne[u]; od[u][r] = no[u]; }
            }
            // every thread is done with this round's pair data and A before the next round's
            // rotations read A and overwrite them; the next round reads snxt, written before the
            // round's first barrier, and writes the array read before it
            __syncthreads();
            int* const t2 = scur;
            scur = snxt;
            snxt = t2;
        }
    }
    if (tid == 0 && sweeps_out) sweeps_out[b] = sweep;
    for (int i = tid; i < p; i += NTH) {
        const double di = a[pk(i, i)];
        int rank = 0;
        for (int j = 0; j < p; ++j) {
            const double dj = a[pk(j, j)];
            rank += (dj > di) || (dj == di && j < i);
        }
        evals[b * p + rank] = di;
        rnk[i] = rank;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
        const int k = k0 + u;
        if (k >= H) continue;
        const int pe = scur[2 * k], po = scur[2 * k + 1];
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            const int x = x0 + r;
            if (x >= p) continue;
            if (pe < p) {
                if (V32) V32[b * (int64_t)p * p + x * p + rnk[pe]] = ev[u][r];
                if (V64) V64[b * (int64_t)p * p + x * p + rnk[pe]] = ev[u][r];
            }
            if (po < p) {
                if (V32) V32[b * (int64_t)p * p + x * p + rnk[po]] = od[u][r];
                if (V64) V64[b * (int64_t)p * p + x * p + rnk[po]] = od[u][r];
            }
        }
    }
}

static size_t jacobi_reg_bytes(int p) {
    const int P = p + (p & 1), H = P / 2;
    return (size_t)2 * H * sizeof(double) + (size_t)(5 * H + 3 * P + 1) * sizeof(int) + 8 +
           (size_t)p * (p + 1) / 2 * sizeof(double) + 16;
}

// ------------------------------------------------------------------ SPD whitening
// Symmetric Gaussian elimination S = L D L^T (rank-revealing: a pivot below rcond2 times the
// largest is dropped), E = L^{-1}; Wt = E^T D^{-1/2}.  One workgroup per matrix.
// LDL^T block form, nb = 32 pivots per panel J:
//   1. the 32 x 32 diagonal block in LDS, one barrier per pivot: pivots (rank-revealing drop
//      rule), L11^{-1};
//   2. panel rows of S right of the block, U12 = L11^{-1} S12, and the panel rows of
//      E = L^{-1} (columns < J + 32), Ep = L11^{-1} E_panel — v_mfma_f64_16x16x4f64 tiles of
//      32 rows x 16 columns (one wave per column block), written to the LDS panel (32 x p: Ep
//      in columns < J + 32, U12 right of them) and Ep also to E (U12 is read by this panel
//      only: S's panel rows are not written back);
//   3. trailing S (upper tiles) -= G^T U12 with G = diag(1/d) U12, trailing E rows -= G^T Ep,
//      both operands from the LDS panel; each wave takes its tiles two at a time with the
//      destination tiles' loads issued before the MFMAs.
// Three workgroup barriers per panel; S and E (fp64 p x p per matrix) stay in global memory
// (L2) and only the current panel's 32 rows live in LDS (256 p bytes: p <= ~560; larger p
// read the panel in place from L2, <false>).  Round 6: the trailing updates read their
// operands from the LDS panel instead of L2, two tiles per wave at a time (the same fp64
// values, MFMAs and sums in the same order: the same bits; p = 192 0.23 -> 0.18 ms at B = 1,
// 0.33 -> 0.24 ms at B = 256, tools/bench_whiten.py).
constexpr int kWmThreads = 512;
// LDS panel pitch in doubles, = 16 mod 32: of a 16 x 4 fragment read, rows k and k + 1 (one
// 32-lane half) fall on disjoint halves of the banks
__host__ __device__ inline int wm_pitch(int p) { return p + (48 - p % 32) % 32; }
constexpr int kWmWaves = kWmThreads / 64;


template <bool LP>   // LP: the panel rows in LDS (p <= 512); else read in place from L2 (any p)
__global__ __launch_bounds__(kWmThreads) void spd_whiten_mfma_kernel(double* __restrict__ S_all, int p, double rc2,
                                                                     double* __restrict__ E_all,
                                                                     float* __restrict__ W32, int* __restrict__ info) {
    extern __shared__ __attribute__((aligned(16))) double wm_smem[];
    double* piv = wm_smem;          // p pivots (inf for dropped)
    double* Li = piv + p;           // 32 x 33: L11^{-1} of the current panel (row-major, padded)
    double* rp = Li + 32 * 33;      // 32: 1 / pivot (0 for dropped) of the current panel
    double* Bk = rp + 32;           // 32 x 33: the diagonal block being factored
    const int pp = wm_pitch(p);     // LDS panel pitch
    double* PP = Bk + 32 * 33;      // 32 x pp: Ep (columns < J + 32) | U12 (columns >= J + 32)
    __shared__ int bad;
    __shared__ double dmax_s;
    __shared__ double red[16];
    const int64_t b = blockIdx.x;
    double* S = S_all + b * (int64_t)p * p;
    double* E = E_all + b * (int64_t)p * p;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int l16 = lane & 15, lk = lane >> 4;
    for (int i = wid; i < p; i += kWmWaves)
        for (int c = lane; c < p; c += 64) E[(int64_t)i * p + c] = (i == c) ? 1.0 : 0.0;
    double dm = 0.0;
    for (int j = tid; j < p; j += kWmThreads) dm = fmax(dm, fabs(S[(int64_t)j * p + j]));
    for (int o = 32; o > 0; o >>= 1) {
        const int2 x = __builtin_bit_cast(int2, dm);
        int2 y;
        y.x = __shfl_xor(x.x, o, 64);
        y.y = __shfl_xor(x.y, o, 64);
        dm = fmax(dm, __builtin_bit_cast(double, y));
    }
    if (lane == 0) red[wid] = dm;
    if (tid == 0) bad = 0;
    __syncthreads();
    if (tid == 0) {
        double m = 0.0;
        for (int w = 0; w < kWmWaves; ++w) m = fmax(m, red[w]);
        dmax_s = m;
    }
    __syncthreads();
    const double dmax = dmax_s;
    for (int J = 0; J < p; J += 32) {
        const int nb = min(32, p - J);
        const int t0 = J + nb;
        // ---- 1. diagonal block (wave 0)
        // the symmetric block (Bk) and L11^{-1} (Li) in LDS; thread (row r = tid / 16, columns
        // c = tid % 16 and c + 16) applies the row operation of pivot k to its elements: within a
        // step nothing it reads (row k, column k) is written, so one barrier per pivot
        {
            const int r = tid >> 4, c0 = tid & 15;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c = c0 + 16 * h;
                const int a = min(r, c), e = max(r, c);
                Bk[r * 33 + c] = (r < nb && c < nb) ? S[(int64_t)(J + a) * p + J + e] : 0.0;
                Li[r * 33 + c] = (c == r) ? 1.0 : 0.0;
            }
            __syncthreads();
            int nbad = 0;
            for (int k = 0; k < nb; ++k) {
                const double d = Bk[k * 33 + k];
                const bool drop = !(d > 1e-300 && d > dmax * rc2);
                nbad += drop;
                if (tid == 0) {
                    piv[J + k] = drop ? __longlong_as_double(0x7ff0000000000000ll) : d;
                    rp[k] = drop ? 0.0 : 1.0 / d;
                }
                if (!drop && r > k && r < nb) {
                    const double f = Bk[r * 33 + k] / d;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int c = c0 + 16 * h;
                        if (c > k && c < nb) Bk[r * 33 + c] -= f * Bk[k * 33 + c];
                        else if (c <= k) Li[r * 33 + c] -= f * Li[k * 33 + c];
                    }
                }
                __syncthreads();
            }
            if (tid == 0) bad += nbad;
        }
        __syncthreads();
        // ---- 2. U12 = L11^{-1} S12 (columns >= t0) and Ep = L11^{-1} E_panel (columns < t0)
        // into the LDS panel (Ep also to E); one wave per 16-column block, both 16-row halves
        const int ncs = (p - t0 + 15) / 16, nce = (t0 + 15) / 16;
        for (int cb = wid; cb < ncs + nce; cb += kWmWaves) {
            const bool isS = cb < ncs;
            double* M = isS ? S : E;
            const int c0 = isS ? t0 + 16 * cb : 16 * (cb - ncs);
            const int clim = isS ? p : t0;
            const int col = c0 + l16;
            f64x4v acc[2] = {f64x4v{0.0, 0.0, 0.0, 0.0}, f64x4v{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
            for (int k0 = 0; k0 < 32; k0 += 4) {
                const int k = k0 + lk;
                const double bv = (k < nb && col < clim) ? M[(int64_t)(J + k) * p + col] : 0.0;
                acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(Li[l16 * 33 + k], bv, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(Li[(16 + l16) * 33 + k], bv, acc[1], 0, 0, 0);
            }
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int k = 16 * h + lk + 4 * r;
                    if (col < clim) {
                        const double v = k < nb ? acc[h][r] : 0.0;
                        if (LP) PP[k * pp + col] = v;
                        if ((!isS || !LP) && k < nb) M[(int64_t)(J + k) * p + col] = v;
                    }
                }
        }
        __syncthreads();
        // ---- 3. trailing updates with G^T[i][k] = U12[k][i] / d_k:
        //   S[i][c] -= sum_k G^T[i][k] U12[k][c]  (16 x 16 tiles on or above the diagonal)
        //   E[i][c] -= sum_k G^T[i][k] Ep[k][c]   (rows i >= t0, columns c < t0)
        const int nt = (p - t0 + 15) / 16;
        const int nst = nt * (nt + 1) / 2, net = nt * nce;
        auto tile_of = [&](int t, int& i0, int& c0, double*& M) {
            if (t < nst) {  // upper tile (ti, tj), tj >= ti
                int tj = (int)((sqrtf(8.0f * (float)t + 1.0f) - 1.0f) * 0.5f);
                if (tj * (tj + 1) / 2 > t) --tj;
                if ((tj + 1) * (tj + 2) / 2 <= t) ++tj;
                i0 = t0 + 16 * (t - tj * (tj + 1) / 2);
                c0 = t0 + 16 * tj;
                M = S;
            } else {
                i0 = t0 + 16 * ((t - nst) / nce);
                c0 = 16 * ((t - nst) % nce);
                M = E;
            }
        };
        for (int t = wid; t < nst + net; t += 2 * kWmWaves) {
            const int tb = t + kWmWaves;
            const bool two = tb < nst + net;
            int i0[2] = {0, 0}, c0[2] = {0, 0};
            double* M[2] = {S, S};
            tile_of(t, i0[0], c0[0], M[0]);
            if (two) tile_of(tb, i0[1], c0[1], M[1]);
            double dv[2][4];
#pragma unroll
            for (int u = 0; u < 2; ++u) {   // the destination tiles first: their loads fly under the MFMAs
                const int clim = (M[u] == S) ? p : t0;
                const int col = c0[u] + l16;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = i0[u] + lk + 4 * r;
                    dv[u][r] = (u == 0 || two) && i < p && col < clim ? M[u][(int64_t)i * p + col] : 0.0;
                }
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                if (u == 1 && !two) break;
                const int clim = (M[u] == S) ? p : t0;
                const int col = c0[u] + l16, arow = i0[u] + l16;
                f64x4v acc = f64x4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int k0 = 0; k0 < 32; k0 += 4) {
                    const int k = k0 + lk;
                    const bool kv = k < nb;
                    const double av = (kv && arow < p) ? (LP ? PP[k * pp + arow] : S[(int64_t)(J + k) * p + arow]) * rp[k] : 0.0;
                    const double bv = (kv && col < clim) ? (LP ? PP[k * pp + col] : M[u][(int64_t)(J + k) * p + col]) : 0.0;
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = i0[u] + lk + 4 * r;
                    if (i < p && col < clim) M[u][(int64_t)i * p + col] = dv[u][r] - acc[r];
                }
            }
        }
        __syncthreads();
    }
    if (tid == 0) info[b] = bad;
    // Wt[a][c] = E[c][a] / sqrt(piv[c])  (upper triangular; 0 for dropped pivots); staged in S
    for (int a = wid; a < p; a += kWmWaves)
        for (int c = lane; c < p; c += 64) {
            const double v = (c >= a) ? E[(int64_t)c * p + a] / sqrt(piv[c]) : 0.0;
            if (W32) W32[b * (int64_t)p * p + (int64_t)a * p + c] = (float)v;
            S[(int64_t)a * p + c] = v;
        }
}

// ------------------------------------------------------------------ extreme Ritz values
// The cheap outer iterations of the rank-r solver only need the two ends of the Ritz spectrum
// (the filter's bounds theta_0 and its cut theta_{p-1}); a full Jacobi eigensolve for them
// (values only, off-norm 1e-2) costs several sweeps of a chain of rotations.  Here: `steps`
// Lanczos iterations on S = (T + T^T) / 2 held in LDS as fp32 (fp32 products over a quarter of
// the rows per wave, fp64 recurrences in wave 0: no barrier inside a reduction), then the
// extreme eigenvalues of the Lanczos tridiagonal by 64-point multisection on Sturm counts (fp64,
// to the last bit of the bracket).  They approach S's extremes from inside, to ~1e-6 relative
// after a few dozen steps even on flat spectra; a lost orthogonality only duplicates converged
// values.  One workgroup per matrix, deterministic (fixed start vector, fixed sum orders).
constexpr int kLzThreads = 256, kLzMaxP = 192, kLzMaxPG = 512, kLzMaxSteps = 64;

__device__ __forceinline__ int lz_sturm(const double* al, const double* b2, int m, double x) {
    int cnt = 0;
    double d = 1.0;
    for (int k = 0; k < m; ++k) {
        d = (al[k] - x) - (k > 0 ? b2[k] / d : 0.0);
        if (d == 0.0) d = -1e-300;
        cnt += d < 0.0;
    }
    return cnt;
}

// Q: 64-row groups per lane (p <= 64 Q).  GT: p > 192, T is read in place (fp64, L2-resident
// after the first step; S v from T's columns, the Rayleigh-Ritz matrix being symmetric to its
// rounding) instead of an fp32 copy of S in LDS
template <int Q, bool GT, int NT>
__global__ __launch_bounds__(NT) void extreme_eigs_kernel(const double* __restrict__ T_all, int p, int steps,
                                                         double* __restrict__ ends) {
    extern __shared__ __attribute__((aligned(16))) float lz_t[];   // S, p x p fp32 (row j at j p), !GT
    __shared__ float vf[64 * Q];                                   // current Lanczos vector (fp32 copy)
    __shared__ float part[NT / 64][64 * Q];                        // per-wave partial products
    __shared__ double al[kLzMaxSteps], b2[kLzMaxSteps];            // alpha_k, beta_k^2
    __shared__ int m_s;
    const int64_t b = blockIdx.x;
    const double* T = T_all + b * (int64_t)p * p;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if constexpr (!GT) {
        for (int e = tid; e < p * p; e += NT) lz_t[e] = (float)T[e];   // coalesced
        __syncthreads();
        for (int e = tid; e < p * p; e += NT) {   // S = (T + T^T) / 2, each pair once
            const int j = e / p, i = e % p;
            if (i < j) {
                const float v = 0.5f * (lz_t[e] + lz_t[i * p + j]);
                lz_t[e] = v;
                lz_t[i * p + j] = v;
            }
        }
    }
    // wave 0 owns the vectors: lane l holds entries l + 64 q (fp64)
    double v[Q], vp[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) v[q] = vp[q] = 0.0;
    if (wid == 0) {
        double ss = 0.0;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int i = lane + 64 * q;
            if (i < p) {
                uint32_t h = (uint32_t)i * 2654435761u ^ 0x9E3779B9u;
                h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15;
                v[q] = ((double)(h & 0xffffu) / 65536.0 + 0.5) * ((h & 0x10000u) ? 1.0 : -1.0);
                ss += v[q] * v[q];
            }
        }
        const double inv = 1.0 / sqrt(wave_sum(ss));
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            v[q] *= inv;
            if (lane + 64 * q < p) vf[lane + 64 * q] = (float)v[q];
        }
        if (lane == 0) m_s = steps;
    }
    __syncthreads();
    constexpr int NWV = NT / 64;
    const int jc = (p + NWV - 1) / NWV, j0 = wid * jc, j1 = min(p, j0 + jc);
    double beta = 0.0;
    for (int k = 0; k < steps; ++k) {
        // partial products of S v over this wave's rows j (S symmetric: column reads coalesce);
        // Q independent chains per lane (rows i = lane + 64 q; beyond p: row 0, unused), four
        // rows j per step so the reads of several j are in flight
        {
            int ii[Q];
            float a[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                ii[q] = lane + 64 * q < p ? lane + 64 * q : 0;
                a[q] = 0.f;
            }
            int j = j0;
            for (; j + 4 <= j1; j += 4) {
                float t[4][Q], vj[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    vj[u] = vf[j + u];
#pragma unroll
                    for (int q = 0; q < Q; ++q)
                        t[u][q] = GT ? (float)T[(int64_t)(j + u) * p + ii[q]] : lz_t[(j + u) * p + ii[q]];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int q = 0; q < Q; ++q) a[q] = __builtin_fmaf(t[u][q], vj[u], a[q]);
            }
            for (; j < j1; ++j) {
                const float vj = vf[j];
#pragma unroll
                for (int q = 0; q < Q; ++q)
                    a[q] = __builtin_fmaf(GT ? (float)T[(int64_t)j * p + ii[q]] : lz_t[j * p + ii[q]], vj, a[q]);
            }
#pragma unroll
            for (int q = 0; q < Q; ++q)
                if (lane + 64 * q < p) part[wid][lane + 64 * q] = a[q];
        }
        __syncthreads();
        if (wid == 0) {
            double w[Q], a = 0.0;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int i = lane + 64 * q;
                w[q] = 0.0;
                if (i < p) {
                    double acc = 0.0;
#pragma unroll
                    for (int wv = 0; wv < NWV; ++wv) acc += (double)part[wv][i];
                    w[q] = acc;
                    w[q] -= beta * vp[q];
                    a += w[q] * v[q];
                }
            }
            a = wave_sum(a);
            double ss = 0.0;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                w[q] -= a * v[q];
                ss += w[q] * w[q];
            }
            ss = wave_sum(ss);
            if (lane == 0) {
                al[k] = a;
                b2[k + 1 < kLzMaxSteps ? k + 1 : 0] = ss;
            }
            beta = sqrt(ss);
            // breakdown (an invariant subspace: its values are exact) or the last step
            const int stop = !(beta > 1e-30 * fabs(a)) || k + 1 == steps;
            if (stop && lane == 0) m_s = k + 1;
            const double inv = stop ? 0.0 : 1.0 / beta;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                vp[q] = v[q];
                v[q] = w[q] * inv;
                if (lane + 64 * q < p) vf[lane + 64 * q] = (float)v[q];
            }
        }
        __syncthreads();
        if (m_s != steps || k + 1 == steps) break;
    }
    // extreme eigenvalues of the m x m tridiagonal: wave 0 the largest, wave 1 the smallest
    const int m = m_s;
    if (wid < 2) {
        double lo = INFINITY, hi = -INFINITY;
        for (int k = 0; k < m; ++k) {
            const double r = (k > 0 ? sqrt(b2[k]) : 0.0) + (k + 1 < m ? sqrt(b2[k + 1]) : 0.0);
            lo = fmin(lo, al[k] - r);
            hi = fmax(hi, al[k] + r);
        }
        const double pad = 1e-12 * fmax(fabs(lo), fabs(hi)) + 1e-300;
        double a = lo - pad, c = hi + pad;   // count(a) = 0, count(c) = m
        bool bad = !(a == a) || !(c == c);
        for (int it = 0; it < 9 && !bad; ++it) {   // 65^-9 of the Gershgorin width: fp64 resolution
            const double x = a + (c - a) * (double)(lane + 1) / 65.0;
            const int cnt = lz_sturm(al, b2, m, x);
            if (wid == 0) {   // largest: the first x with every eigenvalue below it
                const uint64_t msk = __ballot(cnt == m);
                const int jf = msk ? __builtin_ctzll(msk) : 64;
                const double nc = jf < 64 ? a + (c - a) * (double)(jf + 1) / 65.0 : c;
                const double na = jf > 0 ? a + (c - a) * (double)jf / 65.0 : a;
                a = na; c = nc;
            } else {          // smallest: the last x with no eigenvalue below it
                const uint64_t msk = __ballot(cnt == 0);
                const int jl = __builtin_popcountll(msk);   // counts are monotone in x: a prefix
                const double na = jl > 0 ? a + (c - a) * (double)jl / 65.0 : a;
                const double nc = jl < 64 ? a + (c - a) * (double)(jl + 1) / 65.0 : c;
                a = na; c = nc;
            }
        }
        if (lane == 0) ends[2 * b + wid] = bad ? NAN : 0.5 * (a + c);
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

// Product-error estimate of the rank-r projection from the Ritz pairs (see cq_ritz_product_error):
// vector i's residual e_i tilts it toward eigenvectors outside the block by ~||e_i|| / gap_i
// (gap_i = theta_i - theta_{p-1}, the block's smallest Ritz value bounding the unconverged
// complement), which moves the projection of Y by that angle times sigma_i = sqrt(theta_i).
__global__ void ritz_prod_final_kernel(const double* part, int nchunks, int64_t p, int64_t r,
                                       const double* theta, const double* ysq, float* out) {
    __shared__ double red[16];
    const int64_t b = blockIdx.x;
    const double t0 = fabs(theta[b * p]), tp = theta[b * p + p - 1];
    double acc = 0.0;
    for (int64_t c = threadIdx.x; c < r; c += blockDim.x) {
        double s = 0.0;
        for (int t = 0; t < nchunks; ++t) s += part[(b * nchunks + t) * r + c];
        const double th = fmax(theta[b * p + c], 0.0);
        const double gap = fmax(th - tp, 1e-3 * t0);
        acc += s * th / (gap * gap);
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) a += red[i];
        const double y2 = ysq[b];
        out[b] = (float)(y2 > 0 ? sqrt(a / y2) : sqrt(a));
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
    const int64_t tot = batch * M * N;
    const unsigned rgrid = (unsigned)std::min<int64_t>(ceil_div(tot, 256), 4096);
    const bool al4 = lda % 4 == 0 && ldb % 4 == 0 && stride_a % 4 == 0 && stride_b % 4 == 0 &&
                     reinterpret_cast<uintptr_t>(A) % 16 == 0 && reinterpret_cast<uintptr_t>(B) % 16 == 0;
    if (al4 && trans_a == trans_b) {
        const int sym = (A == B && lda == ldb && stride_a == stride_b && M == N) ? 1 : 0;
        if (trans_a)
            gram_f64_mfma_kernel<true><<<grid, kGramThreads, 0, s>>>(M, N, K, kchunk, splits, A, lda, stride_a, B,
                                                                     ldb, stride_b, sym, reinterpret_cast<double*>(ws));
        else
            gram_f64_mfma_kernel<false><<<grid, kGramThreads, 0, s>>>(M, N, K, kchunk, splits, A, lda, stride_a, B,
                                                                      ldb, stride_b, sym, reinterpret_cast<double*>(ws));
        if (sym)
            gram_reduce_sym_kernel<<<rgrid, 256, 0, s>>>(reinterpret_cast<double*>(ws), M, splits, batch, C);
        else
            gram_reduce_kernel<<<rgrid, 256, 0, s>>>(reinterpret_cast<double*>(ws), M * N, splits, batch, C);
        return check_launch("cq_gram_f64");
    }
    gram_f64_kernel<<<grid, kGramThreads, 0, s>>>(M, N, K, kchunk, splits, A, trans_a, lda,
                                                   stride_a, B, trans_b, ldb, stride_b,
                                                   reinterpret_cast<double*>(ws));
    gram_reduce_kernel<<<rgrid, 256, 0, s>>>(reinterpret_cast<double*>(ws), M * N, splits, batch, C);
    return check_launch("cq_gram_f64");
}

int cq_spd_whiten(double* S, int64_t p, int64_t batch, float* Wt32, double* Wt64, int* info,
                  void* stream) {
    return cq_spd_whiten_rcond(S, p, batch, 1e-30, Wt32, Wt64, info, stream);
}

int cq_spd_whiten_rcond(double* S, int64_t p, int64_t batch, double rcond2, float* Wt32, double* Wt64, int* info,
                        void* stream) {
    CQ_REQUIRE(S && p > 0 && batch > 0 && info && Wt64, "cq_spd_whiten: bad args (Wt64 is required scratch)");
    CQ_REQUIRE(rcond2 >= 0.0, "cq_spd_whiten: rcond2 must be >= 0");
    hipStream_t s = as_stream(stream);
    // E is built in Wt64 (scratch); the final fp64 Wt is left in S (ABI 4: no device copy to
    // Wt64 -- the copy was 0.46 ms per B = 256, p = 192 call, ~18 ms per config-2 step)
    const size_t wsm = (size_t)(p + 2 * 32 * 33 + 32) * sizeof(double);
    const size_t wlm = wsm + (size_t)32 * wm_pitch((int)p) * sizeof(double);
    CQ_REQUIRE(wsm <= 64 * 1024, "cq_spd_whiten: p too large");
    if (wlm <= 150 * 1024)
        spd_whiten_mfma_kernel<true><<<(unsigned)batch, kWmThreads, wlm, s>>>(S, (int)p, rcond2, Wt64, Wt32, info);
    else
        spd_whiten_mfma_kernel<false><<<(unsigned)batch, kWmThreads, wsm, s>>>(S, (int)p, rcond2, Wt64, Wt32, info);
    return check_launch("cq_spd_whiten");
}

size_t cq_jacobi_workspace(int64_t p, int64_t batch) {
    if (p > kBlockJacobiMinP) return cq::bj_workspace(p, batch);
    return 16;  // the register/LDS kernel needs none
}

int cq_jacobi_eigh(double* A, int64_t p, int64_t batch, int max_sweeps, double tol, double* evals,
                   float* V32, double* V64, int* sweeps_out, void* ws, size_t ws_bytes,
                   void* stream) {
    CQ_REQUIRE(A && evals && p > 0 && batch > 0 && max_sweeps > 0, "cq_jacobi_eigh: bad args");
    CQ_REQUIRE(p <= 4096, "cq_jacobi_eigh: p too large");
    if (!ws || ws_bytes < cq_jacobi_workspace(p, batch))
        return set_error(CQ_EWORKSPACE, "cq_jacobi_eigh: workspace too small");
    hipStream_t s = as_stream(stream);
    if (p > kBlockJacobiMinP)  // A does not fit one CU's LDS: block Jacobi over many workgroups
        return cq::bj_eigh(A, p, batch, max_sweeps, tol, evals, V32, V64, sweeps_out, ws, ws_bytes, s);
    // p <= 192: fp64 A packed in LDS, V in registers (no per-round memory traffic for V)
    const size_t lreg = jacobi_reg_bytes((int)p);
    CQ_REQUIRE(lreg <= 160 * 1024, "cq_jacobi_eigh: LDS budget");
    if (p <= 64)
        jacobi_reg_kernel<1, 2, 2, 1024><<<(unsigned)batch, 1024, lreg, s>>>(A, (int)p, max_sweeps, tol, evals, V32, V64, sweeps_out);
    else if (p <= 128)
        jacobi_reg_kernel<2, 4, 2, 1024><<<(unsigned)batch, 1024, lreg, s>>>(A, (int)p, max_sweeps, tol, evals, V32, V64, sweeps_out);
    else
        jacobi_reg_kernel<3, 6, 1, 1024><<<(unsigned)batch, 1024, lreg, s>>>(A, (int)p, max_sweeps, tol, evals, V32, V64, sweeps_out);
    return check_launch("cq_jacobi_eigh");
}

size_t cq_jacobi_staged_workspace(int64_t p, int64_t batch) { return cq::bj_workspace(p, batch); }

int cq_jacobi_eigh_staged(double* A, int64_t p, int64_t batch, int phase, int nsweeps, double tol, int want_vectors,
                          double* evals, float* V32, double* V64, int* sweeps_out, int* pending_out, void* ws,
                          size_t ws_bytes, void* stream) {
    CQ_REQUIRE(A && p >= 2 && p <= 4096 && batch > 0, "cq_jacobi_eigh_staged: bad args");
    CQ_REQUIRE(phase > 0 && phase <= (BJ_BEGIN | BJ_SWEEPS | BJ_END), "cq_jacobi_eigh_staged: bad phase");
    CQ_REQUIRE(!(phase & BJ_SWEEPS) || nsweeps > 0, "cq_jacobi_eigh_staged: nsweeps must be > 0");
    CQ_REQUIRE(!(phase & BJ_END) || (evals && (!want_vectors || V32 || V64)), "cq_jacobi_eigh_staged: outputs");
    if (!ws || ws_bytes < cq_jacobi_staged_workspace(p, batch))
        return set_error(CQ_EWORKSPACE, "cq_jacobi_eigh_staged: workspace too small");
    return cq::bj_stage(A, p, batch, phase, nsweeps, tol, want_vectors != 0, evals, V32, V64, sweeps_out, pending_out,
                        ws, ws_bytes, as_stream(stream));
}

int cq_extreme_eigs(const double* T, int64_t p, int64_t batch, int steps, double* ends, void* stream) {
    CQ_REQUIRE(T && ends && p >= 2 && batch > 0 && batch <= 2147483647, "cq_extreme_eigs: bad args");
    CQ_REQUIRE(p <= kLzMaxPG, "cq_extreme_eigs: p > %d", kLzMaxPG);
    CQ_REQUIRE(steps >= 1 && steps < kLzMaxSteps, "cq_extreme_eigs: steps must be in [1, %d)", kLzMaxSteps);
    hipStream_t s = as_stream(stream);
    // p <= 192: S's fp32 copy in LDS, four waves; above: T read in place by sixteen waves (a
    // quarter of the rows each would leave each step's matvec latency-bound on L2), Q = the
    // 64-row groups p needs
    if (p <= kLzMaxP)
        extreme_eigs_kernel<3, false, kLzThreads><<<(unsigned)batch, kLzThreads, (size_t)p * p * sizeof(float), s>>>(
            T, (int)p, steps, ends);
    else if (p <= 320)
        extreme_eigs_kernel<5, true, 1024><<<(unsigned)batch, 1024, 0, s>>>(T, (int)p, steps, ends);
    else if (p <= 384)
        extreme_eigs_kernel<6, true, 1024><<<(unsigned)batch, 1024, 0, s>>>(T, (int)p, steps, ends);
    else
        extreme_eigs_kernel<8, true, 1024><<<(unsigned)batch, 1024, 0, s>>>(T, (int)p, steps, ends);
    return check_launch("cq_extreme_eigs");
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

int cq_ritz_product_error(const float* X, const float* Z, const double* theta, int64_t k, int64_t p, int64_t r,
                          int64_t batch, const double* ysq, float* out, void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(X && Z && theta && ysq && out && k > 0 && p > 0 && r > 0 && r < p,
               "cq_ritz_product_error: bad args");
    if (!ws || ws_bytes < cq_ritz_workspace(k, r, batch))
        return set_error(CQ_EWORKSPACE, "cq_ritz_product_error: workspace too small");
    hipStream_t s = as_stream(stream);
    const int64_t nch = std::min<int64_t>(64, std::max<int64_t>(1, k / 64));
    const int64_t rows_per = ceil_div(k, nch);
    double* part = reinterpret_cast<double*>(ws);
    ritz_partial_kernel<<<dim3((unsigned)nch, (unsigned)batch), 256, 0, s>>>(X, Z, theta, k, p, r, rows_per, part);
    ritz_prod_final_kernel<<<(unsigned)batch, 256, 0, s>>>(part, (int)nch, p, r, theta, ysq, out);
    return check_launch("cq_ritz_product_error");
}

}  // extern "C"
