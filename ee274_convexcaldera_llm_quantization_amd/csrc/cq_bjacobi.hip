// Block Jacobi symmetric eigensolver spread over many workgroups per matrix, for the
// Rayleigh-Ritz matrices that do not fit one CU's LDS (p > 192: rank 256 at config 5,
// p = 384; rank 200 in main.py:176, p = 288).  Replaces the one-CU global-memory Jacobi
// (cq_small.hip jacobi_kernel), which serialised a p = 384 solve on one CU at ~77 ms.
//
// The p indices are cut into nblk blocks of NB = 32.  A sweep is nblk - 1 steps of the
// round-robin pairing of blocks; in a step every pair (a, c) forms a 64 x 64 subproblem:
//   bj_solve_kernel   (one workgroup per pair): the subproblem A[P, P] (P = a u c) lives in
//                     LDS and is diagonalised by cyclic two-sided Jacobi (threshold rotations,
//                     the same rule as the one-CU kernels); it writes back the diagonalised
//                     block and V_P (64 x 64, fp64);
//   bj_update_kernel  (one workgroup per off-diagonal pair-block (P, Q), plus one per pair
//                     for the eigenvector rows): A[P, Q] <- V_P^T A[P, Q] V_Q, Vt[P, :] <-
//                     V_P^T Vt[P, :].  Blocks whose pairs did not rotate are left alone.
// Both kernels also leave per-block off-diagonal / diagonal square sums; bj_check_kernel
// turns them into the per-matrix stop test off^2 <= tol^2 sum a_ii^2 after every sweep
// (a converged matrix's later workgroups exit at entry; the caller's sweep budget bounds the
// launches, no host synchronisation inside).  Everything is fp64.
#include "cq_common.h"

namespace cq {
namespace {

constexpr int NB = 32;        // block size
constexpr int D = 2 * NB;     // subproblem dimension
constexpr int LDP = D + 1;    // padded LDS row (fp64): column walks hit different banks
constexpr int BT = 256;       // threads per workgroup
#ifndef CQ_BJ_INNER
#define CQ_BJ_INNER 1
#endif
constexpr int kInnerMax = CQ_BJ_INNER;  // inner sweeps per subproblem and step (partial solves: see DESIGN.md)

// round-robin pairing of n (even) items, round rd, slot q: (i < j)
__device__ __forceinline__ void rr(int n, int rd, int q, int& i, int& j) {
    const int n1 = n - 1;
    if (q == 0) { i = n1; j = rd; }
    else {
        i = rd + q; if (i >= n1) i -= n1;
        j = rd - q; if (j < 0) j += n1;
    }
    if (i > j) { const int t = i; i = j; j = t; }
}

// global index of subproblem row u for the pair (a, c) of blocks; -1 past p (or a virtual
// block when nblk was rounded up to even)
__device__ __forceinline__ int gidx(int a, int c, int u, int p) {
    const int g = (u < NB ? a : c) * NB + (u & (NB - 1));
    return g < p ? g : -1;
}

// 1 / x and 1 / sqrt(x) from the hardware seeds (v_rcp_f64, v_rsq_f64) and two Newton steps
// each: ~1 ulp, without the correctly rounded division / square-root sequences (round 6:
// the 32 rotations of a subproblem round are a serial step between two barriers)
__device__ __forceinline__ double nr_rcp(double x) {
    double y = __builtin_amdgcn_rcp(x);
    y = __builtin_fma(__builtin_fma(-x, y, 1.0), y, y);
    return __builtin_fma(__builtin_fma(-x, y, 1.0), y, y);
}
__device__ __forceinline__ double nr_rsq(double x) {   // x >= 1 here
    double y = __builtin_amdgcn_rsq(x);
    y = __builtin_fma(0.5 * y, __builtin_fma(-x * y, y, 1.0), y);
    return __builtin_fma(0.5 * y, __builtin_fma(-x * y, y, 1.0), y);
}

// the rotation that annihilates a_ij: th = (a_jj - a_ii) / (2 a_ij), t = sgn(th) / (|th| +
// sqrt(1 + th^2)), c = 1 / sqrt(1 + t^2), s = t c (c^2 + s^2 = 1 to a few ulp: the rotation
// stays orthogonal; the annihilation itself need not be exact)
__device__ __forceinline__ void rot_params(double aii, double ajj, double aij, double thr, double& c, double& s) {
    c = 1.0; s = 0.0;
    if (fabs(aij) > 1e-300 && aij * aij > (thr * thr) * fabs(aii * ajj)) {
        const double th = (ajj - aii) * nr_rcp(2.0 * aij);
        const double q = 1.0 + th * th;   // (|th| > 1e100: t = 1 / (2 th), th^2 would overflow)
        const double t = fabs(th) > 1e100 ? 0.5 * nr_rcp(th) : (th >= 0 ? 1.0 : -1.0) * nr_rcp(fabs(th) + q * nr_rsq(q));
        c = nr_rsq(1.0 + t * t);
        s = t * c;
    }
}

// NT threads per matrix: 256, or 1024 for small batches (one caldera() call: these one-matrix
// passes over p^2 elements are memory-latency chains on one CU)
template <int NT>
__global__ __launch_bounds__(NT) void bj_init_kernel(double* __restrict__ A_all, int p, double* __restrict__ Vt_all,
                                                     int* __restrict__ done, int* __restrict__ sweeps,
                                                     double tol) {
    const int64_t b = blockIdx.x;
    double* A = A_all + b * (int64_t)p * p;
    __shared__ double red[16];
    double off = 0.0, dg = 0.0;
    for (int64_t t = threadIdx.x; t < (int64_t)p * p; t += NT) {
        const int i = (int)(t / p), c = (int)(t % p);
        if (Vt_all) Vt_all[b * (int64_t)p * p + t] = (i == c) ? 1.0 : 0.0;
        if (i < c) {  // symmetrise (Rayleigh-Ritz matrices carry rounding asymmetry)
            const double s = 0.5 * (A[(int64_t)i * p + c] + A[(int64_t)c * p + i]);
            A[(int64_t)i * p + c] = s;
            A[(int64_t)c * p + i] = s;
            off += 2.0 * s * s;
        } else if (i == c) {
            const double v = A[(int64_t)i * p + i];
            dg += v * v;
        }
    }
    const double offs = block_sum_f64(off, red);
    const double dgs = block_sum_f64(dg, red);
    if (threadIdx.x == 0) {
        done[b] = (offs <= tol * tol * dgs) ? 1 : 0;
        sweeps[b] = 0;
    }
}

// One workgroup per (pair q, matrix b): diagonalise the 64 x 64 subproblem in LDS.  ST threads:
// 256, or 1024 when the launch has fewer subproblems than the chip has CUs (a single caldera()
// call: 3 pairs at p = 192), so each round's rotation updates take a quarter of the time
// (every element is updated by one thread with the same arithmetic either way).
template <int ST>
__global__ __launch_bounds__(ST) void bj_solve_kernel(double* __restrict__ A_all, int p, int nblk, int step,
                                                      double thr, double* __restrict__ Vs_all,
                                                      int* __restrict__ rot_all, const int* __restrict__ done,
                                                      double* __restrict__ part_off, double* __restrict__ part_dg,
                                                      int nslots) {
    const int q = blockIdx.x, npair = nblk / 2;
    const int64_t b = blockIdx.y;
    if (done[b]) return;
    __shared__ double As[D * LDP];
    __shared__ double Vsm[D * LDP];
    __shared__ double2 csn[NB];   // (cos, sin) of slot q's rotation: one 16-byte read
    __shared__ int2 pij[NB];      // its (i, j): one 8-byte read
    __shared__ int gi[D];
    __shared__ int any_rot;
    __shared__ double red[16];
    const int tid = threadIdx.x;
    double* A = A_all + b * (int64_t)p * p;
    int a, c;
    rr(nblk, step, q, a, c);
    if (tid < D) gi[tid] = gidx(a, c, tid, p);
    __syncthreads();
    for (int t = tid; t < D * D; t += ST) {
        const int u = t / D, v = t % D;
        const int gu = gi[u], gv = gi[v];
        As[u * LDP + v] = (gu >= 0 && gv >= 0) ? A[(int64_t)gu * p + gv] : 0.0;
        Vsm[u * LDP + v] = (u == v) ? 1.0 : 0.0;
    }
    __syncthreads();
    int rotated = 0;
    for (int inner = 0; inner < kInnerMax; ++inner) {
        if (tid == 0) any_rot = 0;
        __syncthreads();
        for (int rd = 0; rd < D - 1; ++rd) {
            if (tid < NB) {
                int i, j;
                rr(D, rd, tid, i, j);
                double cc, ss;
                rot_params(As[i * LDP + i], As[j * LDP + j], As[i * LDP + j], thr, cc, ss);
                if (ss != 0.0) any_rot = 1;
                csn[tid] = make_double2(cc, ss); pij[tid] = make_int2(i, j);
            }
            __syncthreads();
            // A <- J^T A J on the 32 x 32 pair-blocks (each element belongs to one block)
            for (int t = tid; t < NB * NB; t += ST) {
                const int qa = t / NB, qb = t % NB;
                const double2 ra = csn[qa], rb = csn[qb];
                const double sa = ra.y, sb = rb.y;
                if (sa == 0.0 && sb == 0.0) continue;
                const double ca = ra.x, cb = rb.x;
                const int2 ea = pij[qa], eb = pij[qb];
                const int ia = ea.x, ja = ea.y, ib = eb.x, jb = eb.y;
                const double x00 = As[ia * LDP + ib], x01 = As[ia * LDP + jb];
                const double x10 = As[ja * LDP + ib], x11 = As[ja * LDP + jb];
                const double y00 = cb * x00 - sb * x01, y01 = sb * x00 + cb * x01;
                const double y10 = cb * x10 - sb * x11, y11 = sb * x10 + cb * x11;
                double z00 = ca * y00 - sa * y10, z10 = sa * y00 + ca * y10;
                double z01 = ca * y01 - sa * y11, z11 = sa * y01 + ca * y11;
                if (qa == qb) { z01 = 0.0; z10 = 0.0; }  // the annihilated pair
                As[ia * LDP + ib] = z00; As[ia * LDP + jb] = z01;
                As[ja * LDP + ib] = z10; As[ja * LDP + jb] = z11;
            }
            // V <- V J (columns i, j of every row)
            for (int t = tid; t < D * NB; t += ST) {
                const int u = t / NB, qq = t % NB;
                const double2 rq = csn[qq];
                const double ss = rq.y;
                if (ss == 0.0) continue;
                const double cc = rq.x;
                const int2 eq = pij[qq];
                const int i = eq.x, j = eq.y;
                const double vi = Vsm[u * LDP + i], vj = Vsm[u * LDP + j];
                Vsm[u * LDP + i] = cc * vi - ss * vj;
                Vsm[u * LDP + j] = ss * vi + cc * vj;
            }
            __syncthreads();
        }
        const int anyr = any_rot;
        __syncthreads();
        if (!anyr) break;
        rotated = 1;
    }
    // write back the (block-)diagonalised subproblem, its V, and its square sums
    double off = 0.0, dg = 0.0;
    for (int t = tid; t < D * D; t += ST) {
        const int u = t / D, v = t % D;
        const int gu = gi[u], gv = gi[v];
        if (gu < 0 || gv < 0) continue;
        const double x = As[u * LDP + v];
        if (rotated) A[(int64_t)gu * p + gv] = x;
        if (u == v) dg += x * x; else off += x * x;
    }
    double* Vs = Vs_all + (b * npair + q) * (int64_t)(D * D);
    if (rotated)
        for (int t = tid; t < D * D; t += ST) Vs[t] = Vsm[(t / D) * LDP + (t % D)];
    const double offs = block_sum_f64(off, red);
    const double dgs = block_sum_f64(dg, red);
    if (tid == 0) {
        rot_all[b * npair + q] = rotated;
        part_off[b * nslots + q] = offs;
        part_dg[b * npair + q] = dgs;
    }
}

// 64 x 64 x 64 fp64 product C = X Y on v_mfma_f64_16x16x4f64 (products and sums in fp64,
// as the fp64 FMA loop it replaces): wave w owns the 32 x 32 quadrant (rows 32 (w >> 1),
// columns 32 (w & 1)) as 2 x 2 tiles; xa(i, k) / yb(k, j) fetch the operands (global/L2 or
// LDS).  Result C[32 (w >> 1) + 16 ti + (lane >> 4) + 4 r][32 (w & 1) + 16 tj + (lane & 15)]
// = acc[ti][tj][r] (the f64 MFMA's C/D map).
using f64x4v = __attribute__((ext_vector_type(4))) double;

template <class FX, class FY>
__device__ __forceinline__ void mfma64(FX xa, FY yb, f64x4v (&acc)[2][2], int wid, int lane) {
    const int ri = 32 * (wid >> 1), cj = 32 * (wid & 1), l16 = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f64x4v{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int k0 = 0; k0 < D; k0 += 4) {
        const int k = k0 + lk;
        const double a0 = xa(ri + l16, k), a1 = xa(ri + 16 + l16, k);
        const double b0 = yb(k, cj + l16), b1 = yb(k, cj + 16 + l16);
        acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
}

// Workgroups [0, npair*(npair-1)): off-diagonal pair-block (P, Q), A[P,Q] <- V_P^T A[P,Q] V_Q
// (operands straight from L2 into the MFMAs; T = V_P^T A[P,Q] re-laid out through LDS).
// Workgroups [npair*(npair-1), + npair * nch) (with eigenvectors): Vt[P, x0:x0+64] <-
// V_P^T Vt[P, x0:x0+64], one 64-column chunk each.  33 KB of LDS: several workgroups per CU.
__global__ __launch_bounds__(BT) void bj_update_kernel(double* __restrict__ A_all, int p, int nblk, int step,
                                                       const double* __restrict__ Vs_all,
                                                       const int* __restrict__ rot_all, const int* __restrict__ done,
                                                       double* __restrict__ Vt_all, double* __restrict__ part_off,
                                                       int nslots) {
    const int npair = nblk / 2, noff = npair * (npair - 1);
    const int w = blockIdx.x;
    const int64_t b = blockIdx.y;
    if (done[b]) return;
    __shared__ double Ms[D * LDP];
    __shared__ int gP[D], gQ[D];
    __shared__ double red[16];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int ri = 32 * (wid >> 1), cj = 32 * (wid & 1), l16 = lane & 15, lk = lane >> 4;
    double* A = A_all + b * (int64_t)p * p;
    const int* rot = rot_all + b * npair;
    const double* Vs = Vs_all + b * npair * (int64_t)(D * D);
    f64x4v acc[2][2];
    if (w < noff) {
        const int P = w / (npair - 1);
        int Q = w % (npair - 1);
        if (Q >= P) ++Q;
        int a, c, e, f;
        rr(nblk, step, P, a, c);
        rr(nblk, step, Q, e, f);
        if (tid < D) { gP[tid] = gidx(a, c, tid, p); gQ[tid] = gidx(e, f, tid, p); }
        __syncthreads();
        const bool rp = rot[P] != 0, rq = rot[Q] != 0;
        auto apq = [&](int k, int j) -> double {
            const int gu = gP[k], gv = gQ[j];
            return (gu >= 0 && gv >= 0) ? A[(int64_t)gu * p + gv] : 0.0;
        };
        double off = 0.0;
        if (rp || rq) {
            const double* VP = Vs + (int64_t)P * D * D;
            const double* VQ = Vs + (int64_t)Q * D * D;
            if (rp) {  // T = V_P^T A_PQ into Ms
                mfma64([&](int i, int k) { return VP[k * D + i]; }, apq, acc, wid, lane);
#pragma unroll
                for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            Ms[(ri + 16 * ti + lk + 4 * r) * LDP + cj + 16 * tj + l16] = acc[ti][tj][r];
            } else {
                for (int t = tid; t < D * D; t += BT) Ms[(t / D) * LDP + (t % D)] = apq(t / D, t % D);
            }
            __syncthreads();
            if (rq) {  // C = T V_Q
                mfma64([&](int i, int k) { return Ms[i * LDP + k]; }, [&](int k, int j) { return VQ[k * D + j]; },
                       acc, wid, lane);
            } else {
#pragma unroll
                for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                    for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            acc[ti][tj][r] = Ms[(ri + 16 * ti + lk + 4 * r) * LDP + cj + 16 * tj + l16];
            }
#pragma unroll
            for (int ti = 0; ti < 2; ++ti)
#pragma unroll
                for (int tj = 0; tj < 2; ++tj)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int gu = gP[ri + 16 * ti + lk + 4 * r], gv = gQ[cj + 16 * tj + l16];
                        if (gu >= 0 && gv >= 0) {
                            const double x = acc[ti][tj][r];
                            A[(int64_t)gu * p + gv] = x;
                            off += x * x;
                        }
                    }
        } else {
            for (int t = tid; t < D * D; t += BT) {
                const double x = apq(t / D, t % D);
                off += x * x;
            }
        }
        const double offs = block_sum_f64(off, red);
        if (tid == 0) part_off[b * nslots + npair + w] = offs;
        return;
    }
    // eigenvector rows of pair P, one 64-column chunk
    const int nch = (p + D - 1) / D;
    const int P = (w - noff) / nch, x0 = ((w - noff) % nch) * D;
    if (!Vt_all || !rot[P]) return;
    int a, c;
    rr(nblk, step, P, a, c);
    if (tid < D) gP[tid] = gidx(a, c, tid, p);
    __syncthreads();
    const double* VP = Vs + (int64_t)P * D * D;
    double* Vt = Vt_all + b * (int64_t)p * p;
    mfma64([&](int i, int k) { return VP[k * D + i]; },
           [&](int k, int l) {
               const int gu = gP[k];
               return (gu >= 0 && x0 + l < p) ? Vt[(int64_t)gu * p + x0 + l] : 0.0;
           },
           acc, wid, lane);
    __syncthreads();  // every wave has read the chunk's rows before any is overwritten
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
        for (int tj = 0; tj < 2; ++tj)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gu = gP[ri + 16 * ti + lk + 4 * r], l = cj + 16 * tj + l16;
                if (gu >= 0 && x0 + l < p) Vt[(int64_t)gu * p + x0 + l] = acc[ti][tj][r];
            }
}

__global__ void bj_check_kernel(const double* __restrict__ part_off, const double* __restrict__ part_dg, int nslots,
                                int npair, double tol, int* __restrict__ done, int* __restrict__ sweeps) {
    const int64_t b = blockIdx.x;
    if (done[b]) return;
    __shared__ double red[16];
    double off = 0.0, dg = 0.0;
    for (int i = threadIdx.x; i < nslots; i += blockDim.x) off += part_off[b * nslots + i];
    for (int i = threadIdx.x; i < npair; i += blockDim.x) dg += part_dg[b * npair + i];
    const double offs = block_sum_f64(off, red);
    const double dgs = block_sum_f64(dg, red);
    if (threadIdx.x == 0) {
        sweeps[b] += 1;
        if (offs <= tol * tol * dgs) done[b] = 1;
    }
}

// Descending eigenvalues by rank counting (ties by index); column rank(i) of V = Vt row i.
template <int NT>
__global__ __launch_bounds__(NT) void bj_finish_kernel(const double* __restrict__ A_all, int p,
                                                       const double* __restrict__ Vt_all, double* __restrict__ evals,
                                                       float* __restrict__ V32, double* __restrict__ V64,
                                                       const int* __restrict__ sweeps, int* __restrict__ sweeps_out,
                                                       int* __restrict__ rank_ws) {
    extern __shared__ double fdg[];   // the diagonal (p values): the ranks read it p times
    const int64_t b = blockIdx.x;
    const double* A = A_all + b * (int64_t)p * p;
    int* rk = rank_ws + b * (int64_t)p;
    for (int i = threadIdx.x; i < p; i += NT) fdg[i] = A[(int64_t)i * p + i];
    __syncthreads();
    for (int i = threadIdx.x; i < p; i += NT) {
        const double di = fdg[i];
        int r = 0;
        for (int j = 0; j < p; ++j) {
            const double dj = fdg[j];
            r += (dj > di) || (dj == di && j < i);
        }
        evals[b * p + r] = di;
        rk[i] = r;
    }
    if (threadIdx.x == 0 && sweeps_out) sweeps_out[b] = sweeps[b];
    if (!Vt_all) return;
    __syncthreads();
    const double* Vt = Vt_all + b * (int64_t)p * p;
    for (int64_t t = threadIdx.x; t < (int64_t)p * p; t += NT) {
        const int i = (int)(t / p), x = (int)(t % p);
        const double v = Vt[t];
        if (V32) V32[b * (int64_t)p * p + (int64_t)x * p + rk[i]] = (float)v;
        if (V64) V64[b * (int64_t)p * p + (int64_t)x * p + rk[i]] = v;
    }
}

}  // namespace

size_t bj_workspace(int64_t p, int64_t batch) {
    const int64_t nblk = ceil_div(p, NB) + (ceil_div(p, NB) & 1);
    const int64_t npair = nblk / 2;
    const int64_t nslots = npair + npair * (npair - 1);
    size_t s = align_up((size_t)batch * p * p * sizeof(double), 256);           // Vt
    s += align_up((size_t)batch * npair * D * D * sizeof(double), 256);           // V_P
    s += align_up((size_t)batch * nslots * sizeof(double), 256);                  // off partials
    s += align_up((size_t)batch * npair * sizeof(double), 256);                   // dg partials
    s += align_up((size_t)batch * npair * sizeof(int), 256);                      // rotated
    s += align_up((size_t)batch * sizeof(int), 256) * 2;                          // done, sweeps
    s += align_up((size_t)batch * p * sizeof(int), 256);                          // ranks
    return s;
}

__global__ void bj_pending_kernel(const int* __restrict__ done, int64_t batch, int* __restrict__ pending) {
    int c = 0;
    for (int64_t b = threadIdx.x; b < batch; b += blockDim.x) c += done[b] ? 0 : 1;
    c = wave_sum(c);
    if (threadIdx.x == 0) *pending = c;
}

// Block-Jacobi eigensolver in stages, every stage stream-ordered (no host read-back inside):
//   BJ_BEGIN   V = I, per-matrix done flags and sweep counts cleared;
//   BJ_SWEEPS  nsweeps sweeps; a matrix whose off-norm test passed (bj_check_kernel) has
//              done[b] set and every later workgroup of it exits at entry; pending_out (device
//              int, optional) = matrices still unconverged after these sweeps;
//   BJ_END     eigenvalues (descending) and eigenvectors out, per-matrix sweep counts.
// The state (A in place, Vt, flags) lives in the caller's workspace between stages, so a
// caller that reads pending_out can launch further sweeps only where they are needed.
int bj_stage(double* A, int64_t p, int64_t batch, int phase, int nsweeps, double tol, bool want_v, double* evals,
             float* V32, double* V64, int* sweeps_out, int* pending_out, void* ws, size_t ws_bytes, hipStream_t s) {
    if (ws_bytes < bj_workspace(p, batch)) return set_error(CQ_EWORKSPACE, "cq_jacobi_eigh: workspace too small");
    const int nblk = (int)(ceil_div(p, NB) + (ceil_div(p, NB) & 1));
    const int npair = nblk / 2, noff = npair * (npair - 1), nslots = npair + noff;
    const int nch = (int)ceil_div(p, D);  // 64-column chunks of the eigenvector rows
    char* w = reinterpret_cast<char*>(ws);
    auto take = [&](size_t bytes) { char* r = w; w += align_up(bytes, 256); return r; };
    double* Vt = reinterpret_cast<double*>(take((size_t)batch * p * p * sizeof(double)));
    double* Vs = reinterpret_cast<double*>(take((size_t)batch * npair * D * D * sizeof(double)));
    double* poff = reinterpret_cast<double*>(take((size_t)batch * nslots * sizeof(double)));
    double* pdg = reinterpret_cast<double*>(take((size_t)batch * npair * sizeof(double)));
    int* rot = reinterpret_cast<int*>(take((size_t)batch * npair * sizeof(int)));
    int* done = reinterpret_cast<int*>(take((size_t)batch * sizeof(int)));
    int* sweeps = reinterpret_cast<int*>(take((size_t)batch * sizeof(int)));
    int* ranks = reinterpret_cast<int*>(take((size_t)batch * p * sizeof(int)));
    const double thr = fmax(1e-17, 0.5 * tol / sqrt((double)p));
    if (phase & BJ_BEGIN)
    {
        if (batch < kCUs)
            bj_init_kernel<1024><<<(unsigned)batch, 1024, 0, s>>>(A, (int)p, want_v ? Vt : nullptr, done, sweeps, tol);
        else
            bj_init_kernel<BT><<<(unsigned)batch, BT, 0, s>>>(A, (int)p, want_v ? Vt : nullptr, done, sweeps, tol);
    }
    if (phase & BJ_SWEEPS) {
        for (int sw = 0; sw < nsweeps; ++sw) {
            for (int st = 0; st < nblk - 1; ++st) {
                if (npair * batch < kCUs)
                    bj_solve_kernel<1024><<<dim3((unsigned)npair, (unsigned)batch), 1024, 0, s>>>(
                        A, (int)p, nblk, st, thr, Vs, rot, done, poff, pdg, nslots);
                else
                    bj_solve_kernel<BT><<<dim3((unsigned)npair, (unsigned)batch), BT, 0, s>>>(
                        A, (int)p, nblk, st, thr, Vs, rot, done, poff, pdg, nslots);
                const int nupd = noff + (want_v ? npair * nch : 0);   // 0: one pair, values only
                if (nupd > 0)
                    bj_update_kernel<<<dim3((unsigned)nupd, (unsigned)batch), BT, 0, s>>>(
                        A, (int)p, nblk, st, Vs, rot, done, want_v ? Vt : nullptr, poff, nslots);
            }
            bj_check_kernel<<<(unsigned)batch, 64, 0, s>>>(poff, pdg, nslots, npair, tol, done, sweeps);
        }
        if (pending_out) bj_pending_kernel<<<1, 64, 0, s>>>(done, batch, pending_out);
    }
    if (phase & BJ_END)
    {
        const size_t fl = (size_t)p * sizeof(double);
        if (batch < kCUs)
            bj_finish_kernel<1024><<<(unsigned)batch, 1024, fl, s>>>(A, (int)p, want_v ? Vt : nullptr, evals, V32, V64,
                                                                     sweeps, sweeps_out, ranks);
        else
            bj_finish_kernel<BT><<<(unsigned)batch, BT, fl, s>>>(A, (int)p, want_v ? Vt : nullptr, evals, V32, V64,
                                                                 sweeps, sweeps_out, ranks);
    }
    return check_launch("cq_jacobi_eigh (block Jacobi)");
}

int bj_eigh(double* A, int64_t p, int64_t batch, int max_sweeps, double tol, double* evals, float* V32,
            double* V64, int* sweeps_out, void* ws, size_t ws_bytes, hipStream_t s) {
    return bj_stage(A, p, batch, BJ_BEGIN | BJ_SWEEPS | BJ_END, max_sweeps, tol, V32 || V64, evals, V32, V64,
                    sweeps_out, nullptr, ws, ws_bytes, s);
}

}  // namespace cq
