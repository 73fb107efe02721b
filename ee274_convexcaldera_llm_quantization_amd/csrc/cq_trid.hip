// Symmetric eigensolver for the Rayleigh-Ritz matrices with p <= 192 (cq_jacobi_eigh's
// default path there): Householder reduction to tridiagonal form, eigenvalues by bisection on
// Sturm counts, eigenvectors of the tridiagonal by twisted factorisations, back-transformation
// by the stored reflectors.  Replaces the one-CU cyclic Jacobi, whose p/2 rotations per round
// hit LDS banks at random (the circle-method pairs are scattered in index space) and whose
// 4-8 sweeps cost ~5 ms per batch at p = 192; here every step walks rows of A contiguously.
//
//   trd_kernel   (4 waves per matrix; A packed upper in LDS, 148 KB at p = 192): for
//                j = 0..p-3 the reflector H_j = I - tau v v^T (v[j+1] = 1, LAPACK dlarfg)
//                annihilating A[j][j+2..], then y = tau A' v (per-wave column sums over
//                interleaved rows with lane-owned outputs + 8-lane row dot products),
//                w = y - (tau/2)(y.v) v and the rank-2 update A' -= v w^T + w v^T; every
//                access walks a row of the packed triangle.  Writes d, e, tau and the
//                reflectors (column j of H).
//   tri_eig_kernel  eigenvalue i (descending) by bisection (thread i, Sturm counts with
//                LAPACK's pivmin safeguard); with vectors, the twisted factorisation of
//                T - lambda I (forward LDL^T, backward UDU^T, twist at min |gamma|) gives the
//                eigenvector, normalised into V32.  A relative gap below 1e-9 flags the
//                matrix (inverse-iteration vectors of a near-degenerate pair are not
//                orthogonal): the host then reruns the batch on the Jacobi path.
//   trd_back_kernel  V = H_0 ... H_{p-3} Z with Z in LDS (fp32 storage, fp64 arithmetic).
// Everything before the fp32 eigenvector storage is fp64.
#include "cq_common.h"

namespace cq {
namespace {

constexpr int kTriThreads = 256;

__device__ __forceinline__ int pku(int p, int i, int j) {  // packed upper, i <= j
    return i * p - ((i * (i - 1)) >> 1) + (j - i);
}

constexpr int kTrdWaves = 4;

__global__ __launch_bounds__(64 * kTrdWaves) void trd_kernel(const double* __restrict__ A_all, int p,
                                                            double* __restrict__ H_all, double* __restrict__ dv_all,
                                                            double* __restrict__ ev_all,
                                                            double* __restrict__ tau_all,
                                                            unsigned long long* __restrict__ clk) {
    extern __shared__ double tsm[];
    unsigned long long tp[6] = {0, 0, 0, 0, 0, 0}, t0 = 0;
    auto mark = [&](int ph) {
        if (clk) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            if (ph > 0) tp[ph - 1] += t - t0;
            t0 = t;
        }
    };
    const int P2 = p * (p + 1) / 2;
    double* a = tsm;
    double* vb = a + P2;
    double* wb = vb + p;
    double* yr = wb + p;
    double* ycp = yr + p;  // kTrdWaves x p partial column sums
    __shared__ double red[kTrdWaves];
    const int64_t b = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: row indices stay scalar
    const double* Ag = A_all + b * (int64_t)p * p;
    double* H = H_all + b * (int64_t)p * p;
    double* dv = dv_all + b * p;
    double* ev = ev_all + b * p;
    double* tv = tau_all + b * p;
    for (int i = wid; i < p; i += kTrdWaves)
        for (int c = i + lane; c < p; c += 64) a[pku(p, i, c)] = 0.5 * (Ag[(int64_t)i * p + c] + Ag[(int64_t)c * p + i]);
    __syncthreads();
    const int g = tid >> 3, q = tid & 7;  // 32 row groups of 8 lanes
    for (int j = 0; j + 2 < p; ++j) {
        const int j1 = j + 1;
        mark(0);
        double xs = 0.0;  // squared norm of A[j][j+2..p-1]
        for (int c = j1 + 1 + tid; c < p; c += 64 * kTrdWaves) {
            const double x = a[pku(p, j, c)];
            xs += x * x;
        }
        xs = wave_sum(xs);
        if (lane == 0) red[wid] = xs;
        __syncthreads();
        xs = 0.0;
#pragma unroll
        for (int w = 0; w < kTrdWaves; ++w) xs += red[w];
        const double alpha = a[pku(p, j, j1)];
        double tau = 0.0, beta = alpha, scal = 0.0;
        if (xs > 0.0) {
            const double nrm = sqrt(alpha * alpha + xs);
            beta = alpha >= 0.0 ? -nrm : nrm;
            tau = (beta - alpha) / beta;
            scal = 1.0 / (alpha - beta);
        }
        // v (v[j1] = 1) into LDS and H's column j
        for (int k = j1 + tid; k < p; k += 64 * kTrdWaves) {
            const double v = k == j1 ? 1.0 : a[pku(p, j, k)] * scal;
            vb[k] = v;
            H[(int64_t)k * p + j] = v;
        }
        if (tid == 0) {
            dv[j] = a[pku(p, j, j)];
            ev[j] = beta;
            tv[j] = tau;
        }
        __syncthreads();
        mark(1);
        if (tau == 0.0) continue;  // uniform
        // column part (diagonal included), rows i = j1 + wid + kTrdWaves t:
        //   ycp[wid][k] = sum_i a[i][k] v_i over this wave's rows i <= k (lane-owned k)
        // (RU rows per iteration: all their LDS loads are issued before the first FMA -- one
        // wave per SIMD, so latency is hidden by independent loads, not by other waves)
        constexpr int RU = 8;
        double yk[3] = {0.0, 0.0, 0.0};
        for (int i = j1 + wid; i < p; i += RU * kTrdWaves) {
            double vi[RU], av[RU][3];
            int rb[RU];  // packed offset of row ii, minus ii (scalar)
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                const int ii = i + u * kTrdWaves;
                rb[u] = pku(p, min(ii, p - 1), min(ii, p - 1)) - min(ii, p - 1);
                vi[u] = vb[min(ii, p - 1)];
#pragma unroll
                for (int s2 = 0; s2 < 3; ++s2) {
                    const int k = j1 + lane + 64 * s2;
                    // unconditional load from a clamped address, masked afterwards (no
                    // divergent branch around the load, so all of them stay in flight)
                    const bool ok = ii < p && k >= ii && k < p;
                    const double x = a[rb[u] + min(max(k, ii), p - 1)];
                    av[u][s2] = ok ? x : 0.0;
                }
            }
#pragma unroll
            for (int u = 0; u < RU; ++u)
#pragma unroll
                for (int s2 = 0; s2 < 3; ++s2) yk[s2] += av[u][s2] * vi[u];
        }
#pragma unroll
        for (int s2 = 0; s2 < 3; ++s2) {
            const int k = j1 + lane + 64 * s2;
            if (k < p) ycp[wid * p + k] = yk[s2];
        }
        mark(2);
        // row part: yr[i] = sum_{k > i} a[i][k] v_k, 32 rows at a time, 8 lanes per row
        for (int i0 = j1; i0 < p; i0 += 32) {
            const int i = i0 + g;
            double sr = 0.0;
            if (i < p) {
                const int base = pku(p, i, i);
                for (int k = i + 1 + q; k < p; k += 8 * RU) {
                    double av[RU], bv[RU];
#pragma unroll
                    for (int u = 0; u < RU; ++u) {
                        const int kk = k + 8 * u, kc = min(kk, p - 1);
                        const double x = a[base + kc - i], y = vb[kc];
                        av[u] = kk < p ? x : 0.0;
                        bv[u] = y;
                    }
#pragma unroll
                    for (int u = 0; u < RU; ++u) sr += av[u] * bv[u];
                }
            }
            sr += __shfl_xor(sr, 1, 64);
            sr += __shfl_xor(sr, 2, 64);
            sr += __shfl_xor(sr, 4, 64);
            if (q == 0 && i < p) yr[i] = sr;
        }
        __syncthreads();
        mark(3);
        // y = tau (column + row parts); w = y - (tau / 2)(y . v) v
        double yv = 0.0;
        for (int k = j1 + tid; k < p; k += 64 * kTrdWaves) {
            double y = yr[k];
#pragma unroll
            for (int w = 0; w < kTrdWaves; ++w) y += ycp[w * p + k];
            y *= tau;
            wb[k] = y;
            yv += y * vb[k];
        }
        yv = wave_sum(yv);
        if (lane == 0) red[wid] = yv;
        __syncthreads();
        yv = 0.0;
#pragma unroll
        for (int w = 0; w < kTrdWaves; ++w) yv += red[w];
        const double al2 = -0.5 * tau * yv;
        for (int k = j1 + tid; k < p; k += 64 * kTrdWaves) wb[k] += al2 * vb[k];
        __syncthreads();
        mark(4);
        // A' -= v w^T + w v^T (upper), rows i = j1 + wid + kTrdWaves t, lanes over k >= i
        double vk[3], wk[3];
#pragma unroll
        for (int s2 = 0; s2 < 3; ++s2) {
            const int k = j1 + lane + 64 * s2;
            vk[s2] = k < p ? vb[k] : 0.0;
            wk[s2] = k < p ? wb[k] : 0.0;
        }
        for (int i = j1 + wid; i < p; i += RU * kTrdWaves) {
            double vi[RU], wi[RU], av[RU][3];
            int rb[RU];
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                const int ii = i + u * kTrdWaves;
                rb[u] = pku(p, min(ii, p - 1), min(ii, p - 1)) - min(ii, p - 1);
                vi[u] = vb[min(ii, p - 1)];
                wi[u] = wb[min(ii, p - 1)];
#pragma unroll
                for (int s2 = 0; s2 < 3; ++s2) {
                    const int k = j1 + lane + 64 * s2;
                    const bool ok = ii < p && k >= ii && k < p;
                    const double x = a[rb[u] + min(max(k, ii), p - 1)];
                    av[u][s2] = ok ? x : 0.0;
                }
            }
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                const int ii = i + u * kTrdWaves;
#pragma unroll
                for (int s2 = 0; s2 < 3; ++s2) {
                    const int k = j1 + lane + 64 * s2;
                    if (ii < p && k >= ii && k < p) a[rb[u] + k] = av[u][s2] - (vi[u] * wk[s2] + wi[u] * vk[s2]);
                }
            }
        }
        __syncthreads();
        mark(5);
    }
    if (clk && tid == 0)
        for (int ph = 0; ph < 5; ++ph) atomicAdd(clk + ph, tp[ph]);
    if (tid == 0) {
        if (p >= 2) {
            dv[p - 2] = a[pku(p, p - 2, p - 2)];
            ev[p - 2] = a[pku(p, p - 2, p - 1)];
            tv[p - 2] = 0.0;
        }
        dv[p - 1] = a[pku(p, p - 1, p - 1)];
        tv[p - 1] = 0.0;
        ev[p - 1] = 0.0;
    }
}

// Sturm count: number of eigenvalues of the tridiagonal (d, e2 = e^2) below x
__device__ __forceinline__ int sturm_count(const double* d, const double* e2, int p, double x, double pivmin) {
    double t = d[0] - x;
    if (fabs(t) < pivmin) t = -pivmin;
    int c = t < 0.0;
    for (int k = 1; k < p; ++k) {
        t = d[k] - x - e2[k - 1] / t;
        if (fabs(t) < pivmin) t = -pivmin;
        c += t < 0.0;
    }
    return c;
}

// scratch per matrix: [2][p][kTriThreads] doubles (D+ / D- of each thread's eigenvalue)
__global__ __launch_bounds__(kTriThreads) void tri_eig_kernel(const double* __restrict__ dv_all,
                                                             const double* __restrict__ ev_all, int p,
                                                             double* __restrict__ evals, float* __restrict__ Z_all,
                                                             double* __restrict__ scr_all, int* __restrict__ flag) {
    extern __shared__ double esm[];
    double* d = esm;
    double* e = d + p;
    double* e2 = e + p;
    double* lam = e2 + p;
    __shared__ double red[16];
    const int64_t b = blockIdx.x;
    const int tid = threadIdx.x;
    for (int k = tid; k < p; k += kTriThreads) {
        d[k] = dv_all[b * p + k];
        const double ek = k + 1 < p ? ev_all[b * p + k] : 0.0;
        e[k] = ek;
        e2[k] = ek * ek;
    }
    __syncthreads();
    // Gershgorin bounds and the pivot floor (LAPACK dstebz: pivmin = safe_min * max(1, max e^2))
    double gl = 1e300, gu = -1e300, me2 = 0.0;
    for (int k = 0; k < p; ++k) {
        const double r = (k > 0 ? fabs(e[k - 1]) : 0.0) + (k + 1 < p ? fabs(e[k]) : 0.0);
        gl = fmin(gl, d[k] - r);
        gu = fmax(gu, d[k] + r);
        if (k + 1 < p) me2 = fmax(me2, e2[k]);
    }
    const double tnorm = fmax(fabs(gl), fabs(gu));
    const double pivmin = 2.2250738585072014e-308 * fmax(1.0, me2);
    gl -= 2.0 * 2.2e-16 * tnorm * p + 2.0 * pivmin;
    gu += 2.0 * 2.2e-16 * tnorm * p + 2.0 * pivmin;
    // eigenvalue i (descending) = the (p-1-i)-th smallest
    if (tid < p) {
        const int m = p - 1 - tid;
        double lo = gl, hi = gu;
        for (int it = 0; it < 200; ++it) {
            const double mid = 0.5 * (lo + hi);
            if (hi - lo <= 2.0 * 2.2e-16 * fmax(fabs(lo), fabs(hi)) + pivmin || mid <= lo || mid >= hi) break;
            if (sturm_count(d, e2, p, mid, pivmin) > m) hi = mid;
            else lo = mid;
        }
        lam[tid] = 0.5 * (lo + hi);
        evals[b * p + tid] = lam[tid];
    }
    __syncthreads();
    if (!Z_all) return;
    // near-degenerate neighbours: flag the matrix for the Jacobi path
    int bad = 0;
    if (tid + 1 < p && lam[tid] - lam[tid + 1] <= 1e-9 * fmax(tnorm, 1e-300)) bad = 1;
    bad = __syncthreads_or(bad);
    if (bad) {
        if (tid == 0) flag[b] = 1;
        return;
    }
    if (tid >= p) return;
    // twisted factorisation of T - lambda I: D+ forward, D- backward, twist r = argmin |gamma|
    double* Dp = scr_all + b * (int64_t)2 * p * kTriThreads;
    double* Dm = Dp + (int64_t)p * kTriThreads;
    auto DP = [&](int k) -> double& { return Dp[(int64_t)k * kTriThreads + tid]; };
    auto DM = [&](int k) -> double& { return Dm[(int64_t)k * kTriThreads + tid]; };
    const double l = lam[tid];
    double t = d[0] - l;
    if (fabs(t) < pivmin) t = -pivmin;
    DP(0) = t;
    for (int k = 0; k + 1 < p; ++k) {
        t = d[k + 1] - l - e2[k] / t;
        if (fabs(t) < pivmin) t = -pivmin;
        DP(k + 1) = t;
    }
    t = d[p - 1] - l;
    if (fabs(t) < pivmin) t = -pivmin;
    DM(p - 1) = t;
    for (int k = p - 2; k >= 0; --k) {
        t = d[k] - l - e2[k] / t;
        if (fabs(t) < pivmin) t = -pivmin;
        DM(k) = t;
    }
    int r = 0;
    double gmin = 1e308;
    for (int k = 0; k < p; ++k) {
        const double gk = fabs(DP(k) + DM(k) - (d[k] - l));
        if (gk < gmin) { gmin = gk; r = k; }
    }
    // x_r = 1; below r: x_k = -(e_k / D+_k) x_{k+1}; above r: x_{k+1} = -(e_k / D-_{k+1}) x_k
    // (x stored over the D+ / D- slots as they are consumed)
    double nrm2 = 1.0;
    double x = 1.0;
    for (int k = r - 1; k >= 0; --k) {
        x = -(e[k] / DP(k)) * x;
        DP(k) = x;
        nrm2 += x * x;
    }
    x = 1.0;
    for (int k = r; k + 1 < p; ++k) {
        x = -(e[k] / DM(k + 1)) * x;
        DM(k + 1) = x;
        nrm2 += x * x;
    }
    const double inv = 1.0 / sqrt(nrm2);
    float* Z = Z_all + b * (int64_t)p * p;
    for (int k = 0; k < p; ++k) {
        const double xk = k < r ? DP(k) : (k == r ? 1.0 : DM(k));
        Z[(int64_t)k * p + tid] = (float)(xk * inv);
    }
}

// V = H_0 H_1 ... H_{p-3} Z: reflectors applied last-first to Z (LDS, fp32 storage)
__global__ __launch_bounds__(kTriThreads) void trd_back_kernel(const double* __restrict__ H_all,
                                                              const double* __restrict__ tau_all, int p,
                                                              float* __restrict__ V_all, const int* __restrict__ flag) {
    extern __shared__ __attribute__((aligned(16))) char bsm_raw[];
    double* vb = reinterpret_cast<double*>(bsm_raw);
    float* Z = reinterpret_cast<float*>(vb + p);
    const int64_t b = blockIdx.x;
    if (flag[b]) return;
    const int tid = threadIdx.x;
    float* V = V_all + b * (int64_t)p * p;
    const double* H = H_all + b * (int64_t)p * p;
    for (int t = tid; t < p * p; t += kTriThreads) Z[t] = V[t];
    for (int j = p - 3; j >= 0; --j) {
        const double tau = tau_all[b * p + j];
        __syncthreads();
        for (int i = j + 1 + tid; i < p; i += kTriThreads) vb[i] = H[(int64_t)i * p + j];
        __syncthreads();
        if (tau == 0.0 || tid >= p) continue;
        double s = 0.0;
        for (int i = j + 1; i < p; ++i) s += vb[i] * (double)Z[i * p + tid];
        s *= tau;
        for (int i = j + 1; i < p; ++i) Z[i * p + tid] = (float)((double)Z[i * p + tid] - s * vb[i]);
    }
    __syncthreads();
    for (int t = tid; t < p * p; t += kTriThreads) V[t] = Z[t];
}

}  // namespace

size_t trid_workspace(int64_t p, int64_t batch) {
    return align_up((size_t)batch * p * p * sizeof(double), 256)           // reflectors
           + 3 * align_up((size_t)batch * p * sizeof(double), 256)          // d, e, tau
           + align_up((size_t)batch * 2 * p * kTriThreads * sizeof(double), 256)  // twisted-factorisation scratch
           + align_up((size_t)batch * sizeof(int), 256);                     // near-degenerate flags
}

bool trid_supported(int64_t p) {
    return p >= 1 && p <= 192 && (size_t)(p * (p + 1) / 2 + (3 + kTrdWaves) * p) * sizeof(double) <= 160 * 1024;
}

// Returns 0 with *fallback = 1 when some matrix needs the Jacobi path (near-degenerate pair).
int trid_eigh(const double* A, int64_t p, int64_t batch, double* evals, float* V32, void* ws, size_t ws_bytes,
              hipStream_t s, int* fallback) {
    *fallback = 0;
    if (ws_bytes < trid_workspace(p, batch)) return set_error(CQ_EWORKSPACE, "cq_jacobi_eigh: workspace too small");
    char* w = reinterpret_cast<char*>(ws);
    auto take = [&](size_t bytes) { char* r = w; w += align_up(bytes, 256); return r; };
    double* H = reinterpret_cast<double*>(take((size_t)batch * p * p * sizeof(double)));
    double* dv = reinterpret_cast<double*>(take((size_t)batch * p * sizeof(double)));
    double* ev = reinterpret_cast<double*>(take((size_t)batch * p * sizeof(double)));
    double* tv = reinterpret_cast<double*>(take((size_t)batch * p * sizeof(double)));
    double* scr = reinterpret_cast<double*>(take((size_t)batch * 2 * p * kTriThreads * sizeof(double)));
    int* flag = reinterpret_cast<int*>(take((size_t)batch * sizeof(int)));
    if (hipMemsetAsync(flag, 0, (size_t)batch * sizeof(int), s) != hipSuccess)
        return set_error(CQ_EHIP, "cq_jacobi_eigh: memset failed");
    const size_t la = (size_t)(p * (p + 1) / 2 + (3 + kTrdWaves) * p) * sizeof(double);
    static unsigned long long* clk = [] {
        unsigned long long* c = nullptr;
        if (getenv("CQ_TRD_CLOCK") && hipMalloc(&c, 8 * sizeof(unsigned long long)) == hipSuccess)
            (void)hipMemset(c, 0, 8 * sizeof(unsigned long long));
        return c;
    }();
    trd_kernel<<<(unsigned)batch, 64 * kTrdWaves, la, s>>>(A, (int)p, H, dv, ev, tv, clk);
    if (clk && getenv("CQ_TRD_CLOCK")[0] == 'p') {
        unsigned long long h[5];
        (void)hipStreamSynchronize(s);
        (void)hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
        fprintf(stderr, "trd clocks (sum over matrices): v %llu col %llu row %llu w %llu upd %llu\n", h[0], h[1],
                h[2], h[3], h[4]);
        (void)hipMemset(clk, 0, 8 * sizeof(unsigned long long));
    }
    tri_eig_kernel<<<(unsigned)batch, kTriThreads, 4 * p * sizeof(double), s>>>(dv, ev, (int)p, evals, V32, scr,
                                                                               flag);
    if (V32) {
        const size_t lb = (size_t)p * sizeof(double) + (size_t)p * p * sizeof(float);
        trd_back_kernel<<<(unsigned)batch, kTriThreads, lb, s>>>(H, tv, (int)p, V32, flag);
        int* hf = new int[batch];
        const bool ok = hipMemcpyAsync(hf, flag, batch * sizeof(int), hipMemcpyDeviceToHost, s) == hipSuccess &&
                        hipStreamSynchronize(s) == hipSuccess;
        for (int64_t i = 0; ok && i < batch; ++i) *fallback |= hf[i];
        delete[] hf;
        if (!ok) return check_launch("cq_jacobi_eigh (tridiagonal flags)");
    }
    return check_launch("cq_jacobi_eigh (tridiagonal)");
}

}  // namespace cq

using namespace cq;

extern "C" {

size_t cq_tridiag_workspace(int64_t p, int64_t batch) { return trid_workspace(p, batch); }

int cq_tridiag_eigh(const double* A, int64_t p, int64_t batch, double* evals, float* V32, void* ws,
                    size_t ws_bytes, int* fallback, void* stream) {
    CQ_REQUIRE(A && evals && fallback && batch > 0 && trid_supported(p), "cq_tridiag_eigh: bad args (p <= 192)");
    return trid_eigh(A, p, batch, evals, V32, ws, ws_bytes, as_stream(stream), fallback);
}

}  // extern "C"
