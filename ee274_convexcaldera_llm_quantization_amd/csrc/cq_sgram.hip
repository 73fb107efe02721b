// The solver's Gram G = Y Y^T from the sparse 2-bit codes (the LR step's SVD operand,
// alg.py:211-217, Y = (W - Q) diag(ycol), m <= n).
//
// With 2-bit whole-matrix absmax codes (quantization.py:93-105, k = 1) Q = s c, c in {-1, 0, 1},
// and |c| = 1 only where |x| > s / 2: ~1 % of the codes.  With w = ycol^2 and E = W - (s/2) c:
//   G = W diag(w) W^T - s (P + P^T),   P = E diag(w) c^T        (k x k, k = m, contraction n)
// because E c^T + c E^T = W c^T + c W^T - s c c^T.  A = W diag(w) W^T does not depend on Q: the
// engine forms it once per run (cq_gemm_x3 Gram of W's halves, fp32 upper triangle).  Each LR
// step then only needs the sparse product P (~1 % of a dense product's work) and one elementwise
// pass that writes G's K-blocked split halves (the operand layout of the Chebyshev filter,
// identical to cq_gemm_x3's sym_out output):
//   sgram_count_kernel   nonzero codes per row of c;
//   sgram_slices_kernel  rows sorted by count, per 64-row slice the widest -> sliced-ELL offsets;
//   sgram_fill_kernel    the ELL entries (l << 2 | code + 1), per row in an order that keeps the
//                        lanes of a step in different LDS bank groups (l mod 16); a slice holds
//                        64 rows of similar count (padding ~ a few %)
//   sgram_spmm_kernel    P[i, j] = sum_{l in row j of c} c_jl (E_il w_l): a workgroup stages R
//                        rows of E (fp32, l-major, R values per l) in LDS and sweeps every row j
//                        of c with one lane per j (64 rows per wave, coalesced ELL reads);
//   sgram_combine_kernel G = A - s (P + P^T) per 64 x 64 tile pair (I <= J), P^T through LDS,
//                        split halves written at (i, j) and mirrored (j, i).
// Every sum runs in a fixed order (per row j the fill order): results are deterministic.
#include "cq_common.h"

namespace cq {

constexpr int SG_SLICE = 64;

// nonzero 2-bit offset-binary fields (code != 0 <=> field != 1) in a 32-bit word of 16 codes
__device__ __forceinline__ uint32_t sg_nz_mask(uint32_t word) {
    const uint32_t x = word ^ 0x55555555u;
    return (x | (x >> 1)) & 0x55555555u;
}

// code u (0..15) of a little-endian word: byte u / 4, MSB-first within the byte
__device__ __forceinline__ uint32_t sg_field(uint32_t word, int u) {
    return (word >> (8 * (u >> 2) + 6 - 2 * (u & 3))) & 3u;
}

// code u (0..15) of the field whose low bit is at bit position p (p even)
__device__ __forceinline__ int sg_u_of_bit(int p) { return 4 * (p >> 3) + ((6 - (p & 7)) >> 1); }

// Per row: the nonzero count and, with W (fp16, the codes' layout) given, the row's part of
// ||(W - s c) diag(ycol)||^2 - ||W diag(ycol)||^2 = sum over its nonzero codes of
// wcol[l] (s^2 - 2 s c W[j, l]) (fp64; wcol = ycol^2, NULL = 1): ||Y||_F^2 of the LR step
// without a pass over Y (the per-matrix sum in row order in sgram_slices_kernel)
__global__ __launch_bounds__(256) void sgram_count_kernel(const uint8_t* __restrict__ packed, int64_t k, int64_t L,
                                                          int32_t* __restrict__ row_nnz, const _Float16* __restrict__ W,
                                                          const float* __restrict__ qscale,
                                                          const float* __restrict__ wcol, double* __restrict__ row_corr,
                                                          int64_t Lh, int32_t* __restrict__ row_nnz1, int64_t wcs) {
    const int lane = threadIdx.x & 63;
    const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t b = blockIdx.y;
    if (wcol) wcol += b * wcs;  // per-matrix column weights (stride 0: shared)
    if (j >= k) return;
    const uint32_t* row = reinterpret_cast<const uint32_t*>(packed + b * (k * L / 4) + j * (L / 4));
    const int64_t nw = L / 16;
    uint32_t cnt = 0, cnt1 = 0;
    double corr = 0.0;
    const double s = W ? (double)qscale[b] : 0.0;
    const _Float16* Wr = W ? W + b * k * L + j * L : nullptr;
    const int64_t nw1 = Lh / 16;   // words of the contraction's first part (l < Lh)
    for (int64_t w = lane; w < nw; w += 64) {
        const uint32_t word = row[w];
        uint32_t nz = sg_nz_mask(word);
        cnt += __popc(nz);
        if (w < nw1) cnt1 += __popc(nz);
        if (W) {
            while (nz) {
                const int p = __builtin_ctz(nz);
                nz &= nz - 1u;
                const int64_t l = 16 * w + sg_u_of_bit(p);
                const double c = (double)((int)((word >> p) & 3u) - 1);
                const double t = s * s - 2.0 * s * c * (double)(float)Wr[l];
                corr += wcol ? (double)wcol[l] * t : t;
            }
        }
    }
    cnt = wave_sum(cnt);
    if (lane == 0) row_nnz[b * k + j] = (int32_t)cnt;
    if (row_nnz1) {
        cnt1 = wave_sum(cnt1);
        if (lane == 0) row_nnz1[b * k + j] = (int32_t)cnt1;
    }
    if (W) {
        corr = wave_sum(corr);
        if (lane == 0) row_corr[b * k + j] = corr;
    }
}

// one workgroup per matrix: the rows sorted by nonzero count (descending; ties in row order --
// a deterministic counting sort), so a 64-row slice's width (its widest row) wastes little
// padding; perm[b, p] = the row at sorted position p; slice widths and their exclusive prefix
// (in 64-entry rows): slice_off has ns + 1 entries per matrix, total[b] = entries of matrix b
constexpr int SG_BINS = 1024;

__global__ __launch_bounds__(256) void sgram_slices_kernel(const int32_t* __restrict__ row_nnz, int64_t k,
                                                           int32_t* __restrict__ perm, int64_t* __restrict__ slice_off,
                                                           int64_t* __restrict__ total, const double* __restrict__ row_corr,
                                                           double* __restrict__ corr_out,
                                                           const int32_t* __restrict__ row_nnz1,
                                                           int32_t* __restrict__ slice_w1) {
    // stable counting sort, the four waves on four contiguous row ranges: per-wave bin counts,
    // bin starts (descending), each wave's base per bin = start + the counts of the waves before
    // it; then every wave places its rows in row order (ballots per distinct bin of a 64-row chunk)
    __shared__ int32_t hist[SG_BINS];
    __shared__ int32_t wbase[4][SG_BINS];
    const int64_t b = blockIdx.x;
    const int32_t* nz = row_nnz + b * k;
    int32_t* pm = perm + b * k;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t per = (k + 255) / 256 * 64;   // rows per wave, whole 64-row chunks
    const int64_t r0 = wv * per, r1 = min<int64_t>(k, r0 + per);
    for (int v = threadIdx.x; v < SG_BINS; v += blockDim.x)
        for (int w = 0; w < 4; ++w) wbase[w][v] = 0;
    __syncthreads();
    for (int64_t j = r0 + lane; j < r1; j += 64) atomicAdd(&wbase[wv][min(nz[j], SG_BINS - 1)], 1);
    __syncthreads();
    for (int v = threadIdx.x; v < SG_BINS; v += blockDim.x)
        hist[v] = wbase[0][v] + wbase[1][v] + wbase[2][v] + wbase[3][v];
    __syncthreads();
    if (threadIdx.x == 0) {
        int32_t acc = 0;  // descending: bin v starts after every row with a larger count
        for (int v = SG_BINS - 1; v >= 0; --v) {
            const int32_t c = hist[v];
            hist[v] = acc;
            acc += c;
        }
    }
    __syncthreads();
    for (int v = threadIdx.x; v < SG_BINS; v += blockDim.x) {
        int32_t acc = hist[v];
        for (int w = 0; w < 4; ++w) {
            const int32_t c = wbase[w][v];
            wbase[w][v] = acc;
            acc += c;
        }
    }
    __syncthreads();
    {
        const uint64_t lt = (1ull << lane) - 1ull;
        int32_t* base_w = wbase[wv];
        for (int64_t c0 = r0; c0 < r1; c0 += 64) {
            const int64_t j = c0 + lane;
            const int bin = j < r1 ? min(nz[j], SG_BINS - 1) : -1;
            uint64_t todo = __ballot(j < r1);
            while (todo) {
                const int leader = __builtin_ctzll(todo);
                const int bl = __shfl(bin, leader, 64);
                const uint64_t mk = __ballot(bin == bl);
                const int base = base_w[bl];
                if (bin == bl) pm[base + __popcll(mk & lt)] = (int32_t)j;
                __builtin_amdgcn_wave_barrier();
                if (lane == leader) base_w[bl] = base + __popcll(mk);
                __builtin_amdgcn_wave_barrier();
                todo &= ~mk;
            }
        }
    }
    if (row_corr) {   // the rows' norm corrections: fixed per-thread subsets, fixed reduction
        __shared__ double red[16];
        double cs = 0.0;
        for (int64_t j = threadIdx.x; j < k; j += blockDim.x) cs += row_corr[b * k + j];
        cs = block_sum_f64(cs, red);
        if (threadIdx.x == 0) corr_out[b] = cs;
    }
    __syncthreads();
    const int64_t ns = (k + SG_SLICE - 1) / SG_SLICE;
    int64_t* so = slice_off + b * (ns + 1);
    // l-split (row_nnz1 given): a slice holds its rows' first-part entries (l < Lh) in its
    // first w1 64-entry rows and the second part's after them, each part padded to the
    // slice's widest row of that part
    const int32_t* nz1 = row_nnz1 ? row_nnz1 + b * k : nullptr;
    for (int64_t s = threadIdx.x; s < ns; s += blockDim.x) {
        int32_t w = 0, w1 = 0, w2 = 0;
        for (int64_t p = s * SG_SLICE; p < (s + 1) * SG_SLICE && p < k; ++p) {
            const int32_t c = nz[pm[p]], c1 = nz1 ? nz1[pm[p]] : c;
            w = max(w, c);
            w1 = max(w1, c1);
            w2 = max(w2, c - c1);
        }
        so[s + 1] = nz1 ? w1 + w2 : w;  // widths, prefixed below
        if (slice_w1) slice_w1[b * ns + s] = nz1 ? w1 : w;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t acc = 0;
        so[0] = 0;
        for (int64_t s = 1; s <= ns; ++s) {
            acc += so[s];
            so[s] = acc;
        }
        total[b] = acc * SG_SLICE;
    }
}

constexpr int SG_FILL_CAP = 256;   // rows with more nonzeros take the plain order (LDS: 6 workgroups per CU)
constexpr int SG_FILL_RW = 4;   // sorted positions (rows) per wave

// Entry order.  The SpMM reads E's l-th 16-byte slab entry (LDS bank group l mod 16) for the 64
// rows of a slice at once, one lane per row; lanes whose entries share a bank group at the same
// step serialise.  Step t of the row at sorted position q (mod 16) therefore takes an entry of
// residue (q + t) mod 16 while it has one (neighbouring lanes then read different groups), else
// one of the residue with the most entries left (ties: the smaller residue); within a residue in
// increasing l.  Rows longer than SG_FILL_CAP take the plain residue-rotated order
// (sg_fill_plain).  One wave per SG_FILL_RW rows: each row's nonzeros are compacted in l order
// (one pass over its words) and stably counting-sorted by residue; the greedy order then runs
// for the SG_FILL_RW rows at once, 16 lanes (one per residue) each.
// l-split: entries with l < Lh go to the row's first part (out), the others to its second part
// (out2: the slice's first-part width further on); Lh >= L: one part.  n1 = first-part entries
__device__ void sg_fill_plain(const uint32_t* __restrict__ row, int64_t nw, int q, int lane, uint32_t* out,
                              uint32_t* out2, int64_t nw1, int& n1) {
    int64_t base = 0, base2 = 0;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int i = 0; i < 16; ++i) {
        const int u = (q + i) & 15;
        for (int64_t w0 = 0; w0 < nw; w0 += 64) {
            const int64_t w = w0 + lane;
            const uint32_t f = w < nw ? sg_field(row[w], u) : 1u;
            const bool nz = f != 1u, first = w < nw1;
            const uint64_t m1 = __ballot(nz && first), m2 = __ballot(nz && !first);
            const uint32_t e = (uint32_t)((16 * w + u) << 2) | f;
            if (nz && first) out[(base + __popcll(m1 & lt)) * SG_SLICE] = e;
            if (nz && !first) out2[(base2 + __popcll(m2 & lt)) * SG_SLICE] = e;
            base += __popcll(m1);
            base2 += __popcll(m2);
        }
    }
    n1 = (int)base;
}

__global__ __launch_bounds__(256, 6) void sgram_fill_kernel(const uint8_t* __restrict__ packed, int64_t k, int64_t L,
                                                         const int32_t* __restrict__ row_nnz,
                                                         const int32_t* __restrict__ perm,
                                                         const int64_t* __restrict__ slice_off,
                                                         const int32_t* __restrict__ slice_w1, int64_t Lh,
                                                         int64_t stride_ell, uint32_t* __restrict__ ell) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t p0 = ((int64_t)blockIdx.x * 4 + wv) * SG_FILL_RW;
    const int64_t b = blockIdx.y;
    if (p0 >= k) return;
    __shared__ uint32_t nat[4][SG_FILL_CAP];
    __shared__ uint32_t grp[4][SG_FILL_RW][SG_FILL_CAP];
    __shared__ int rsb[4][SG_FILL_RW][2][16], rcb[4][SG_FILL_RW][2][16];
    const int64_t nw = L / 16;
    const bool split = Lh < L;
    const int64_t nw1 = split ? Lh / 16 : nw;
    const int np = split ? 2 : 1;   // parts of the contraction
    const int64_t ns = (k + SG_SLICE - 1) / SG_SLICE;
    const uint64_t lt = (1ull << lane) - 1ull;
    int cntr[SG_FILL_RW];   // entries of each row (< 0: written in the plain order)
    int c1r[SG_FILL_RW];    // of them in the first part (l < Lh)
    uint32_t* outr[SG_FILL_RW];
    int64_t widr[SG_FILL_RW], w1r[SG_FILL_RW];
#pragma unroll
    for (int r = 0; r < SG_FILL_RW; ++r) {
        cntr[r] = 0;
        c1r[r] = 0;
        outr[r] = nullptr;
        widr[r] = 0;
        w1r[r] = 0;
        const int64_t p = p0 + r;
        if (p >= k) continue;
        const int64_t j = perm[b * k + p];
        const int64_t s = p / SG_SLICE;
        const int64_t off = slice_off[b * (ns + 1) + s];
        widr[r] = slice_off[b * (ns + 1) + s + 1] - off;
        w1r[r] = split ? slice_w1[b * ns + s] : widr[r];
        outr[r] = ell + b * stride_ell + off * SG_SLICE + (p % SG_SLICE);
        const uint32_t* row = reinterpret_cast<const uint32_t*>(packed + b * (k * L / 4) + j * (L / 4));
        if (row_nnz[b * k + j] > SG_FILL_CAP) {
            int n1 = 0;
            sg_fill_plain(row, nw, (int)(p & 15), lane, outr[r], outr[r] + w1r[r] * SG_SLICE, nw1, n1);
            cntr[r] = -row_nnz[b * k + j];   // written; padding below
            c1r[r] = n1;
            continue;
        }
        // the row's nonzeros in increasing l: per word, codes u = 0..15 in order (the first
        // part, l < Lh, is the prefix of c1 entries)
        int cnt = 0, cnt1 = 0;
        for (int64_t w0 = 0; w0 < nw; w0 += 64) {
            const int64_t w = w0 + lane;
            const uint32_t word = w < nw ? row[w] : 0x55555555u;
            uint32_t um = 0;
#pragma unroll
            for (int u = 0; u < 16; ++u) um |= (uint32_t)(sg_field(word, u) != 1u) << u;
            const int c = __builtin_popcount(um);
            int pre = 0, tot = 0;
#pragma unroll
            for (int bt = 0; bt < 5; ++bt) {
                const uint64_t mk = __ballot((c >> bt) & 1);
                pre += __popcll(mk & lt) << bt;
                tot += __popcll(mk) << bt;
            }
            if (split) {
                const int cf = w < nw1 ? c : 0;
#pragma unroll
                for (int bt = 0; bt < 5; ++bt) cnt1 += __popcll(__ballot((cf >> bt) & 1)) << bt;
            }
            int pos = cnt + pre;
            while (um) {
                const int u = __builtin_ctz(um);
                um &= um - 1u;
                nat[wv][pos++] = (uint32_t)((16 * w + u) << 2) | sg_field(word, u);
            }
            cnt += tot;
        }
        c1r[r] = split ? cnt1 : cnt;
        __builtin_amdgcn_wave_barrier();
        // per part: stable counting sort by residue (l mod 16) into grp (part 1 after part 0):
        // counts, starts, ranks (16 ballots a batch)
        for (int h = 0; h < np; ++h) {
            const int base = h ? c1r[r] : 0, cn = h ? cnt - c1r[r] : c1r[r];
            int cntu = 0;   // lane u < 16: entries of residue u
            for (int i0 = 0; i0 < cn; i0 += 64) {
                const int i = i0 + lane;
                const int res = i < cn ? (int)((nat[wv][base + i] >> 2) & 15u) : 16;
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const int m = __popcll(__ballot(res == u));
                    if (lane == u) cntu += m;
                }
            }
            int start = cntu;   // exclusive prefix over lanes 0..15
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                const int v = __shfl_up(start, o, 64);
                if ((lane & 15) >= o) start += v;
            }
            start -= cntu;
            start += base;
            if (lane < 16) {
                rsb[wv][r][h][lane] = start;
                rcb[wv][r][h][lane] = cntu;
            }
            int seen = 0;   // lane u < 16: entries of residue u already placed
            for (int i0 = 0; i0 < cn; i0 += 64) {
                const int i = i0 + lane;
                const uint32_t e = i < cn ? nat[wv][base + i] : 0u;
                const int res = i < cn ? (int)((e >> 2) & 15u) : 16;
                int dst = 0;
#pragma unroll
                for (int u = 0; u < 16; ++u) {
                    const uint64_t mk = __ballot(res == u);
                    const int su = __shfl(start + seen, u, 64);
                    if (res == u) dst = su + __popcll(mk & lt);
                    if (lane == u) seen += __popcll(mk);
                }
                if (i < cn) grp[wv][r][dst] = e;
            }
        }
        cntr[r] = cnt;
        __builtin_amdgcn_wave_barrier();
    }
    // greedy order per part, the SG_FILL_RW rows at once: lane = 16 g + u (row g, residue u)
    const int g = lane >> 4, u = lane & 15;
    const int q = (int)((p0 + g) & 15);
    for (int h = 0; h < np; ++h) {
        int myc = 0, mys = 0, mycnt = 0;
        uint32_t* myout = nullptr;
        int T = 0;
#pragma unroll
        for (int r = 0; r < SG_FILL_RW; ++r) {
            const int cn = cntr[r] <= 0 ? 0 : (h ? cntr[r] - c1r[r] : c1r[r]);
            if (g == r) {
                mycnt = cn;
                myout = outr[r] ? outr[r] + (h ? w1r[r] * SG_SLICE : 0) : nullptr;
            }
            T = cn > T ? cn : T;
        }
        if (mycnt > 0) {
            myc = rcb[wv][g][h][u];
            mys = rsb[wv][g][h][u];
        }
        int taken = 0;
        for (int t = 0; t < T; ++t) {
            const int d = (q + t) & 15;
            const int remd = __shfl(myc - taken, 16 * g + d, 64);
            int key = ((myc - taken) << 4) | (15 - u);
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) key = max(key, __shfl_xor(key, o, 64));
            const int sel = remd > 0 ? d : 15 - (key & 15);
            const int at = __shfl(mys + taken, 16 * g + sel, 64);
            if (t < mycnt) {
                if (u == 0) myout[(int64_t)t * SG_SLICE] = grp[wv][g][at];
                if (u == sel) ++taken;
            }
        }
    }
    // padding (code 0): the first part at l = 0, the second at l = Lh (inside its staged slab)
#pragma unroll
    for (int r = 0; r < SG_FILL_RW; ++r) {
        if (!outr[r]) continue;
        const int tot = cntr[r] < 0 ? -cntr[r] : cntr[r];
        for (int64_t t = c1r[r] + lane; t < w1r[r]; t += 64) outr[r][t * SG_SLICE] = 1u;
        if (split) {
            const uint32_t pad = (uint32_t)(Lh << 2) | 1u;
            for (int64_t t = w1r[r] + (tot - c1r[r]) + lane; t < widr[r]; t += 64) outr[r][t * SG_SLICE] = pad;
        }
    }
}

// one 64-row slice of the sorted ELL for the R staged rows: acc[r] = P[i0 + r, perm[64 s + lane]].
// The ELL loads (L2) are software-pipelined SG_PF entries ahead of the LDS reads and FMAs.
constexpr int SG_PF = 6;
constexpr int SG_WAVES = 16, SG_THREADS = 64 * SG_WAVES;

// E slab layout: planes of SG_PL rows, each plane l-major with SG_PL floats per l (16 bytes
// for R >= 4: the l-th entry starts in LDS bank group l mod 16)
template <int R>
__device__ __forceinline__ int64_t sg_slab_at(int64_t L, int64_t l, int r) {
    constexpr int PL = R < 4 ? R : 4;
    return (int64_t)(r / PL) * PL * L + l * PL + (r % PL);
}

template <int R>
__device__ __forceinline__ void sg_slice(const float* __restrict__ slab, int64_t L, const uint32_t* __restrict__ ep,
                                         int64_t width, float (&acc)[R], int64_t lbase = 0) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.f;
    constexpr int PL = R < 4 ? R : 4;
    auto fma_entry = [&](uint32_t e) {
        const float c = (float)((int)(e & 3u) - 1);
        const int64_t l = (int64_t)(e >> 2) - lbase;   // the slab holds l in [lbase, lbase + L)
#pragma unroll
        for (int pl = 0; pl < R / PL; ++pl) {
            const float* v = slab + (int64_t)pl * PL * L + l * PL;
#pragma unroll
            for (int r = 0; r < PL; ++r) acc[pl * PL + r] = __builtin_fmaf(c, v[r], acc[pl * PL + r]);
        }
    };
    int64_t t = 0;
    if (width >= SG_PF) {
        uint32_t cur[SG_PF];
#pragma unroll
        for (int q = 0; q < SG_PF; ++q) cur[q] = ep[q * SG_SLICE];
        for (t = SG_PF; t + SG_PF <= width; t += SG_PF) {
            uint32_t nxt[SG_PF];
#pragma unroll
            for (int q = 0; q < SG_PF; ++q) nxt[q] = ep[(t + q) * SG_SLICE];
#pragma unroll
            for (int q = 0; q < SG_PF; ++q) fma_entry(cur[q]);
#pragma unroll
            for (int q = 0; q < SG_PF; ++q) cur[q] = nxt[q];
        }
#pragma unroll
        for (int q = 0; q < SG_PF; ++q) fma_entry(cur[q]);
    }
    for (; t < width; ++t) fma_entry(ep[t * SG_SLICE]);
}

// P[b, i0 + r, j] for r < R and every row j of c.  LDS: E rows i0 .. i0 + R - 1 as
// the l-major slab (sg_slab_at, fp32), E_il = (W_il - (s/2) c_il) * w_l.  Wave wv takes the slices wv,
// wv + 16, ...; with NSW > 0 (ceil(ns / 16) <= NSW) it keeps all of its results in registers and
// the R output rows are assembled in LDS (the slab's space, k <= L, j-major) and stored over j
// -- the sorted slices' rows are scattered over j, so direct stores would be 4-byte scatters
template <int R, int NSW, bool SPLIT = false>
__global__ __launch_bounds__(1024) void sgram_spmm_kernel(const _Float16* __restrict__ W, const uint8_t* __restrict__ packed,
                                                         const float* __restrict__ qscale, const float* __restrict__ wcol,
                                                         int64_t k, int64_t L, const uint32_t* __restrict__ ell,
                                                         const int32_t* __restrict__ perm,
                                                         const int64_t* __restrict__ slice_off,
                                                         const int32_t* __restrict__ slice_w1, int64_t Lh,
                                                         int64_t stride_ell, float* __restrict__ P, int64_t wcs) {
    extern __shared__ __attribute__((aligned(16))) float slab[];
    const int64_t b = blockIdx.y;
    if (wcol) wcol += b * wcs;  // per-matrix column weights (stride 0: shared)
    const int64_t i0 = (int64_t)blockIdx.x * R;
    const float hs = 0.5f * qscale[b];
    const int64_t KL = k * L;
    const int64_t Ls = SPLIT ? Lh : L;   // l-values a slab holds (SPLIT: each part of the contraction)
    // stage E for l in [la, lb): per plane, a thread loads 8 consecutive l of each of its PL rows
    // (16-byte W and 2-byte code loads) and stores the 8 l-entries (PL floats each) in an order
    // rotated by its lane (t mod 8): the 8 lanes of a ds_write_b128 group then hit 8 different
    // bank groups instead of one (the entries of consecutive lanes lie 128 bytes apart)
    constexpr int PL = R < 4 ? R : 4;
    auto stage = [&](int64_t la, int64_t lb) {
#pragma unroll
    for (int pl = 0; pl < R / PL; ++pl) {
        for (int64_t l0 = la + (int64_t)threadIdx.x * 8; l0 < lb; l0 += SG_THREADS * 8) {
            float e[PL][8];
#pragma unroll
            for (int r = 0; r < PL; ++r) {
                const int64_t i = i0 + pl * PL + r;
                if (i < k) {
                    const int64_t el = b * KL + i * L + l0;
                    const uint4 raw = *reinterpret_cast<const uint4*>(W + el);
                    const _Float16* hv = reinterpret_cast<const _Float16*>(&raw);
                    const uint16_t two = *reinterpret_cast<const uint16_t*>(packed + el / 4);
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const uint32_t byte = (u < 4) ? (two & 0xffu) : (two >> 8);
                        const float c = (float)((int)((byte >> (6 - 2 * (u & 3))) & 3u) - 1);
                        e[r][u] = (float)hv[u] - hs * c;
                        if (wcol) e[r][u] *= wcol[l0 + u];
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < 8; ++u) e[r][u] = 0.f;
                }
            }
            const int rot = threadIdx.x & 7;
#pragma unroll
            for (int sh = 1; sh < 8; sh <<= 1) {  // e[r][u] <- e[r][(u + rot) & 7], log shifter
                if (rot & sh) {
#pragma unroll
                    for (int r = 0; r < PL; ++r) {
                        float t8[8];
#pragma unroll
                        for (int u = 0; u < 8; ++u) t8[u] = e[r][(u + sh) & 7];
#pragma unroll
                        for (int u = 0; u < 8; ++u) e[r][u] = t8[u];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                float* dst = slab + (int64_t)pl * PL * Ls + (l0 - la + ((u + rot) & 7)) * PL;
                if constexpr (PL == 4) *reinterpret_cast<float4*>(dst) = make_float4(e[0][u], e[1][u], e[2][u], e[3][u]);
                else *reinterpret_cast<float2*>(dst) = make_float2(e[0][u], e[1][u]);
            }
        }
    }
    };
    stage(0, SPLIT ? Lh : L);
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t ns = (k + SG_SLICE - 1) / SG_SLICE;
    const int64_t* so = slice_off + b * (ns + 1);
    const uint32_t* eb = ell + b * stride_ell + lane;
    const int32_t* pm = perm + b * k;
    float* Pb = P + b * k * k;
    if constexpr (NSW > 0) {
        float acc[NSW][R];
#pragma unroll
        for (int q = 0; q < NSW; ++q) {
            const int64_t s = wv + SG_WAVES * q;
            if (s < ns) sg_slice<R>(slab, L, eb + so[s] * SG_SLICE, so[s + 1] - so[s], acc[q]);
        }
        __syncthreads();  // every wave is done with the slab: it becomes the k x R output block
        // (j-major, one 16- or 8-byte store per PL rows: few LDS writes for the scattered j)
#pragma unroll
        for (int q = 0; q < NSW; ++q) {
            const int64_t p = (wv + SG_WAVES * q) * SG_SLICE + lane;
            if (p < k) {
                float* dst = slab + pm[p] * R;
#pragma unroll
                for (int pl = 0; pl < R / PL; ++pl) {
                    if constexpr (PL == 4)
                        *reinterpret_cast<float4*>(dst + 4 * pl) = make_float4(acc[q][4 * pl], acc[q][4 * pl + 1],
                                                                              acc[q][4 * pl + 2], acc[q][4 * pl + 3]);
                    else *reinterpret_cast<float2*>(dst) = make_float2(acc[q][0], acc[q][1]);
                }
            }
        }
        __syncthreads();
        // one j per thread: its R values (contiguous in LDS) to the R rows of P, coalesced over j
        for (int64_t j = threadIdx.x; j < k; j += SG_THREADS) {
            float v[R];
#pragma unroll
            for (int pl = 0; pl < R / PL; ++pl) {
                if constexpr (PL == 4) {
                    const float4 x = *reinterpret_cast<const float4*>(slab + j * R + 4 * pl);
                    v[4 * pl] = x.x; v[4 * pl + 1] = x.y; v[4 * pl + 2] = x.z; v[4 * pl + 3] = x.w;
                } else {
                    const float2 x = *reinterpret_cast<const float2*>(slab + j * R);
                    v[0] = x.x; v[1] = x.y;
                }
            }
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (i0 + r < k) Pb[(i0 + r) * k + j] = v[r];
        }
    } else if constexpr (NSW < 0) {
        // output block of its own after the slab (k x R, j-major): each slice's results go to
        // LDS as soon as they are done (nothing held in registers), then stored over j.
        // SPLIT (l-split ELL, the 11008-long contractions): R = 4 rows of E fit the LDS only
        // half a contraction at a time, so each slice's first part (l < Lh) is swept against
        // the slab of l in [0, Lh), then the slab is restaged with l in [Lh, L) and the second
        // parts are added: every workgroup still reads the ELL once, but half as many do it
        // as with R = 2 rows over the whole contraction
        float* outb = slab + (int64_t)R * Ls;
        const int32_t* w1 = SPLIT ? slice_w1 + b * ns : nullptr;
        for (int64_t s = wv; s < ns; s += SG_WAVES) {
            float acc[R];
            sg_slice<R>(slab, Ls, eb + so[s] * SG_SLICE, SPLIT ? w1[s] : so[s + 1] - so[s], acc);
            const int64_t p = s * SG_SLICE + lane;
            if (p < k) {
#pragma unroll
                for (int r = 0; r < R; ++r) outb[(int64_t)pm[p] * R + r] = acc[r];
            }
        }
        if constexpr (SPLIT) {
            __syncthreads();   // every wave is done with the first part's slab
            stage(Lh, L);
            __syncthreads();
            for (int64_t s = wv; s < ns; s += SG_WAVES) {
                float acc[R];
                sg_slice<R>(slab, Ls, eb + (so[s] + w1[s]) * SG_SLICE, so[s + 1] - so[s] - w1[s], acc, Lh);
                const int64_t p = s * SG_SLICE + lane;
                if (p < k) {
#pragma unroll
                    for (int r = 0; r < R; ++r) outb[(int64_t)pm[p] * R + r] += acc[r];
                }
            }
        }
        __syncthreads();
        for (int64_t j = threadIdx.x; j < k; j += SG_THREADS) {
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (i0 + r < k) Pb[(i0 + r) * k + j] = outb[j * R + r];
        }
    } else {
        for (int64_t s = wv; s < ns; s += SG_WAVES) {
            float acc[R];
            sg_slice<R>(slab, L, eb + so[s] * SG_SLICE, so[s + 1] - so[s], acc);
            const int64_t p = s * SG_SLICE + lane;
            if (p < k) {
                const int64_t j = pm[p];
#pragma unroll
                for (int r = 0; r < R; ++r)
                    if (i0 + r < k) Pb[(i0 + r) * k + j] = acc[r];
            }
        }
    }
}

__device__ __forceinline__ float sg_split_scale(double bound) {
    int e = 0;
    if (bound > 0.0 && isfinite(bound)) frexp(bound, &e);
    return ldexpf(1.f, 14 - e);
}

// G = A - s (P + P^T) for the 64 x 64 tile pair (I, J), I <= J: halves at (i, j) and (j, i)
// of the K-blocked split (element (i, j) at (j / 32) k 32 + i 32 + j % 32); fp32 G too if given
__global__ __launch_bounds__(256) void sgram_combine_kernel(const float* __restrict__ A, const float* __restrict__ P,
                                                            const float* __restrict__ qscale, int64_t k,
                                                            const double* __restrict__ bound, float out_scale,
                                                            _Float16* __restrict__ Gh, _Float16* __restrict__ Gl,
                                                            float* __restrict__ scale_out, float* __restrict__ inv_out,
                                                            float* __restrict__ G32) {
    __shared__ float pt[64][65];  // pt[a][c] = P[J0 + a][I0 + c], then the G tile v[i][j]
    const int64_t b = blockIdx.y;
    const int64_t nt = k / 64;
    int64_t t = blockIdx.x, I = 0;
    while (t >= nt - I) { t -= nt - I; ++I; }
    const int64_t J = I + t;
    const int64_t I0 = I * 64, J0 = J * 64;
    const float s = qscale[b];
    const float gs = sg_split_scale(bound[b]);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        scale_out[b] = gs;
        inv_out[b] = 1.f / (gs * out_scale);
    }
    const int64_t KK = k * k;
    const float* Pb = P + b * KK;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;   // 16 x 16 threads, 4 columns each
    for (int a = ty; a < 64; a += 16) {
        const float4 v = *reinterpret_cast<const float4*>(Pb + (J0 + a) * k + I0 + 4 * tx);
        pt[a][4 * tx] = v.x; pt[a][4 * tx + 1] = v.y; pt[a][4 * tx + 2] = v.z; pt[a][4 * tx + 3] = v.w;
    }
    __syncthreads();
    float g[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int a = ty + 16 * q;                 // row i = I0 + a, columns j = J0 + 4 tx .. + 3
        const float4 av = *reinterpret_cast<const float4*>(A + b * KK + (I0 + a) * k + J0 + 4 * tx);
        const float4 pv = *reinterpret_cast<const float4*>(Pb + (I0 + a) * k + J0 + 4 * tx);
        const float aa[4] = {av.x, av.y, av.z, av.w}, pp[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
        for (int u = 0; u < 4; ++u) g[q][u] = aa[u] - s * (pp[u] + pt[4 * tx + u][a]);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int u = 0; u < 4; ++u) pt[ty + 16 * q][4 * tx + u] = g[q][u];
    __syncthreads();
    _Float16* Ohb = Gh + b * KK;
    _Float16* Olb = Gl + b * KK;
    // (i, j), i <= j: row i = I0 + a, 4 columns j
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int a = ty + 16 * q;
        const int64_t i = I0 + a, j = J0 + 4 * tx;
        _Float16 h[4], l[4];
        bool any = false;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float hsv = pt[a][4 * tx + u] * gs;
            h[u] = (_Float16)hsv;
            l[u] = (_Float16)(hsv - (float)h[u]);
            any |= j + u >= i;
        }
        const int64_t o = (j >> 5) * (k * 32) + i * 32 + (j & 31);
        if (j >= i) {
            *reinterpret_cast<uint2*>(Ohb + o) = *reinterpret_cast<const uint2*>(h);
            *reinterpret_cast<uint2*>(Olb + o) = *reinterpret_cast<const uint2*>(l);
        } else if (any) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (j + u >= i) { Ohb[o + u] = h[u]; Olb[o + u] = l[u]; }
        }
        if (G32) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (j + u >= i) G32[b * KK + i * k + j + u] = pt[a][4 * tx + u];
        }
    }
    // mirror (j, i), j > i: row j = J0 + a, 4 columns i = I0 + 4 tx .. + 3
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int a = ty + 16 * q;
        const int64_t j = J0 + a, i = I0 + 4 * tx;
        _Float16 h[4], l[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float hsv = pt[4 * tx + u][a] * gs;
            h[u] = (_Float16)hsv;
            l[u] = (_Float16)(hsv - (float)h[u]);
        }
        const int64_t o = (i >> 5) * (k * 32) + j * 32 + (i & 31);
        if (i + 3 < j) {
            *reinterpret_cast<uint2*>(Ohb + o) = *reinterpret_cast<const uint2*>(h);
            *reinterpret_cast<uint2*>(Olb + o) = *reinterpret_cast<const uint2*>(l);
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u < j) { Ohb[o + u] = h[u]; Olb[o + u] = l[u]; }
        }
        if (G32) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u < j) G32[b * KK + j * k + i + u] = pt[4 * tx + u][a];
        }
    }
}

// ------------------------------------------------------------------ packed-code helpers
// Packed 2-bit code matrices: offset binary (field = c + 1), 16 codes per little-endian 32-bit
// word, code u of a word at bits 8 (u / 4) + 6 - 2 (u % 4) (bytes MSB-first).

__device__ __forceinline__ uint32_t sg_put(uint32_t f, int u) { return f << (8 * (u >> 2) + 6 - 2 * (u & 3)); }

// Transpose of packed 2-bit codes (rows x cols -> cols x rows), a tile of 256 x 256 codes per
// workgroup: thread (i, j) loads the 16 x 16 block of input rows 16 i.., word j (16 lanes read a
// row's 64 contiguous bytes), transposes it in registers and parks the 16 output words in LDS;
// then thread q writes output row q's 16 words of the tile (64 contiguous bytes).
__global__ __launch_bounds__(256) void codes_transpose_kernel(const uint32_t* __restrict__ in, int64_t rows,
                                                              int64_t cols, uint32_t* __restrict__ out) {
    __shared__ uint32_t t[256][17];
    const int64_t b = blockIdx.z;
    const int64_t wr = cols / 16, wc = rows / 16;   // words per input / output row
    const int64_t r0 = (int64_t)blockIdx.y * 256, c0 = (int64_t)blockIdx.x * 256;
    const int tid = threadIdx.x, i = tid >> 4, j = tid & 15;
    const int64_t ir = r0 + 16 * i, iw = c0 / 16 + j;
    if (ir < rows && iw < wr) {
        const uint32_t* src = in + b * rows * wr + ir * wr + iw;
        uint32_t w[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) w[r] = src[r * wr];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            uint32_t o = 0;
#pragma unroll
            for (int r = 0; r < 16; ++r) o |= sg_put(sg_field(w[r], u), r);
            t[16 * j + u][i] = o;   // output row c0 + 16 j + u, word r0 / 16 + i
        }
    }
    __syncthreads();
    const int64_t orow = c0 + tid;
    if (orow < cols) {
        uint32_t* dst = out + b * cols * wc + orow * wc + r0 / 16;
        const int64_t nwv = wc - r0 / 16 < 16 ? wc - r0 / 16 : 16;
        if (nwv == 16 && (wc & 3) == 0) {   // 16-byte aligned rows
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<uint4*>(dst + 4 * q) = make_uint4(t[tid][4 * q], t[tid][4 * q + 1], t[tid][4 * q + 2],
                                                                    t[tid][4 * q + 3]);
        } else {
            for (int q = 0; q < nwv; ++q) dst[q] = t[tid][q];
        }
    }
}

// out[row, :] = sum over the nonzero codes c (col) of row `row` of c w[col] X[col, :] (X: cols x r,
// row stride ldx; w NULL = 1), times roww[row] if given: the sparse-code product of the LR step
// (U^T c, c V).  One wave per row: the row's nonzero codes are compacted into a per-wave LDS list
// (in increasing word order; fixed order, deterministic), then consumed CM_G at a time with the
// X-row loads of all CM_G in flight; lane l owns r-values l, l + 64, ...  The words of a row
// (CM_WPL per lane and block of 64 CM_WPL words) are loaded in one batch, and the next row's
// first block while the current row is consumed.  TRANS: out is r x rows (ld ldo), written
// through an LDS tile of the workgroup's 64 rows (coalesced over rows); else rows x r.
// list entries per wave: a row of c^T holds ~1 % nonzeros (~40 at 4096 columns); a fuller
// block is consumed in parts (the small list keeps 4 workgroups per CU in LDS)
constexpr int CM_LIST = 256;
constexpr int CM_WPL = 4;       // words per lane per block
constexpr int CM_G = 16;        // entries per gather batch
template <int RV, bool TRANS>
__global__ __launch_bounds__(256) void codes_matmul_kernel(const uint32_t* __restrict__ packed, int64_t rows,
                                                           int64_t cols, const float* __restrict__ X, int64_t ldx,
                                                           int64_t sx, const float* __restrict__ w,
                                                           const float* __restrict__ roww, int r,
                                                           float* __restrict__ out, int64_t ldo, int64_t so,
                                                           int64_t ws_, int64_t rws) {
    extern __shared__ __attribute__((aligned(16))) uint32_t cm_lds[];
    uint32_t* list = cm_lds + (threadIdx.x >> 6) * CM_LIST;
    float* tile = reinterpret_cast<float*>(cm_lds + 4 * CM_LIST);   // TRANS: [r][65]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t b = blockIdx.y, row0 = (int64_t)blockIdx.x * 64;
    if (w) w += b * ws_;        // per-matrix column / row weights (stride 0: shared)
    if (roww) roww += b * rws;
    const int64_t nw = cols / 16;
    const uint32_t* pb = packed + b * rows * nw;
    const float* Xb = X + b * sx;
    const uint64_t lt = (1ull << lane) - 1ull;
    constexpr int64_t BLK = 64 * CM_WPL;   // words per block
    auto load_block = [&](int64_t row, int64_t w0, uint32_t (&wd)[CM_WPL]) {
#pragma unroll
        for (int t = 0; t < CM_WPL; ++t) {
            const int64_t wi = w0 + 64 * t + lane;
            wd[t] = (row < rows && wi < nw) ? pb[row * nw + wi] : 0x55555555u;
        }
    };
    float acc[RV];
    int cnt = 0;
    auto consume = [&]() {
        for (int t0 = 0; t0 < cnt; t0 += CM_G) {
            float cv[CM_G], xv[CM_G][RV];
#pragma unroll
            for (int e = 0; e < CM_G; ++e) {
                const bool live = t0 + e < cnt;
                const uint32_t en = live ? list[t0 + e] : 1u;   // padding: code 0 at column 0
                const int64_t col = en >> 2;
                cv[e] = (float)((int)(en & 3u) - 1);
                if (w && live) cv[e] *= w[col];
                const float* xr = Xb + col * ldx;
#pragma unroll
                for (int k = 0; k < RV; ++k) xv[e][k] = (lane + 64 * k < r) ? xr[lane + 64 * k] : 0.f;
            }
#pragma unroll
            for (int e = 0; e < CM_G; ++e)
#pragma unroll
                for (int k = 0; k < RV; ++k) acc[k] = __builtin_fmaf(cv[e], xv[e][k], acc[k]);
        }
        cnt = 0;
    };
    uint32_t cur[CM_WPL];
    load_block(row0 + wv * 16, 0, cur);
    for (int q = 0; q < 16; ++q) {
        const int lr = wv * 16 + q;
        const int64_t row = row0 + lr;
#pragma unroll
        for (int k = 0; k < RV; ++k) acc[k] = 0.f;
        for (int64_t w0 = 0; w0 < nw; w0 += BLK) {
            // compact this block's nonzero codes into the list (ballot prefix of the counts)
#pragma unroll
            for (int t = 0; t < CM_WPL; ++t) {
                uint32_t nz = sg_nz_mask(cur[t]);
                const int c = __builtin_popcount(nz);
                int pre = 0, tot = 0;
#pragma unroll
                for (int bt = 0; bt < 5; ++bt) {
                    const uint64_t mk = __ballot((c >> bt) & 1);
                    pre += __popcll(mk & lt) << bt;
                    tot += __popcll(mk) << bt;
                }
                const int64_t wi = w0 + 64 * t + lane;
                if (cnt + tot <= CM_LIST) {
                    int pos = cnt + pre;
                    while (nz) {
                        const int p = __builtin_ctz(nz);
                        nz &= nz - 1u;
                        list[pos++] = (uint32_t)((16 * wi + sg_u_of_bit(p)) << 2) | ((cur[t] >> p) & 3u);
                    }
                    cnt += tot;
                } else {   // the list cannot take this word group: in lane order, a list-full at a time
                    for (int src = 0; src < 64; ++src) {
                        const uint32_t wsrc = (uint32_t)__shfl((int)cur[t], src, 64);
                        uint32_t nzs = sg_nz_mask(wsrc);
                        const int64_t wis = w0 + 64 * t + src;
                        while (nzs) {   // wave-uniform
                            const int p = __builtin_ctz(nzs);
                            nzs &= nzs - 1u;
                            if (cnt == CM_LIST) {
                                __builtin_amdgcn_wave_barrier();
                                consume();
                                __builtin_amdgcn_wave_barrier();
                            }
                            if (lane == 0) list[cnt] = (uint32_t)((16 * wis + sg_u_of_bit(p)) << 2) | ((wsrc >> p) & 3u);
                            ++cnt;
                        }
                    }
                }
            }
            // the next block of this row, or the first block of the next row, in flight while
            // this list is consumed
            if (w0 + BLK < nw) load_block(row, w0 + BLK, cur);
            else if (q + 1 < 16) load_block(row + 1, 0, cur);
            __builtin_amdgcn_wave_barrier();
            consume();
            __builtin_amdgcn_wave_barrier();
        }
        if (roww && row < rows) {
            const float rw = roww[row];
#pragma unroll
            for (int k = 0; k < RV; ++k) acc[k] *= rw;
        }
        if constexpr (TRANS) {
#pragma unroll
            for (int k = 0; k < RV; ++k)
                if (lane + 64 * k < r) tile[(lane + 64 * k) * 65 + lr] = acc[k];
        } else if (row < rows) {
            float* o = out + b * so + row * ldo;
#pragma unroll
            for (int k = 0; k < RV; ++k)
                if (lane + 64 * k < r) o[lane + 64 * k] = acc[k];
        }
    }
    if constexpr (TRANS) {
        __syncthreads();
        for (int64_t e = threadIdx.x; e < (int64_t)r * 64; e += 256) {
            const int64_t idx = e / 64, lr = e % 64;
            if (row0 + lr < rows) out[b * so + idx * ldo + row0 + lr] = tile[idx * 65 + lr];
        }
    }
}

// per matrix: the part of ||(W - s c) diag(ycol)||_F^2 that the nonzero codes add to
// ||W diag(ycol)||_F^2, sum over them of w[col] (s^2 - 2 s c W[row, col]) (w = ycol^2, NULL = 1),
// in fp64 in a fixed order (wave wv: rows wv, wv + 16, ...; fixed reduction): deterministic
__global__ __launch_bounds__(1024) void codes_ysq_corr_kernel(const uint32_t* __restrict__ packed,
                                                              const _Float16* __restrict__ W,
                                                              const float* __restrict__ qscale,
                                                              const float* __restrict__ w, int64_t rows,
                                                              int64_t cols, double* __restrict__ out, int64_t wst) {
    __shared__ double red[16];
    const int64_t b = blockIdx.x;
    if (w) w += b * wst;  // per-matrix column weights (stride 0: shared)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const double s = (double)qscale[b];
    const int64_t nw = cols / 16;
    const uint32_t* pb = packed + b * rows * nw;
    const _Float16* Wb = W + b * rows * cols;
    double acc = 0.0;
    for (int64_t row = wv; row < rows; row += 16) {
        for (int64_t wi = lane; wi < nw; wi += 64) {
            const uint32_t word = pb[row * nw + wi];
            uint32_t nz = sg_nz_mask(word);
            while (nz) {
                const int p = __builtin_ctz(nz);
                nz &= nz - 1u;
                const int64_t col = 16 * wi + sg_u_of_bit(p);
                const double c = (double)((int)((word >> p) & 3u) - 1);
                const double x = (double)(float)Wb[row * cols + col];
                const double t = s * s - 2.0 * s * c * x;
                acc += w ? (double)w[col] * t : t;
            }
        }
    }
    const double tot = block_sum_f64(acc, red);
    if (threadIdx.x == 0) out[b] = tot;
}

// Y = X^T for fp16 (batch x rows x cols -> batch x cols x rows), 64 x 64 tiles through LDS
__global__ __launch_bounds__(256) void transpose_f16_kernel(const uint16_t* __restrict__ in, int64_t rows, int64_t cols,
                                                            uint16_t* __restrict__ out) {
    __shared__ uint16_t t[64][66];
    const int64_t b = blockIdx.z, r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const uint16_t* src = in + b * rows * cols;
    for (int i = ty; i < 64; i += 4)
        if (r0 + i < rows && c0 + tx < cols) t[i][tx] = src[(r0 + i) * cols + c0 + tx];
    __syncthreads();
    uint16_t* dst = out + b * rows * cols;
    for (int i = ty; i < 64; i += 4)
        if (c0 + i < cols && r0 + tx < rows) dst[(c0 + i) * rows + r0 + tx] = t[tx][i];
}

}  // namespace cq

using namespace cq;

extern "C" {

int cq_codes_transpose(const uint8_t* packed, int bits, int64_t batch, int64_t rows, int64_t cols, uint8_t* out,
                       void* stream) {
    CQ_REQUIRE(packed && out, "cq_codes_transpose: null argument");
    CQ_REQUIRE(bits == 2, "cq_codes_transpose: 2-bit codes only");
    CQ_REQUIRE(batch > 0 && batch < 65536 && rows > 0 && cols > 0 && rows % 16 == 0 && cols % 16 == 0,
               "cq_codes_transpose: bad shape (rows, cols multiples of 16)");
    const dim3 grid((unsigned)ceil_div(cols, 256), (unsigned)ceil_div(rows, 256), (unsigned)batch);
    codes_transpose_kernel<<<grid, 256, 0, as_stream(stream)>>>(reinterpret_cast<const uint32_t*>(packed), rows,
                                                                cols, reinterpret_cast<uint32_t*>(out));
    return check_launch("cq_codes_transpose");
}

int cq_codes_matmul(const uint8_t* packed, int bits, int64_t batch, int64_t rows, int64_t cols, const float* X,
                    int64_t ldx, int64_t stride_x, const float* colw, int64_t colw_stride, const float* roww,
                    int64_t roww_stride, int64_t r, float* out, int64_t ldo, int64_t stride_out, int trans,
                    void* stream) {
    CQ_REQUIRE(packed && X && out, "cq_codes_matmul: null argument");
    CQ_REQUIRE(bits == 2, "cq_codes_matmul: 2-bit codes only");
    CQ_REQUIRE(batch > 0 && batch < 65536 && rows > 0 && cols > 0 && cols % 16 == 0 && cols < (1ll << 29),
               "cq_codes_matmul: bad shape");
    CQ_REQUIRE(r > 0 && r <= 256 && ldx >= r, "cq_codes_matmul: r must be in 1..256 and <= ldx");
    const dim3 grid((unsigned)ceil_div(rows, 64), (unsigned)batch);
    const size_t lds = 4 * CM_LIST * sizeof(uint32_t) + (trans ? (size_t)r * 65 * sizeof(float) : 0);
    hipStream_t s = as_stream(stream);
    const uint32_t* pk = reinterpret_cast<const uint32_t*>(packed);
#define CQ_CM(RV, T) codes_matmul_kernel<RV, T><<<grid, 256, lds, s>>>(pk, rows, cols, X, ldx, stride_x, colw, roww, (int)r, \
                                                                       out, ldo, stride_out, colw_stride, roww_stride)
    const int rv = (int)ceil_div(r, 64);
    if (trans) {
        if (rv == 1) CQ_CM(1, true); else if (rv == 2) CQ_CM(2, true); else if (rv == 3) CQ_CM(3, true); else CQ_CM(4, true);
    } else {
        if (rv == 1) CQ_CM(1, false); else if (rv == 2) CQ_CM(2, false); else if (rv == 3) CQ_CM(3, false); else CQ_CM(4, false);
    }
#undef CQ_CM
    return check_launch("cq_codes_matmul");
}

int cq_codes_ysq_corr(const uint8_t* packed, int bits, const void* W, int dtype, const float* qscale, const float* colw,
                      int64_t colw_stride, int64_t batch, int64_t rows, int64_t cols, double* out, void* stream) {
    CQ_REQUIRE(packed && W && qscale && out, "cq_codes_ysq_corr: null argument");
    CQ_REQUIRE(bits == 2 && dtype == CQ_F16, "cq_codes_ysq_corr: 2-bit codes, fp16 W only");
    CQ_REQUIRE(batch > 0 && batch < 65536 && rows > 0 && cols > 0 && cols % 16 == 0, "cq_codes_ysq_corr: bad shape");
    codes_ysq_corr_kernel<<<(unsigned)batch, 1024, 0, as_stream(stream)>>>(
        reinterpret_cast<const uint32_t*>(packed), reinterpret_cast<const _Float16*>(W), qscale, colw, rows, cols, out, colw_stride);
    return check_launch("cq_codes_ysq_corr");
}

int cq_transpose_f16(const uint16_t* X, int64_t batch, int64_t rows, int64_t cols, uint16_t* Y, void* stream) {
    CQ_REQUIRE(X && Y && X != Y, "cq_transpose_f16: null or aliased argument");
    CQ_REQUIRE(batch > 0 && batch < 65536 && rows > 0 && cols > 0, "cq_transpose_f16: bad shape");
    const dim3 grid((unsigned)ceil_div(cols, 64), (unsigned)ceil_div(rows, 64), (unsigned)batch);
    transpose_f16_kernel<<<grid, 256, 0, as_stream(stream)>>>(X, rows, cols, Y);
    return check_launch("cq_transpose_f16");
}

int cq_sgram_count(const uint8_t* packed, int bits, int64_t batch, int64_t k, int64_t L, int32_t* row_nnz,
                   int32_t* perm, int64_t* slice_off, int64_t* total, int64_t Lh, int32_t* row_nnz1,
                   int32_t* slice_w1, const void* W, const float* qscale, const float* wcol, int64_t wcol_stride,
                   double* corr_ws, double* corr_out, void* stream) {
    CQ_REQUIRE(packed && row_nnz && perm && slice_off && total, "cq_sgram_count: null argument");
    CQ_REQUIRE(bits == 2, "cq_sgram_count: 2-bit codes only");
    CQ_REQUIRE(batch > 0 && batch < 65536 && k > 0 && L > 0 && L % 64 == 0, "cq_sgram_count: bad shape");
    CQ_REQUIRE(!W || (qscale && corr_ws && corr_out), "cq_sgram_count: the norm correction needs qscale, corr_ws, corr_out");
    CQ_REQUIRE(Lh >= L || (Lh > 0 && Lh % 64 == 0 && 2 * Lh >= L && row_nnz1 && slice_w1),
               "cq_sgram_count: an l-split needs Lh % 64 == 0, Lh >= L / 2, row_nnz1 and slice_w1");
    const bool split = Lh < L;
    hipStream_t s = as_stream(stream);
    sgram_count_kernel<<<dim3((unsigned)ceil_div(k, 4), (unsigned)batch), 256, 0, s>>>(
        packed, k, L, row_nnz, reinterpret_cast<const _Float16*>(W), qscale, wcol, corr_ws, split ? Lh : L,
        split ? row_nnz1 : nullptr, wcol_stride);
    sgram_slices_kernel<<<(unsigned)batch, 256, 0, s>>>(row_nnz, k, perm, slice_off, total, W ? corr_ws : nullptr,
                                                        corr_out, split ? row_nnz1 : nullptr, slice_w1);
    return check_launch("cq_sgram_count");
}

int cq_sgram_fill(const uint8_t* packed, int bits, int64_t batch, int64_t k, int64_t L, const int32_t* row_nnz,
                  const int32_t* perm, const int64_t* slice_off, const int32_t* slice_w1, int64_t Lh,
                  int64_t stride_ell, uint32_t* ell, void* stream) {
    CQ_REQUIRE(packed && row_nnz && perm && slice_off && ell, "cq_sgram_fill: null argument");
    CQ_REQUIRE(bits == 2, "cq_sgram_fill: 2-bit codes only");
    CQ_REQUIRE(batch > 0 && batch < 65536 && k > 0 && L > 0 && L % 64 == 0 && L < (1ll << 29),
               "cq_sgram_fill: bad shape");
    CQ_REQUIRE(Lh >= L || (Lh > 0 && Lh % 64 == 0 && 2 * Lh >= L && slice_w1), "cq_sgram_fill: bad l-split");
    sgram_fill_kernel<<<dim3((unsigned)ceil_div(k, 4 * SG_FILL_RW), (unsigned)batch), 256, 0, as_stream(stream)>>>(
        packed, k, L, row_nnz, perm, slice_off, slice_w1, Lh < L ? Lh : L, stride_ell, ell);
    return check_launch("cq_sgram_fill");
}

int cq_sgram_rows(int64_t L) {
    for (int r : {8, 4, 2})
        if ((size_t)L * r * sizeof(float) <= 150 * 1024) return r;
    return 0;
}

int64_t cq_sgram_split(int64_t k, int64_t L) {
    // two rows of E fit the LDS but not four: stage four rows half a contraction at a time when
    // the half-slab and the k x 4 output block fit (config 3's and config 4's 11008 contractions)
    if (cq_sgram_rows(L) != 2 || L % 64) return L;
    const int64_t Lh = ceil_div(L / 2, (int64_t)64) * 64;
    return ((size_t)Lh * 4 + (size_t)k * 4) * sizeof(float) <= 150 * 1024 ? Lh : L;
}

int cq_sgram_spmm(int dtype, const void* W, const uint8_t* packed, const float* qscale, const float* wcol,
                  int64_t wcol_stride, int64_t batch, int64_t k, int64_t L, const uint32_t* ell, const int32_t* perm,
                  const int64_t* slice_off, const int32_t* slice_w1, int64_t Lh, int64_t stride_ell, float* P,
                  void* stream) {
    CQ_REQUIRE(W && packed && qscale && ell && perm && slice_off && P, "cq_sgram_spmm: null argument");
    CQ_REQUIRE(dtype == CQ_F16, "cq_sgram_spmm: fp16 W only");
    CQ_REQUIRE(batch > 0 && batch < 65536 && k > 0 && L % 64 == 0, "cq_sgram_spmm: bad shape");
    hipStream_t s = as_stream(stream);
    const _Float16* Wh = reinterpret_cast<const _Float16*>(W);
    if (Lh < L) {   // l-split ELL (cq_sgram_split): R = 4 rows, two slabs of Lh values
        CQ_REQUIRE(Lh == cq_sgram_split(k, L) && slice_w1, "cq_sgram_spmm: Lh must be cq_sgram_split(k, L)");
        const size_t lds = ((size_t)Lh * 4 + (size_t)k * 4) * sizeof(float);
        sgram_spmm_kernel<4, -1, true><<<dim3((unsigned)ceil_div(k, 4), (unsigned)batch), SG_THREADS, lds, s>>>(
            Wh, packed, qscale, wcol, k, L, ell, perm, slice_off, slice_w1, Lh, stride_ell, P, wcol_stride);
        return check_launch("cq_sgram_spmm");
    }
    const int R = cq_sgram_rows(L);
    CQ_REQUIRE(R > 0, "cq_sgram_spmm: rows of %lld values do not fit the LDS", (long long)L);
    size_t lds = (size_t)L * R * sizeof(float);
    const dim3 grid((unsigned)ceil_div(k, R), (unsigned)batch);
    const int64_t nsw = ceil_div(ceil_div(k, SG_SLICE), SG_WAVES);  // slices per wave
    // the register-held form needs k <= L (the output block reuses the slab's LDS) and fits the
    // 128-VGPR budget of 16 waves per CU only at R = 8 (4 slices per wave): at R = 4 / 2 its 8 /
    // 16 inlined slice loops spilled to scratch (cfg3's R = 2 SpMM ran 587 ms instead of ~20)
    const bool held = k <= L && nsw * R <= 32 && R == 8;
    // R = 4 / 2: results through an LDS output block of their own where slab + block fit
    const bool ldsout = !held && R < 8 && lds + (size_t)k * R * sizeof(float) <= 150 * 1024;
    if (ldsout) lds += (size_t)k * R * sizeof(float);
#define CQ_SP(RR, NN) sgram_spmm_kernel<RR, NN><<<grid, SG_THREADS, lds, s>>>(Wh, packed, qscale, wcol, k, L, ell, \
                                                                             perm, slice_off, nullptr, L, stride_ell, P, \
                                                                             wcol_stride)
    if (R == 8) {
        if (held) CQ_SP(8, 4); else CQ_SP(8, 0);
    } else if (R == 4) {
        if (ldsout) CQ_SP(4, -1); else CQ_SP(4, 0);
    } else {
        if (ldsout) CQ_SP(2, -1); else CQ_SP(2, 0);
    }
#undef CQ_SP
    return check_launch("cq_sgram_spmm");
}

int cq_sgram_combine(const float* A, const float* P, const float* qscale, int64_t batch, int64_t k,
                     const double* bound, float out_scale, uint16_t* Gh, uint16_t* Gl, float* scale_out,
                     float* inv_out, float* G32, void* stream) {
    CQ_REQUIRE(A && P && qscale && bound && Gh && Gl && scale_out && inv_out, "cq_sgram_combine: null argument");
    CQ_REQUIRE(batch > 0 && batch < 65536 && k > 0 && k % 64 == 0 && out_scale > 0.f, "cq_sgram_combine: bad shape");
    const int64_t nt = k / 64;
    sgram_combine_kernel<<<dim3((unsigned)(nt * (nt + 1) / 2), (unsigned)batch), 256, 0, as_stream(stream)>>>(
        A, P, qscale, k, bound, out_scale, reinterpret_cast<_Float16*>(Gh), reinterpret_cast<_Float16*>(Gl),
        scale_out, inv_out, G32);
    return check_launch("cq_sgram_combine");
}

}  // extern "C"
