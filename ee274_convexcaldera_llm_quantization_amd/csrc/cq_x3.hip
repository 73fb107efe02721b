// Split-fp16 ("f16x3") products with the symmetric Gram G for the rank-r solver's
// Chebyshev filter (the dominant cost of the SVD replacing alg.py:217).
//
// Every fp32 operand x is carried as two fp16 halves, x*s = hi + lo with hi = f16(x*s) and
// lo = f16(x*s - hi) (s a power of two), so x*s is represented to 2^-22 relative.  A product
// sum_k a_k b_k is then hi_a hi_b + hi_a lo_b + lo_a hi_b (the dropped lo_a lo_b term is
// 2^-22 relative), each term one v_mfma_f32_16x16x32_f16 with fp32 accumulation: three fp16
// MFMAs give fp32-grade products (measured error at or below the fp32 MFMA GEMM's,
// DESIGN.md) on the fp16 matrix cores.
//
// Layout: the filter iterates on X^T (p x k, row-major) so both operands are K-contiguous:
//   C[j][i] = sum_k Xt[j][k] G[i][k]   ( = (G X)^T since G = G^T )
// gemm_x3v_kernel: tile 192 (rows of Xt) x 384 (rows of G) x 32, 768 threads = 12 waves of
// 96 x 64 (6 x 4 blocks of 16 x 16), operands global -> LDS by LDS-DMA into a 2-stage ring
// (144 KB; a 4-slot ring of hi halves only for the single-product steps), XOR-swizzled 16-B
// chunks so fragment reads are conflict-free; the transposed MFMA operand order gives each
// lane 4 consecutive output columns for a vectorised epilogue (Chebyshev recurrence, split
// halves of the next iterate, or the Gram's mirrored K-blocked halves).
#include <type_traits>
#include <numeric>

#include "cq_x3.h"

namespace cq {

__device__ __forceinline__ float sym_split_scale(double bound) {
    int e = 0;
    if (bound > 0.0 && isfinite(bound)) frexp(bound, &e);
    return ldexpf(1.f, 14 - e);
}

// ------------------------------------------------------------------ LDS images
// LDS images are linear per wave-instruction (16 rows x 64 B) with the 16-B chunk index
// XOR-swizzled on the global source address by xg_swz(row), a permutation of the row quad
// q = (row >> 2) & 3.  gfx950 serves a ds_read_b128 in four 16-lane groups, {0-3, 12-15,
// 20-27}, {4-11, 16-19, 28-31} and the same +32 (MI355X_MICROARCH.md, LDS banking): for the
// 16x16x32 fragment reads (lane = row l16 + 16 x chunk lq) a group holds rows of all four quads
// at two chunks, so q -> {0, 2, 3, 1} (not q itself, which left every group 2-way conflicted:
// 4 conflict cycles per read in the PMC counters) puts its 16 lanes on 16 different 16-byte
// bank slots; the 32x32x16 reads (32 rows x one chunk) stay conflict-free.
constexpr int XG_BK = 32;

__device__ __forceinline__ int xg_swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

__device__ __forceinline__ f16x8g xg_frag(const _Float16* img, int row, int chunk) {
    const int pc = chunk ^ xg_swz(row);
    return *reinterpret_cast<const f16x8g*>(img + row * XG_BK + pc * 8);
}

// ------------------------------------------------------------------ wide-tile LDS-DMA variant
// Tile 192 x 384 x 32 (12 waves of 96 x 64, 3 x 2 blocks of v_mfma_f32_32x32x16_f16), two
// 72 KB stages.  Per K step the CU loads 72 KB for 2x the MFMA work of the 192 x 192 tile
// (48 KB): the X^T slice is re-read by half as many tiles, which is what bounds the filter
// product (per-CU load path, ~10 B/clk/CU).
constexpr int XW_BM = 192, XW_BN = 384, XW_BK = 32;
constexpr int XW_THREADS = 768;
constexpr int XW_APART = XW_BM * XW_BK, XW_BPART = XW_BN * XW_BK;   // halves
constexpr int XW_STAGE = 2 * XW_APART + 2 * XW_BPART;
constexpr size_t XW_LDS_BYTES = (size_t)2 * XW_STAGE * sizeof(_Float16);  // 144 KB
constexpr int XW_PER_WAVE = (2 * XW_BM / 16 + 2 * XW_BN / 16) / (XW_THREADS / 64);  // 6
static_assert(XW_PER_WAVE == 6, "load split");

// One 16-B-per-lane LDS-DMA load (default cache policy: non-temporal loads of the once-read
// B panels measured 0.5-3 % slower, profiles/r04aq_nt_ab)
__device__ __forceinline__ void xw_load(const _Float16* src, _Float16* dst) {
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// Load plan: the wave-uniform part of each of this wave's 6 LDS-DMA loads (which image,
// which 16-row group) is scalar; the per-lane part is a 32-bit element offset computed once
// per tile, so a K step costs one 64-bit add per load (keeps the loop free of spills).
__device__ __forceinline__ void xw_plan(const X3K& a, int64_t m0, int64_t n0, int wid, int lane,
                                        uint32_t (&off)[XW_PER_WAVE]) {
#pragma unroll
    for (int u = 0; u < XW_PER_WAVE; ++u) {
        const int I = wid * XW_PER_WAVE + u;  // 0..71: Ah 0-11, Al 12-23, Bh 24-47, Bl 48-71
        const bool isA = I < 24;
        const int part = isA ? (I >= 12) : (I >= 48);
        const int sub = isA ? (I - 12 * part) : (I - 24 - 24 * part);
        const int row = 16 * sub + (lane >> 2);
        const int c = (lane & 3) ^ xg_swz(row);
        const int64_t lim = isA ? a.M : a.N;
        int64_t gr = (isA ? m0 : n0) + row;
        gr = gr < lim ? gr : lim - 1;
        off[u] = (uint32_t)(isA ? (a.a_blocked ? gr * 32 + c * 8 : gr * a.lda + c * 8)
                                : (a.b_blocked ? gr * 32 + c * 8 : gr * a.ldb + c * 8));
    }
}

__device__ __forceinline__ void xw_issue(const X3K& a, int64_t b, int64_t k0, _Float16* stage, int wid,
                                         const uint32_t (&off)[XW_PER_WAVE]) {
#pragma unroll
    for (int u = 0; u < XW_PER_WAVE; ++u) {
        const int I = wid * XW_PER_WAVE + u;
        const bool isA = I < 24;
        const int part = isA ? (I >= 12) : (I >= 48);
        const int sub = isA ? (I - 12 * part) : (I - 24 - 24 * part);
        const _Float16* base = isA ? (part ? a.Al : a.Ah) + b * a.sa + (a.a_blocked ? (k0 >> 5) * (a.lda * 32) : k0)
                                   : (part ? a.Bl : a.Bh) + b * a.sb + (a.b_blocked ? (k0 >> 5) * (a.ldb * 32) : k0);
        _Float16* dst = stage + (isA ? part * XW_APART : 2 * XW_APART + part * XW_BPART) + (16 * sub) * XW_BK;
        xw_load(base + off[u], dst);
    }
}

// Hi-only load plan (single product): the 36 hi-half wave-instructions of a stage spread
// 3 per wave (Ah 0-11, Bh 12-35).
constexpr int XW1_PER_WAVE = 3;
__device__ __forceinline__ void xw1_plan(const X3K& a, int64_t m0, int64_t n0, int wid, int lane,
                                         uint32_t (&off)[XW1_PER_WAVE]) {
#pragma unroll
    for (int u = 0; u < XW1_PER_WAVE; ++u) {
        const int I = wid * XW1_PER_WAVE + u;
        const bool isA = I < 12;
        const int sub = isA ? I : I - 12;
        const int row = 16 * sub + (lane >> 2);
        const int c = (lane & 3) ^ xg_swz(row);
        const int64_t lim = isA ? a.M : a.N;
        int64_t gr = (isA ? m0 : n0) + row;
        gr = gr < lim ? gr : lim - 1;
        off[u] = (uint32_t)(isA ? (a.a_blocked ? gr * 32 + c * 8 : gr * a.lda + c * 8)
                                : (a.b_blocked ? gr * 32 + c * 8 : gr * a.ldb + c * 8));
    }
}

// The 192 x 384 tile's K loop (shared by the filter/Gram product and the fused Q update):
// acc = A[m0.., :] B[n0.., :]^T over K, split-fp16 products; nt = 0 leaves acc = 0.
__device__ __forceinline__ void xw_mainloop(const X3K& a, int64_t b, int64_t m0, int64_t n0, int64_t nt,
                                            _Float16* smem, int wid, int lane, int wm, int wn,
                                            f32x16v (&acc)[3][2]) {
    const int lr = lane & 31, lh = lane >> 5;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    wid = __builtin_amdgcn_readfirstlane(wid);  // wave-uniform: load selection stays scalar
    uint32_t off[XW_PER_WAVE];
    if (nt > 0) {
        xw_plan(a, m0, n0, wid, lane, off);
        xw_issue(a, b, 0, smem, wid, off);
    }
    for (int64_t t = 0; t < nt; ++t) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // stage t landed everywhere; stage t-1 fully read
        if (t + 1 < nt) xw_issue(a, b, (t + 1) * XW_BK, smem + ((t + 1) & 1) * XW_STAGE, wid, off);
        const _Float16* sA = smem + (t & 1) * XW_STAGE;
        const _Float16* sB = sA + 2 * XW_APART;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            const int ch = 2 * s2 + lh;
            f16x8 ah[3], al[3], bh[2], bl[2];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int row = 96 * wm + 32 * i + lr;
                ah[i] = xg_frag(sA, row, ch);
                al[i] = xg_frag(sA + XW_APART, row, ch);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = 64 * wn + 32 * j + lr;
                bh[j] = xg_frag(sB, row, ch);
                bl[j] = xg_frag(sB + XW_BPART, row, ch);
            }
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bh[j], acc[i][j], 0, 0, 0);
                }
        }
    }
}

// ------------------------------------------------------------------ 16x16x32 MFMA variant
// Same tile, ring and LDS image as gemm_x3w_kernel; each wave's 96 x 64 block is 6 x 4
// v_mfma_f32_16x16x32_f16 tiles (one MFMA per 32-deep K step and product instead of two
// 32x32x16).  Under the chip's power limit the 16x16x32 form runs at a higher clock for the
// same work (MI355X_MICROARCH.md: ~1.15x the FLOP/s of 32x32x16 in bare loops).
// PERMB: block j's B fragment row for output register index t = 4 lq + r is LDS row
// 64 wn + 16 (t >> 2) + 4 j + (t & 3), so lane (l16, lq) ends up holding the 16 consecutive
// B rows 64 wn + 16 lq + [0, 16) in acc[i][0..3][0..3] (used by the fused Q update).
template <bool PERMB = false>
__device__ __forceinline__ void xv_mainloop(const X3K& a, int64_t b, int64_t m0, int64_t n0, int64_t nt,
                                            _Float16* smem, int wid, int lane, int wm, int wn,
                                            f32x4v (&acc)[6][4], int64_t kb = 0) {
    const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    wid = __builtin_amdgcn_readfirstlane(wid);
    uint32_t off[XW_PER_WAVE];
    auto issue = [&](int64_t k0, _Float16* st) { xw_issue(a, b, kb * XW_BK + k0, st, wid, off); };
    if (nt > 0) {
        xw_plan(a, m0, n0, wid, lane, off);
        issue(0, smem);
    }
    // a wave whose 96 x 64 output block lies wholly past the matrix edge (ragged last tiles)
    // or, for a symmetric Gram (tri), wholly below the diagonal is never stored: it runs only
    // its share of the loads and barriers, no fragment reads or MFMAs (fewer MFMA joules;
    // measured time-neutral — the workgroup still waits for its live waves at every barrier:
    // Gram 6.16 vs 6.13 ms, filter 2.65 vs 2.65 ms at B = 128/32, CQ_X3_NOSKIP=1 A/B;
    // per-strip or per-block skips inside the K loop make the allocator spill the accumulators)
    // (PERMB: a fragment's 16 columns interleave with stride 16 across the wave's 64; the
    // wave-level test below only needs the block's first row and column)
    const int64_t rs0 = m0 + 96 * wm, cs0 = n0 + 64 * wn;
    uint32_t live = (rs0 < a.M && cs0 < a.N && (!a.tri || cs0 + 63 >= rs0)) ? 1u : 0u;
    live = __builtin_amdgcn_readfirstlane(live);
    if (!live) {  // the wave's whole 96 x 64 block is dead: its share of the loads and barriers only
        for (int64_t t = 0; t < nt; ++t) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if (t + 1 < nt) issue((t + 1) * XW_BK, smem + ((t + 1) & 1) * XW_STAGE);
        }
        return;
    }
    for (int64_t t = 0; t < nt; ++t) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // stage t landed everywhere; stage t-1 fully read
        if (t + 1 < nt) issue((t + 1) * XW_BK, smem + ((t + 1) & 1) * XW_STAGE);
        const _Float16* sA = smem + (t & 1) * XW_STAGE;
        const _Float16* sB = sA + 2 * XW_APART;
        f16x8 bh[4], bl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = PERMB ? 64 * wn + 16 * (l16 >> 2) + 4 * j + (l16 & 3) : 64 * wn + 16 * j + l16;
            bh[j] = xg_frag(sB, row, lq);
            bl[j] = xg_frag(sB + XW_BPART, row, lq);
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int row = 96 * wm + 16 * i + l16;
            const f16x8 ah = xg_frag(sA, row, lq);
            const f16x8 al = xg_frag(sA + XW_APART, row, lq);
#pragma unroll
            for (int j = 0; j < 4; ++j) {  // transposed block: lanes run over A rows, registers over B rows
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], al, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl[j], ah, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], ah, acc[i][j], 0, 0, 0);
            }
        }
    }
}

// Single-product (hi x hi) K loop on a 4-slot ring: only the hi halves are loaded, so a
// stage is 36 KB (A hi 192 x 32 | B hi 384 x 32) and four fit the 144 KB the 2-stage split
// ring uses.  Loads of steps t+1..t+3 are issued while step t computes (counted vmcnt
// across the raw s_barrier: 3 LDS-DMA wave-instructions per wave and step): a hi-only step
// has a third of the split product's MFMA work, too little to cover an HBM round trip with
// one stage ahead.  Same fragments, MFMAs and accumulation order as xv_mainloop<false, true>.
constexpr int XV1_NS = 4;
constexpr int XV1_STAGE = XW_APART + XW_BPART;  // halves
static_assert((size_t)XV1_NS * XV1_STAGE * sizeof(_Float16) <= XW_LDS_BYTES, "single-product ring fits the LDS");

__device__ __forceinline__ void xv1_issue(const X3K& a, int64_t b, int64_t k0, _Float16* stage, int wid,
                                          const uint32_t (&off)[XW1_PER_WAVE]) {
#pragma unroll
    for (int u = 0; u < XW1_PER_WAVE; ++u) {
        const int I = wid * XW1_PER_WAVE + u;
        const bool isA = I < 12;
        const int sub = isA ? I : I - 12;
        const _Float16* base = isA ? a.Ah + b * a.sa + (a.a_blocked ? (k0 >> 5) * (a.lda * 32) : k0)
                                   : a.Bh + b * a.sb + (a.b_blocked ? (k0 >> 5) * (a.ldb * 32) : k0);
        _Float16* dst = stage + (isA ? 0 : XW_APART) + (16 * sub) * XW_BK;
        xw_load(base + off[u], dst);
    }
}

__device__ __forceinline__ void xv1_wait(int64_t after) {
    // this wave's loads of the stages issued after step t (at most XV1_NS - 2 = 2 at the wait,
    // step t + 3 being issued after it) may stay in flight
    if (after >= 2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (after == 1) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void xv1_mainloop(const X3K& a, int64_t b, int64_t m0, int64_t n0, int64_t nt,
                                             _Float16* smem, int wid, int lane, int wm, int wn,
                                             f32x4v (&acc)[6][4], int64_t kb = 0) {
    static_assert(XV1_NS == 4 && XW1_PER_WAVE == 3, "xv1_wait's counts");
    const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    wid = __builtin_amdgcn_readfirstlane(wid);
    uint32_t off[XW1_PER_WAVE];
    if (nt > 0) {
        xw1_plan(a, m0, n0, wid, lane, off);
        for (int64_t s = 0; s < XV1_NS - 1 && s < nt; ++s)
            xv1_issue(a, b, (kb + s) * XW_BK, smem + s * XV1_STAGE, wid, off);
    }
    const int64_t rs0 = m0 + 96 * wm, cs0 = n0 + 64 * wn;
    uint32_t live = (rs0 < a.M && cs0 < a.N && (!a.tri || cs0 + 63 >= rs0)) ? 1u : 0u;
    live = __builtin_amdgcn_readfirstlane(live);
    if (!live) {  // dead 96 x 64 block: its share of the loads and barriers only
        for (int64_t t = 0; t < nt; ++t) {
            xv1_wait(nt - 1 - t);
            __builtin_amdgcn_s_barrier();
            if (t + XV1_NS - 1 < nt)
                xv1_issue(a, b, (kb + t + XV1_NS - 1) * XW_BK, smem + ((t + XV1_NS - 1) & (XV1_NS - 1)) * XV1_STAGE,
                          wid, off);
        }
        return;
    }
    for (int64_t t = 0; t < nt; ++t) {
        xv1_wait(nt - 1 - t);
        __builtin_amdgcn_s_barrier();  // stage t landed everywhere; the slot of t - 1 fully read
        // slot (t + 3) % 4 last held step t - 1, whose reads every wave finished before this barrier
        if (t + XV1_NS - 1 < nt)
            xv1_issue(a, b, (kb + t + XV1_NS - 1) * XW_BK, smem + ((t + XV1_NS - 1) & (XV1_NS - 1)) * XV1_STAGE, wid,
                      off);
        const _Float16* sA = smem + (t & (XV1_NS - 1)) * XV1_STAGE;
        const _Float16* sB = sA + XW_APART;
        f16x8 bh[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) bh[j] = xg_frag(sB, 64 * wn + 16 * j + l16, lq);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const f16x8 ah = xg_frag(sA, 96 * wm + 16 * i + l16, lq);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], ah, acc[i][j], 0, 0, 0);
        }
    }
}

// Exact-B K loop (two products, al x bh + ah x bh): B is an fp16 matrix itself (W's halves
// under a split scale >= 1: lo = 0), so Bl is neither loaded nor multiplied.  A stage is
// 48 KB (A hi | A lo | B hi) and three fit the 144 KB: loads of steps t+1, t+2 are in flight
// while step t computes (4 LDS-DMA wave-instructions per wave and step, counted vmcnt across
// the barrier as in xv1_mainloop).  The same MFMAs in the same order as xv_mainloop minus the
// ah x bl term, whose product is exactly zero: the same bits.
constexpr int XV2_NS = 3;
constexpr int XV2_STAGE = 2 * XW_APART + XW_BPART;  // halves
constexpr int XW2_PER_WAVE = 4;
static_assert((size_t)XV2_NS * XV2_STAGE * sizeof(_Float16) <= XW_LDS_BYTES, "exact-B ring fits the LDS");
static_assert(XW2_PER_WAVE * (XW_THREADS / 64) == 2 * XW_BM / 16 + XW_BN / 16, "exact-B load split");

__device__ __forceinline__ void xw2_plan(const X3K& a, int64_t m0, int64_t n0, int wid, int lane,
                                         uint32_t (&off)[XW2_PER_WAVE]) {
#pragma unroll
    for (int u = 0; u < XW2_PER_WAVE; ++u) {
        const int I = wid * XW2_PER_WAVE + u;  // 0..47: Ah 0-11, Al 12-23, Bh 24-47
        const bool isA = I < 24;
        const int sub = isA ? I % 12 : I - 24;
        const int row = 16 * sub + (lane >> 2);
        const int c = (lane & 3) ^ xg_swz(row);
        const int64_t lim = isA ? a.M : a.N;
        int64_t gr = (isA ? m0 : n0) + row;
        gr = gr < lim ? gr : lim - 1;
        off[u] = (uint32_t)(isA ? (a.a_blocked ? gr * 32 + c * 8 : gr * a.lda + c * 8)
                                : (a.b_blocked ? gr * 32 + c * 8 : gr * a.ldb + c * 8));
    }
}

__device__ __forceinline__ void xv2_issue(const X3K& a, int64_t b, int64_t k0, _Float16* stage, int wid,
                                          const uint32_t (&off)[XW2_PER_WAVE]) {
#pragma unroll
    for (int u = 0; u < XW2_PER_WAVE; ++u) {
        const int I = wid * XW2_PER_WAVE + u;
        const bool isA = I < 24;
        const int part = I >= 12 && isA;
        const int sub = isA ? I % 12 : I - 24;
        const _Float16* base = isA ? (part ? a.Al : a.Ah) + b * a.sa + (a.a_blocked ? (k0 >> 5) * (a.lda * 32) : k0)
                                   : a.Bh + b * a.sb + (a.b_blocked ? (k0 >> 5) * (a.ldb * 32) : k0);
        _Float16* dst = stage + (isA ? part * XW_APART : 2 * XW_APART) + (16 * sub) * XW_BK;
        xw_load(base + off[u], dst);
    }
}

__device__ __forceinline__ void xv2_wait(int64_t after) {
    // this wave's loads of the stage issued after step t (at most XV2_NS - 2 = 1 at the wait,
    // step t + 2 being issued after it) may stay in flight
    if (after >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void xv2_mainloop(const X3K& a, int64_t b, int64_t m0, int64_t n0, int64_t nt,
                                             _Float16* smem, int wid, int lane, int wm, int wn,
                                             f32x4v (&acc)[6][4], int64_t kb = 0) {
    static_assert(XV2_NS == 3 && XW2_PER_WAVE == 4, "xv2_wait's counts");
    const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    wid = __builtin_amdgcn_readfirstlane(wid);
    uint32_t off[XW2_PER_WAVE];
    if (nt > 0) {
        xw2_plan(a, m0, n0, wid, lane, off);
        for (int64_t s = 0; s < XV2_NS - 1 && s < nt; ++s)
            xv2_issue(a, b, (kb + s) * XW_BK, smem + s * XV2_STAGE, wid, off);
    }
    const int64_t rs0 = m0 + 96 * wm, cs0 = n0 + 64 * wn;
    uint32_t live = (rs0 < a.M && cs0 < a.N && (!a.tri || cs0 + 63 >= rs0)) ? 1u : 0u;
    live = __builtin_amdgcn_readfirstlane(live);
    int slot = 0, nslot = XV2_NS - 1;  // slot of step t, slot the stage of step t + 2 goes to
    if (!live) {  // dead 96 x 64 block: its share of the loads and barriers only
        for (int64_t t = 0; t < nt; ++t) {
            xv2_wait(nt - 1 - t);
            __builtin_amdgcn_s_barrier();
            if (t + XV2_NS - 1 < nt) xv2_issue(a, b, (kb + t + XV2_NS - 1) * XW_BK, smem + nslot * XV2_STAGE, wid, off);
            nslot = nslot == XV2_NS - 1 ? 0 : nslot + 1;
        }
        return;
    }
    for (int64_t t = 0; t < nt; ++t) {
        xv2_wait(nt - 1 - t);
        __builtin_amdgcn_s_barrier();  // stage t landed everywhere; the slot of t - 1 fully read
        if (t + XV2_NS - 1 < nt) xv2_issue(a, b, (kb + t + XV2_NS - 1) * XW_BK, smem + nslot * XV2_STAGE, wid, off);
        {
            const _Float16* sA = smem + slot * XV2_STAGE;
            const _Float16* sB = sA + 2 * XW_APART;
            f16x8 bh[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) bh[j] = xg_frag(sB, 64 * wn + 16 * j + l16, lq);
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const int row = 96 * wm + 16 * i + l16;
                const f16x8 ah = xg_frag(sA, row, lq);
                const f16x8 al = xg_frag(sA + XW_APART, row, lq);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], al, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], ah, acc[i][j], 0, 0, 0);
                }
            }
        }
        slot = slot == XV2_NS - 1 ? 0 : slot + 1;
        nslot = nslot == XV2_NS - 1 ? 0 : nslot + 1;
    }
}

// Gram tile order.  Only the tiles on or above the diagonal are launched: 384 x 384 blocks
// (I, J >= I) of tiles tm = 2I, 2I + 1 (192 rows) by tn = J.  The blocks are enumerated per
// matrix in 4 x 4 super-blocks (row-major over super-blocks, then over their blocks), and
// the launch index is dealt to the XCDs (workgroup i runs on XCD i % 8) in runs of
// GRAM_RUN consecutive tiles of that order: the 32 tiles an XCD holds at a time share 8 row
// and 4 column panels of Y instead of ~30 of each, so their K slices are re-read from the
// XCD's L2 rather than from the memory-side cache, and all XCDs stay on the same one or two
// matrices (whose operands fit that 256 MB cache).  The order changes nothing in a tile's
// arithmetic.
constexpr int GRAM_SB = 4, GRAM_RUN = 32;

__device__ __forceinline__ int64_t gram_block_tiles(int64_t I, int64_t tiles_m) {
    return 2 * I + 1 < tiles_m ? 2 : 1;
}

__device__ void gram_tile(const X3K& a, int64_t orig, int64_t& b, int64_t& tm, int64_t& tn) {
    const int64_t live = a.tiles_live, total = live * a.batch;
    constexpr int64_t S = 8 * GRAM_RUN;
    int64_t lin = orig;
    if (orig < total / S * S) {
        const int64_t k = orig / 8, x = orig % 8;
        lin = (k / GRAM_RUN) * S + x * GRAM_RUN + k % GRAM_RUN;
    }
    b = lin / live;
    int64_t j = lin % live;
    const int64_t nb = a.tiles_n, nsb = (nb + GRAM_SB - 1) / GRAM_SB;
    for (int64_t si = 0; si < nsb; ++si) {
        for (int64_t sj = si; sj < nsb; ++sj) {
            const int64_t i1 = min<int64_t>(GRAM_SB * si + GRAM_SB, nb), j1 = min<int64_t>(GRAM_SB * sj + GRAM_SB, nb);
            for (int64_t I = GRAM_SB * si; I < i1; ++I) {
                const int64_t per = gram_block_tiles(I, a.tiles_m);
                const int64_t jb = max<int64_t>(GRAM_SB * sj, I);
                const int64_t cnt = (j1 > jb ? j1 - jb : 0) * per;
                if (j < cnt) {
                    tn = jb + j / per;
                    tm = 2 * I + j % per;
                    return;
                }
                j -= cnt;
            }
        }
    }
    tm = tn = 0;  // unreachable for lin < total
}

// XM: 0 = three split products, 1 = one hi x hi product, 2 = exact B (two products, Bl unread)
template <int XM>
__global__ __launch_bounds__(XW_THREADS, 1) void gemm_x3v_kernel(X3K a) {
    extern __shared__ __attribute__((aligned(16))) char xv_smem_raw[];
    _Float16* smem = reinterpret_cast<_Float16*>(xv_smem_raw);
    int64_t tn, tm, b;
    if (a.sym_out) {
        gram_tile(a, blockIdx.x, b, tm, tn);
    } else {
        const int64_t total = a.tiles_n * a.tiles_m * a.batch;
        const int64_t orig = a.ksplit > 1 ? blockIdx.x / a.ksplit : blockIdx.x;   // split-K: chunk fastest
        const int64_t q = total / 8, r8 = total % 8, xcd = orig % 8;
        const int64_t lin = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
        // row tiles fastest: when A has more than one 192-row tile (the filter at p > 192), the
        // tiles sharing one 384-row panel of B (G) run together on one XCD and read its K slices
        // once from HBM and again from L2
        tm = lin % a.tiles_m;
        tn = (lin / a.tiles_m) % a.tiles_n;
        b = lin / (a.tiles_n * a.tiles_m);
    }
    const int64_t m0 = tm * XW_BM, n0 = tn * XW_BN;
    if (a.tri && n0 + XW_BN <= m0) return;

    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid & 1, wn = wid >> 1;  // rows 96 wm .. +96, cols 64 wn .. +64
    const int l16 = lane & 15, lq = lane >> 4;

    f32x4v acc[6][4];
    const bool live = !a.active || a.active[b];
    const int64_t nk = a.K / XW_BK;
    int64_t kb = 0, kn = nk;
    if (a.ksplit > 1) {   // this workgroup's K chunk
        const int64_t ks = blockIdx.x % a.ksplit;
        kb = ks * nk / a.ksplit;
        kn = (ks + 1) * nk / a.ksplit - kb;
    }
    if constexpr (XM == 1) {
        xv1_mainloop(a, b, m0, n0, live ? kn : 0, smem, wid, lane, wm, wn, acc, kb);
    } else if constexpr (XM == 2) {
        xv2_mainloop(a, b, m0, n0, live ? kn : 0, smem, wid, lane, wm, wn, acc, kb);
    } else {
        xv_mainloop<false>(a, b, m0, n0, live ? kn : 0, smem, wid, lane, wm, wn, acc, kb);
    }

    const float sc = a.inv_scale[b];
    if (a.ksplit > 1) {   // partial products (times the operand scale) for x3_splitk_epi_kernel
        float* part = a.part + ((blockIdx.x % a.ksplit) * a.batch + b) * a.M * a.N;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int64_t row = m0 + 96 * wm + 16 * i + l16;
            if (row >= a.M) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t col = n0 + 64 * wn + 16 * j + 4 * lq;
                if (col >= a.N) continue;
                // N % 4 == 0 (host check): 4 columns, 16-byte aligned
                *reinterpret_cast<float4*>(part + row * a.N + col) =
                    make_float4(acc[i][j][0] * sc, acc[i][j][1] * sc, acc[i][j][2] * sc, acc[i][j][3] * sc);
            }
        }
        return;
    }
    if (a.sym_out) {
        // symmetric Gram: entries on/above the diagonal are written at (row, col) and, mirrored,
        // at (col, row) of the K-blocked split (the lower triangle of a straddling tile is not
        // used, so the split is exactly symmetric); (fp32 C too if given)
        const float gs = sym_split_scale(a.out_bound[b]);
        if (tm == 0 && tn == 0 && threadIdx.x == 0) {
            a.scale_out[b] = gs;
            a.inv_out[b] = 1.f / (gs * a.out_scale);
        }
        const int64_t M = a.M;
        _Float16* Oh = a.Oh + b * a.so;
        _Float16* Ol = a.Ol + b * a.so;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int64_t row = m0 + 96 * wm + 16 * i + l16;
            if (row >= M) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t col = n0 + 64 * wn + 16 * j + 4 * lq;
                if (col + 3 < row || col >= a.N) continue;
                _Float16 h[4], l[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v = acc[i][j][r] * sc;
                    if (a.C && col + r >= row && col + r < a.N) a.C[b * a.sc + row * a.ldc + col + r] = v;
                    const float hs = v * gs;
                    h[r] = (_Float16)hs;
                    l[r] = (_Float16)(hs - (float)h[r]);
                }
                const int64_t o = (col >> 5) * (M * 32) + row * 32 + (col & 31);
                if (col >= row && col + 3 < a.N) {
                    *reinterpret_cast<uint2*>(Oh + o) = *reinterpret_cast<const uint2*>(h);
                    *reinterpret_cast<uint2*>(Ol + o) = *reinterpret_cast<const uint2*>(l);
                } else {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (col + r >= row && col + r < a.N) { Oh[o + r] = h[r]; Ol[o + r] = l[r]; }
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {  // mirror (col + r, row)
                    const int64_t c = col + r;
                    if (c > row && c < a.N) {
                        const int64_t om = (row >> 5) * (M * 32) + c * 32 + (row & 31);
                        Oh[om] = h[r];
                        Ol[om] = l[r];
                    }
                }
            }
        }
        return;
    }
    const float al_ = !live ? 0.f : a.alpha_v ? a.alpha_v[b] : 1.f;
    const float be_ = !live ? 0.f : a.beta_v ? a.beta_v[b] : 0.f;
    const float ga_ = !live ? 1.f : a.gamma_v ? a.gamma_v[b] : 0.f;
    bool ovf = false;
    uint32_t amx = 0u;   // |C| max bits (absmax_out)
    // lane = C row (A row), registers r = 4 consecutive C columns: 16-byte fp32 and 8-byte
    // fp16 accesses (host guarantees N % 4 == 0 and 16-byte aligned rows)
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    auto al8 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; };
    const bool vec = (a.N & 3) == 0 && (a.ldc & 3) == 0 && (a.sc & 3) == 0 && al16(a.C) &&
                     (!a.P || ((a.ldp & 3) == 0 && (a.sp & 3) == 0 && al16(a.P))) &&
                     (!a.D || ((a.ldd & 3) == 0 && (a.sd & 3) == 0 && al16(a.D))) &&
                     (!a.Oh || ((a.o_blocked || (a.ldo & 3) == 0) && (a.so & 3) == 0 && al8(a.Oh) && al8(a.Ol)));
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int64_t row = m0 + 96 * wm + 16 * i + l16;
        if (row >= a.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t col = n0 + 64 * wn + 16 * j + 4 * lq;
            if (col >= a.N) continue;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = al_ * (acc[i][j][r] * sc);
            if (a.colw) {
                const float* cw = a.colw + b * a.scolw;
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (col + r < a.N) v[r] *= cw[col + r];
            }
            if (vec) {
                if (a.P && be_ != 0.f) {
                    const float4 pv = *reinterpret_cast<const float4*>(a.P + b * a.sp + row * a.ldp + col);
                    v[0] += be_ * pv.x; v[1] += be_ * pv.y; v[2] += be_ * pv.z; v[3] += be_ * pv.w;
                }
                if (a.D && ga_ != 0.f) {
                    const float4 dv = *reinterpret_cast<const float4*>(a.D + b * a.sd + row * a.ldd + col);
                    v[0] += ga_ * dv.x; v[1] += ga_ * dv.y; v[2] += ga_ * dv.z; v[3] += ga_ * dv.w;
                }
                *reinterpret_cast<float4*>(a.C + b * a.sc + row * a.ldc + col) = make_float4(v[0], v[1], v[2], v[3]);
                if (a.Ct) {   // C^T: lanes l16 (consecutive rows) make 64-byte runs per column
#pragma unroll
                    for (int r = 0; r < 4; ++r) a.Ct[b * a.sct + (col + r) * a.M + row] = v[r];
                }
                if (a.absmax_out)
                    amx = max(amx, max(max(abs_bits(v[0]), abs_bits(v[1])), max(abs_bits(v[2]), abs_bits(v[3]))));
                if (a.Oh) {
                    _Float16 h[4], l[4];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float hs = v[r] * a.out_scale;
                        h[r] = (_Float16)hs;
                        l[r] = (_Float16)(hs - (float)h[r]);
                        ovf |= !(fabsf(hs) < 65504.f);
                    }
                    const int64_t o = b * a.so + (a.o_blocked ? (col >> 5) * (a.M * 32) + row * 32 + (col & 31)
                                                              : row * a.ldo + col);
                    *reinterpret_cast<uint2*>(a.Oh + o) = *reinterpret_cast<const uint2*>(h);
                    *reinterpret_cast<uint2*>(a.Ol + o) = *reinterpret_cast<const uint2*>(l);
                }
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t c = col + r;
                    if (c >= a.N) continue;
                    float w = v[r];
                    if (a.P && be_ != 0.f) w += be_ * a.P[b * a.sp + row * a.ldp + c];
                    if (a.D && ga_ != 0.f) w += ga_ * a.D[b * a.sd + row * a.ldd + c];
                    a.C[b * a.sc + row * a.ldc + c] = w;
                    if (a.Ct) a.Ct[b * a.sct + c * a.M + row] = w;
                    amx = max(amx, abs_bits(w));
                    if (a.Oh) {
                        const float hs = w * a.out_scale;
                        const _Float16 h = (_Float16)hs;
                        const int64_t o = b * a.so + (a.o_blocked ? (c >> 5) * (a.M * 32) + row * 32 + (c & 31)
                                                                  : row * a.ldo + c);
                        a.Oh[o] = h;
                        a.Ol[o] = (_Float16)(hs - (float)h);
                        ovf |= !(fabsf(hs) < 65504.f);
                    }
                }
            }
        }
    }
    if (ovf) atomicOr(a.overflow + b, 1);
    if (a.absmax_out) {
        amx = wave_max_u32(amx);
        if (lane == 0 && amx) atomicMax(a.absmax_out + b, amx);
    }
}


// ------------------------------------------------------------------ 256 x 256 tile variant
// For the rank-256 products (config 5: the LPLR loop's Y Rw^T and L^T res, the normal-equation
// multiplies, all with r = 256 as M or N), where the 192 x 384 tile leaves a third of every
// tile idle (256 = 192 + 64 rows, or 256 of 384 columns).  Tile 256 x 256 x 32: 8 waves of
// 128 x 64 (8 x 4 blocks of v_mfma_f32_16x16x32_f16, 128 accumulator VGPRs, two waves per
// SIMD), the same LDS image (16-row x 64-B pieces, swizzled chunks), the same fragment reads
// and MFMA order per block as xv_mainloop<false> (al x bh, ah x bl, ah x bh per K step), so a
// block's sum is the same bits as the 192 x 384 kernel's; the same per-element bytes per flop
// (2/256 + 2/256 vs 2/192 + 2/384).  Two 64 KB stages.  Plain products only (C = alpha A B^T
// scale): M % 256 == 0, N % 256 == 0, no split-K / P / D / split output / colw.
constexpr int XS_BM = 256, XS_BN = 256, XS_THREADS = 512;
constexpr int XS_APART = XS_BM * XW_BK, XS_BPART = XS_BN * XW_BK;   // halves
constexpr int XS_STAGE = 2 * XS_APART + 2 * XS_BPART;
constexpr size_t XS_LDS_BYTES = (size_t)2 * XS_STAGE * sizeof(_Float16);  // 128 KB
constexpr int XS_PER_WAVE = (2 * XS_BM / 16 + 2 * XS_BN / 16) / (XS_THREADS / 64);  // 8
static_assert(XS_PER_WAVE == 8, "load split");

__device__ __forceinline__ void xs_plan(const X3K& a, int64_t m0, int64_t n0, int wid, int lane,
                                        uint32_t (&off)[XS_PER_WAVE]) {
#pragma unroll
    for (int u = 0; u < XS_PER_WAVE; ++u) {
        const int I = wid * XS_PER_WAVE + u;  // 0..63: Ah 0-15, Al 16-31, Bh 32-47, Bl 48-63
        const bool isA = I < 32;
        const int sub = I & 15;
        const int row = 16 * sub + (lane >> 2);
        const int c = (lane & 3) ^ xg_swz(row);
        const int64_t gr = (isA ? m0 : n0) + row;
        off[u] = (uint32_t)(isA ? (a.a_blocked ? gr * 32 + c * 8 : gr * a.lda + c * 8)
                                : (a.b_blocked ? gr * 32 + c * 8 : gr * a.ldb + c * 8));
    }
}

__device__ __forceinline__ void xs_issue(const X3K& a, int64_t b, int64_t k0, _Float16* stage, int wid,
                                         const uint32_t (&off)[XS_PER_WAVE]) {
#pragma unroll
    for (int u = 0; u < XS_PER_WAVE; ++u) {
        const int I = wid * XS_PER_WAVE + u;
        const bool isA = I < 32;
        const int part = (I >> 4) & 1;
        const int sub = I & 15;
        const _Float16* base = isA ? (part ? a.Al : a.Ah) + b * a.sa + (a.a_blocked ? (k0 >> 5) * (a.lda * 32) : k0)
                                   : (part ? a.Bl : a.Bh) + b * a.sb + (a.b_blocked ? (k0 >> 5) * (a.ldb * 32) : k0);
        _Float16* dst = stage + (isA ? part * XS_APART : 2 * XS_APART + part * XS_BPART) + (16 * sub) * XW_BK;
        xw_load(base + off[u], dst);
    }
}

__global__ __launch_bounds__(XS_THREADS, 1) void gemm_x3s_kernel(X3K a) {
    extern __shared__ __attribute__((aligned(16))) char xs_smem_raw[];
    _Float16* smem = reinterpret_cast<_Float16*>(xs_smem_raw);
    const int64_t total = a.tiles_n * a.tiles_m * a.batch;
    const int64_t orig = blockIdx.x;
    const int64_t q = total / 8, r8 = total % 8, xcd = orig % 8;
    const int64_t lin = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
    const int64_t tm = lin % a.tiles_m, tn = (lin / a.tiles_m) % a.tiles_n, b = lin / (a.tiles_n * a.tiles_m);
    const int64_t m0 = tm * XS_BM, n0 = tn * XS_BN;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid & 1, wn = wid >> 1;  // rows 128 wm .. +128, cols 64 wn .. +64
    const int l16 = lane & 15, lq = lane >> 4;
    f32x4v acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    uint32_t off[XS_PER_WAVE];
    xs_plan(a, m0, n0, wid, lane, off);
    const int64_t nt = a.K / XW_BK;
    xs_issue(a, b, 0, smem, wid, off);
    for (int64_t t = 0; t < nt; ++t) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // stage t landed everywhere; stage t-1 fully read
        if (t + 1 < nt) xs_issue(a, b, (t + 1) * XW_BK, smem + ((t + 1) & 1) * XS_STAGE, wid, off);
        const _Float16* sA = smem + (t & 1) * XS_STAGE;
        const _Float16* sB = sA + 2 * XS_APART;
        f16x8 bh[4], bl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = 64 * wn + 16 * j + l16;
            bh[j] = xg_frag(sB, row, lq);
            bl[j] = xg_frag(sB + XS_BPART, row, lq);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int row = 128 * wm + 16 * i + l16;
            const f16x8 ah = xg_frag(sA, row, lq);
            const f16x8 al = xg_frag(sA + XS_APART, row, lq);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], al, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl[j], ah, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], ah, acc[i][j], 0, 0, 0);
            }
        }
    }
    // C = alpha (acc scale), the same two roundings as gemm_x3v_kernel's epilogue
    const float sc = a.inv_scale[b], al = a.alpha_v ? a.alpha_v[b] : 1.f;
    uint32_t mx = 0u;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int64_t row = m0 + 128 * wm + 16 * i + l16;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t col = n0 + 64 * wn + 16 * j + 4 * lq;
            const float4 v = make_float4(al * (acc[i][j][0] * sc), al * (acc[i][j][1] * sc), al * (acc[i][j][2] * sc),
                                         al * (acc[i][j][3] * sc));
            *reinterpret_cast<float4*>(a.C + b * a.sc + row * a.ldc + col) = v;
            mx = max(mx, max(max(abs_bits(v.x), abs_bits(v.y)), max(abs_bits(v.z), abs_bits(v.w))));
        }
    }
    if (a.absmax_out) {
        mx = wave_max_u32(mx);
        if (lane == 0 && mx) atomicMax(a.absmax_out + b, mx);
    }
}

// Split-K epilogue: C = alpha (sum of the ksplit partials, in chunk order) + beta P + gamma D,
// and the split halves of C, as gemm_x3v_kernel's epilogue does (inactive matrices: C = D).
// One thread per 4 consecutive columns (N % 4 == 0).
__global__ __launch_bounds__(256) void x3_splitk_epi_kernel(X3K a) {
    const int64_t nq = a.N / 4;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t b = blockIdx.y;
    const bool in = t < a.M * nq;
    uint32_t amx = 0u;
    if (in) {
    const int64_t row = t / nq, col = 4 * (t % nq);
    const bool live = !a.active || a.active[b];
    const float al_ = !live ? 0.f : a.alpha_v ? a.alpha_v[b] : 1.f;
    const float be_ = !live ? 0.f : a.beta_v ? a.beta_v[b] : 0.f;
    const float ga_ = !live ? 1.f : a.gamma_v ? a.gamma_v[b] : 0.f;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < a.ksplit; ++ks) {
        const float4 pv = *reinterpret_cast<const float4*>(a.part + ((ks * a.batch + b) * a.M + row) * a.N + col);
        s[0] += pv.x; s[1] += pv.y; s[2] += pv.z; s[3] += pv.w;
    }
    bool ovf = false;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float w = al_ * s[r];
        if (a.colw) w *= a.colw[b * a.scolw + col + r];
        if (a.P && be_ != 0.f) w += be_ * a.P[b * a.sp + row * a.ldp + col + r];
        if (a.D && ga_ != 0.f) w += ga_ * a.D[b * a.sd + row * a.ldd + col + r];
        a.C[b * a.sc + row * a.ldc + col + r] = w;
        if (a.Ct) a.Ct[b * a.sct + (col + r) * a.M + row] = w;
        amx = max(amx, abs_bits(w));
        if (a.Oh) {
            const float hs = w * a.out_scale;
            const _Float16 h = (_Float16)hs;
            const int64_t c = col + r;
            const int64_t o = b * a.so + (a.o_blocked ? (c >> 5) * (a.M * 32) + row * 32 + (c & 31) : row * a.ldo + c);
            a.Oh[o] = h;
            a.Ol[o] = (_Float16)(hs - (float)h);
            ovf |= !(fabsf(hs) < 65504.f);
        }
    }
    if (ovf) atomicOr(a.overflow + b, 1);
    }
    if (a.absmax_out) {   // (every lane reaches the wave reduction)
        amx = wave_max_u32(amx);
        if ((threadIdx.x & 63) == 0 && amx) atomicMax(a.absmax_out + b, amx);
    }
}

// ------------------------------------------------------------------ fused Q update
// maybe_update_Q (alg.py:253-283) + quantize_matrix (alg.py:245-250, quantization.py:244-269)
// without materialising the residual: res = W - L R is recomputed per 192 x 384 tile from
// the split-fp16 halves of L (m x r) and R^T (n x r) (K = r; r = 0: res = W exactly) in two
// passes over W:
//   pass 0: per-matrix max |res| (uint bits, NaN sorts above inf like torch.max) -> atomicMax;
//   pass 1: scale = max(absmax, eps); code = rint((res / scale) k) (IEEE division, then the
//           multiply, round-half-even: the reference's two roundings); packed offset-binary
//           codes (c + k, MSB-first: 4 per byte at 2 bits, 2 per byte at 4 bits) or int8/int16
//           codes; sum_j w_j (deq - res)^2 per tile in fp64 (deterministic 2-stage sum).
// Both passes evaluate res with identical code, so pass 1 sees pass 0's values bit for bit.

template <int PASS, int BITS>
__global__ __launch_bounds__(XW_THREADS, 1) void q_update_x3_kernel(QUK q) {
    extern __shared__ __attribute__((aligned(16))) char qu_smem_raw[];
    _Float16* smem = reinterpret_cast<_Float16*>(qu_smem_raw);
    const X3K& a = q.x;
    const int64_t tiles = a.tiles_n * a.tiles_m;
    const int64_t total = tiles * a.batch;
    const int64_t orig = blockIdx.x;
    const int64_t qq = total / 8, r8 = total % 8, xcd = orig % 8;
    const int64_t lin = (xcd < r8 ? xcd * (qq + 1) : r8 * (qq + 1) + (xcd - r8) * qq) + orig / 8;
    const int64_t tile = lin % tiles;
    const int64_t tn = tile % a.tiles_n, tm = tile / a.tiles_n;
    const int64_t b = lin / tiles;
    const int64_t m0 = tm * XW_BM, n0 = tn * XW_BN;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid & 1, wn = wid >> 1;
    const int lr = lane & 31, lh = lane >> 5;

    // transposed product: A operand = R^T (tile rows = columns of W), B operand = L (tile
    // columns = rows of W), so each lane owns one row of W and holds 4 runs of 4 consecutive
    // columns: W loads are 8-byte vectors and 4 two-bit codes make one byte in-lane
    f32x16v acc[3][2];
    xw_mainloop(a, b, m0, n0, a.K / XW_BK, smem, wid, lane, wm, wn, acc);
    const float sc = a.K > 0 ? a.inv_scale[b] : 0.f;
    const int64_t MN = q.m * q.n;
    const _Float16* Wh = reinterpret_cast<const _Float16*>(q.W) + b * MN;
    const float* Wf = reinterpret_cast<const float*>(q.W) + b * MN;

    constexpr float kq = (float)((1 << (BITS - 1)) - 1);
    uint32_t mx = 0;
    double err = 0.0;
    float s = 0.f;
    if (PASS == 1) s = quant_scale(q.absmax[b], q.eps);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int64_t row = n0 + 64 * wn + 32 * j + lr;  // row of W (tile column)
        if (row >= q.m) continue;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                const int64_t col = m0 + 96 * wm + 32 * i + 8 * g4 + 4 * lh;  // 4 consecutive columns
                if (col >= q.n) continue;  // n % 4 == 0: a run is all in or all out
                const int64_t e = row * q.n + col;
                float w4[4];
                if (q.wf16) {
                    const uint2 raw = *reinterpret_cast<const uint2*>(Wh + e);
                    const _Float16* hv = reinterpret_cast<const _Float16*>(&raw);
#pragma unroll
                    for (int u = 0; u < 4; ++u) w4[u] = (float)hv[u];
                } else {
                    const float4 f = *reinterpret_cast<const float4*>(Wf + e);
                    w4[0] = f.x; w4[1] = f.y; w4[2] = f.z; w4[3] = f.w;
                }
                float v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    v[u] = a.K > 0 ? w4[u] - acc[i][j][4 * g4 + u] * sc : w4[u];  // res = W - L R (alg.py:262)
                if (PASS == 0) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) mx = max(mx, abs_bits(v[u]));
                } else {
                    float c[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        c[u] = quant_code(v[u], s, kq);
                        const float d = dequant(c[u], kq, s) - v[u];
                        err += (double)(d * d) * (q.ew ? (double)q.ew[b * q.sew + col + u] : 1.0);
                    }
                    if constexpr (BITS <= 4) {
                        if (q.packed) {
                            uint32_t uq[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) uq[u] = (uint32_t)((int)c[u] + (int)kq);
                            if (BITS == 2) {
                                q.packed[(b * MN + e) / 4] = (uint8_t)((uq[0] << 6) | (uq[1] << 4) | (uq[2] << 2) | uq[3]);
                            } else {
                                *reinterpret_cast<uchar2*>(q.packed + (b * MN + e) / 2) =
                                    make_uchar2((uint8_t)((uq[0] << 4) | uq[1]), (uint8_t)((uq[2] << 4) | uq[3]));
                            }
                        }
                    }
                    if (q.codes) {
                        if (BITS <= 8)
                            *reinterpret_cast<char4*>(reinterpret_cast<int8_t*>(q.codes) + b * MN + e) =
                                make_char4((signed char)(int)c[0], (signed char)(int)c[1], (signed char)(int)c[2],
                                           (signed char)(int)c[3]);
                        else
                            *reinterpret_cast<short4*>(reinterpret_cast<int16_t*>(q.codes) + b * MN + e) =
                                make_short4((short)(int)c[0], (short)(int)c[1], (short)(int)c[2], (short)(int)c[3]);
                    }
                }
            }
    }
    if (PASS == 0) {
        mx = wave_max_u32(mx);
        if (lane == 0 && mx) atomicMax(q.absmax + b, mx);
    } else if (q.part) {
        __shared__ double red[16];
        const double tsum = block_sum_f64(err, red);
        if (threadIdx.x == 0) q.part[b * tiles + tile] = tsum;
    }
}

// Fused Q update on the 16x16x32 ring (default): A = L halves (tile rows = rows of W),
// B = R^T halves with PERMB, so each lane owns 16 consecutive columns of one W row: W loads
// of 32 B (fp16) per lane, one 32-bit store of 16 two-bit codes (64 bits at 4 bits), and a
// wave-instruction covers 16 rows x 64 columns.  Same two passes and arithmetic as
// q_update_x3_kernel (res = W - L R with identical code in both passes).  n % 16 == 0.
template <int PASS, int BITS, int DT>
__global__ __launch_bounds__(XW_THREADS, 1) void q_update_v_kernel(QUK q) {
    extern __shared__ __attribute__((aligned(16))) char qv_smem_raw[];
    _Float16* smem = reinterpret_cast<_Float16*>(qv_smem_raw);
    const X3K& a = q.x;
    const int64_t tiles = a.tiles_n * a.tiles_m;
    const int64_t total = tiles * a.batch;
    const int64_t orig = blockIdx.x;
    const int64_t qq = total / 8, r8 = total % 8, xcd = orig % 8;
    const int64_t lin = (xcd < r8 ? xcd * (qq + 1) : r8 * (qq + 1) + (xcd - r8) * qq) + orig / 8;
    const int64_t tile = lin % tiles;
    const int64_t tn = tile % a.tiles_n, tm = tile / a.tiles_n;
    const int64_t b = lin / tiles;
    const int64_t m0 = tm * XW_BM, n0 = tn * XW_BN;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wm = wid & 1, wn = wid >> 1;
    const int l16 = lane & 15, lq = lane >> 4;

    f32x4v acc[6][4];
    xv_mainloop<true>(a, b, m0, n0, a.K / XW_BK, smem, wid, lane, wm, wn, acc);
    const float sc = a.K > 0 ? a.inv_scale[b] : 0.f;
    const int64_t MN = q.m * q.n;
    const _Float16* Wh = reinterpret_cast<const _Float16*>(q.W) + b * MN;
    const float* Wf = reinterpret_cast<const float*>(q.W) + b * MN;
    constexpr float kq = (float)((1 << (BITS - 1)) - 1);
    uint32_t mx = 0;
    double err = 0.0;
    float s = 0.f;
    if (PASS == 1) s = quant_scale(q.absmax[b], q.eps);
    const float ys = 1.f / s, yk = 1.f / kq;  // IEEE reciprocals for div_rn
    const int64_t col = n0 + 64 * wn + 16 * lq;  // this lane's 16 consecutive columns
    const bool colok = col < q.n;                 // n % 16 == 0: a run is all in or all out
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int64_t row = m0 + 96 * wm + 16 * i + l16;
        if (row >= q.m || !colok) continue;
        const int64_t e = row * q.n + col;
        // W kept packed (fp16: 8 registers) and converted 4 columns at a time
        uint4 wr[4];
        if (DT == CQ_F16) {
            wr[0] = *reinterpret_cast<const uint4*>(Wh + e);
            wr[1] = *reinterpret_cast<const uint4*>(Wh + e + 8);
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) wr[u] = *reinterpret_cast<const uint4*>(Wf + e + 4 * u);
        }
        uint32_t pk[4] = {0u, 0u, 0u, 0u};  // packed / int8 code words
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float w;
                if (DT == CQ_F16) {
                    const uint32_t pr = (&wr[j >> 1].x)[(j & 1) * 2 + (r >> 1)];
                    w = (float)__builtin_bit_cast(_Float16, (uint16_t)((r & 1) ? (pr >> 16) : (pr & 0xffffu)));
                } else {
                    w = __uint_as_float((&wr[j].x)[r]);
                }
                v[r] = a.K > 0 ? w - acc[i][j][r] * sc : w;  // res = W - L R (alg.py:262)
            }
            if (PASS == 0) {
#pragma unroll
                for (int r = 0; r < 4; ++r) mx = max(mx, abs_bits(v[r]));
                continue;
            }
            int cq[4];
            float e4[4];
            float4 wv = make_float4(1.f, 1.f, 1.f, 1.f);
            if (q.ew) wv = *reinterpret_cast<const float4*>(q.ew + b * q.sew + col + 4 * j);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float c = quant_code_r(v[r], s, ys, kq);
                const float d = dequant_r(c, kq, yk, s) - v[r];
                e4[r] = (d * d) * (&wv.x)[r];
                cq[r] = (int)c;
            }
            err += (double)((e4[0] + e4[1]) + (e4[2] + e4[3]));  // fp32 within a run of 4, fp64 across
            if (BITS == 2) {  // byte j = codes 4j..4j+3, MSB-first (offset binary c + 1)
                const uint32_t by = ((uint32_t)(cq[0] + 1) << 6) | ((uint32_t)(cq[1] + 1) << 4) |
                                    ((uint32_t)(cq[2] + 1) << 2) | (uint32_t)(cq[3] + 1);
                pk[0] |= by << (8 * j);
            } else if (BITS == 4) {  // bytes 2j, 2j+1 = codes (4j, 4j+1), (4j+2, 4j+3)
                const uint32_t b0 = ((uint32_t)(cq[0] + 7) << 4) | (uint32_t)(cq[1] + 7);
                const uint32_t b1 = ((uint32_t)(cq[2] + 7) << 4) | (uint32_t)(cq[3] + 7);
                pk[j >> 1] |= (b0 | (b1 << 8)) << (16 * (j & 1));
            } else if (BITS == 8) {
                pk[j] = (uint32_t)(uint8_t)(int8_t)cq[0] | ((uint32_t)(uint8_t)(int8_t)cq[1] << 8) |
                        ((uint32_t)(uint8_t)(int8_t)cq[2] << 16) | ((uint32_t)(uint8_t)(int8_t)cq[3] << 24);
            } else if (q.codes) {
                *reinterpret_cast<short4*>(reinterpret_cast<int16_t*>(q.codes) + b * MN + e + 4 * j) =
                    make_short4((short)cq[0], (short)cq[1], (short)cq[2], (short)cq[3]);
            }
            if (BITS <= 4 && q.codes) {  // unpacked int8 codes alongside the packed bytes
                *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(q.codes) + b * MN + e + 4 * j) =
                    (uint32_t)(uint8_t)(int8_t)cq[0] | ((uint32_t)(uint8_t)(int8_t)cq[1] << 8) |
                    ((uint32_t)(uint8_t)(int8_t)cq[2] << 16) | ((uint32_t)(uint8_t)(int8_t)cq[3] << 24);
            }
        }
        if (PASS == 1) {
            if (BITS == 2 && q.packed) *reinterpret_cast<uint32_t*>(q.packed + (b * MN + e) / 4) = pk[0];
            if (BITS == 4 && q.packed) *reinterpret_cast<uint2*>(q.packed + (b * MN + e) / 2) = make_uint2(pk[0], pk[1]);
            if (BITS == 8 && q.codes)
                *reinterpret_cast<uint4*>(reinterpret_cast<int8_t*>(q.codes) + b * MN + e) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
        }
        asm volatile("" ::: "memory");  // keep the row blocks' W loads from being hoisted together (VGPRs)
    }
    if (PASS == 0) {
        mx = wave_max_u32(mx);
        if (lane == 0 && mx) atomicMax(q.absmax + b, mx);
    } else if (q.part) {
        __shared__ double red[16];
        const double tsum = block_sum_f64(err, red);
        if (threadIdx.x == 0) q.part[b * tiles + tile] = tsum;
    }
}

// First Q step (r = 0, max|W| known): a plain streaming quantise of W, 16 consecutive
// elements per thread per step (32-byte fp16 loads, one 32-bit store of 16 two-bit codes),
// no LDS and no MFMA, so many workgroups per CU keep HBM busy.  Same arithmetic as pass 1 of
// the fused kernels with res = W.  n % 16 == 0; per-block fp64 error partials in part.
template <int DT, int BITS, bool FAST, bool EW>
__device__ __forceinline__ void qstream_group(const QUK& q, int64_t b, int64_t MN, int64_t e, const uint4 (&wr)[4],
                                              const float4 (&ewv)[4], float s, float ys, float yk, double& err) {
    // EW: error column weights (loaded with the group's W); without them the squared errors
    // are not multiplied by 1 (the same sums).  The 2-bit fast path dequantises as c s (k = 1:
    // (c / 1) s is exactly c s) and packs each 8 codes by FMAs on integral floats (below 2^16,
    // exact), as pass 1 of the fused Q update does: ~10 VALU instructions per element instead of
    // ~20, which made this HBM stream VALU-bound (0.60 of HBM at B = 256)
    constexpr float kq = (float)((1 << (BITS - 1)) - 1);
    uint32_t pk[4] = {0u, 0u, 0u, 0u};
    constexpr bool PK2 = BITS == 2 && FAST;
    // 2-bit: element 8 h + 4 j' + r has weight 2^(8 j' + 6 - 2 r) in the h-th 16 bits
    constexpr float wt[4] = {64.f, 16.f, 4.f, 1.f};
    float a2[2] = {0.f, 0.f};
    if (PK2) a2[0] = a2[1] = (64.f + 16.f + 4.f + 1.f) * 257.f;   // the +1 offsets of 8 codes
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int cq[4];
        float cf[4];
        float e4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v;
            if (DT == CQ_F16) {
                const uint32_t pr = (&wr[j >> 1].x)[(j & 1) * 2 + (r >> 1)];
                v = (float)__builtin_bit_cast(_Float16, (uint16_t)((r & 1) ? (pr >> 16) : (pr & 0xffffu)));
            } else {
                v = __uint_as_float((&wr[j].x)[r]);
            }
            float c, dq;
            if (FAST && BITS == 2) {
                c = rintf(div_fast(v, s, ys));
                dq = c * s;
            } else if (FAST) {
                c = rintf(div_fast(v, s, ys) * kq);
                dq = div_fast(c, kq, yk) * s;
            } else {
                c = quant_code(v, s, kq);
                dq = dequant(c, kq, s);
            }
            const float d = dq - v;
            e4[r] = EW ? (d * d) * (&ewv[j].x)[r] : d * d;
            cf[r] = c;
            if (!PK2) cq[r] = (int)c;
        }
        err += (double)((e4[0] + e4[1]) + (e4[2] + e4[3]));  // fp32 within a run of 4, fp64 across
        if (PK2) {
            const float wj = (j & 1) ? 256.f : 1.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) a2[j >> 1] = __builtin_fmaf(cf[r], wt[r] * wj, a2[j >> 1]);
        } else if (BITS == 2) {
            pk[0] |= (((uint32_t)(cq[0] + 1) << 6) | ((uint32_t)(cq[1] + 1) << 4) | ((uint32_t)(cq[2] + 1) << 2) |
                      (uint32_t)(cq[3] + 1)) << (8 * j);
        } else if (BITS == 4) {
            const uint32_t b0 = ((uint32_t)(cq[0] + 7) << 4) | (uint32_t)(cq[1] + 7);
            const uint32_t b1 = ((uint32_t)(cq[2] + 7) << 4) | (uint32_t)(cq[3] + 7);
            pk[j >> 1] |= (b0 | (b1 << 8)) << (16 * (j & 1));
        } else if (BITS == 8) {
            pk[j] = (uint32_t)(uint8_t)(int8_t)cq[0] | ((uint32_t)(uint8_t)(int8_t)cq[1] << 8) |
                    ((uint32_t)(uint8_t)(int8_t)cq[2] << 16) | ((uint32_t)(uint8_t)(int8_t)cq[3] << 24);
        } else if (q.codes) {
            *reinterpret_cast<short4*>(reinterpret_cast<int16_t*>(q.codes) + b * MN + e + 4 * j) =
                make_short4((short)cq[0], (short)cq[1], (short)cq[2], (short)cq[3]);
        }
        if (BITS <= 4 && q.codes) {
            if (PK2) {
#pragma unroll
                for (int r = 0; r < 4; ++r) cq[r] = (int)cf[r];
            }
            *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(q.codes) + b * MN + e + 4 * j) =
                (uint32_t)(uint8_t)(int8_t)cq[0] | ((uint32_t)(uint8_t)(int8_t)cq[1] << 8) |
                ((uint32_t)(uint8_t)(int8_t)cq[2] << 16) | ((uint32_t)(uint8_t)(int8_t)cq[3] << 24);
        }
    }
    if (PK2) pk[0] = (uint32_t)a2[0] | ((uint32_t)a2[1] << 16);
    if (BITS == 2 && q.packed) *reinterpret_cast<uint32_t*>(q.packed + (b * MN + e) / 4) = pk[0];
    if (BITS == 4 && q.packed) *reinterpret_cast<uint2*>(q.packed + (b * MN + e) / 2) = make_uint2(pk[0], pk[1]);
    if (BITS == 8 && q.codes)
        *reinterpret_cast<uint4*>(reinterpret_cast<int8_t*>(q.codes) + b * MN + e) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
}

template <int DT>
__device__ __forceinline__ void qstream_load(const QUK& q, int64_t b, int64_t MN, int64_t e, uint4 (&wr)[4]) {
    if (DT == CQ_F16) {
        const _Float16* Wh = reinterpret_cast<const _Float16*>(q.W) + b * MN + e;
        wr[0] = *reinterpret_cast<const uint4*>(Wh);
        wr[1] = *reinterpret_cast<const uint4*>(Wh + 8);
    } else {
        const float* Wf = reinterpret_cast<const float*>(q.W) + b * MN + e;
#pragma unroll
        for (int u = 0; u < 4; ++u) wr[u] = *reinterpret_cast<const uint4*>(Wf + 4 * u);
    }
}

template <int DT>
__device__ __forceinline__ void qstream_load(const QUK& q, int64_t b, int64_t MN, int64_t e, uint4 (&wr)[4],
                                             float4 (&ewv)[4], bool load_ew = true) {
    // the group's error column weights ride with its W (a load issued at use would expose an
    // L2 round trip per group: config 3's diagonal-H first Q step ran at 0.42 of HBM);
    // load_ew false: the caller holds them (a thread whose columns do not change)
    if (!load_ew) return qstream_load<DT>(q, b, MN, e, wr);
    if (q.ew) {
        const float* ew = q.ew + b * q.sew + e % q.n;
#pragma unroll
        for (int j = 0; j < 4; ++j) ewv[j] = *reinterpret_cast<const float4*>(ew + 4 * j);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) ewv[j] = make_float4(1.f, 1.f, 1.f, 1.f);
    }
    if (DT == CQ_F16) {
        const _Float16* Wh = reinterpret_cast<const _Float16*>(q.W) + b * MN + e;
        wr[0] = *reinterpret_cast<const uint4*>(Wh);
        wr[1] = *reinterpret_cast<const uint4*>(Wh + 8);
    } else {
        const float* Wf = reinterpret_cast<const float*>(q.W) + b * MN + e;
#pragma unroll
        for (int u = 0; u < 4; ++u) wr[u] = *reinterpret_cast<const uint4*>(Wf + 4 * u);
    }
}

// First Q step (r = 0, max|W| known): a plain streaming quantise of W, 16 consecutive
// elements per thread per group, the next group's load in flight (32-byte fp16 loads, one
// 32-bit store of 16 two-bit codes), no LDS and no MFMA, so many workgroups per CU keep HBM
// busy.  Same arithmetic as pass 1 of the fused kernels with res = W.  n % 16 == 0;
// per-block fp64 error partials in part.
template <int DT, int BITS, bool EW>
__global__ __launch_bounds__(256) void quant_w_stream_kernel(QUK q) {
    constexpr float kq = (float)((1 << (BITS - 1)) - 1);
    const int64_t b = blockIdx.y;
    const int64_t MN = q.m * q.n;
    const int64_t ng = MN / 16;
    const float s = quant_scale(q.absmax[b], q.eps);
    const float ys = 1.f / s, yk = 1.f / kq;  // IEEE reciprocals for div_rn
    double err = 0.0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    // a grid stride that is a multiple of the row length (the launcher picks one when there are
    // error weights) keeps each thread on the same 16 columns: their weights are loaded once
    const bool ewfix = EW && ((stride * 16) % q.n) == 0;
    if (div_fast_ok(s)) {  // uniform: the common case, branch-free correctly rounded division
        uint4 nx[4];  // the next group's W (and weights), loaded while this one is quantised
        float4 nw[4];
        if (g < ng) qstream_load<DT>(q, b, MN, g * 16, nx, nw, EW);
        if (!EW) {
#pragma unroll
            for (int u = 0; u < 4; ++u) nw[u] = make_float4(1.f, 1.f, 1.f, 1.f);   // unused
        }
        if (ewfix || !EW) {
            // columns fixed per thread (or no weights): W two groups ahead (~100 KB of loads in
            // flight per CU at 6 waves per SIMD)
            uint4 nx2[4];
            if (g + stride < ng) qstream_load<DT>(q, b, MN, (g + stride) * 16, nx2);
            for (; g < ng; g += stride) {
                uint4 cur[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) { cur[u] = nx[u]; nx[u] = nx2[u]; }
                if (g + 2 * stride < ng) qstream_load<DT>(q, b, MN, (g + 2 * stride) * 16, nx2);
                qstream_group<DT, BITS, true, EW>(q, b, MN, g * 16, cur, nw, s, ys, yk, err);
            }
        }
        for (; g < ng; g += stride) {
            uint4 cur[4];
            float4 cw[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) { cur[u] = nx[u]; cw[u] = nw[u]; }
            if (g + stride < ng) qstream_load<DT>(q, b, MN, (g + stride) * 16, nx, nw);
            qstream_group<DT, BITS, true, EW>(q, b, MN, g * 16, cur, cw, s, ys, yk, err);
        }
    } else {  // non-finite / subnormal scale: IEEE divisions
        for (; g < ng; g += stride) {
            uint4 w0[4];
            float4 ew0[4];
            qstream_load<DT>(q, b, MN, g * 16, w0, ew0, EW);
            if (!EW) {
#pragma unroll
                for (int u = 0; u < 4; ++u) ew0[u] = make_float4(1.f, 1.f, 1.f, 1.f);
            }
            qstream_group<DT, BITS, false, EW>(q, b, MN, g * 16, w0, ew0, s, ys, yk, err);
        }
    }
    if (q.part) {
        __shared__ double red[16];
        const double tsum = block_sum_f64(err, red);
        if (threadIdx.x == 0) q.part[b * gridDim.x + blockIdx.x] = tsum;
    }
}

__global__ void q_update_finalize_kernel(const uint32_t* absmax, const double* part, int64_t tiles, int64_t batch,
                                         float eps, float* scale, double* err_out) {
    const int64_t b = blockIdx.x;
    if (b >= batch) return;
    double s = 0.0;
    for (int64_t t = threadIdx.x; t < tiles; t += 64) s += part[b * tiles + t];
    s = wave_sum(s);  // one wave: fixed order -> deterministic
    if (threadIdx.x == 0) {
        if (scale) scale[b] = quant_scale(absmax[b], eps);
        if (err_out) err_out[b] = s;
    }
}


// ------------------------------------------------------------------ fused residual + split
// One pass over W and the packed Q codes for the LR step (alg.py:124 res = W - Q, :211
// Y = res * sqrt(h)): writes any of res (fp32), Y (fp32), the K-blocked split halves of Y
// over its columns (A/B operand of Y Y^T) and over its rows (operand of U^T Y / Y^T Y), and
// ||Y||^2 (fp64, deterministic per-tile partials).  The split scale is a per-matrix power of
// two from the bound |Y| <= (max|W| + Q_scale) * max(ycol), so no absmax pass is needed.
// Tile 32 rows x 64 columns per step, 256 threads (8 consecutive columns each).
template <int DT, int BITS>
__global__ __launch_bounds__(256) void residual_split_kernel(
    const void* __restrict__ Ws, const uint8_t* __restrict__ qc, const float* __restrict__ qscale,
    const float* __restrict__ ycol, const float* __restrict__ wmax, float ycmax, int64_t m, int64_t n,
    float* __restrict__ res, float* __restrict__ Y, _Float16* __restrict__ hi, _Float16* __restrict__ lo,
    _Float16* __restrict__ thi, _Float16* __restrict__ tlo, float* __restrict__ scale_out,
    double* __restrict__ part, const float* __restrict__ ycol_hi, float ychmax, float* __restrict__ scale_hi_out,
    int64_t ycs, const float* __restrict__ ycmax_v, const float* __restrict__ ychmax_v) {
    __shared__ float tile[64][33];
    __shared__ double red[4];
    constexpr float k = BITS == 32 ? 1.f : (float)((1 << (BITS - 1)) - 1);
    const int64_t b = blockIdx.z;
    const int64_t MN = m * n;
    const float qs = qc ? qscale[b] : 0.f;
    // per-matrix column weights (distinct diagonal Hessians): this matrix's row of ycol / ycol_hi
    // and its own bounds
    if (ycol) ycol += b * ycs;
    if (ycol_hi) ycol_hi += b * ycs;
    if (ycmax_v) ycmax = ycmax_v[b];
    if (ychmax_v) ychmax = ychmax_v[b];
    int e2 = 0;
    {
        const float bnd = (wmax[b] + qs) * ycmax;
        if (bnd > 0.f && isfinite(bnd)) frexpf(bnd, &e2);
    }
    // fp16 W alone (no codes, no column weights): a scale >= 1 keeps W * sc exact in fp16
    // (lo = 0), so the lo halves may be skipped and their products dropped (gemm_x3 b_exact)
    const bool exact = DT == CQ_F16 && !qc && !ycol;
    const float sc = exact ? fmaxf(ldexpf(1.f, 14 - e2), 1.f) : ldexpf(1.f, 14 - e2);
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && scale_out) scale_out[b] = sc;
    // ycol_hi: the column-blocked halves (hi/lo) are of res * ycol_hi instead, at their own scale
    float sch = sc;
    if (ycol_hi) {
        int e3 = 0;
        const float bnd = (wmax[b] + qs) * ychmax;
        if (bnd > 0.f && isfinite(bnd)) frexpf(bnd, &e3);
        sch = ldexpf(1.f, 14 - e3);
        if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) scale_hi_out[b] = sch;
    }
    const int t = threadIdx.x;
    const int r = t >> 3, c8 = (t & 7) * 8;          // row in tile, first of 8 columns
    const int64_t j0 = (int64_t)blockIdx.x * 64;
    double acc = 0.0;
    const int rows_per = (int)gridDim.y;
    for (int64_t i0 = (int64_t)blockIdx.y * 32; i0 < m; i0 += (int64_t)rows_per * 32) {
        const int64_t i = i0 + r, j = j0 + c8;
        const int64_t e = b * MN + i * n + j;
        float w[8];
        if (DT == CQ_F16) {
            const uint4 raw = *reinterpret_cast<const uint4*>(reinterpret_cast<const _Float16*>(Ws) + e);
            const _Float16* hv = reinterpret_cast<const _Float16*>(&raw);
#pragma unroll
            for (int u = 0; u < 8; ++u) w[u] = (float)hv[u];
        } else {
            const float4 f0 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(Ws) + e);
            const float4 f1 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(Ws) + e + 4);
            w[0] = f0.x; w[1] = f0.y; w[2] = f0.z; w[3] = f0.w; w[4] = f1.x; w[5] = f1.y; w[6] = f1.z; w[7] = f1.w;
        }
        float q[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) q[u] = 0.f;
        if (qc) {
            const int64_t eq = e;  // element index (codes follow the row-major element order)
            if (BITS == 2) {
                const uint16_t two = *reinterpret_cast<const uint16_t*>(qc + eq / 4);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t byte = (u < 4) ? (two & 0xffu) : (two >> 8);
                    const int sh = 6 - 2 * (u & 3);
                    q[u] = dequant((float)((int)((byte >> sh) & 3u) - 1), k, qs);
                }
            } else if (BITS == 4) {
                const uint32_t four = *reinterpret_cast<const uint32_t*>(qc + eq / 2);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t byte = (four >> (8 * (u >> 1))) & 0xffu;
                    const uint32_t v = (u & 1) ? (byte & 15u) : (byte >> 4);
                    q[u] = dequant((float)((int)v - 7), k, qs);
                }
            } else if (BITS == 8) {
                const int8_t* cp = reinterpret_cast<const int8_t*>(qc) + eq;
#pragma unroll
                for (int u = 0; u < 8; ++u) q[u] = dequant((float)cp[u], k, qs);
            } else if (BITS == 32) {  // dense fp32 Q (codebook methods); qscale = bound on |Q|
                const float4 f0 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(qc) + eq);
                const float4 f1 = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(qc) + eq + 4);
                q[0] = f0.x; q[1] = f0.y; q[2] = f0.z; q[3] = f0.w; q[4] = f1.x; q[5] = f1.y; q[6] = f1.z; q[7] = f1.w;
            } else {
                const int16_t* cp = reinterpret_cast<const int16_t*>(qc) + eq;
#pragma unroll
                for (int u = 0; u < 8; ++u) q[u] = dequant((float)cp[u], k, qs);
            }
        }
        float rv[8], yv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            rv[u] = w[u] - q[u];
            yv[u] = ycol ? rv[u] * ycol[j + u] : rv[u];
            acc += (double)yv[u] * (double)yv[u];
        }
        if (res) {
            *reinterpret_cast<float4*>(res + e) = make_float4(rv[0], rv[1], rv[2], rv[3]);
            *reinterpret_cast<float4*>(res + e + 4) = make_float4(rv[4], rv[5], rv[6], rv[7]);
        }
        if (Y) {
            *reinterpret_cast<float4*>(Y + e) = make_float4(yv[0], yv[1], yv[2], yv[3]);
            *reinterpret_cast<float4*>(Y + e + 4) = make_float4(yv[4], yv[5], yv[6], yv[7]);
        }
        if (hi) {  // blocked over columns: (j / 32) * m * 32 + i * 32 + j % 32
            _Float16 h8[8], l8[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const float xs = ycol_hi ? rv[u] * ycol_hi[j + u] * sch : yv[u] * sc;
                h8[u] = (_Float16)xs;
                l8[u] = (_Float16)(xs - (float)h8[u]);
            }
            const int64_t o = b * MN + (j >> 5) * m * 32 + i * 32 + (j & 31);
            *reinterpret_cast<uint4*>(hi + o) = *reinterpret_cast<const uint4*>(h8);
            if (lo) *reinterpret_cast<uint4*>(lo + o) = *reinterpret_cast<const uint4*>(l8);
        }
        if (thi) {  // blocked over rows (Y^T as a row-major n x m operand): (i / 32) * n * 32 + j * 32 + i % 32
#pragma unroll
            for (int u = 0; u < 8; ++u) tile[c8 + u][r] = yv[u] * sc;
            __syncthreads();
            const int jc = t >> 2, r8 = (t & 3) * 8;   // column of the tile, 8 consecutive rows
            _Float16 h8[8], l8[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const float xs = tile[jc][r8 + u];
                h8[u] = (_Float16)xs;
                l8[u] = (_Float16)(xs - (float)h8[u]);
            }
            const int64_t o = b * MN + (i0 >> 5) * n * 32 + (j0 + jc) * 32 + r8;
            *reinterpret_cast<uint4*>(thi + o) = *reinterpret_cast<const uint4*>(h8);
            if (tlo) *reinterpret_cast<uint4*>(tlo + o) = *reinterpret_cast<const uint4*>(l8);
            __syncthreads();
        }
    }
    if (part) {
        acc = wave_sum(acc);
        if ((t & 63) == 0) red[t >> 6] = acc;
        __syncthreads();
        if (t == 0) part[(b * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
    }
}

__global__ void sum_tile_parts_kernel(const double* __restrict__ part, int64_t nparts, double* __restrict__ out) {
    const int64_t b = blockIdx.x;
    double s = 0.0;
    for (int64_t t = threadIdx.x; t < nparts; t += 64) s += part[b * nparts + t];
    s = wave_sum(s);
    if (threadIdx.x == 0) out[b] = s;
}

template <int DT>
__global__ void absmax_dt_kernel(const void* __restrict__ X, int64_t n_per, uint32_t* __restrict__ out) {
    const int64_t b = blockIdx.y;
    uint32_t mx = 0;
    // 16-byte vector loads (8 halves / 4 floats per load) where the rows allow it
    constexpr int V = DT == CQ_F16 ? 8 : 4;
    const bool vec = n_per % V == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
    if (vec) {
        const uint4* Xv = reinterpret_cast<const uint4*>(X) + b * (n_per / V);
        for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n_per / V; q += (int64_t)gridDim.x * blockDim.x) {
            const uint4 r = Xv[q];
            if (DT == CQ_F16) {
                const _Float16* h = reinterpret_cast<const _Float16*>(&r);
#pragma unroll
                for (int u = 0; u < 8; ++u) mx = max(mx, abs_bits((float)h[u]));
            } else {
                mx = max(mx, max(max(abs_bits(__uint_as_float(r.x)), abs_bits(__uint_as_float(r.y))),
                                 max(abs_bits(__uint_as_float(r.z)), abs_bits(__uint_as_float(r.w)))));
            }
        }
        mx = wave_max_u32(mx);
        if ((threadIdx.x & 63) == 0 && mx) atomicMax(out + b, mx);
        return;
    }
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n_per; q += (int64_t)gridDim.x * blockDim.x) {
        const float v = DT == CQ_F16 ? (float)reinterpret_cast<const _Float16*>(X)[b * n_per + q]
                                     : reinterpret_cast<const float*>(X)[b * n_per + q];
        mx = max(mx, abs_bits(v));
    }
    mx = wave_max_u32(mx);
    if ((threadIdx.x & 63) == 0 && mx) atomicMax(out + b, mx);
}

// ------------------------------------------------------------------ split / transpose helpers

// Per-batch power-of-two scale s = 2^(14 - ceil(log2 max_i G_ii)) for a PSD G (|G_ij| <=
// max diag), so the scaled hi halves stay <= 2^14 (fp16 max 65504) with headroom; the
// kernel stores 1 / (s * x_scale) for the GEMM epilogue and s for the split.
__global__ void sym_scale_kernel(const float* __restrict__ G, int64_t n, int64_t ldg, int64_t sg,
                                 float x_scale, float* __restrict__ s_out, float* __restrict__ inv_out) {
    const int64_t b = blockIdx.x;
    float m = 0.f;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) m = fmaxf(m, fabsf(G[b * sg + i * ldg + i]));
    m = wave_max(m);
    __shared__ float red[16];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float mm = 0.f;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) mm = fmaxf(mm, red[w]);
        int e = 0;
        if (mm > 0.f && isfinite(mm)) {
            frexpf(mm, &e);  // mm in [2^(e-1), 2^e)
        }
        const float s = ldexpf(1.f, 14 - e);
        s_out[b] = s;
        inv_out[b] = 1.f / (s * x_scale);
    }
}

__global__ void split_kernel(const float* __restrict__ X, int64_t n_per, const float* __restrict__ s_v,
                             float s_fixed, _Float16* __restrict__ hi, _Float16* __restrict__ lo, int64_t batch) {
    const int64_t tot4 = batch * n_per / 4;
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < tot4; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = q * 4;
        const int64_t o = e;
        const float s = s_v ? s_v[e / n_per] : s_fixed;
        const float4 v = *reinterpret_cast<const float4*>(X + e);
        const float xs[4] = {v.x * s, v.y * s, v.z * s, v.w * s};
        _Float16 h[4], l[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            h[u] = (_Float16)xs[u];
            l[u] = (_Float16)(xs[u] - (float)h[u]);
        }
        *reinterpret_cast<uint2*>(hi + o) = *reinterpret_cast<const uint2*>(h);
        *reinterpret_cast<uint2*>(lo + o) = *reinterpret_cast<const uint2*>(l);
    }
}

// Split of a symmetric matrix of which only the upper triangle (j >= i) is valid: 64 x 64
// tiles, lower tiles read from the transposed upper tile through LDS.
__device__ __forceinline__ int64_t blk_off(int64_t i, int64_t j, int64_t n, int blocked) {
    return blocked ? ((j >> 5) * n * 32 + i * 32 + (j & 31)) : (i * n + j);
}

__global__ __launch_bounds__(256) void sym_split_upper_kernel(const float* __restrict__ G, int64_t n,
                                                              const float* __restrict__ s_v,
                                                              _Float16* __restrict__ hi, _Float16* __restrict__ lo,
                                                              int blocked) {
    __shared__ float tile[64][65];
    const int64_t b = blockIdx.z;
    const int64_t ti = blockIdx.y, tj = blockIdx.x;
    const float* Gb = G + b * n * n;
    const float s = s_v[b];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const bool lower = ti > tj;
    const int64_t si = lower ? tj : ti, sj = lower ? ti : tj;  // source tile (upper)
    for (int r = ty; r < 64; r += 4) {
        const int64_t i = si * 64 + r, j = sj * 64 + tx;
        // inside a diagonal tile, take (min, max) so only upper entries are read
        float v = 0.f;
        if (i < n && j < n) v = (j >= i) ? Gb[i * n + j] : Gb[j * n + i];
        tile[r][tx] = v;
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int64_t i = ti * 64 + r, j = tj * 64 + tx;
        if (i < n && j < n) {
            const float v = (lower ? tile[tx][r] : tile[r][tx]) * s;
            const _Float16 h = (_Float16)v;
            const int64_t o = b * n * n + blk_off(i, j, n, blocked);
            hi[o] = h;
            lo[o] = (_Float16)(v - (float)h);
        }
    }
}

// Per-batch max |x| as uint bits (atomicMax into a zeroed buffer), then
// s[b] = 2^(log2_target - e) with max in [2^(e-1), 2^e): the scaled values stay below 2^log2_target.
__global__ void absmax_bits_kernel(const float* __restrict__ X, int64_t n_per, uint32_t* __restrict__ out) {
    const int64_t b = blockIdx.y;
    const float* Xb = X + b * n_per;
    uint32_t m = 0;
    const int64_t n4 = n_per / 4;
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
        const float4 v = *reinterpret_cast<const float4*>(Xb + 4 * q);
        m = max(m, max(max(abs_bits(v.x), abs_bits(v.y)), max(abs_bits(v.z), abs_bits(v.w))));
    }
    for (int64_t q = 4 * n4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n_per;
         q += (int64_t)gridDim.x * blockDim.x)
        m = max(m, abs_bits(Xb[q]));
    m = wave_max_u32(m);
    if ((threadIdx.x & 63) == 0 && m) atomicMax(out + b, m);
}

__global__ void pow2_scale_kernel(float* __restrict__ s, int64_t batch, int log2_target) {
    const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (b >= batch) return;
    const float mm = __uint_as_float(reinterpret_cast<const uint32_t*>(s)[b]);
    int e = 0;
    if (mm > 0.f && isfinite(mm)) frexpf(mm, &e);
    s[b] = ldexpf(1.f, log2_target - e);
}

// K-blocked split (ncols % 32 == 0): element (row, col) of a rows x ncols matrix goes to
// (col / 32) * rows * 32 + row * 32 + col % 32 — the K-blocked operand layout of cq_gemm_x3.
// grid (rows / 4, batch): one row per wave, no integer division.
__global__ __launch_bounds__(256) void split_blocked_kernel(const float* __restrict__ X, int64_t rows, int64_t ncols,
                                                            const float* __restrict__ s_v, float s_fixed,
                                                            _Float16* __restrict__ hi, _Float16* __restrict__ lo) {
    const int64_t b = blockIdx.y;
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= rows) return;
    const float s = s_v ? s_v[b] : s_fixed;
    const float* xr = X + b * rows * ncols + row * ncols;
    _Float16* hb = hi + b * rows * ncols + row * 32;
    _Float16* lb = lo + b * rows * ncols + row * 32;
    for (int64_t c = 4 * (threadIdx.x & 63); c < ncols; c += 256) {
        const float4 v = *reinterpret_cast<const float4*>(xr + c);
        const float xs[4] = {v.x * s, v.y * s, v.z * s, v.w * s};
        _Float16 h[4], l[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            h[u] = (_Float16)xs[u];
            l[u] = (_Float16)(xs[u] - (float)h[u]);
        }
        const int64_t o = (c >> 5) * rows * 32 + (c & 31);
        *reinterpret_cast<uint2*>(hb + o) = *reinterpret_cast<const uint2*>(h);
        *reinterpret_cast<uint2*>(lb + o) = *reinterpret_cast<const uint2*>(l);
    }
}

// Batched transpose Y = X^T (X rows x cols, row-major) through a 64 x 65 LDS tile, with an
// optional fp16 split of Y (scale s).  VEC (rows % 8 == 0, cols % 4 == 0, 16-byte aligned
// buffers; the solver's k x p blocks): 16-byte loads of X, and each thread writes 8
// consecutive Y columns of one Y row -- two 16-byte fp32 stores and one 16-byte store per
// half -- instead of one 4-byte and two 2-byte stores per element (the tile's column reads
// (8 g + q) x 65 + i, lane = (i, g), hit 64 different banks).  The same values either way.
template <bool VEC>
__global__ __launch_bounds__(256) void transpose_split_kernel(const float* __restrict__ X, int64_t rows, int64_t cols,
                                                              float* __restrict__ Y, _Float16* __restrict__ hi,
                                                              _Float16* __restrict__ lo, float s_fixed,
                                                              const float* __restrict__ s_v, int blocked) {
    __shared__ float tile[64][65];
    const int64_t b = blockIdx.z;
    const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
    const float* Xb = X + b * rows * cols;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int64_t ob = b * rows * cols;
    const float s = s_v ? s_v[b] : s_fixed;
    if constexpr (VEC) {
        // load: 64 rows x 16 float4, 4 per thread (thread t: rows t / 16 + 16 u, float4 t % 16)
        const int q4 = threadIdx.x & 15, rq = threadIdx.x >> 4;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = rq + 16 * u;
            const int64_t r = r0 + i, c = c0 + 4 * q4;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (r < rows && c < cols) v = *reinterpret_cast<const float4*>(Xb + r * cols + c);
            tile[i][4 * q4] = v.x; tile[i][4 * q4 + 1] = v.y; tile[i][4 * q4 + 2] = v.z; tile[i][4 * q4 + 3] = v.w;
        }
        __syncthreads();
        // store: Y row orow = c0 + i (64 of them), columns r0 + 8 g .. + 7 (g = 0..7): 512 tasks,
        // 2 per thread; a wave covers 8 Y rows x 64 columns
        const int g = threadIdx.x & 7, il = threadIdx.x >> 3;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = il + 32 * u;
            const int64_t orow = c0 + i, ocol = r0 + 8 * g;
            if (orow >= cols || ocol >= rows) continue;
            float v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = tile[8 * g + q][i];
            if (Y) {
                float* yp = Y + ob + orow * rows + ocol;
                *reinterpret_cast<float4*>(yp) = make_float4(v[0], v[1], v[2], v[3]);
                *reinterpret_cast<float4*>(yp + 4) = make_float4(v[4], v[5], v[6], v[7]);
            }
            if (hi) {
                _Float16 h[8], l[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const float xs = v[q] * s;
                    h[q] = (_Float16)xs;
                    l[q] = (_Float16)(xs - (float)h[q]);
                }
                const int64_t o = blocked ? ob + (ocol >> 5) * cols * 32 + orow * 32 + (ocol & 31) : ob + orow * rows + ocol;
                *reinterpret_cast<uint4*>(hi + o) = *reinterpret_cast<const uint4*>(h);
                *reinterpret_cast<uint4*>(lo + o) = *reinterpret_cast<const uint4*>(l);
            }
        }
        return;
    }
    for (int i = ty; i < 64; i += 4) {
        const int64_t r = r0 + i, c = c0 + tx;
        tile[i][tx] = (r < rows && c < cols) ? Xb[r * cols + c] : 0.f;
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {
        const int64_t orow = c0 + i, ocol = r0 + tx;  // Y is cols x rows
        if (orow < cols && ocol < rows) {
            const float v = tile[tx][i];
            if (Y) Y[ob + orow * rows + ocol] = v;
            if (hi) {
                const float xs = v * s;
                const _Float16 h = (_Float16)xs;
                // Y is cols x rows: K-blocked halves put (orow, ocol) at (ocol/32)*cols*32 + orow*32 + ocol%32
                const int64_t o = blocked ? ob + (ocol >> 5) * cols * 32 + orow * 32 + (ocol & 31) : ob + orow * rows + ocol;
                hi[o] = h;
                lo[o] = (_Float16)(xs - (float)h);
            }
        }
    }
}


}  // namespace cq

using namespace cq;

extern "C" {

int cq_sym_split_f16(const float* G, int64_t n, int64_t batch, int upper_only, int blocked, float x_scale,
                     uint16_t* Gh, uint16_t* Gl, float* scale_out, float* inv_scale_out, void* stream) {
    CQ_REQUIRE(G && Gh && Gl && scale_out && inv_scale_out, "cq_sym_split_f16: null pointer");
    CQ_REQUIRE(n > 0 && batch > 0 && (n * n) % 4 == 0, "cq_sym_split_f16: bad shape");
    CQ_REQUIRE(x_scale > 0.f, "cq_sym_split_f16: x_scale must be > 0");
    hipStream_t s = as_stream(stream);
    sym_scale_kernel<<<(unsigned)batch, 256, 0, s>>>(G, n, n, n * n, x_scale, scale_out, inv_scale_out);
    CQ_REQUIRE(!blocked || n % 32 == 0, "cq_sym_split_f16: blocked layout needs n % 32 == 0");
    if (upper_only || blocked) {
        CQ_REQUIRE(batch < 65536, "cq_sym_split_f16: batch too large");
        const unsigned t64 = (unsigned)ceil_div(n, 64);
        sym_split_upper_kernel<<<dim3(t64, t64, (unsigned)batch), 256, 0, s>>>(
            G, n, scale_out, reinterpret_cast<_Float16*>(Gh), reinterpret_cast<_Float16*>(Gl), blocked);
        return check_launch("cq_sym_split_f16");
    }
    const int64_t tot4 = batch * n * n / 4;
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(tot4, 256), 8192);
    split_kernel<<<grid, 256, 0, s>>>(G, n * n, scale_out, 1.f, reinterpret_cast<_Float16*>(Gh),
                                      reinterpret_cast<_Float16*>(Gl), batch);
    return check_launch("cq_sym_split_f16");
}

int cq_pow2_scale(const float* X, int64_t n_per, int64_t batch, int log2_target, float* scale_out, void* stream) {
    CQ_REQUIRE(X && scale_out, "cq_pow2_scale: null pointer");
    CQ_REQUIRE(n_per > 0 && batch > 0 && batch < 65536 && n_per % 4 == 0, "cq_pow2_scale: bad shape");
    CQ_REQUIRE(log2_target > -100 && log2_target < 100, "cq_pow2_scale: bad target");
    hipStream_t s = as_stream(stream);
    if (hipMemsetAsync(scale_out, 0, batch * sizeof(float), s) != hipSuccess)
        return set_error(CQ_EHIP, "cq_pow2_scale: memset failed");
    const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n_per / 4, 256), std::max<int64_t>(1, 2048 / batch)));
    absmax_bits_kernel<<<dim3(gx, (unsigned)batch), 256, 0, s>>>(X, n_per, reinterpret_cast<uint32_t*>(scale_out));
    pow2_scale_kernel<<<(unsigned)ceil_div(batch, 256), 256, 0, s>>>(scale_out, batch, log2_target);
    return check_launch("cq_pow2_scale");
}

int cq_pow2_from_absmax(float* scale_inout, int64_t batch, int log2_target, void* stream) {
    CQ_REQUIRE(scale_inout && batch > 0, "cq_pow2_from_absmax: bad args");
    CQ_REQUIRE(log2_target > -100 && log2_target < 100, "cq_pow2_from_absmax: bad target");
    pow2_scale_kernel<<<(unsigned)ceil_div(batch, 256), 256, 0, as_stream(stream)>>>(scale_inout, batch, log2_target);
    return check_launch("cq_pow2_from_absmax");
}

int cq_split_f16(const float* X, int64_t n_per, int64_t batch, const float* scale_v, float scale, uint16_t* hi,
                 uint16_t* lo, int64_t blocked_ncols, void* stream) {
    CQ_REQUIRE(X && hi && lo, "cq_split_f16: null pointer");
    CQ_REQUIRE(n_per > 0 && batch > 0 && n_per % 4 == 0, "cq_split_f16: n_per must be a positive multiple of 4");
    CQ_REQUIRE(blocked_ncols == 0 || (blocked_ncols % 32 == 0 && n_per % blocked_ncols == 0),
               "cq_split_f16: blocked layout needs ncols % 32 == 0 dividing n_per");
    const int64_t tot4 = batch * n_per / 4;
    const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(tot4, 256), 8192);
    if (blocked_ncols) {
        const int64_t rows = n_per / blocked_ncols;
        CQ_REQUIRE(batch < 65536, "cq_split_f16: batch too large");
        split_blocked_kernel<<<dim3((unsigned)ceil_div(rows, 4), (unsigned)batch), 256, 0, as_stream(stream)>>>(
            X, rows, blocked_ncols, scale_v, scale, reinterpret_cast<_Float16*>(hi), reinterpret_cast<_Float16*>(lo));
        return check_launch("cq_split_f16");
    }
    split_kernel<<<grid, 256, 0, as_stream(stream)>>>(X, n_per, scale_v, scale, reinterpret_cast<_Float16*>(hi),
                                                      reinterpret_cast<_Float16*>(lo), batch);
    return check_launch("cq_split_f16");
}

int cq_transpose_split(const float* X, int64_t rows, int64_t cols, int64_t batch, float* Y, uint16_t* hi,
                       uint16_t* lo, float scale, const float* scale_v, int blocked, void* stream) {
    CQ_REQUIRE(!blocked || rows % 32 == 0, "cq_transpose_split: blocked halves need rows % 32 == 0");
    CQ_REQUIRE(X && (Y || (hi && lo)), "cq_transpose_split: null pointer");
    CQ_REQUIRE(!hi == !lo, "cq_transpose_split: hi and lo go together");
    CQ_REQUIRE(rows > 0 && cols > 0 && batch > 0 && batch < 65536, "cq_transpose_split: bad shape");
    dim3 grid((unsigned)ceil_div(cols, 64), (unsigned)ceil_div(rows, 64), (unsigned)batch);
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool vec = rows % 8 == 0 && cols % 4 == 0 && al16(X) && (!Y || al16(Y)) && (!hi || (al16(hi) && al16(lo)));
    if (vec)
        transpose_split_kernel<true><<<grid, 256, 0, as_stream(stream)>>>(
            X, rows, cols, Y, reinterpret_cast<_Float16*>(hi), reinterpret_cast<_Float16*>(lo), scale, scale_v, blocked);
    else
        transpose_split_kernel<false><<<grid, 256, 0, as_stream(stream)>>>(
            X, rows, cols, Y, reinterpret_cast<_Float16*>(hi), reinterpret_cast<_Float16*>(lo), scale, scale_v, blocked);
    return check_launch("cq_transpose_split");
}


static int64_t qu_tiles(int64_t m, int64_t n) {
    return std::max(ceil_div(n, XW_BM) * ceil_div(m, XW_BN), ceil_div(m, XW_BM) * ceil_div(n, XW_BN));
}

// the single-recompute 2-bit path's buffers (qp_launch_cand) for one of its geometries (rows
// per wave, waves): overflow flags | list-B counts | pass-2 partials | corrections | list-A
// counts | list-B group ids | list-B residuals | list-A entries
static size_t qu_cand_geom(int64_t m, int64_t n, int64_t batch, int rpw, int nw, int64_t* regions_out,
                           int64_t* cap_out, int64_t* capa_out = nullptr) {
    const int64_t regions = ceil_div(m, (int64_t)rpw * nw) * nw, groups = (int64_t)rpw * n / 8;
    const bool big = m * n >= QP_BIG_NUMEL;
    const int64_t cap = ceil_div(groups * (big ? QP_CAPB_PERMILLE_BIG : QP_CAPB_PERMILLE_SMALL), (int64_t)1000);
    const int64_t capa = ceil_div(groups * (big ? QP_CAPA_PERMILLE_BIG : QP_CAPA_PERMILLE_SMALL), (int64_t)1000);
    if (regions_out) *regions_out = regions;
    if (cap_out) *cap_out = cap;
    if (capa_out) *capa_out = capa;
    return align_up((size_t)batch * 4, 256) + align_up((size_t)batch * regions * 4, 256) +
           align_up((size_t)batch * regions * 8, 256) * 2 + align_up((size_t)batch * regions * 4, 256) +
           align_up((size_t)batch * regions * cap * 4, 256) + align_up((size_t)batch * regions * cap * 32, 256) +
           (size_t)batch * regions * capa * 8;
}
static size_t qu_cand_bytes(int64_t m, int64_t n, int64_t batch) {
    return std::max(qu_cand_geom(m, n, batch, qp_cand_rows(128), qp_cand_waves(128), nullptr, nullptr),
                    qu_cand_geom(m, n, batch, qp_cand_rows(256), qp_cand_waves(256), nullptr, nullptr));
}

size_t cq_q_update_workspace(int64_t m, int64_t n, int64_t batch, int with_hint) {
    // tile counts of both Q-update kernels (q_update_v_kernel tiles W as m x n, the 32x32
    // kernel as n x m)
    const int64_t tiles = qu_tiles(m, n);
    // absmax bits | error partials | list path (only when a scale hint will be passed)
    return (size_t)align_up((size_t)batch * sizeof(uint32_t), 256) +
           align_up((size_t)batch * tiles * sizeof(double), 256) +
           (with_hint ? qu_cand_bytes(m, n, batch) : 0);
}

int cq_q_update_list_geometry(int64_t m, int64_t n, int64_t r, int64_t* rows_out, int64_t* cap_out,
                              int64_t* capb_out) {
    CQ_REQUIRE(rows_out && cap_out, "cq_q_update_list_geometry: null argument");
    if (!(r > 0 && r % XW_BK == 0 && qp_cand_ok(m, n, (int)r)))
        return set_error(CQ_EINVAL, "cq_q_update_list_geometry: (m, n, r) do not take the list path");
    const int rpw = qp_cand_rows((int)r);
    int64_t capb = 0;
    qu_cand_geom(m, n, 1, rpw, qp_cand_waves((int)r), nullptr, &capb, cap_out);
    if (capb_out) *capb_out = capb;
    *rows_out = rpw;
    return CQ_OK;
}

int cq_q_update_x3(int dtype, const void* W, int64_t m, int64_t n, int64_t r, int64_t batch, const uint16_t* Lh,
                   const uint16_t* Ll, const uint16_t* Rth, const uint16_t* Rtl, const float* inv_scale, int bits,
                   float eps, void* codes, uint8_t* packed, float* scale_out, const float* err_w,
                   int64_t err_w_stride, double* err_out, const float* absmax_in, const float* scale_hint,
                   int* fallback_out, void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(W && m > 0 && n > 0 && batch > 0 && r >= 0, "cq_q_update_x3: bad shape");
    CQ_REQUIRE(dtype == CQ_F16 || dtype == CQ_F32, "cq_q_update_x3: dtype must be f16/f32");
    if (bits != 2 && bits != 4 && bits != 8 && bits != 16) return set_error(CQ_EINVAL, "Bit-width not supported!");
    CQ_REQUIRE(r == 0 || (Lh && Ll && Rth && Rtl && inv_scale), "cq_q_update_x3: null factor halves");
    CQ_REQUIRE(r % XW_BK == 0, "cq_q_update_x3: rank must be a multiple of 32");
    CQ_REQUIRE(n % 4 == 0, "cq_q_update_x3: n must be a multiple of 4");
    CQ_REQUIRE(!packed || bits <= 4, "cq_q_update_x3: packing needs bits <= 4");
    CQ_REQUIRE(codes || packed, "cq_q_update_x3: no code output");
    if (!ws || ws_bytes < cq_q_update_workspace(m, n, batch, scale_hint != nullptr))
        return set_error(CQ_EWORKSPACE, "cq_q_update_x3: workspace too small");
    QUK q;
    X3K& a = q.x;
    memset(&q, 0, sizeof(q));  // a_blocked = b_blocked = 0, no active mask, no list path
    auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool vk = n % 16 == 0 && al16(W) && (!codes || al16(codes)) && (!packed || al16(packed)) &&
                    (!err_w || (al16(err_w) && err_w_stride % 4 == 0));
    if (vk) {
        // A operand L (m x r): tile rows run over W's rows; B operand R^T (n x r): tile
        // columns over W's columns (see q_update_v_kernel)
        a.M = m; a.N = n;
        a.Ah = reinterpret_cast<const _Float16*>(Lh); a.Al = reinterpret_cast<const _Float16*>(Ll);
        a.lda = r; a.sa = m * r;
        a.Bh = reinterpret_cast<const _Float16*>(Rth); a.Bl = reinterpret_cast<const _Float16*>(Rtl);
        a.ldb = r; a.sb = n * r;
        a.tiles_n = ceil_div(n, XW_BN);
        a.tiles_m = ceil_div(m, XW_BM);
    } else {
        // A operand R^T (n x r): tile rows run over W's columns; B operand L (m x r): tile
        // columns run over W's rows (see q_update_x3_kernel)
        a.M = n; a.N = m;
        a.Ah = reinterpret_cast<const _Float16*>(Rth); a.Al = reinterpret_cast<const _Float16*>(Rtl);
        a.lda = r; a.sa = n * r;
        a.Bh = reinterpret_cast<const _Float16*>(Lh); a.Bl = reinterpret_cast<const _Float16*>(Ll);
        a.ldb = r; a.sb = m * r;
        a.tiles_n = ceil_div(m, XW_BN);
        a.tiles_m = ceil_div(n, XW_BM);
    }
    a.K = r; a.batch = batch;
    a.inv_scale = inv_scale;
    const int64_t tiles = a.tiles_n * a.tiles_m;
    CQ_REQUIRE(tiles * batch < (1ll << 31), "cq_q_update_x3: grid too large");
    q.W = W; q.wf16 = dtype == CQ_F16; q.m = m; q.n = n;
    q.absmax = reinterpret_cast<uint32_t*>(ws);
    q.part = reinterpret_cast<double*>(reinterpret_cast<char*>(ws) + align_up((size_t)batch * sizeof(uint32_t), 256));
    q.eps = eps; q.codes = codes; q.packed = packed; q.scale = scale_out; q.ew = err_w; q.sew = err_w ? err_w_stride : 0;
    hipStream_t s = as_stream(stream);
    const bool known = absmax_in && r == 0;  // max|W| bits given: skip the absmax pass
    if (known) {
        if (hipMemcpyAsync(q.absmax, absmax_in, batch * sizeof(uint32_t), hipMemcpyDeviceToDevice, s) != hipSuccess)
            return set_error(CQ_EHIP, "cq_q_update_x3: copy failed");
    } else if (hipMemsetAsync(q.absmax, 0, batch * sizeof(uint32_t), s) != hipSuccess) {
        return set_error(CQ_EHIP, "cq_q_update_x3: memset failed");
    }
    const unsigned grid = (unsigned)(tiles * batch);
    // row-panel kernel (q_update_p_kernel): K <= 256, m % 16 == 0, n % 32 == 0, 16-B aligned
    const bool pk = r > 0 && r <= QP_KMAX && m % 16 == 0 && n % QP_BN == 0 && vk && al16(Lh) && al16(Ll) &&
                    al16(Rth) && al16(Rtl);
    // single recompute (2-bit packed codes, fp16 W, previous scale given):
    // pass 2 + candidate lists + code kernel, pass 1 only where a list cannot be complete
    if (pk && !known && scale_hint && bits == 2 && packed && !codes && dtype == CQ_F16 &&
        qp_cand_ok(m, n, (int)r)) {
        int64_t regions = 0, cap = 0, capa = 0;
        qu_cand_geom(m, n, batch, qp_cand_rows((int)r), qp_cand_waves((int)r), &regions, &cap, &capa);
        char* c = reinterpret_cast<char*>(q.part) + align_up((size_t)batch * tiles * sizeof(double), 256);
        q.ovf = reinterpret_cast<uint32_t*>(c); c += align_up((size_t)batch * 4, 256);
        q.cnt = reinterpret_cast<uint32_t*>(c); c += align_up((size_t)batch * regions * 4, 256);
        q.part0 = reinterpret_cast<double*>(c); c += align_up((size_t)batch * regions * 8, 256);
        q.partF = reinterpret_cast<double*>(c); c += align_up((size_t)batch * regions * 8, 256);
        q.cntA = reinterpret_cast<uint32_t*>(c); c += align_up((size_t)batch * regions * 4, 256);
        q.gid = reinterpret_cast<uint32_t*>(c); c += align_up((size_t)batch * regions * cap * 4, 256);
        q.gval = reinterpret_cast<float4*>(c); c += align_up((size_t)batch * regions * cap * 32, 256);
        q.la = reinterpret_cast<uint2*>(c);
        q.cap = cap;
        q.capA = capa;
        q.hint = scale_hint;
        q.fb_out = fallback_out;
        q.x.batch = batch;
        if (hipMemsetAsync(q.ovf, 0, batch * sizeof(uint32_t), s) != hipSuccess)
            return set_error(CQ_EHIP, "cq_q_update_x3: memset failed");
        if (qp_launch_cand(q, Lh, Ll, Rth, Rtl, (int)r, batch, eps, scale_out, err_out, s) < 0)
            return set_error(CQ_EINVAL, "cq_q_update_x3: grid too large");
        return check_launch("cq_q_update_x3");
    }
    if (fallback_out && hipMemsetAsync(fallback_out, 0, batch * sizeof(int), s) != hipSuccess)
        return set_error(CQ_EHIP, "cq_q_update_x3: memset failed");
    if (pk && !known) {
        q.x.batch = batch;
        const int64_t p1 = qp_launch(q, dtype, bits, Lh, Ll, Rth, Rtl, (int)r, batch, s);
        if (p1 < 0) return set_error(CQ_EINVAL, "cq_q_update_x3: grid too large");
        q_update_finalize_kernel<<<(unsigned)batch, 64, 0, s>>>(q.absmax, q.part, p1, batch, eps, scale_out, err_out);
        return check_launch("cq_q_update_x3");
    }
    if (known && vk) {  // r = 0 with max|W| known: one streaming pass over W
        int64_t gx = std::max<int64_t>(1, std::min<int64_t>(tiles, ceil_div(m * n / 16, 256)));
        if (err_w) {  // a stride of whole rows: each thread keeps its 16 columns (and their weights);
                      // rounded down, as the workspace holds `tiles` error partials per matrix
            const int64_t g16 = n / 16, unit = g16 / std::gcd<int64_t>(g16, 256);
            if (gx >= unit) gx = gx / unit * unit;
        }
        CQ_REQUIRE(batch < 65536, "cq_q_update_x3: batch too large");
        const dim3 sg((unsigned)gx, (unsigned)batch);
#define CQ_QS(DT, B) do { if (q.ew) quant_w_stream_kernel<DT, B, true><<<sg, 256, 0, s>>>(q); \
                             else quant_w_stream_kernel<DT, B, false><<<sg, 256, 0, s>>>(q); } while (0)
        if (dtype == CQ_F16) {
            switch (bits) { case 2: CQ_QS(CQ_F16, 2); break; case 4: CQ_QS(CQ_F16, 4); break;
                            case 8: CQ_QS(CQ_F16, 8); break; default: CQ_QS(CQ_F16, 16); }
        } else {
            switch (bits) { case 2: CQ_QS(CQ_F32, 2); break; case 4: CQ_QS(CQ_F32, 4); break;
                            case 8: CQ_QS(CQ_F32, 8); break; default: CQ_QS(CQ_F32, 16); }
        }
#undef CQ_QS
        q_update_finalize_kernel<<<(unsigned)batch, 64, 0, s>>>(q.absmax, q.part, gx, batch, eps, scale_out, err_out);
        return check_launch("cq_q_update_x3");
    }
#define CQ_QU(B) do { if (vk && dtype == CQ_F16) { \
                          if (!known) q_update_v_kernel<0, B, CQ_F16><<<grid, XW_THREADS, XW_LDS_BYTES, s>>>(q); \
                          q_update_v_kernel<1, B, CQ_F16><<<grid, XW_THREADS, XW_LDS_BYTES, s>>>(q); } \
                      else if (vk) { if (!known) q_update_v_kernel<0, B, CQ_F32><<<grid, XW_THREADS, XW_LDS_BYTES, s>>>(q); \
                                     q_update_v_kernel<1, B, CQ_F32><<<grid, XW_THREADS, XW_LDS_BYTES, s>>>(q); } \
                      else { if (!known) q_update_x3_kernel<0, B><<<grid, XW_THREADS, XW_LDS_BYTES, s>>>(q); \
                             q_update_x3_kernel<1, B><<<grid, XW_THREADS, XW_LDS_BYTES, s>>>(q); } } while (0)
    switch (bits) {
        case 2: CQ_QU(2); break;
        case 4: CQ_QU(4); break;
        case 8: CQ_QU(8); break;
        default: CQ_QU(16); break;
    }
#undef CQ_QU
    q_update_finalize_kernel<<<(unsigned)batch, 64, 0, s>>>(q.absmax, q.part, tiles, batch, eps, scale_out, err_out);
    return check_launch("cq_q_update_x3");
}


int cq_absmax(int dtype, const void* X, int64_t n_per, int64_t batch, float* out, void* stream) {
    CQ_REQUIRE(X && out && n_per > 0 && batch > 0 && batch < 65536, "cq_absmax: bad args");
    CQ_REQUIRE(dtype == CQ_F16 || dtype == CQ_F32, "cq_absmax: dtype must be f16/f32");
    hipStream_t s = as_stream(stream);
    if (hipMemsetAsync(out, 0, batch * sizeof(float), s) != hipSuccess) return set_error(CQ_EHIP, "cq_absmax: memset");
    const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(n_per, 256), std::max<int64_t>(1, 4096 / batch)));
    if (dtype == CQ_F16) absmax_dt_kernel<CQ_F16><<<dim3(gx, (unsigned)batch), 256, 0, s>>>(X, n_per, reinterpret_cast<uint32_t*>(out));
    else absmax_dt_kernel<CQ_F32><<<dim3(gx, (unsigned)batch), 256, 0, s>>>(X, n_per, reinterpret_cast<uint32_t*>(out));
    return check_launch("cq_absmax");  // max |x| bits are the float's bits: out reads as float
}

size_t cq_residual_split_workspace(int64_t m, int64_t n, int64_t batch) {
    const int64_t gy = std::max<int64_t>(1, std::min<int64_t>(m / 32, 16));
    return (size_t)batch * gy * ceil_div(n, 64) * sizeof(double);
}

int cq_residual_split(int dtype, const void* Ws, const uint8_t* packed, const float* qscale, int bits,
                      const float* ycol, float ycol_max, const float* wmax, int64_t batch, int64_t m, int64_t n,
                      float* res_out, float* Y_out, uint16_t* hi, uint16_t* lo, uint16_t* thi, uint16_t* tlo,
                      float* scale_out, double* sq_out, const float* ycol_hi, float ycol_hi_max, float* scale_hi_out,
                      int64_t ycol_stride, const float* ycol_max_v, const float* ycol_hi_max_v,
                      void* ws, size_t ws_bytes, void* stream) {
    CQ_REQUIRE(Ws && wmax && batch > 0 && batch < 65536 && m > 0 && n > 0, "cq_residual_split: bad args");
    CQ_REQUIRE(m % 32 == 0 && n % 64 == 0, "cq_residual_split: m % 32 and n % 64 must be 0");
    CQ_REQUIRE(!packed || qscale, "cq_residual_split: scale required with codes");
    CQ_REQUIRE(!packed || bits == 2 || bits == 4 || bits == 8 || bits == 16 || bits == 32, "Bit-width not supported!");
    const bool exact = dtype == CQ_F16 && !packed && !ycol;  // lo = 0: the lo halves are optional
    CQ_REQUIRE((!lo || hi) && (!tlo || thi) && (exact || (!hi == !lo && !thi == !tlo)),
               "cq_residual_split: halves go in pairs (lo optional only for fp16 W without codes or ycol)");
    CQ_REQUIRE((!hi && !thi) || scale_out, "cq_residual_split: halves need scale_out");
    CQ_REQUIRE(!ycol_hi || (hi && lo && scale_hi_out), "cq_residual_split: ycol_hi needs hi, lo and scale_hi_out");
    CQ_REQUIRE(!sq_out || (ws && ws_bytes >= cq_residual_split_workspace(m, n, batch)), "cq_residual_split: workspace too small");
    const int64_t gy = std::max<int64_t>(1, std::min<int64_t>(m / 32, 16));
    dim3 grid((unsigned)(n / 64), (unsigned)gy, (unsigned)batch);
    hipStream_t s = as_stream(stream);
    double* part = sq_out ? reinterpret_cast<double*>(ws) : nullptr;
    auto h = [](uint16_t* p) { return reinterpret_cast<_Float16*>(p); };
#define CQ_RS(DT, B) residual_split_kernel<DT, B><<<grid, 256, 0, s>>>(Ws, packed, qscale, ycol, wmax, ycol_max, m, n, \
        res_out, Y_out, h(hi), h(lo), h(thi), h(tlo), scale_out, part, ycol_hi, ycol_hi_max, scale_hi_out, \
        ycol_stride, ycol_max_v, ycol_hi_max_v)
    const int bsel = packed ? bits : 2;
    if (dtype == CQ_F16) {
        switch (bsel) { case 2: CQ_RS(CQ_F16, 2); break; case 4: CQ_RS(CQ_F16, 4); break;
                        case 8: CQ_RS(CQ_F16, 8); break; case 32: CQ_RS(CQ_F16, 32); break; default: CQ_RS(CQ_F16, 16); }
    } else {
        switch (bsel) { case 2: CQ_RS(CQ_F32, 2); break; case 4: CQ_RS(CQ_F32, 4); break;
                        case 8: CQ_RS(CQ_F32, 8); break; case 32: CQ_RS(CQ_F32, 32); break; default: CQ_RS(CQ_F32, 16); }
    }
#undef CQ_RS
    if (sq_out) sum_tile_parts_kernel<<<(unsigned)batch, 64, 0, s>>>(part, gy * (n / 64), sq_out);
    return check_launch("cq_residual_split");
}

int cq_gemm_x3(const cq_x3_args* g, void* stream) {
    CQ_REQUIRE(g, "cq_gemm_x3: null args");
    CQ_REQUIRE(g->Ah && g->Al && g->Bh && (g->Bl || g->single || g->b_exact) && (g->C || g->sym_out) && g->inv_scale,
               "cq_gemm_x3: null operand");
    CQ_REQUIRE(!g->sym_out || (g->tri && g->out_h && g->out_l && g->out_bound && g->scale_out && g->inv_out &&
                               g->out_scale > 0.f && g->N % 32 == 0),
               "cq_gemm_x3: sym_out needs tri, out_h/out_l, out_bound, scale_out, inv_out, N % 32 == 0");
    CQ_REQUIRE(g->M > 0 && g->N > 0 && g->K > 0 && g->batch > 0, "cq_gemm_x3: bad shape");
    CQ_REQUIRE(g->K % XW_BK == 0, "cq_gemm_x3: K must be a multiple of 32");
    CQ_REQUIRE(g->lda % 8 == 0 && g->ldb % 8 == 0 && g->stride_a % 8 == 0 && g->stride_b % 8 == 0,
               "cq_gemm_x3: operand rows must be 16-byte aligned");
    CQ_REQUIRE((g->a_blocked ? g->lda >= g->M : g->lda >= g->K) && (g->b_blocked ? g->ldb >= g->N : g->ldb >= g->K) &&
                   g->ldc >= g->N,
               "cq_gemm_x3: leading dimension too small");
    CQ_REQUIRE(!g->out_h == !g->out_l, "cq_gemm_x3: out_h and out_l go together");
    CQ_REQUIRE(!g->out_h || g->sym_out || (g->overflow && g->out_scale > 0.f),
               "cq_gemm_x3: split output needs overflow flags");
    CQ_REQUIRE(!g->beta_v || g->P, "cq_gemm_x3: beta_v needs P");
    CQ_REQUIRE(!g->gamma_v || g->D, "cq_gemm_x3: gamma_v needs D");
    X3K a;
    a.M = g->M; a.N = g->N; a.K = g->K; a.batch = g->batch;
    a.Ah = reinterpret_cast<const _Float16*>(g->Ah); a.Al = reinterpret_cast<const _Float16*>(g->Al);
    a.lda = g->lda; a.sa = g->stride_a;
    a.Bh = reinterpret_cast<const _Float16*>(g->Bh); a.Bl = reinterpret_cast<const _Float16*>(g->Bl);
    a.ldb = g->ldb; a.sb = g->stride_b;
    a.inv_scale = g->inv_scale;
    a.C = g->C; a.ldc = g->ldc; a.sc = g->stride_c;
    a.P = g->P; a.ldp = g->ldp; a.sp = g->stride_p;
    a.D = g->D; a.ldd = g->ldd; a.sd = g->stride_d;
    a.alpha_v = g->alpha_v; a.beta_v = g->beta_v; a.gamma_v = g->gamma_v;
    a.Oh = reinterpret_cast<_Float16*>(g->out_h); a.Ol = reinterpret_cast<_Float16*>(g->out_l);
    a.ldo = g->ldo; a.so = g->stride_o; a.out_scale = g->out_scale;
    a.overflow = g->overflow;
    CQ_REQUIRE(!g->tri || (g->M == g->N && !g->P && !g->D && (!g->out_h || g->sym_out)),
               "cq_gemm_x3: tri needs a square plain product");
    a.single = g->single;
    a.colw = g->colw;
    a.scolw = g->stride_colw;
    a.absmax_out = g->absmax_out;
    a.Ct = g->Ct;
    a.sct = g->stride_ct;
    CQ_REQUIRE(!g->Ct || (!g->sym_out && !g->tri && g->C), "cq_gemm_x3: Ct needs a non-symmetric product with C");
    CQ_REQUIRE(!g->absmax_out || (!g->sym_out && !g->tri), "cq_gemm_x3: absmax_out needs a plain product");
    CQ_REQUIRE(!g->colw || (!g->sym_out && !g->tri), "cq_gemm_x3: colw needs a plain product");
    // single + sym_out: the Gram of an exactly-fp16 operand (lo = 0; A = W W^T of the sparse-code
    // Gram, sgram.py): the split products add exact zeros, so one product gives the same bits
    a.sym_out = g->sym_out;
    a.out_bound = g->out_bound;
    a.scale_out = g->scale_out;
    a.inv_out = g->inv_out;
    a.tri = g->tri;
    a.b_blocked = g->b_blocked;
    a.active = g->active;
    a.a_blocked = g->a_blocked;
    a.o_blocked = g->o_blocked;
    CQ_REQUIRE(!g->o_blocked || g->N % 32 == 0, "cq_gemm_x3: blocked split output needs N % 32 == 0");
    CQ_REQUIRE(!g->a_blocked || g->lda >= g->M, "cq_gemm_x3: blocked A needs lda = rows >= M");
    CQ_REQUIRE(!g->active || g->D, "cq_gemm_x3: active needs D (the pass-through value)");
    CQ_REQUIRE(!g->b_blocked || g->ldb >= g->N, "cq_gemm_x3: blocked B needs ldb = rows >= N");
    a.tiles_n = ceil_div(g->N, XW_BN);
    a.tiles_m = ceil_div(g->M, XW_BM);
    int64_t total = a.tiles_n * a.tiles_m * a.batch;
    a.tiles_live = 0;
    if (a.sym_out) {  // tiles with tn >= tm / 2 (XW_BN = 2 XW_BM): the rest lie below the diagonal
        static_assert(XW_BN == 2 * XW_BM, "Gram tile enumeration");
        for (int64_t tm = 0; tm < a.tiles_m; ++tm) a.tiles_live += std::max<int64_t>(0, a.tiles_n - (tm >> 1));
        total = a.tiles_live * a.batch;
    }
    a.ksplit = g->ksplit > 1 ? g->ksplit : 1;
    a.part = g->split_ws;
    if (a.ksplit > 1) {
        CQ_REQUIRE(!a.tri && !a.sym_out && a.part && a.C && g->N % 4 == 0 && a.ksplit <= g->K / XW_BK,
                   "cq_gemm_x3: split-K needs a plain product with C, N % 4 == 0, split_ws, ksplit <= K / 32");
        total *= a.ksplit;
    }
    CQ_REQUIRE(total < (1ll << 31), "cq_gemm_x3: grid too large");
    // the 256 x 256 tile where the 192 x 384 one would leave over 15 % of its MFMA work idle
    // (rank-256 products), for plain split products
    const bool sq = !a.single && !g->b_exact && !a.tri && !a.sym_out && a.ksplit == 1 && !a.P && !a.D && !a.Oh && !a.Ct &&
                    !a.colw && !a.active && g->M % XS_BM == 0 && g->N % XS_BN == 0 && g->ldc % 4 == 0 &&
                    g->stride_c % 4 == 0 && (reinterpret_cast<uintptr_t>(g->C) & 15) == 0 &&
                    (double)(a.tiles_m * XW_BM) * (double)(a.tiles_n * XW_BN) > 1.15 * (double)g->M * (double)g->N;
    if (sq) {
        a.tiles_m = g->M / XS_BM;
        a.tiles_n = g->N / XS_BN;
        const int64_t tot = a.tiles_m * a.tiles_n * a.batch;
        CQ_REQUIRE(tot < (1ll << 31), "cq_gemm_x3: grid too large");
        gemm_x3s_kernel<<<(unsigned)tot, XS_THREADS, XS_LDS_BYTES, as_stream(stream)>>>(a);
        return check_launch("cq_gemm_x3");
    }
    if (a.single) gemm_x3v_kernel<1><<<(unsigned)total, XW_THREADS, XW_LDS_BYTES, as_stream(stream)>>>(a);
    else if (g->b_exact) gemm_x3v_kernel<2><<<(unsigned)total, XW_THREADS, XW_LDS_BYTES, as_stream(stream)>>>(a);
    else gemm_x3v_kernel<0><<<(unsigned)total, XW_THREADS, XW_LDS_BYTES, as_stream(stream)>>>(a);
    if (a.ksplit > 1)
        x3_splitk_epi_kernel<<<dim3((unsigned)ceil_div(g->M * (g->N / 4), 256), (unsigned)g->batch), 256, 0,
                               as_stream(stream)>>>(a);
    return check_launch("cq_gemm_x3");
}

}  // extern "C"
