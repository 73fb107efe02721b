// Row-panel fused Q update: maybe_update_Q (alg.py:253-283) + quantize_matrix
// (alg.py:245-250, quantization.py:244-269) for K = r <= 256, both passes of the absmax /
// quantise pair on res = W - L R recomputed on split-fp16 MFMAs (see qp_body).  Its own
// translation unit so that it builds without SLP vectorisation (build.py), which keeps the
// per-element epilogue in scalar fp32 instructions.
#include "cq_x3.h"

namespace cq {

// ------------------------------------------------------------------ row-panel fused Q update
// Same two passes and per-element arithmetic as q_update_v_kernel (res = W - L R on
// split-fp16 MFMAs, absmax pass, quantise pass), organised for K = r <= 256: a workgroup owns
// a panel of QP_WAVES * 16 * RB rows of W and walks its columns in chunks of 32.  Each wave
// keeps its L rows' fragments (hi and lo, all of K) in VGPRs for the whole panel, so L is
// read once per panel; the chunk's R^T rows are staged once per workgroup in LDS by LDS-DMA
// (double buffer) and shared by every wave.  Per output element the load path then carries
// 2 B of W plus 512 B / (rows per panel) of R^T halves (1 B at 512 rows) instead of ~4 B of
// operand tiles with the 192 x 384 tiles.  Transposed MFMA (A = R^T, B = L) with the R^T rows
// of a chunk permuted so each lane owns 8 consecutive columns of one W row: 16-byte W loads.
//
// W stream (fp16 W, WL): a chunk's W rows come by LDS-DMA into a ring of QP_WD slots, each
// wave filling and reading only its own 16-row x 64-B pieces (no extra barrier), QP_WD - 1
// chunks ahead of the compute (~4.6 us of MFMA work at QP_WD = 5): with the W registers of
// the previous design only 1-2 chunks could be in flight, and every chunk waited out an HBM
// round trip (pass 0 3.3 ms, pass 1 5.0 ms per B = 256 call against a ~1.6 ms MFMA floor).
// The end-of-chunk wait is counted (the ring's newest slot stays in flight); only pass 1's
// code stores, gathered over 16 chunks into whole 128-B row segments, need a full drain
// (vmcnt also counts stores, which may complete out of order with the loads).
constexpr int QP_WAVES = 8;               // default waves per workgroup (template parameter NW);
                                          // the 2-bit list path at K <= 128 runs 12 (qp_cand_waves)
constexpr int QP_WD = 5;                  // W ring slots (WL path)
constexpr size_t QP_LDS_MAX = 156 * 1024;

// LDS halves of one R^T stage (hi rows, then lo rows; RROW = 32 KSMAX halves per R^T row) and
// of one W ring slot (NW waves x RB row blocks x 16 rows x 32 columns)
__host__ __device__ constexpr int qp_rstage(int ksmax) { return 2 * QP_BN * 32 * ksmax; }
__host__ __device__ constexpr int qp_wslot(int nw, int rb) { return nw * rb * 512; }
__host__ __device__ constexpr size_t qp_lds_bytes(int nw, int rb, int ksmax, bool wl) {
    // (W ring: + two 32-float slots of the error column weights of a chunk, pass 2)
    return (size_t)(2 * qp_rstage(ksmax) + (wl ? QP_WD * qp_wslot(nw, rb) + 2 * 64 : 0)) * 2;
}

// 16-B chunk swizzle of an LDS row: the 16 rows one MFMA fragment read touches (rows
// 8 a + b + 4 c, a, b < 4) land on 16 different chunk positions mod 16 (bank-conflict free)
__device__ __forceinline__ int qp_swz(int row) { return (row & 3) | (((row >> 3) & 3) << 2); }

// LDS-DMA of chunk n0's R^T rows (both halves) into a stage of RROW-half rows: each
// wave-instruction fills 512 / RROW whole rows (1 KB), 64 / NW... instructions per wave; lane
// slot (lane % (RROW / 8)) holds logical 16-B chunk slot ^ swz(row)
template <int NW, int RROW>
__device__ __forceinline__ void qp_issue_r(const uint16_t* __restrict__ Rh, const uint16_t* __restrict__ Rl,
                                           int64_t n0, int K, _Float16* stage, int wid, int lane) {
    constexpr int RPI = 512 / RROW;            // rows per wave-instruction
    constexpr int LPR = RROW / 8;              // lanes per row
    constexpr int NI = 2 * QP_BN / RPI;        // instructions per stage
    // waves take instructions wid, wid + NW, ... (NW need not divide NI: the counted waits
    // only count the W loads issued after a stage)
#pragma unroll
    for (int u = 0; u < (NI + NW - 1) / NW; ++u) {
        const int I = wid + u * NW;
        if (I >= NI) break;
        const int half = I / (NI / 2), rowbase = RPI * (I % (NI / 2));
        const int row = rowbase + lane / LPR;
        const int logical = (lane % LPR) ^ qp_swz(row);
        const int kc = 8 * logical < K ? 8 * logical : 0;   // past K: any valid address (unused)
        const uint16_t* src = (half ? Rl : Rh) + (n0 + row) * (int64_t)K + kc;
        _Float16* dst = stage + (half * QP_BN + rowbase) * RROW;
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
}

template <int RROW>
__device__ __forceinline__ f16x8g qp_frag(const _Float16* stage, int half, int row, int chunk) {
    return *reinterpret_cast<const f16x8g*>(stage + (half * QP_BN + row) * RROW + 8 * (chunk ^ qp_swz(row)));
}

// The single-recompute path's completeness test for matrix b with scale s: every nonzero
// 2-bit code needs |res| > s / 2, and the list holds every |res| >= tau, so the list is
// complete when 2 tau <= s (exact), no wave's list overflowed, and the quotients take the
// branch-free division (as pass 1 would).  Otherwise pass 1 recomputes the matrix.
__device__ __forceinline__ bool qp_fallback(const QUK& q, int64_t b, float s) {
    const float h = q.hint[b];
    if (!(h > 0.f && h <= 0x1p127f)) return true;
    const float tau = QP_TAU * h;
    return q.ovf[b] != 0u || !div_fast_ok(s) || !(2.f * tau <= s);
}

// max(m, |a|, |b|) in one v_max3_f32 with |.| source modifiers (fmaxf would first canonicalise
// each |x| by a v_max_f32 of its own).  A NaN operand is dropped, not propagated: pass 2
// catches NaN residuals through its error sum instead.
__device__ __forceinline__ float qp_max3_abs(float m, float a, float b) {
    float r;
    asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}

// RB row-blocks of 16 rows per wave; K = r <= 32 KSMAX.  FAST (pass 1): the scale is a
// finite normal number and |res| <= scale, so x / s and c / k take the branch-free correctly
// rounded division (div_fast; same results as IEEE division), and 2-bit dequantisation is
// c * s (k = 1: (c / 1) * s is exactly c * s).  The per-element arithmetic is scalar fp32 in
// this translation unit, compiled without SLP vectorisation: beside MFMAs a packed
// v_pk_{mul,add,fma}_f32 costs ~13 issue cycles more than the two scalar ops it replaces
// (MI355X_MICROARCH.md, "price of one filler beside MFMAs"), and pass 1's epilogue is
// issue-bound (~1000 instructions per 32-column chunk and wave with packed pairs).
template <int PASS, int BITS, int DT, int RB, int KSMAX, bool FAST, int NW, bool WL>
__device__ __forceinline__ void qp_body(const QUK& q, const uint16_t* __restrict__ Lh, const uint16_t* __restrict__ Ll,
                                        const uint16_t* __restrict__ Rh, const uint16_t* __restrict__ Rl, int K,
                                        int panels, _Float16* smem, int64_t orig) {
    static_assert(!WL || DT == CQ_F16, "the W ring carries fp16 W");
    static_assert(PASS != 2 || (WL && BITS == 2), "the candidate pass runs on the W ring, 2-bit codes");
    constexpr int ROWS = NW * 16 * RB;
    constexpr int WV = DT == CQ_F16 ? 1 : 2;        // uint4 per lane-run of 8 W elements
    constexpr int RROW = 32 * KSMAX;                 // halves per R^T row in LDS
    constexpr int RSTAGE = qp_rstage(KSMAX);
    constexpr int WSLOT = qp_wslot(NW, RB);
    // pass 1 packed 2-bit codes: a row's code bytes of GRP chunks are gathered before one store
    // (E = GRP / 4 entries of 8 B per lane, lanes lq = 0..3 of the row side by side)
    constexpr int GRP = WL ? 16 : 4, E = GRP / 4;
    const int64_t m = q.m, n = q.n, MN = m * n;
    // XCD-aware order: the panels of one matrix run on one XCD (R^T chunks shared in its L2)
    const int64_t total = (int64_t)panels * q.x.batch;
    const int64_t qq = total / 8, r8 = total % 8, xcd = orig % 8;
    const int64_t lin = (xcd < r8 ? xcd * (qq + 1) : r8 * (qq + 1) + (xcd - r8) * qq) + orig / 8;
    const int64_t b = lin / panels, panel = lin % panels;
    const float* __restrict__ ewb = q.ew ? q.ew + b * q.sew : nullptr;  // this matrix's error weights
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int l16 = lane & 15, lq = lane >> 4;
    const int KS = K / 32;
    const uint16_t* Lhb = Lh + b * m * (int64_t)K;
    const uint16_t* Llb = Ll + b * m * (int64_t)K;
    const uint16_t* Rhb = Rh + b * n * (int64_t)K;
    const uint16_t* Rlb = Rl + b * n * (int64_t)K;
    const int64_t row0 = panel * ROWS + wid * 16 * RB;   // this wave's first W row

    // this wave's L fragments: row block rb, K step ks, lane (l16 row, lq chunk)
    f16x8g lh[RB][KSMAX], ll[RB][KSMAX];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
        const int64_t row = row0 + 16 * rb + l16;
#pragma unroll
        for (int ks = 0; ks < KSMAX; ++ks) {
            if (ks < KS && row < m) {
                const int64_t o = row * K + 32 * ks + 8 * lq;
                lh[rb][ks] = *reinterpret_cast<const f16x8g*>(Lhb + o);
                ll[rb][ks] = *reinterpret_cast<const f16x8g*>(Llb + o);
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) { lh[rb][ks][e] = (_Float16)0.f; ll[rb][ks][e] = (_Float16)0.f; }
            }
        }
    }
    const float sc = q.x.inv_scale[b];
    const _Float16* Wh = reinterpret_cast<const _Float16*>(q.W) + b * MN;
    const float* Wf = reinterpret_cast<const float*>(q.W) + b * MN;
    constexpr float kq = (float)((1 << (BITS - 1)) - 1);
    float s = 0.f;
    if (PASS == 1) s = quant_scale(q.absmax[b], q.eps);
    const float ys = 1.f / s, yk = 1.f / kq;
    uint32_t mx = 0;
    double err = 0.0;
    // pass 2: candidate threshold (|res| >= tau as order-preserving bits; an invalid hint keeps
    // only non-finite values and the matrix falls back) and this wave's list region
    float tau = __builtin_inff();
    float mxf = 0.f;   // pass 2: max |res| (non-negative floats order as their bits)
    if (PASS == 2) {
        const float h = q.hint[b];
        if (h > 0.f && h <= 0x1p127f) tau = QP_TAU * h;
    }
    const int64_t region = (b * panels + panel) * NW + wid;
    int gcur = 0, gcurA = 0;   // pass 2: list-B groups / list-A entries this wave has listed
    uint2* const laR = PASS == 2 ? q.la + region * q.capA : nullptr;
    float4* const gvR = PASS == 2 ? q.gval + 2 * region * q.cap : nullptr;
    uint32_t* const gidR = PASS == 2 ? q.gid + region * q.cap : nullptr;
    const int capA = PASS == 2 ? (int)q.capA : 0, capB = PASS == 2 ? (int)q.cap : 0;
    // A-row t (MFMA row) of 16-column block c <-> chunk column 8 (t / 4) + 4 c + t % 4: the
    // lane (l16, lq) then owns chunk columns 8 lq .. 8 lq + 7 of W row l16 (per row block)
    const int acol0 = 8 * (l16 >> 2) + (l16 & 3);   // + 4 c
    const int64_t nchunks = n / QP_BN;
    auto w_elem = [&](int rb, int64_t n0) {          // this lane's first W element of chunk n0
        const int64_t row = row0 + 16 * rb + l16;
        return (row < m ? row : m - 1) * n + n0 + 8 * lq;
    };
    auto load_w = [&](int64_t n0, uint4 (&dst)[RB][WV]) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const int64_t e = w_elem(rb, n0);
            if (DT == CQ_F16) {
                dst[rb][0] = *reinterpret_cast<const uint4*>(Wh + e);
            } else {
                dst[rb][0] = *reinterpret_cast<const uint4*>(Wf + e);
                dst[rb][WV - 1] = *reinterpret_cast<const uint4*>(Wf + e + 4);
            }
        }
    };
    _Float16* wring = smem + 2 * RSTAGE;
    // pass 2 with error column weights: a chunk's 32 weights ride with its R^T stage (LDS-DMA
    // by 8 lanes of wave 0, issued before the W loads, so the counted wait covers them), read
    // from LDS in the epilogue -- a global load there would drain the W ring
    float* ewslot = reinterpret_cast<float*>(wring + QP_WD * WSLOT);
    const bool ewl = PASS == 2 && WL && q.ew != nullptr;
    auto issue_ew = [&](int64_t chn) {
        if (ewl && wid == 0 && lane < 8)
            __builtin_amdgcn_global_load_lds((const void*)(ewb + chn * QP_BN + 4 * lane),
                                             (__attribute__((address_space(3))) void*)(ewslot + 32 * (chn & 1)), 16, 0,
                                             0);
    };
    // WL: this wave's RB pieces (16 rows x 64 B) of chunk chn into ring slot `slot` by LDS-DMA
    auto issue_w = [&](int64_t chn, int slot) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            _Float16* dst = wring + slot * WSLOT + (wid * RB + rb) * 512;
            __builtin_amdgcn_global_load_lds((const void*)(Wh + w_elem(rb, chn * QP_BN)),
                                             (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        }
    };
    // the chunk's products: acc[rb][c][i] is (W row row0 + 16 rb + l16, column n0 + 8 lq + 4 c + i);
    // split: al x lh, ah x ll, ah x lh per K step (the one order both passes use)
    auto mma = [&](const _Float16* st, f32x4v (&acc)[RB][2]) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int c = 0; c < 2; ++c) acc[rb][c] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KSMAX; ++ks) {
            if (ks < KS) {
                f16x8g ah[2], al[2];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    ah[c] = qp_frag<RROW>(st, 0, acol0 + 4 * c, 4 * ks + lq);
                    al[c] = qp_frag<RROW>(st, 1, acol0 + 4 * c, 4 * ks + lq);
                }
#pragma unroll
                for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[c], lh[rb][ks], acc[rb][c], 0, 0, 0);
                        acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[c], ll[rb][ks], acc[rb][c], 0, 0, 0);
                        acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[c], lh[rb][ks], acc[rb][c], 0, 0, 0);
                    }
            }
        }
    };
    // res = W - L R (alg.py:262) of row block rb: v[u] = element u of the lane's 8 columns
    // (acc[rb][u / 4][u % 4]; the product times the power-of-two scale is exact, then one
    // rounding in the subtraction, as the reference's fp32 W - L @ R)
    auto resid = [&](const uint4 (&wc)[RB][WV], const f32x4v (&acc)[RB][2], int rb, float (&v)[8]) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (DT == CQ_F16) {
                // one fma: the product times the power-of-two scale is exact, so w - acc sc
                // rounded once is the same number as the multiply then subtract of the fp32
                // path (v_fma_mix_f32 reads the f16 half of W's register directly)
                const uint32_t pr = (&wc[rb][0].x)[u >> 1];
                const float w = (float)__builtin_bit_cast(_Float16, (uint16_t)((u & 1) ? (pr >> 16) : (pr & 0xffffu)));
                v[u] = __builtin_fmaf(-acc[rb][u >> 2][u & 3], sc, w);
            } else {
                const float w = __uint_as_float((&wc[rb][u >> 2].x)[u & 3]);
                const float pv = acc[rb][u >> 2][u & 3] * sc;
                v[u] = w - pv;
            }
        }
    };
    auto vmax = [&](const float (&v)[8], uint32_t cur) {
#pragma unroll
        for (int u = 0; u < 8; u += 2) cur = max(cur, max(abs_bits(v[u]), abs_bits(v[u + 1])));
        return cur;
    };
    uint2 seg[RB][E];   // pass 1, 2-bit packed: a row's code bytes of the current GRP-chunk group
    // chunk ch's products and epilogue on W wc and R^T stage st; returns whether it issued
    // global stores (then only a full vmcnt drain is a safe wait)
    // passes 0 and 2, K <= 128 (UPF): the chunk's R^T fragments (both halves, every K step: 64 VGPRs) are read
    // from LDS once, behind one wait, and each row block's MFMAs are followed by its epilogue,
    // so the epilogue's VALU work of row block rb overlaps the MFMAs of rb + 1 (independent
    // registers) instead of waiting for all of them; the MFMA order per accumulator (K steps,
    // then al x lh, ah x ll, ah x lh) is the same as mma()'s, so the sums are bit-identical.
    constexpr bool UPF = KSMAX <= 4 && (PASS == 0 || PASS == 2) && NW <= 8;
    auto compute = [&](int64_t ch, const uint4 (&wc)[RB][WV], const _Float16* st) -> bool {
        const int64_t n0 = ch * QP_BN;
        bool stored = false;
        f32x4v acc[RB][2];
        f16x8g fh[UPF ? KSMAX : 1][2], fl[UPF ? KSMAX : 1][2];
        if constexpr (UPF) {
#pragma unroll
            for (int ks = 0; ks < KSMAX; ++ks)
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    if (ks < KS) {
                        fh[ks][c] = qp_frag<RROW>(st, 0, acol0 + 4 * c, 4 * ks + lq);
                        fl[ks][c] = qp_frag<RROW>(st, 1, acol0 + 4 * c, 4 * ks + lq);
                    }
                }
        } else {
            mma(st, acc);
        }
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            if constexpr (UPF) {
#pragma unroll
                for (int c = 0; c < 2; ++c) acc[rb][c] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < KSMAX; ++ks) {
                    if (ks < KS) {
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fl[ks][c], lh[rb][ks], acc[rb][c], 0, 0, 0);
                            acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fh[ks][c], ll[rb][ks], acc[rb][c], 0, 0, 0);
                            acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fh[ks][c], lh[rb][ks], acc[rb][c], 0, 0, 0);
                        }
                    }
                }
            }
            const int64_t row = row0 + 16 * rb + l16;
            if (row >= m) continue;
            const int64_t e = row * n + n0 + 8 * lq;
            float v[8];
            resid(wc, acc, rb, v);
            if (PASS == 0) {
                mx = vmax(v, mx);
                continue;
            }
            if constexpr (PASS == 2) {
                // absmax; the error every element has with code 0 (d = 0 - x; fp32 over the
                // lane's 8 elements, fp64 across); and the candidates |res| >= tau, as lane
                // masks (v_cmp with the |.| modifier).  A lane group with exactly one candidate
                // goes to list A (its element index and residual), one with two or more to
                // list B (the whole group); the count runs bit-sliced on the masks (scalar
                // instructions), the slot of a lane comes from one ballot per list, so the list
                // order, hence every later sum, is deterministic.  The stores are followed by a
                // full drain at the chunk's end (compute() returns true).
                // (the per-element tests as 64-lane masks from the start: kept as lane booleans
                // the compiler materialises the count's and/or chain in VALU registers)
                uint64_t c[8];
                float e8 = 0.f;
#pragma unroll
                for (int u = 0; u < 8; ++u) c[u] = __ballot(__builtin_fabsf(v[u]) >= tau);
#pragma unroll
                for (int u = 0; u < 8; u += 2) mxf = qp_max3_abs(mxf, v[u], v[u + 1]);
                if (ewl) {
                    const float* wv = ewslot + 32 * (ch & 1) + 8 * lq;
#pragma unroll
                    for (int u = 0; u < 8; ++u) e8 = __builtin_fmaf(v[u] * v[u], wv[u], e8);
                } else {
#pragma unroll
                    for (int u = 0; u < 8; ++u) e8 = __builtin_fmaf(v[u], v[u], e8);
                }
                err += (double)e8;
                uint64_t any = c[0], two = 0;
#pragma unroll
                for (int u = 1; u < 8; ++u) {
                    two |= any & c[u];
                    any |= c[u];
                }
                const uint64_t mA = any & ~two, mB = two;
                if (mA | mB) {
                    stored = true;
                    if (__builtin_amdgcn_inverse_ballot_w64(mA)) {   // list A: the one candidate's index and residual
                        const int pos = gcurA + (int)__builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(mA >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mA, 0u));
                        if (pos < capA) {
                            // its position u1 bit by bit from the masks, its residual by a
                            // three-level select on those bits
                            const bool b0 = __builtin_amdgcn_inverse_ballot_w64(c[1] | c[3] | c[5] | c[7]);
                            const bool b1 = __builtin_amdgcn_inverse_ballot_w64(c[2] | c[3] | c[6] | c[7]);
                            const bool b2 = __builtin_amdgcn_inverse_ballot_w64(c[4] | c[5] | c[6] | c[7]);
                            const uint32_t u1 = (b0 ? 1u : 0u) | (b1 ? 2u : 0u) | (b2 ? 4u : 0u);
                            const float p0 = b0 ? v[1] : v[0], p1 = b0 ? v[3] : v[2];
                            const float p2 = b0 ? v[5] : v[4], p3 = b0 ? v[7] : v[6];
                            const float x1 = b2 ? (b1 ? p3 : p2) : (b1 ? p1 : p0);
                            laR[pos] = make_uint2((uint32_t)e + u1, __float_as_uint(x1));
                        }
                    }
                    if (__builtin_amdgcn_inverse_ballot_w64(mB)) {  // list B: the whole group
                        const int pos = gcur + (int)__builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(mB >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mB, 0u));
                        if (pos < capB) {
                            gvR[2 * pos] = make_float4(v[0], v[1], v[2], v[3]);
                            gvR[2 * pos + 1] = make_float4(v[4], v[5], v[6], v[7]);
                            gidR[pos] = (uint32_t)e;
                        }
                    }
                    gcurA += __builtin_popcountll(mA);
                    gcur += __builtin_popcountll(mB);
                }
                continue;
            }
            float cf[8];   // codes (integral floats)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float e4[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const float x = v[4 * h + t];
                    float c, dq;
                    if (FAST) {
                        // div_fast: q = x y, r = x - q s (FMA), q + r y
                        const float qd = x * ys;
                        const float rr = __builtin_fmaf(-qd, s, x);
                        const float z = __builtin_fmaf(rr, ys, qd) * kq;
                        c = rintf(z);
                        if (BITS == 2) {
                            dq = c * s;
                        } else {
                            const float qk = c * yk;
                            const float rk = __builtin_fmaf(-qk, kq, c);
                            dq = __builtin_fmaf(rk, yk, qk) * s;
                        }
                    } else {
                        c = quant_code_r(x, s, ys, kq);
                        dq = dequant_r(c, kq, yk, s);
                    }
                    const float d = dq - x;
                    e4[t] = d * d;
                    cf[4 * h + t] = c;
                }
                if (ewb) {  // error column weights (activation-aware error, alg.py:286-302)
                    const float4 wv = *reinterpret_cast<const float4*>(ewb + n0 + 8 * lq + 4 * h);
                    e4[0] *= wv.x; e4[1] *= wv.y; e4[2] *= wv.z; e4[3] *= wv.w;
                }
                err += (double)((e4[0] + e4[1]) + (e4[2] + e4[3]));  // fp32 within a run of 4, fp64 across
            }
            if (BITS == 2 && q.packed) {
                // bytes: codes 0-3, 4-7, MSB-first offset binary (c + 1): element u's code
                // has weight 2^(8 (u / 4) + 6 - 2 (u % 4)); the sum of (c_u + 1) times these
                // weights is an integer below 2^16, exact in fp32 (FMAs)
                constexpr float wt[8] = {64.f, 16.f, 4.f, 1.f, 16384.f, 4096.f, 1024.f, 256.f};
                float a0 = wt[0] + wt[2] + wt[4] + wt[6], a1 = wt[1] + wt[3] + wt[5] + wt[7];
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    a0 = __builtin_fmaf(cf[2 * p], wt[2 * p], a0);
                    a1 = __builtin_fmaf(cf[2 * p + 1], wt[2 * p + 1], a1);
                }
                const uint32_t w16 = (uint32_t)(a0 + a1);
                // a row's 8 code bytes of this chunk sit in lanes l16 + 16 t (t = 0..3): lane
                // lq == j / E gathers them into entry j % E, and at the end of a group of GRP
                // chunks lanes lq = 0..3 store the row's GRP x 8 contiguous bytes side by side
                // (one 2-B store per lane and chunk left 4.5x the packed bytes in partial-line
                // writes).  m % 16 == 0 keeps a row block, hence the shuffles, wave-uniform.
                const int j = (int)(ch % GRP);
                const uint32_t s0 = (uint32_t)__shfl((int)w16, l16), s1 = (uint32_t)__shfl((int)w16, l16 + 16);
                const uint32_t s2 = (uint32_t)__shfl((int)w16, l16 + 32), s3 = (uint32_t)__shfl((int)w16, l16 + 48);
                const uint2 v8 = make_uint2(s0 | (s1 << 16), s2 | (s3 << 16));
#pragma unroll
                for (int ee = 0; ee < E; ++ee)
                    if (lq == j / E && ee == j % E) seg[rb][ee] = v8;
                if (j == GRP - 1 || ch + 1 == nchunks) {
                    stored = true;
                    uint8_t* dst = q.packed + (b * MN + row * n) / 4 + (ch - j) * 8 + lq * E * 8;
                    if (j == GRP - 1 && E % 2 == 0) {
#pragma unroll
                        for (int ee = 0; ee < E; ee += 2)
                            *reinterpret_cast<uint4*>(dst + 8 * ee) =
                                make_uint4(seg[rb][ee].x, seg[rb][ee].y, seg[rb][ee + 1].x, seg[rb][ee + 1].y);
                    } else {
#pragma unroll
                        for (int ee = 0; ee < E; ++ee)
                            if (lq * E + ee <= j) *reinterpret_cast<uint2*>(dst + 8 * ee) = seg[rb][ee];
                    }
                }
            }
            int cq8[8];
            if (q.codes || (BITS == 4 && q.packed)) {
#pragma unroll
                for (int u = 0; u < 8; ++u) cq8[u] = (int)cf[u];
            }
            if (BITS == 4 && q.packed) {
                stored = true;
                uint32_t w32 = 0;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    w32 |= (((uint32_t)(cq8[2 * j] + 7) << 4) | (uint32_t)(cq8[2 * j + 1] + 7)) << (8 * j);
                *reinterpret_cast<uint32_t*>(q.packed + (b * MN + e) / 2) = w32;
            }
            if (q.codes) {
                stored = true;
                if (BITS <= 8) {
                    uint32_t c0 = 0, c1 = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        c0 |= (uint32_t)(uint8_t)(int8_t)cq8[j] << (8 * j);
                        c1 |= (uint32_t)(uint8_t)(int8_t)cq8[4 + j] << (8 * j);
                    }
                    *reinterpret_cast<uint2*>(reinterpret_cast<int8_t*>(q.codes) + b * MN + e) = make_uint2(c0, c1);
                } else {
                    int16_t* cp = reinterpret_cast<int16_t*>(q.codes) + b * MN + e;
                    *reinterpret_cast<short4*>(cp) = make_short4((short)cq8[0], (short)cq8[1], (short)cq8[2], (short)cq8[3]);
                    *reinterpret_cast<short4*>(cp + 4) = make_short4((short)cq8[4], (short)cq8[5], (short)cq8[6], (short)cq8[7]);
                }
            }
        }
        return stored;
    };
    // vmcnt(N) with expcnt / lgkmcnt at their maxima (not waited); vmcnt in bits [3:0], [15:14]
    auto wait_vm = [](auto n_c) {
        constexpr int nw = decltype(n_c)::value;
        __builtin_amdgcn_s_waitcnt((nw & 15) | ((nw >> 4) << 14) | (0x7 << 4) | (0xF << 8));
    };
    if constexpr (WL) {
        // ring: chunk ch's W in slot ch % QP_WD; at its start the R^T stage of ch + 1 and the W
        // of ch + QP_WD - 1 (into the slot chunk ch - 1 has finished reading) are issued
        static_assert(QP_WD >= 3, "W(ch + 1) must be older than R(ch + 1) at the counted wait");
        qp_issue_r<NW, RROW>(Rhb, Rlb, 0, K, smem, wid, lane);
        issue_ew(0);
        for (int c = 0; c < QP_WD - 1 && c < nchunks; ++c) issue_w(c, c);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // static priority for the youngest wave of each SIMD (waves NW - 4 .. NW - 1, dispatched
        // last: the arbitration losers of every chunk), set once (MI355X_MICROARCH.md, static
        // priority): list pass 2 4.35 -> 4.21 ms per B = 256 call, profiles/r05r_kt_*
        if (wid >= NW - 4) __builtin_amdgcn_s_setprio(1);
        int sw = 0;   // slot of chunk ch
        for (int64_t ch = 0; ch < nchunks; ++ch) {
            if (ch + 1 < nchunks) {
                qp_issue_r<NW, RROW>(Rhb, Rlb, (ch + 1) * QP_BN, K, smem + ((ch + 1) & 1) * RSTAGE, wid, lane);
                issue_ew(ch + 1);
            }
            const bool wlive = ch + QP_WD - 1 < nchunks;
            if (wlive) issue_w(ch + QP_WD - 1, sw == 0 ? QP_WD - 1 : sw - 1);
            uint4 wc[RB][WV];
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
                wc[rb][0] = *reinterpret_cast<const uint4*>(wring + sw * WSLOT + (wid * RB + rb) * 512 + 8 * lane);
            const bool stored = compute(ch, wc, smem + (ch & 1) * RSTAGE);
            // R(ch + 1) and W(ch + 1) landed (W(ch + QP_WD - 1), issued after R(ch + 1), may
            // stay in flight); after stores only a full drain is safe
            if (!stored && wlive) wait_vm(std::integral_constant<int, RB>{});
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();  // next chunk's stage landed everywhere; this chunk's stage fully read
            sw = sw + 1 == QP_WD ? 0 : sw + 1;
        }
    } else {
        // registers: pass 0 keeps W two chunks ahead (three buffers, loop unrolled by 3 so no
        // in-flight destination is copied), pass 1 one chunk ahead
        constexpr int WAHEAD = PASS == 0 ? 2 : 1;
        uint4 wr[RB][WV], wn[RB][WV], w3[PASS == 0 ? RB : 1][WV];
        auto chunk = [&](int64_t ch, uint4 (&wc)[RB][WV], uint4 (&wl)[RB][WV]) {
            if (ch + 1 < nchunks)
                qp_issue_r<NW, RROW>(Rhb, Rlb, (ch + 1) * QP_BN, K, smem + ((ch + 1) & 1) * RSTAGE, wid, lane);
            const bool wlive = ch + WAHEAD < nchunks;
            if (wlive) load_w((ch + WAHEAD) * QP_BN, wl);
            const bool stored = compute(ch, wc, smem + (ch & 1) * RSTAGE);
            if (PASS == 0 && wlive && !stored) wait_vm(std::integral_constant<int, RB * WV>{});
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        };
        qp_issue_r<NW, RROW>(Rhb, Rlb, 0, K, smem, wid, lane);
        load_w(0, wr);
        if (PASS == 0 && nchunks > 1) load_w(QP_BN, wn);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if constexpr (PASS == 0) {
            for (int64_t ch = 0; ch < nchunks; ch += 3) {
                chunk(ch, wr, w3);
                if (ch + 1 < nchunks) chunk(ch + 1, wn, wr);
                if (ch + 2 < nchunks) chunk(ch + 2, w3, wn);
            }
        } else {
            for (int64_t ch = 0; ch < nchunks; ++ch) {
                chunk(ch, wr, wn);
#pragma unroll
                for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                    for (int w = 0; w < WV; ++w) wr[rb][w] = wn[rb][w];  // landed at the chunk's vmcnt(0)
            }
        }
    }
    if (PASS == 2) mx = __float_as_uint(mxf);
    if (PASS == 0 || PASS == 2) {
        mx = wave_max_u32(mx);
        if (lane == 0 && mx) atomicMax(q.absmax + b, mx);
    }
    if (PASS == 2) {
        if (lane == 0) {
            // gcur == cap: every listed group got a slot (pos < cap) -- a full list, not an
            // overflow; past cap the count is clamped and the matrix falls back to pass 1
            q.cnt[region] = (uint32_t)(gcur <= capB ? gcur : capB);
            q.cntA[region] = (uint32_t)(gcurA <= capA ? gcurA : capA);
            if (gcur > capB || gcurA > capA) q.ovf[b] = 1u;
        }
        __shared__ double red2[16];
        const double tsum = block_sum_f64(err, red2);
        if (tid == 0) {
            q.part0[b * panels + panel] = tsum;
            // a NaN residual (the float max above skips it; the error sum does not): the
            // matrix takes pass 1 with a NaN absmax, as the two-pass form would
            if (tsum != tsum) {
                q.ovf[b] = 1u;
                atomicMax(q.absmax + b, 0x7fffffffu);
            }
        }
    } else if (PASS == 1 && q.part) {
        __shared__ double red[16];
        const double tsum = block_sum_f64(err, red);
        if (tid == 0) q.part[b * panels + panel] = tsum;
    }
}

static_assert(qp_lds_bytes(QP_WAVES, 3, 4, true) <= QP_LDS_MAX && qp_lds_bytes(QP_WAVES, 2, 8, true) <= QP_LDS_MAX &&
                  qp_lds_bytes(12, 2, 4, true) <= QP_LDS_MAX,
              "Q-update LDS: R^T stages + W ring fit one CU (160 KB, static reduction scratch aside)");

template <int PASS, int BITS, int DT, int RB, int KSMAX, int NW, bool WL>
__global__ __launch_bounds__(NW * 64, 1) void q_update_p_kernel(QUK q, const uint16_t* __restrict__ Lh,
                                                                   const uint16_t* __restrict__ Ll,
                                                                   const uint16_t* __restrict__ Rh,
                                                                   const uint16_t* __restrict__ Rl, int K,
                                                                   int panels) {
    extern __shared__ __attribute__((aligned(16))) char qp_smem_raw[];
    _Float16* smem = reinterpret_cast<_Float16*>(qp_smem_raw);
    if (PASS == 0 || PASS == 2) {
        qp_body<PASS, BITS, DT, RB, KSMAX, false, NW, WL>(q, Lh, Ll, Rh, Rl, K, panels, smem, blockIdx.x);
        return;
    }
    // which matrix a panel serves (same mapping as qp_body) decides the division path.  The
    // fallback launch of the list path is a grid of one workgroup per CU looping over the panels
    // (gridDim a multiple of 8: a panel keeps its XCD), so that matrices that took the list
    // path cost a check, not a dispatch of a 150-KB-LDS workgroup
    const int64_t total = (int64_t)panels * q.x.batch;
    for (int64_t orig = blockIdx.x; orig < total; orig += gridDim.x) {
        const int64_t qq = total / 8, r8 = total % 8, xcd = orig % 8;
        const int64_t lin = (xcd < r8 ? xcd * (qq + 1) : r8 * (qq + 1) + (xcd - r8) * qq) + orig / 8;
        const float sb = quant_scale(q.absmax[lin / panels], q.eps);
        if (q.only_fallback && !qp_fallback(q, lin / panels, sb)) continue;   // codes came from the list
        if (div_fast_ok(sb)) qp_body<PASS, BITS, DT, RB, KSMAX, true, NW, WL>(q, Lh, Ll, Rh, Rl, K, panels, smem, orig);
        else qp_body<PASS, BITS, DT, RB, KSMAX, false, NW, WL>(q, Lh, Ll, Rh, Rl, K, panels, smem, orig);
    }
}


// ------------------------------------------------------------------ list path: codes + error
// One workgroup per wave region of pass 2 (rpw rows x n): the region's packed 2-bit codes are
// built in LDS (all code 0 = offset-binary 01, then each nonzero code of a listed group flips
// its 2 bits by an LDS xor: 01 -> 10 for c = 1, 01 -> 00 for c = -1) and stored whole; the error correction
// of a nonzero code, (c s - x)^2 - x^2, with pass 1's fp32 arithmetic, summed in fp64 in list
// order (deterministic).  Codes: the same quotient as pass 1 (div_fast of the same residual).
__global__ __launch_bounds__(256) void qp_codes_kernel(QUK q, int panels, int nw, int rpw) {
    extern __shared__ __attribute__((aligned(16))) uint32_t qc_lds[];
    const int64_t region = blockIdx.x;
    const int64_t b = region / ((int64_t)panels * nw);
    const int64_t rem = region % ((int64_t)panels * nw);
    const int64_t r0 = (rem / nw) * (int64_t)nw * rpw + (rem % nw) * (int64_t)rpw;
    const float s = quant_scale(q.absmax[b], q.eps);
    if (qp_fallback(q, b, s)) return;   // pass 1 writes this matrix's codes and errors
    const int tid = threadIdx.x;
    const int64_t m = q.m, n = q.n;
    const int64_t nr = r0 < m ? (m - r0 < rpw ? m - r0 : rpw) : 0;
    __shared__ double red[16];
    double delta = 0.0;
    if (nr > 0) {
        const int64_t words = nr * n / 16;   // 16 codes per 32-bit word
        for (int64_t i = tid; i < words; i += 256) qc_lds[i] = 0x55555555u;
        __syncthreads();
        const float ys = 1.f / s;
        const int64_t cnt = q.cnt[region];
        const uint32_t* gid = q.gid + region * q.cap;
        const float4* gv = q.gval + 2 * region * q.cap;
        const int64_t base = r0 * n;
        // list A (single candidates), then list B (whole groups): a fixed order
        const int64_t cntA = q.cntA[region];
        const uint2* la = q.la + region * q.capA;
        for (int64_t i = tid; i < cntA; i += 256) {
            const uint2 en = la[i];
            const float x = __uint_as_float(en.y);
            const float qd = x * ys;
            const float rr = __builtin_fmaf(-qd, s, x);
            const float c = rintf(__builtin_fmaf(rr, ys, qd) * 1.f);
            if (c != 0.f) {
                const int64_t loc = (int64_t)en.x - base;
                const uint32_t sh = 8u * (uint32_t)((loc >> 2) & 3) + 6u - 2u * (uint32_t)(loc & 3);
                atomicXor(&qc_lds[loc >> 4], (c > 0.f ? 3u : 1u) << sh);
                const float d = c * s - x;
                if (q.ew) {
                    const float w = q.ew[b * q.sew + (int64_t)en.x % n];
                    delta += (double)((d * d) * w) - (double)((x * x) * w);
                } else {
                    delta += (double)(d * d) - (double)(x * x);
                }
            }
        }
        for (int64_t i = tid; i < cnt; i += 256) {
            const float4 v0 = gv[2 * i], v1 = gv[2 * i + 1];
            const float xs[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
            const int64_t loc0 = (int64_t)gid[i] - base;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const float x = xs[u];
                const float qd = x * ys;
                const float rr = __builtin_fmaf(-qd, s, x);
                const float c = rintf(__builtin_fmaf(rr, ys, qd) * 1.f);
                if (c != 0.f) {
                    const int64_t loc = loc0 + u;
                    // element loc: byte loc / 4 (bits 6 - 2 (loc % 4), MSB-first) of word loc / 16
                    const uint32_t sh = 8u * (uint32_t)((loc >> 2) & 3) + 6u - 2u * (uint32_t)(loc & 3);
                    atomicXor(&qc_lds[loc >> 4], (c > 0.f ? 3u : 1u) << sh);
                    const float d = c * s - x;
                    if (q.ew) {
                        const float w = q.ew[b * q.sew + (loc + base) % n];
                        delta += (double)((d * d) * w) - (double)((x * x) * w);
                    } else {
                        delta += (double)(d * d) - (double)(x * x);
                    }
                }
            }
        }
        __syncthreads();
        uint32_t* dst = reinterpret_cast<uint32_t*>(q.packed + (b * m * n + base) / 4);
        for (int64_t i = tid; i < words; i += 256) dst[i] = qc_lds[i];
    }
    const double t = block_sum_f64(delta, red);
    if (tid == 0) q.partF[region] = t;
}

// scale, error and fallback flag per matrix of the list path: pass-2 partials + the code
// kernel's corrections, or pass 1's partials where the matrix fell back (fixed order)
__global__ void qp_finalize_cand_kernel(QUK q, int panels, int nw, float* scale, double* err_out) {
    const int64_t b = blockIdx.x;
    const float s = quant_scale(q.absmax[b], q.eps);
    const bool fb = qp_fallback(q, b, s);
    double acc = 0.0;
    if (fb) {
        for (int t = threadIdx.x; t < panels; t += 64) acc += q.part[b * panels + t];
    } else {
        for (int t = threadIdx.x; t < panels; t += 64) acc += q.part0[b * panels + t];
        for (int t = threadIdx.x; t < panels * nw; t += 64) acc += q.partF[(b * panels) * nw + t];
    }
    acc = wave_sum(acc);
    if (threadIdx.x == 0) {
        if (scale) scale[b] = s;
        if (err_out) err_out[b] = acc;
        if (q.fb_out) q.fb_out[b] = fb ? 1 : 0;
    }
}

// list path geometry: K <= 128 runs 12 waves of 2 row blocks (three waves per SIMD at <= 168
// VGPRs: the fragments are read per K step instead of up front), K <= 256 8 waves of 2
constexpr int QP_CAND_NW_SMALL = 12;
int qp_cand_rows(int K) { (void)K; return 32; }
int qp_cand_waves(int K) { return K <= 128 ? QP_CAND_NW_SMALL : QP_WAVES; }

bool qp_cand_ok(int64_t m, int64_t n, int K) {
    // the code kernel holds a wave region's packed codes (rows x n / 4 bytes) in LDS
    return K > 0 && K <= QP_KMAX && m % 16 == 0 && n % QP_BN == 0 && m * n < (1ll << 31) &&
           (int64_t)qp_cand_rows(K) * n / 4 <= 144 * 1024;
}

int64_t qp_launch_cand(QUK& q, const uint16_t* Lh, const uint16_t* Ll, const uint16_t* Rth, const uint16_t* Rtl,
                       int K, int64_t batch, float eps, float* scale_out, double* err_out, hipStream_t s) {
    const int64_t m = q.m, n = q.n;
    const bool small = K <= 128;
    const int rb = 2, nw = qp_cand_waves(K);
    const int64_t panels = ceil_div(m, (int64_t)nw * 16 * rb);
    if (panels * batch * nw >= (1ll << 31)) return -1;
    const unsigned g = (unsigned)(panels * batch);
    const unsigned gf = (unsigned)std::min<int64_t>(panels * batch, kCUs);   // fallback pass 1
    const int rpw = 16 * rb;
    const size_t lds = (size_t)rpw * n / 4;
    q.only_fallback = 0;
#define CQ_QPC(PS, RBV, KSV, NWV)                                                          \
    q_update_p_kernel<PS, 2, CQ_F16, RBV, KSV, NWV, true><<<PS == 2 ? g : gf, NWV * 64,    \
        qp_lds_bytes(NWV, RBV, KSV, true), s>>>(                                           \
        q, Lh, Ll, Rth, Rtl, K, (int)panels)
    if (small) CQ_QPC(2, 2, 4, QP_CAND_NW_SMALL); else CQ_QPC(2, 2, 8, QP_WAVES);
    qp_codes_kernel<<<(unsigned)(panels * batch * nw), 256, lds, s>>>(q, (int)panels, nw, rpw);
    q.only_fallback = 1;
    if (small) CQ_QPC(1, 2, 4, QP_CAND_NW_SMALL); else CQ_QPC(1, 2, 8, QP_WAVES);
#undef CQ_QPC
    q.only_fallback = 0;
    qp_finalize_cand_kernel<<<(unsigned)batch, 64, 0, s>>>(q, (int)panels, nw, scale_out, err_out);
    (void)eps;
    return panels;
}

int64_t qp_launch(QUK& q, int dtype, int bits, const uint16_t* Lh, const uint16_t* Ll, const uint16_t* Rth,
                  const uint16_t* Rtl, int K, int64_t batch, hipStream_t s) {
    const int64_t m = q.m;
    const bool f16 = dtype == CQ_F16;
    const bool small = K <= 128;
    const int rb0 = (small && f16) ? 3 : 2, rb1 = rb0;
    const int64_t p0 = ceil_div(m, (int64_t)QP_WAVES * 16 * rb0), p1 = ceil_div(m, (int64_t)QP_WAVES * 16 * rb1);
    if (p0 * batch >= (1ll << 31) || p1 * batch >= (1ll << 31)) return -1;
    const uint16_t *lh = Lh, *ll = Ll, *rh = Rth, *rl = Rtl;
    const int Ki = K;
    const unsigned g0 = (unsigned)(p0 * batch), g1 = (unsigned)(p1 * batch);
#define CQ_QP(PS, B, DTV, RBV, KSV, G, P) \
    q_update_p_kernel<PS, B, DTV, RBV, KSV, QP_WAVES, DTV == CQ_F16><<<G, QP_WAVES * 64, \
        qp_lds_bytes(QP_WAVES, RBV, KSV, DTV == CQ_F16), s>>>(q, lh, ll, rh, rl, Ki, (int)P)
#define CQ_QP0(B, DTV, RBV, KSV) CQ_QP(0, B, DTV, RBV, KSV, g0, p0)
#define CQ_QP_B(B) do { \
        if (f16 && small) { CQ_QP0(B, CQ_F16, 3, 4); CQ_QP(1, B, CQ_F16, 3, 4, g1, p1); } \
        else if (f16) { CQ_QP0(B, CQ_F16, 2, 8); CQ_QP(1, B, CQ_F16, 2, 8, g1, p1); } \
        else if (small) { CQ_QP0(B, CQ_F32, 2, 4); CQ_QP(1, B, CQ_F32, 2, 4, g1, p1); } \
        else { CQ_QP0(B, CQ_F32, 2, 8); CQ_QP(1, B, CQ_F32, 2, 8, g1, p1); } } while (0)
    switch (bits) {
        case 2: CQ_QP_B(2); break;
        case 4: CQ_QP_B(4); break;
        case 8: CQ_QP_B(8); break;
        default: CQ_QP_B(16); break;
    }
#undef CQ_QP_B
#undef CQ_QP0
#undef CQ_QP
    return p1;
}

}  // namespace cq
