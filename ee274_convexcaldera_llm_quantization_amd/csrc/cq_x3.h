// Shared definitions of the split-fp16 kernels (cq_x3.hip) and the row-panel fused Q update
// (cq_qupdate.hip): operand-tile argument blocks and vector types.
#pragma once

#include "cq_common.h"

namespace cq {

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using f32x16v = __attribute__((ext_vector_type(16))) float;

struct X3K {
    int64_t M, N, K, batch;
    const _Float16 *Ah, *Al; int64_t lda, sa;
    const _Float16 *Bh, *Bl; int64_t ldb, sb;
    const float* inv_scale;       // per batch
    float* C; int64_t ldc, sc;
    const float* P; int64_t ldp, sp;    // prev (may alias C)
    const float* D; int64_t ldd, sd;    // cur
    const float *alpha_v, *beta_v, *gamma_v;
    _Float16 *Oh, *Ol; int64_t ldo, so;
    float out_scale;
    int* overflow;
    int tri;  // skip tiles entirely below the diagonal (C symmetric; M == N)
    int b_blocked;  // B halves in K-blocked layout [K/32][ldb rows][32] (cq_sym_split_f16 blocked)
    const int* active;  // per batch (NULL = all): inactive entries skip the product, C = D
    int a_blocked;  // A halves K-blocked [K/32][lda rows][32] (lda = rows)
    int o_blocked;  // split output halves K-blocked over C's columns: (col/32)*M*32 + row*32 + col%32
    int64_t tiles_n, tiles_m;
    int64_t tiles_live;        // sym_out: launched tiles per matrix (on or above the diagonal)
    int single;                // one product hi x hi (lo halves not read): ~2^-11 relative
    int sym_out;               // tri Gram: write the blocked split of the symmetric C (mirrored upper)
    const double* out_bound;   // [batch] bound on max|C|: split scale 2^(14 - e)
    float* scale_out;          // [batch] that scale
    float* inv_out;            // [batch] 1 / (scale * out_scale)
    int ksplit;                // > 1: K cut into ksplit chunks, fp32 partials in part (split-K)
    float* part;               // [ksplit][batch][M][N]
    const float* colw = nullptr;  // [N] (or NULL): the product term scaled per C column
    int64_t scolw = 0;            // colw batch stride (0: one vector for every matrix)
    uint32_t* absmax_out = nullptr;  // [batch] (or NULL, plain products): atomic max of |C| bits
    float* Ct = nullptr; int64_t sct = 0;  // C^T too (N x M, row stride M), batch stride sct
};

using f16x8g = __attribute__((ext_vector_type(8))) _Float16;
using f32x4v = __attribute__((ext_vector_type(4))) float;

// Fused Q update arguments (maybe_update_Q alg.py:253-283 + quantize_matrix alg.py:245-250)
struct QUK {
    X3K x;                       // A = L halves, B = R^T halves, inv_scale, K = r, tiling
    const void* W; int wf16;     // W (m x n), fp16 or fp32
    int64_t m, n;
    uint32_t* absmax;            // [batch] bits, zeroed before pass 0
    float eps;
    void* codes;                 // int8 / int16 (m x n), or NULL
    uint8_t* packed;             // packed bytes (m n bits / 8), or NULL
    float* scale;                // [batch] out (pass 1)
    const float* ew;             // error column weights [n] or NULL (= 1)
    int64_t sew = 0;             // ew batch stride (0: one vector for every matrix)
    double* part;                // [batch * tiles] error partials
    // single-recompute 2-bit path (qp_launch cand = true): pass 2 = pass 0 + the error of
    // all-zero codes + a list of the candidates |res| >= tau (tau = QP_TAU x the previous
    // scale); qp_codes_kernel writes the codes from the lists; pass 1 runs only for matrices
    // whose lists cannot be complete (qp_fallback)
    const float* hint;           // [batch] previous Q scale (candidate threshold), or NULL
    uint32_t* ovf;               // [batch] a wave's list overflowed (zeroed before pass 2)
    // two lists per wave region: a lane group (8 elements) with exactly ONE |res| >= tau goes
    // to list A as (element index, residual) -- 8 B; one with two or more to list B as (first
    // element index, 8 residuals) -- 36 B.  ~95 % of the candidate groups are single (~12 % of
    // all groups hold a candidate at 4096^2), so the lists take ~1/4 of whole-group records
    uint32_t* cnt;               // [batch * panels * waves] list-B groups per wave region
    uint32_t* gid;               // [batch * panels * waves * cap] first element index of a group
    float4* gval;                // [.. * cap * 2] the group's 8 residuals (two or more |res| >= tau)
    int64_t cap;                 // list-B groups per wave region
    uint32_t* cntA;              // [batch * panels * waves] list-A entries per wave region
    uint2* la;                   // [.. * capA] (element index, residual bits) of single candidates
    int64_t capA;                // list-A entries per wave region
    double* part0;               // [batch * panels] pass-2 error partials (all codes zero)
    double* partF;               // [batch * panels * waves] code-kernel error corrections
    int only_fallback;           // pass 1: skip matrices that took the list path
    int* fb_out;                 // [batch] 1 = took the two-pass fallback, or NULL
};

constexpr float QP_TAU = 0.45f;           // candidate threshold / previous scale (2 tau <= s needed)
// list capacities, in thousandths of a wave region's 8-element groups.  Measured on the bench
// batches (tools/list_density.py, profiles/r05n_list_density_*.log): the first hinted update
// has the densest lists -- single-candidate groups 7.8 % on average at 4096^2 but up to 13.4 %
// in one 32-row region (the L R part of the residual is not uniform over rows), groups with two
// or more 0.32 % on average, up to 1.07 %; later updates ~5.3 % / 0.14 %; 4096 x 11008 and
// 11008 x 4096 lower.  A region past a capacity overflows and its matrix takes the second
// recompute (correct, slower).  Matrices of at least 2^22 elements get A 15.5 % (1.16x the
// densest region) + B 1.5 % (1.4x): 1.78 B of list per group, ~0.22 B per element, 0.99 GB of workspace at
// the bench's B = 256; smaller ones A 50 % + B 25 % (their candidates are denser, ~31 % of the
// groups at 320 x 544, and their lists small anyway)
constexpr int QP_CAPA_PERMILLE_BIG = 155, QP_CAPB_PERMILLE_BIG = 15, QP_CAPA_PERMILLE_SMALL = 500,
              QP_CAPB_PERMILLE_SMALL = 250;
constexpr int64_t QP_BIG_NUMEL = 1ll << 22;

constexpr int QP_BN = 32;                 // row-panel Q update: columns per chunk
constexpr int QP_KMAX = 256;              // row-panel Q update: largest r

// Row-panel fused Q update (cq_qupdate.hip): both passes of q_update_p_kernel for K = r <= 256,
// m % 16 == 0, n % 32 == 0 and 16-byte aligned operands; q.absmax zeroed, q.part sized for
// the pass-1 panels.  Returns the number of pass-1 panels per matrix (the error partials).
int64_t qp_launch(QUK& q, int dtype, int bits, const uint16_t* Lh, const uint16_t* Ll, const uint16_t* Rth,
                  const uint16_t* Rtl, int K, int64_t batch, hipStream_t s);
// The single-recompute 2-bit path's geometry (rows per wave) and whether it applies: fp16 W,
// K <= 256, a wave region's packed codes fit the code kernel's LDS.
int qp_cand_rows(int K);
int qp_cand_waves(int K);
bool qp_cand_ok(int64_t m, int64_t n, int K);
// Launches pass 2, the code kernel, the fallback pass 1 and the finalize (scale, error,
// fallback flags); q.ovf / q.absmax zeroed, q.list / q.cnt / q.part0 / q.partF sized by
// qp_cand_ws.  Returns the panels per matrix, or -1 when the grid is too large.
int64_t qp_launch_cand(QUK& q, const uint16_t* Lh, const uint16_t* Ll, const uint16_t* Rth, const uint16_t* Rtl,
                       int K, int64_t batch, float eps, float* scale_out, double* err_out, hipStream_t s);

}  // namespace cq
