/*
 * caldera_hip.h — C-ABI of libcaldera_hip.so, the MI355X (gfx950) engine behind the
 * drop-in `caldera()` / `LowMemoryQuantizer` API.
 *
 * The reference (genglongling/EE274_ConvexCaldera_LLM_quantization) is pure Python on
 * PyTorch: it has no native boundary.  Each entry point below replaces the tensor ops of
 * one step of the reference hot path; the replaced reference lines are cited per entry
 * (RCR/ = rank-constrained-regression-main/).  The Python caller is
 * ee274_convexcaldera_llm_quantization_amd/_lib.py (ctypes).
 *
 * Conventions (every export):
 *   - returns int status: 0 = ok, < 0 = error (CQ_E*); cq_last_error() gives a
 *     thread-local message.  No C++ exception crosses the ABI.
 *   - never allocates device memory: the caller passes workspace (size queried with the
 *     matching *_workspace function).  Launches are stream-ordered on `stream`
 *     (a hipStream_t; NULL = default stream) and never synchronise the host.
 *   - all matrices are row-major; "batch" = number of independent matrices of one shape,
 *     laid out at a fixed element stride (stride 0 = broadcast one operand).
 *   - pointers are device pointers unless the name ends in _host.
 *   - column / error weight vectors (a diagonal Hessian's derived weights) carry a batch
 *     stride (ABI 5): 0 = one vector shared by the batch, else matrix b reads its own vector
 *     at w + b * stride -- a batch of layers with distinct diagonal Hessians (main.py:163-165
 *     gives every layer its own Hall[name]) runs in one call.
 */
#ifndef CALDERA_HIP_H
#define CALDERA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CQ_ABI_VERSION 5

#define CQ_OK 0
#define CQ_EINVAL (-1)   /* bad argument (shape, bits, null pointer) */
#define CQ_EHIP (-2)     /* HIP runtime error (launch failed)        */
#define CQ_EWORKSPACE (-3) /* workspace too small                    */

/* dtype tags */
#define CQ_F32 0
#define CQ_F16 1
#define CQ_BF16 2
#define CQ_F64 3

int cq_abi_version(void);
const char* cq_last_error(void);

/* ---------------------------------------------------------------------------------
 * Global RMS scaling.  Replaces RCR/src/caldera/decomposition/alg.py:38-42:
 *   gs = W.square().mean().sqrt().item();  W = W / gs      (evaluated in W's dtype)
 * W: batch x numel of dtype (CQ_F16 | CQ_F32).  gs_out[b] (float) receives the scale as
 * the reference rounds it (fp16 for fp16 W).  Ws_out gets W/gs in W's dtype
 * (half(float(w)/gs) for fp16).  If do_scale == 0, gs = 1 and Ws = W.
 */
size_t cq_rms_scale_workspace(int64_t batch, int64_t numel);
int cq_rms_scale(int dtype, const void* W, int64_t batch, int64_t numel, int do_scale,
                 float* gs_out, void* Ws_out, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Uniform absmax quantiser.  Replaces RCR/src/caldera/utils/quantization.py:244-269
 * (quantize_block, method "uniform"), :93-101 (_quantize_uniform) and :290-295/:103-105
 * (dequantize_block).  x: batch x numel fp32, blocks of block_size consecutive elements
 * (block_size == numel is the whole-matrix case forced by alg.py:247).
 *   scale[b*nblk + j] = max(max|x_blk|, eps)                 (fp32)
 *   code = rint((x / scale) * k),  k = 2^(bits-1) - 1           (int8 for bits<=8, else int16)
 *   deq  = (float(code) / k) * scale
 * Outputs are optional (pass NULL to skip): codes (int8/int16, reference layout),
 * packed (bits 2/4 only: offset-binary c+k, MSB-first, 4 resp. 2 codes per byte),
 * deq (fp32).  If err_w != NULL and err_out != NULL, also accumulates
 *   err_out[b] = sum_ij err_w[j % err_ncols] * (deq_ij - x_ij)^2   (fp64, deterministic)
 * i.e. the numerator of alg.py:286-302 after a Q update with diagonal H.
 */
size_t cq_quantize_workspace(int64_t batch, int64_t numel, int64_t block_size);
int cq_quantize_uniform(const float* x, int64_t batch, int64_t numel, int64_t block_size,
                        int bits, float eps, void* codes, uint8_t* packed, float* deq,
                        float* scale, const float* err_w, int64_t err_ncols, int64_t err_w_stride,
                        double* err_out, void* ws, size_t ws_bytes, void* stream);

/* Same quantiser when the whole-matrix absmax is already known (bits of |x|max as
 * uint32 in absmax_bits[b], e.g. produced by cq_gemm_f32 EPI_RESID).  Replaces
 * alg.py:262-283 (maybe_update_Q / update_Q_non_data_aware) after the fused residual. */
int cq_quantize_uniform_known_max(const float* x, int64_t batch, int64_t numel, int bits,
                                  float eps, const uint32_t* absmax_bits, void* codes,
                                  uint8_t* packed, float* deq, float* scale,
                                  const float* err_w, int64_t err_ncols, int64_t err_w_stride,
                                  double* err_out, void* ws, size_t ws_bytes, void* stream);

/* Dequantise (quantization.py:103-105, :292-295): out[e] = (float(c_e)/k) * scale[e / block_size].
 * codes: int8 (bits <= 8) / int16 (bits 16), or offset-binary packed if `packed` (bits 2/4).
 * total = elements over the whole batch (scales indexed globally). */
int cq_dequant_uniform(const void* codes, int packed, const float* scale, int64_t total,
                       int64_t block_size, int bits, float* out, void* stream);

/* Unpack offset-binary packed codes (layout above) to int8 reference codes. */
int cq_unpack_codes(const uint8_t* packed, int64_t batch, int64_t numel, int bits,
                    int8_t* codes, void* stream);

/* ---------------------------------------------------------------------------------
 * NF4 / NF2 codebook quantiser.  Replaces RCR/src/caldera/utils/quantization.py:39-91
 * (levels, thresholds (l_i + l_{i+1}) / 2, _quantize_nf, _dequantize_nf) with the dispatch
 * of :270-279 / :296-298.  x: batch x numel fp32 in blocks of block_size:
 *   scale = max(max|x_blk|, eps);  idx = #{t : x / scale > thr_t}  (uint8, reference layout)
 *   deq   = level[idx] * scale
 * idx / deq optional; err_out[b] = sum err_w[j % err_ncols] (deq - x)^2 (fp64) if non-NULL. */
size_t cq_quantize_nf_workspace(int64_t batch, int64_t numel, int64_t block_size);
int cq_quantize_nf(const float* x, int64_t batch, int64_t numel, int64_t block_size, int bits, float eps,
                   uint8_t* idx, float* deq, float* scale, const float* err_w, int64_t err_ncols,
                   int64_t err_w_stride, double* err_out, void* ws, size_t ws_bytes, void* stream);
/* out[e] = level[idx[e]] * scale[e / block_size]  (quantization.py:87-91) */
int cq_dequant_nf(const uint8_t* idx, const float* scale, int64_t total, int64_t block_size, int bits,
                  float* out, void* stream);

/* ---------------------------------------------------------------------------------
 * bbint4 / bbint2 (bitsandbytes-style affine codes with 6-sigma outliers).  Replaces
 * quantization.py:107-154 (_quantize_bbint4), :175-222 (_quantize_bbint2) and their dequant
 * :157-172 / :224-243.  Two calls with the same workspace (the outlier list is variable
 * length, so the caller reads n_outliers between them):
 *   cq_bbint_stats: per block mean (reference fp32 order), unbiased std (max eps), outlier
 *     mask |x - mean| > 6 std, min / max of the outlier-replaced block, scale = max((max -
 *     min) / (2^bits - 1), eps) -> bmin, bscale [batch * nblk]; n_outliers[b] per matrix.
 *   cq_bbint_emit: packed codes (uint8, MSB-first, 8/bits per byte, reference layout
 *     (nblk, block_size*bits/8)), deq (fp32, outliers restored), the outlier values and
 *     their int64 (row, col) indices in the (nblk, block_size) view (torch.nonzero order),
 *     all matrices concatenated (matrix b after matrix b-1), err_out as for the uniform
 *     quantiser.  Any output may be NULL (out_vals and out_idx together). */
size_t cq_bbint_workspace(int64_t batch, int64_t numel, int64_t block_size);
int cq_bbint_stats(const float* x, int64_t batch, int64_t numel, int64_t block_size, int bits, float eps,
                   float* bmin, float* bscale, int64_t* n_outliers, void* ws, size_t ws_bytes, void* stream);
int cq_bbint_emit(const float* x, int64_t batch, int64_t numel, int64_t block_size, int bits, const float* bmin,
                  const float* bscale, uint8_t* packed, float* deq, float* out_vals, int64_t* out_idx,
                  const float* err_w, int64_t err_ncols, int64_t err_w_stride, double* err_out, void* ws,
                  size_t ws_bytes, void* stream);
/* out = u * bscale[blk] + bmin[blk] from the packed codes, then out[row*bs + col] = value for
 * each of the n_outliers listed outliers. */
int cq_dequant_bbint(const uint8_t* packed, int bits, const float* bmin, const float* bscale, int64_t total,
                     int64_t block_size, const float* out_vals, const int64_t* out_idx, int64_t n_outliers,
                     float* out, void* stream);

/* ---------------------------------------------------------------------------------
 * Residual builder for the LR update.  Replaces alg.py:124 (residual = W - Q) and the
 * diagonal-H form of alg.py:211 (Y = residual @ H_sqrt @ eigvecs; for diagonal H this is
 * a column scaling by sqrt(h) up to a permutation that LR_init undoes):
 *   res_ij = float(Ws_ij) - (float(c_ij)/k)*scale_b    (Q from packed codes; packed==NULL: Q=0)
 *   Y_ij   = res_ij * ycol[j]                           (ycol == NULL: 1)
 * Ws: fp16 or fp32 (dtype).  Y and/or res_out may be NULL.
 * bits == 32: `packed` is a dense fp32 dequantised Q (the codebook methods nf4/nf2/bbint,
 * whose Q is not an affine function of one scale); `scale` is then unused.
 */
int cq_build_residual(int dtype, const void* Ws, const uint8_t* packed, const float* scale,
                      int bits, const float* ycol, int64_t ycol_stride, int64_t batch, int64_t m, int64_t n,
                      float* Y, float* res_out, void* stream);

/* ---------------------------------------------------------------------------------
 * Batched FP32 GEMM on gfx950 MFMA (v_mfma_f32_32x32x2_f32; exact f32 products).
 * Carries the fp32 products of the hot path: Ritz rotations X V, the fp32 solver filter
 * (fallback after an fp16 overflow, and k % 32 != 0 shapes), R = U^T Y / L = Y V where the
 * split-fp16 path does not apply, the LPLR normal-equation products of alg.py:162-182, the
 * fused residual (alg.py:262) and error (alg.py:182, :286-302) epilogues.  The Gram Y Y^T,
 * the filter's G X and the Rayleigh-Ritz products run on cq_gemm_x3 (split-fp16 MFMA).
 * op(A) is M x K, op(B) is K x N.
 *   epi = CQ_EPI_LINEAR:  C = alpha*op(A)op(B) + beta*C + gamma*D
 *   epi = CQ_EPI_RESID :  C = D - op(A)op(B) (D fp32, or fp16 if d_f16);
 *                          atomicMax(absmax_bits[b], |C|)     (alg.py:262 fused with :262 of quantization.py)
 *   epi = CQ_EPI_WERR  :  no C; err_out[b] += sum_ij w[j]*(D_ij - op(A)op(B)_ij)^2 (fp64,
 *                          deterministic two-stage) — alg.py:182 and :286-302 for diagonal H
 * Strides are in elements between consecutive batch entries (0 = shared).
 */
#define CQ_EPI_LINEAR 0
#define CQ_EPI_RESID 1
#define CQ_EPI_WERR 2

typedef struct cq_gemm_args {
    int64_t M, N, K, batch;
    int trans_a, trans_b;
    const float* A; int64_t lda, stride_a;
    const float* B; int64_t ldb, stride_b;
    float* C; int64_t ldc, stride_c;
    const void* D; int64_t ldd, stride_d; int d_f16;
    float alpha, beta, gamma;
    const float* alpha_v; const float* beta_v; const float* gamma_v; /* optional per-batch
                                       coefficients (device, [batch]); override the scalars */
    int epi;
    uint32_t* absmax_bits;           /* EPI_RESID: [batch], pre-zeroed by caller */
    const float* w; int64_t stride_w; /* EPI_WERR: column weights (may be NULL) */
    double* err_out;                 /* EPI_WERR: [batch] */
    int syrk;                        /* 1: C = alpha op(A) op(B) is symmetric (A = B^T up to
                                        op): only upper 128x128 tiles are computed, then
                                        mirrored (LINEAR, beta = gamma = 0)               */
    int b_triu;                      /* 1: B (not transposed) is upper triangular, B[k][n] = 0
                                        for k > n (a CholQR whitening factor): the K slices
                                        that meet only its zeros are skipped (same bits)   */
} cq_gemm_args;

size_t cq_gemm_workspace(const cq_gemm_args* a);
int cq_gemm_f32(const cq_gemm_args* a, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Small dense kernels of the rank-r solver (replace torch.linalg.svd at alg.py:217,
 * torch.linalg.lstsq at alg.py:163,175 and torch.linalg.eigh at alg.py:23).
 */
/* C[b] (M x N, fp64) = op(A[b])^T-style Gram:  C = A^T B with A K x M, B K x N
 * (trans_a/trans_b: A stored M x K / B stored N x K).  fp32 inputs, fp64 accumulation. */
size_t cq_gram_f64_workspace(int64_t M, int64_t N, int64_t K, int64_t batch);
int cq_gram_f64(int64_t M, int64_t N, int64_t K, int64_t batch, const float* A, int trans_a,
                int64_t lda, int64_t stride_a, const float* B, int trans_b, int64_t ldb,
                int64_t stride_b, double* C, void* ws, size_t ws_bytes, void* stream);

/* SPD whitening by symmetric Gaussian elimination (Cholesky-equivalent):
 * for each b, finds upper-triangular Wt (p x p) with Wt^T S Wt = I, written as fp32
 * (Wt32, may be NULL) and as fp64 over S itself (S is overwritten by Wt).  Wt64 (p x p fp64
 * per matrix) is required scratch; its content is undefined on return (ABI 4: through ABI 3
 * the fp64 Wt was also copied there).  A pivot <= rcond2 * max_j S_jj (or not
 * positive) marks a column dependent on the previous ones: it is dropped (its Wt column is
 * 0), so Wt Wt^T is a generalised inverse and (A^T A) x = A^T y solved through it gives the
 * basic least-squares solution — torch.linalg.lstsq's gelsy semantics (rcond = eps * max(m,
 * n) on A, i.e. rcond2 = rcond^2 on the Gram), the rank decision taken in index order.
 * info[b] = number of dropped pivots (0: full rank).  cq_spd_whiten: rcond2 = 1e-30. */
int cq_spd_whiten_rcond(double* S, int64_t p, int64_t batch, double rcond2, float* Wt32, double* Wt64,
                        int* info, void* stream);
int cq_spd_whiten(double* S, int64_t p, int64_t batch, float* Wt32, double* Wt64,
                  int* info, void* stream);

/* Symmetric eigendecomposition by parallel cyclic Jacobi (fp64), eigenpairs sorted by
 * DESCENDING eigenvalue.  A (p x p) is overwritten; evals[b*p..]; V32/V64 (p x p, columns
 * = eigenvectors), either may be NULL.  sweeps_out[b] = sweeps used (may be NULL). */
size_t cq_jacobi_workspace(int64_t p, int64_t batch);
int cq_jacobi_eigh(double* A, int64_t p, int64_t batch, int max_sweeps, double tol,
                   double* evals, float* V32, double* V64, int* sweeps_out, void* ws,
                   size_t ws_bytes, void* stream);
/* The same eigensolve as a block Jacobi over many workgroups per matrix, in caller-driven
 * stages, each stream-ordered: phase bit 1 = begin (V = I), 2 = nsweeps sweeps (matrices that
 * converged skip the rest; pending_out, a device int, = matrices still unconverged), 4 = end
 * (evals, V32/V64, sweeps_out).  The state stays in ws (cq_jacobi_staged_workspace) between
 * calls, so a caller reading pending_out launches further sweeps only while some are needed.
 * Used for p > 192 (the Rayleigh-Ritz eigensolve of alg.py:217's replacement at rank > 136,
 * e.g. main.py:176's rank 200 and config 5's rank 256), and at any p for small batches (one
 * caldera() call, main.py:189-196), where the one-CU kernel would leave the other CUs idle.
 * want_vectors must be the same in every stage. */
size_t cq_jacobi_staged_workspace(int64_t p, int64_t batch);
int cq_jacobi_eigh_staged(double* A, int64_t p, int64_t batch, int phase, int nsweeps, double tol, int want_vectors,
                          double* evals, float* V32, double* V64, int* sweeps_out, int* pending_out, void* ws,
                          size_t ws_bytes, void* stream);

/* The two ends of the spectrum of each symmetric T (p x p fp64, (T + T^T) / 2 used, not
 * overwritten): ends[2 b] = largest, ends[2 b + 1] = smallest eigenvalue, from `steps`
 * (1 <= steps < 64) Lanczos iterations and bisection on the Lanczos tridiagonal (approach the
 * true ends from inside; exact when the iteration breaks down on an invariant subspace).
 * p <= 512 (p > 192: T read in place, its upper and lower triangle taken as equal).  The
 * rank-r solver's cheap outer iterations take their Chebyshev filter bounds
 * from it instead of a values-only eigensolve (the SVD replacement of alg.py:217). */
int cq_extreme_eigs(const double* T, int64_t p, int64_t batch, int steps, double* ends, void* stream);

/* Ritz residuals: out[b] = max_{i<r} ||Z[:,i] - theta_i X[:,i]||_2 / |theta_0|
 * (X, Z: k x p row-major with ld p).  theta fp64 [b*p..]. */
size_t cq_ritz_workspace(int64_t k, int64_t r, int64_t batch);
int cq_ritz_residual(const float* X, const float* Z, const double* theta, int64_t k,
                     int64_t p, int64_t r, int64_t batch, float* out, void* ws,
                     size_t ws_bytes, void* stream);
/* The rank-r solver's stopping test (replaces the full SVD's exactness, alg.py:217): an
 * estimate of ||(P_r - P_r*) Y||_F / ||Y||_F, the relative error of the rank-r projection of
 * Y from the Ritz pairs:  out[b] = sqrt(sum_{i<r} ||e_i||^2 theta_i / gap_i^2 / ysq[b]),
 * e_i = Z[:,i] - theta_i X[:,i], gap_i = max(theta_i - theta_{p-1}, 1e-3 theta_0), ysq[b] =
 * ||Y||_F^2 = trace(G).  Spectra with a wide spread (activation-weighted Y) need much smaller
 * residuals than flat ones for the same product accuracy; a residual relative to theta_0
 * cannot tell them apart.  r < p.  Workspace: cq_ritz_workspace. */
int cq_ritz_product_error(const float* X, const float* Z, const double* theta, int64_t k, int64_t p, int64_t r,
                          int64_t batch, const double* ysq, float* out, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------
 * Split-fp16 ("f16x3") products with a symmetric Gram, fp32-grade accuracy on the fp16
 * MFMA (the subspace filter of the SVD replacing alg.py:217).  A value x*s (s a power of
 * two) is held as two fp16 halves hi = f16(x*s), lo = f16(x*s - hi); fp16 buffers are
 * passed as uint16_t.
 */
/* Gh/Gl[b] = split of G[b] (n x n PSD, row-major) scaled by scale_out[b] = 2^(14 -
 * ceil(log2 max_i G_ii)); inv_scale_out[b] = 1 / (scale_out[b] * x_scale).  upper_only:
 * only G's upper triangle (j >= i) is read and mirrored into the full split.  blocked:
 * halves written K-blocked, element (i, j) at (j / 32) * n * 32 + i * 32 + j % 32, so a
 * 32-deep K step of any row range is one contiguous run (cq_x3_args.b_blocked). */
int cq_sym_split_f16(const float* G, int64_t n, int64_t batch, int upper_only, int blocked,
                     float x_scale, uint16_t* Gh, uint16_t* Gl, float* scale_out,
                     float* inv_scale_out, void* stream);
/* scale_out[b] = 2^(log2_target - e) with max|X[b]| in [2^(e-1), 2^e) (1 for all-zero X[b]). */
int cq_pow2_scale(const float* X, int64_t n_per, int64_t batch, int log2_target, float* scale_out,
                  void* stream);
/* In place: scale_inout[b] holds the bits of a bound on max|X[b]| (cq_gemm_x3's absmax_out, or a
 * positive fp32 such as a quantiser's scale) on entry and the power-of-two split scale
 * cq_pow2_scale would give for that maximum on exit (no pass over X). */
int cq_pow2_from_absmax(float* scale_inout, int64_t batch, int log2_target, void* stream);
/* hi/lo[b] = split of X[b] (n_per values) scaled by scale_v[b] (or scale if scale_v NULL).
 * blocked_ncols > 0: X[b] is (n_per / ncols) x ncols and the halves are written K-blocked
 * (element (r, c) at (c / 32) * rows * 32 + r * 32 + c % 32; ncols % 32 == 0). */
int cq_split_f16(const float* X, int64_t n_per, int64_t batch, const float* scale_v, float scale,
                 uint16_t* hi, uint16_t* lo, int64_t blocked_ncols, void* stream);
/* Y[b] = X[b]^T (X rows x cols row-major -> Y cols x rows), and/or its split (scale_v[b], or
 * scale if scale_v is NULL); blocked: halves K-blocked over Y's columns (rows % 32 == 0). */
int cq_transpose_split(const float* X, int64_t rows, int64_t cols, int64_t batch, float* Y,
                       uint16_t* hi, uint16_t* lo, float scale, const float* scale_v, int blocked,
                       void* stream);
/* CholQR's product with its triangular factor and the next product's operand in one pass:
 * C[b] = X[b] Wt[b] (X M x p, Wt p x p upper triangular, both row-major and contiguous;
 * p % 32 == 0, p <= 192, M % 32 == 0) and hi/lo[b] = the K-blocked split of C[b]^T at
 * `scale` -- the same bits as cq_gemm_f32 (b_triu) followed by cq_transpose_split (blocked),
 * without the second pass over C (the SVD replacement's CholQR -> Rayleigh-Ritz, alg.py:217). */
int cq_gemm_triu_split(const float* X, const float* Wt, int64_t M, int64_t p, int64_t batch, float* C,
                       uint16_t* hi, uint16_t* lo, float scale, void* stream);

typedef struct cq_x3_args {
    int64_t M, N, K, batch;
    const uint16_t *Ah, *Al;       /* M x K halves (row-major, ld lda, batch stride) */
    int64_t lda, stride_a;
    const uint16_t *Bh, *Bl;       /* N x K halves: op(B)[k][n] = B[n][k] */
    int64_t ldb, stride_b;
    const float* inv_scale;        /* [batch]: 1 / (scale_A * scale_B) */
    float* C;                      /* M x N fp32 */
    int64_t ldc, stride_c;
    const float* P;                /* beta term operand (may alias C) */
    int64_t ldp, stride_p;
    const float* D;                /* gamma term operand */
    int64_t ldd, stride_d;
    const float *alpha_v, *beta_v, *gamma_v;  /* [batch] each; NULL = 1, 0, 0 */
    uint16_t *out_h, *out_l;       /* optional split of C (scale out_scale) */
    int64_t ldo, stride_o;
    float out_scale;
    int* overflow;                 /* [batch]: set to 1 when |C * out_scale| >= 65504 */
    int tri;                       /* C symmetric (M == N, plain product): tiles entirely below
                                      the diagonal are skipped; the upper triangle is exact */
    int b_blocked;                 /* B halves K-blocked (see cq_sym_split_f16); ldb = rows */
    const int* active;             /* [batch] or NULL: entries with active[b] == 0 skip the
                                      product and write C = D (and its split) unchanged */
    int a_blocked;                 /* A halves K-blocked like b_blocked; lda = rows */
    int o_blocked;                 /* out_h/out_l written K-blocked over C's columns (an A
                                      operand of the next product); N % 32 == 0 */
    int sym_out;                   /* with tri: write the split of the symmetric C directly,
                                      K-blocked (o_blocked layout), from its upper triangle
                                      (mirrored), with the per-matrix power-of-two scale
                                      s[b] = 2^(14 - e) for out_bound[b] in [2^(e-1), 2^e);
                                      C (fp32) may be NULL.  Replaces cq_sym_split_f16. */
    const double* out_bound;       /* [batch] bound on max|C[b]| (e.g. ||Y||_F^2 for Y Y^T) */
    float* scale_out;              /* [batch] s[b] */
    float* inv_out;                /* [batch] 1 / (s[b] * out_scale) */
    int single;                    /* one fp16 product hi x hi (Al, Bl not read): ~2^-11
                                      relative, for filter steps whose error later steps damp */
    int ksplit;                    /* > 1 (not with tri/sym_out): the K loop is cut into ksplit
                                      chunks run by separate workgroups (a small batch's few tiles
                                      then fill the chip: one caldera() call), their fp32 partials
                                      summed in chunk order by an epilogue kernel */
    float* split_ws;               /* ksplit x batch x M x N fp32 partials (ksplit > 1) */
    int b_exact;                   /* B is exactly fp16 (Bl = 0, e.g. W's halves under a split
                                      scale >= 1): two products al x bh + ah x bh, Bl not read
                                      (may be NULL); the same bits as the three products */
    const float* colw;             /* [N] or NULL (not with tri / sym_out): the product term of
                                      C column j is scaled by colw[j] before beta P + gamma D
                                      (R = (U^T W) diag(ycol) - s (U^T c) diag(ycol) from W's
                                      exact halves)                                        */
    uint32_t* absmax_out;          /* [batch] or NULL (plain products only): atomic max of the
                                      bits of |C[b]| into absmax_out[b] (zeroed by the caller):
                                      the next product's split scale without a pass over C */
    float* Ct;                     /* N x M fp32 (row stride M, batch stride stride_ct) or NULL
                                      (not with tri / sym_out): C^T as well (ABI 4) -- the
                                      solver's filter and Rayleigh-Ritz products hand their
                                      result back in the k x p layout without a transpose pass */
    int64_t stride_ct;
    int64_t stride_colw;           /* colw batch stride (ABI 5; 0: one vector for every matrix,
                                      N: per-matrix weights -- distinct diagonal Hessians) */
} cq_x3_args;
/* C = alpha * (A B^T) + beta * P + gamma * D, per batch coefficient vectors; K % 32 == 0. */
int cq_gemm_x3(const cq_x3_args* a, void* stream);

/* out[b] = max |X[b]| (n_per values, fp16 or fp32), NaN sorting above inf. */
int cq_absmax(int dtype, const void* X, int64_t n_per, int64_t batch, float* out, void* stream);

/* Fused residual for the LR step.  Replaces alg.py:124 (residual = W - Q) and :211
 * (Y = residual @ H_sqrt for diagonal H), plus the operand preparation of the solver: one
 * pass over W and the packed codes writes any of res (fp32), Y = res * ycol (fp32), the
 * K-blocked split halves of Y over its columns (hi/lo, layout of cq_split_f16 blocked) and
 * over its rows (thi/tlo: Y^T as an n x m operand, blocked), and sq_out[b] = ||Y||_F^2
 * (fp64).  The halves' scale (scale_out[b]) is the power of two for the bound
 * (wmax[b] + Q_scale[b]) * ycol_max >= max|Y|, and at least 1 for fp16 W without codes or
 * ycol: Y's halves are then exact (lo = 0) and lo / tlo may be NULL (gemm_x3 b_exact reads
 * only the hi halves).  ycol_hi (optional, with hi/lo): the column-blocked halves are of
 * res * ycol_hi instead (the weighted Gram's W diag(ycol^2) operand), at the power of two for
 * (wmax[b] + Q_scale[b]) * ycol_hi_max, written to scale_hi_out[b]; everything else keeps ycol.
 * Per-matrix weights (ABI 5): ycol / ycol_hi at + b * ycol_stride, and ycol_max_v[b] /
 * ycol_hi_max_v[b] (when non-NULL) replace the scalar bounds.
 * m % 32 == 0, n % 64 == 0.
 * bits == 32: `packed` is a dense fp32 Q and qscale[b] a bound on max|Q[b]|. */
size_t cq_residual_split_workspace(int64_t m, int64_t n, int64_t batch);
int cq_residual_split(int dtype, const void* Ws, const uint8_t* packed, const float* qscale, int bits,
                      const float* ycol, float ycol_max, const float* wmax, int64_t batch, int64_t m,
                      int64_t n, float* res_out, float* Y_out, uint16_t* hi, uint16_t* lo,
                      uint16_t* thi, uint16_t* tlo, float* scale_out, double* sq_out,
                      const float* ycol_hi, float ycol_hi_max, float* scale_hi_out, int64_t ycol_stride,
                      const float* ycol_max_v, const float* ycol_hi_max_v, void* ws, size_t ws_bytes,
                      void* stream);

/* Gram of the LR step's Y from sparse 2-bit codes (cq_sgram.hip).  Replaces, for m <= n,
 * Q_bits = 2 and a diagonal (or no) H, the Gram Y Y^T of Y = (W - Q) diag(ycol) that the SVD
 * at alg.py:211-217 factors: with Q = s c (c in {-1, 0, 1}, ~1 % nonzero), w = ycol^2 and
 * E = W - (s/2) c, G = W diag(w) W^T - s (P + P^T) with P = E diag(w) c^T.
 *   cq_sgram_count:   row_nnz (batch x k, int32) nonzero codes per row of the packed codes
 *                     (batch x k x L, offset-binary MSB-first), perm (batch x k, int32: rows
 *                     sorted by count, descending, ties in row order), slice_off (batch x (ceil(k/64)
 *                     + 1), int64: sliced-ELL offsets per 64-row slice, in 64-entry rows), total[b] entries;
 *                     with W (fp16, batch x k x L; may be NULL) also corr_out[b] = sum over the
 *                     nonzero codes of wcol[l] (s^2 - 2 s c W[j, l]) (fp64, s = qscale[b], wcol NULL
 *                     = 1; corr_ws: batch x k doubles): ||(W - s c) diag(ycol)||^2 - ||W diag(ycol)||^2
 *                     for wcol = ycol^2, the ||Y||_F^2 of alg.py:211 without a pass over Y;
 *                     l-split (Lh < L, from cq_sgram_split): also row_nnz1 (batch x k, the
 *                     entries with l < Lh) and slice_w1 (batch x ceil(k/64), int32): a slice holds
 *                     its rows' first-part entries in its first slice_w1 64-entry rows, the rest
 *                     after them (each part padded to its widest row); Lh >= L: one part
 *                     (row_nnz1 / slice_w1 may be NULL);
 *   cq_sgram_fill:    the ELL entries (uint32: l << 2 | code + 1) of matrix b at ell + b stride_ell
 *                     (row_nnz, perm, slice_off, slice_w1, Lh as given to cq_sgram_count);
 *   cq_sgram_rows:    rows of E a workgroup stages for contraction length L (0: too long);
 *   cq_sgram_split:   the l-split point Lh for k x L (L: no split): where two rows of E fit the
 *                     LDS but four do not, four are staged half a contraction at a time;
 *   cq_sgram_spmm:    P (batch x k x k fp32) from W (fp16, batch x k x L), the codes, qscale[b] = s
 *                     and wcol (L, may be NULL = 1), over the ELL of cq_sgram_fill (same Lh);
 *   cq_sgram_combine: G = A - s (P + P^T) with A (batch x k x k fp32, upper triangle read) =
 *                     W diag(w) W^T, written as the K-blocked split halves Gh/Gl with
 *                     cq_gemm_x3 sym_out's scale rule (scale_out[b] from bound[b] >= max|G|,
 *                     inv_out[b] = 1 / (scale_out[b] out_scale)); G32 (full fp32 G) optional.
 * k % 64 == 0, L % 64 == 0. */
int cq_sgram_count(const uint8_t* packed, int bits, int64_t batch, int64_t k, int64_t L, int32_t* row_nnz,
                   int32_t* perm, int64_t* slice_off, int64_t* total, int64_t Lh, int32_t* row_nnz1,
                   int32_t* slice_w1, const void* W, const float* qscale, const float* wcol, int64_t wcol_stride,
                   double* corr_ws, double* corr_out, void* stream);
int cq_sgram_fill(const uint8_t* packed, int bits, int64_t batch, int64_t k, int64_t L, const int32_t* row_nnz,
                  const int32_t* perm, const int64_t* slice_off, const int32_t* slice_w1, int64_t Lh,
                  int64_t stride_ell, uint32_t* ell, void* stream);
int cq_sgram_rows(int64_t L);
int64_t cq_sgram_split(int64_t k, int64_t L);
int cq_sgram_spmm(int dtype, const void* W, const uint8_t* packed, const float* qscale, const float* wcol,
                  int64_t wcol_stride, int64_t batch, int64_t k, int64_t L, const uint32_t* ell, const int32_t* perm,
                  const int64_t* slice_off, const int32_t* slice_w1, int64_t Lh, int64_t stride_ell, float* P,
                  void* stream);
int cq_sgram_combine(const float* A, const float* P, const float* qscale, int64_t batch, int64_t k,
                     const double* bound, float out_scale, uint16_t* Gh, uint16_t* Gl, float* scale_out,
                     float* inv_out, float* G32, void* stream);

/* Sparse-code helpers of the LR step (cq_sgram.hip), for 2-bit packed codes c (batch x rows x
 * cols, the layout above):
 *   cq_codes_transpose: c^T (batch x cols x rows, same packing); rows, cols multiples of 16.
 *     Lets the sparse-code Gram run on m > n shapes (G = Y^T Y from W^T and c^T) and the R step
 *     read the codes by column.
 *   cq_codes_matmul: out[b, i, :] = roww[i] sum_{j: c[b,i,j] != 0} c[b,i,j] colw[j] X[b, j, 0:r] (X
 *     row stride ldx, matrix stride stride_x; colw, roww NULL = 1; r <= 256), row-major (ld ldo) or, with
 *     trans, out[b] is r x rows (ld ldo).  Replaces the code part of R = U^T (W - Q) (alg.py:
 *     219-225, via c^T: U^T c) and of L = Y V for m > n; fixed summation order (deterministic).
 *   cq_codes_ysq_corr: out[b] = sum over the nonzero codes of colw[j] (s^2 - 2 s c W[b,i,j])
 *     (fp64, s = qscale[b]): ||(W - s c) diag(ycol)||^2 - ||W diag(ycol)||^2 with colw = ycol^2,
 *     the ||Y||_F^2 of alg.py:211 without a pass over Y.
 *   cq_transpose_f16: Y[b] = X[b]^T for fp16 X (batch x rows x cols). */
int cq_codes_transpose(const uint8_t* packed, int bits, int64_t batch, int64_t rows, int64_t cols, uint8_t* out,
                       void* stream);
int cq_codes_matmul(const uint8_t* packed, int bits, int64_t batch, int64_t rows, int64_t cols, const float* X,
                    int64_t ldx, int64_t stride_x, const float* colw, int64_t colw_stride, const float* roww,
                    int64_t roww_stride, int64_t r, float* out, int64_t ldo, int64_t stride_out, int trans,
                    void* stream);
int cq_codes_ysq_corr(const uint8_t* packed, int bits, const void* W, int dtype, const float* qscale,
                      const float* colw, int64_t colw_stride, int64_t batch, int64_t rows, int64_t cols, double* out,
                      void* stream);
int cq_transpose_f16(const uint16_t* X, int64_t batch, int64_t rows, int64_t cols, uint16_t* Y, void* stream);

/* Fused Q update.  Replaces alg.py:253-283 (maybe_update_Q / update_Q_non_data_aware:
 * res = W - L@R, quantize_matrix) + quantization.py:244-269 (whole-matrix uniform quantise):
 * res is recomputed per tile from the split-fp16 halves of L (m x r) and R^T (n x r,
 * inv_scale[b] = 1 / (scale_L * scale_R)) and never written; two passes over W (absmax, then
 * quantise).  r = 0 (no LR yet): res = W exactly, factor pointers may be NULL.  Outputs:
 * packed offset-binary codes (bits 2/4) and/or int8/int16 codes, scale_out[b] =
 * max(max|res|, eps), err_out[b] = sum_ij err_w[j] (deq - res)^2 (fp64; err_w NULL = 1).
 * absmax_in (r = 0 only, may be NULL): max|W[b]| already known (cq_absmax of the same W),
 * so the absmax pass is skipped and W is read once.
 * scale_hint (may be NULL; may alias scale_out): the previous Q update's scale per matrix.
 * With 2-bit packed codes and fp16 W, LR is then recomputed once: the
 * absmax pass also sums the all-zero-code error and lists every 8-element group holding a
 * |res| >= 0.45 scale_hint (a group with one such element as that element's index and
 * residual, 8 B; a group with more as its 8 residuals, 36 B); the codes come from those lists
 * (a 2-bit code is nonzero only where |res| > scale / 2).  A
 * matrix whose list cannot be complete (scale < 0.9 scale_hint, list overflow, non-normal
 * scale) takes the second recompute; fallback_out[b] (may be NULL) reports it.  The
 * workspace is cq_q_update_workspace(m, n, batch, scale_hint != NULL) bytes.  Codes and
 * scales are those of the two-pass form bit for bit; err_out sums the same fp32 terms in
 * another order (~1e-8 relative). */
size_t cq_q_update_workspace(int64_t m, int64_t n, int64_t batch, int with_hint);
/* Geometry of the single-recompute list path for rank r: rows of W per list region
 * (*rows_out), the capacity of its list of single-candidate groups (*cap_out) and of its list
 * of groups with two or more candidates (*capb_out, may be NULL), per region; a region with
 * more groups of either kind overflows and its matrix takes the second recompute.
 * Returns 0, or CQ_EINVAL when (m, n, r) do not take the list path. */
int cq_q_update_list_geometry(int64_t m, int64_t n, int64_t r, int64_t* rows_out, int64_t* cap_out,
                              int64_t* capb_out);
int cq_q_update_x3(int dtype, const void* W, int64_t m, int64_t n, int64_t r, int64_t batch,
                   const uint16_t* Lh, const uint16_t* Ll, const uint16_t* Rth, const uint16_t* Rtl,
                   const float* inv_scale, int bits, float eps, void* codes, uint8_t* packed,
                   float* scale_out, const float* err_w, int64_t err_w_stride, double* err_out,
                   const float* absmax_in, const float* scale_hint, int* fallback_out, void* ws,
                   size_t ws_bytes, void* stream);

/* Chebyshev 3-term recurrence support and elementwise helpers. */
/* out[b] = sum(x[b]^2 * w[j % ncols]) fp64 (w may be NULL) — denominators of alg.py:298 */
int cq_weighted_sqsum(int dtype, const void* x, int64_t batch, int64_t numel,
                      const float* w, int64_t ncols, int64_t w_stride, double* out, void* ws,
                      size_t ws_bytes, void* stream);
/* out[b] = sum_i x[b][i] * y[b][i], fp64 accumulation; dtype CQ_F32 | CQ_F64.  Workspace
 * as cq_weighted_sqsum (cq_rms_scale_workspace(batch, numel)).  Replaces the separate
 * m x n x r error GEMM of the LPLR loop (alg.py:182): with Y R^T and the r x r Grams
 * already at hand, ||Y - L R||^2 = ||Y||^2 - 2 <L, Y R^T> + <L^T L, R R^T>. */
int cq_batched_dot(int dtype, const void* x, const void* y, int64_t batch, int64_t numel, double* out,
                   void* ws, size_t ws_bytes, void* stream);
/* Y[b][i][j] = op(X[b])[i][j] * rowscale[b*rss + i] * colscale[b*css + j]
 * (op(X)[i][j] = X[i*ldx + j], or X[j*ldx + i] if trans_x; a NULL scale is 1;
 *  a stride of 0 shares the scale vector across the batch). rows x cols is op(X)'s shape. */
int cq_scale_rc(const float* X, int64_t ldx, int64_t stride_x, int trans_x, float* Y,
                int64_t ldy, int64_t stride_y, int64_t rows, int64_t cols, int64_t batch,
                const float* rowscale, int64_t rowscale_stride, const float* colscale,
                int64_t colscale_stride, void* stream);

/* ---------------------------------------------------------------------------------
 * Hessian calibration.  Replaces the activation accumulation of
 * main.py:296-308 (a_aT = A A^T in float64, summed over samples) for the diagonal that
 * diag_Hessians.pt ships (`Hall[name]`, main.py:163).  Activations x (fp32 | fp16 | bf16).
 *
 * cq_act_sqsum_cols: out[j] = (accumulate ? out[j] : 0) + sum_i x[i*ld + j]^2, then * post
 *   (rows x cols, row stride ld): diag(X^T X) of a token-major activation block — the
 *   per-channel sum over tokens.  fp64 accumulation in a fixed order (deterministic).
 * cq_act_sqsum_rows: out[i] = (accumulate ? out[i] : 0) + sum_j x[i*ld + j]^2, then * post
 *   — diag(X X^T) of the reference's `activations.view(D, -1)` (main.py:302-305).
 * post = 1/(idx+1) reproduces main.py:307's running division. */
size_t cq_act_sqsum_workspace(int64_t rows, int64_t cols);
int cq_act_sqsum_cols(int dtype, const void* x, int64_t rows, int64_t cols, int64_t ld, double* out,
                      int accumulate, double post, void* ws, size_t ws_bytes, void* stream);
int cq_act_sqsum_rows(int dtype, const void* x, int64_t rows, int64_t len, int64_t ld, double* out,
                      int accumulate, double post, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CALDERA_HIP_H */
