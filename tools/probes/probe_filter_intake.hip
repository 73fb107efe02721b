// Probe (test infrastructure, not product code): what bounds the split-fp16 filter step
// gemm_x3v_kernel<0> (cq_x3.hip xv_mainloop)?  Same tile (192 x 384 x 32, 12 waves of 96 x 64,
// 16x16x32 MFMAs, 2-stage LDS-DMA ring, swizzled images) on the config-2 B = 256 shapes
// (A = X^T halves 192 x 4096, B = G halves 4096 x 4096, K-blocked), random fp16 operands,
// with parts of the work removed:
//   mode 0  the product as in the engine (loads, fragment reads, 3 MFMAs per block and step)
//   mode 1  G's LDS-DMA loads skipped on every odd K step (per-CU intake -1/3: what a
//           symmetric-tile variant feeding G[I,J] to two products would save)
//   mode 2  no loads after the first stage (intake 0: fragment reads + MFMAs + barriers)
//   mode 3  loads as mode 0, fragments read from LDS once (no per-step fragment reads)
//   mode 4  loads and fragment reads as mode 0, one MFMA per block and step instead of three
//   mode 5  X^T's (A's) LDS-DMA loads skipped after the first stage (G's every step)
//   mode 6  G's (B's) LDS-DMA loads skipped after the first stage (X^T's every step)
//   mode 7  X^T's fragments loaded by each wave straight into registers (global_load, L2/L1-
//           served): row block i's fragments of step t + 1 are loaded into the registers of
//           step t's right after its MFMAs; only G through the LDS-DMA ring
//   mode 8  loads and barriers only (no fragment reads, no MFMAs): the 2-stage ring's intake floor
//   mode 9  a 3-stage ring (round 6): 192 x 192 x 32 tiles (48 KB stages, 3 fit
//           the 144 KB), 12 waves of 48 x 64, stage t + 2 issued at step t (counted vmcnt: two
//           stages in flight instead of one) -- the same MFMAs per output, 1.33x the intake per
//           flop (X^T re-read by twice as many tiles)
//   mode 10 mode 9's loads and barriers only (its intake floor)
//   mode 11 the 192 x 384 tile and 2-slot ring, but G's stage t + 2 issued inside step t: every
//           wave reads its G fragments of step t first (they are already front-loaded), a second
//           barrier, then the G loads of t + 2 into the slot just read (two steps to land instead
//           of one: 2/3 of the intake); X^T's stage t + 1 at the top of step t as before
//   mode 12 mode 11's loads and barriers only
// Results are numerically meaningless for modes 1-6, 8, 10 (stale LDS / reused fragments).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -o probe_filter_intake probe_filter_intake.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

using f16x8 = __attribute__((ext_vector_type(8))) _Float16;
using f32x4v = __attribute__((ext_vector_type(4))) float;

constexpr int BM = 192, BN = 384, BK = 32, THREADS = 768;
constexpr int APART = BM * BK, BPART = BN * BK, STAGE = 2 * APART + 2 * BPART;
constexpr size_t LDS_BYTES = (size_t)2 * STAGE * 2;
constexpr int PER_WAVE = 6;

__device__ __forceinline__ int swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }
__device__ __forceinline__ f16x8 frag(const _Float16* img, int row, int chunk) {
    return *reinterpret_cast<const f16x8*>(img + row * BK + (chunk ^ swz(row)) * 8);
}

__device__ __forceinline__ void issue(const _Float16* Ah, const _Float16* Al, const _Float16* Bh, const _Float16* Bl,
                                      int64_t b, int64_t M, int64_t N, int64_t K, int wid, const uint32_t (&off)[PER_WAVE],
                                      int64_t k0, _Float16* st, bool withB, bool withA = true) {
#pragma unroll
    for (int u = 0; u < PER_WAVE; ++u) {
        const int I = wid * PER_WAVE + u;
        const bool isA = I < 24;
        if (!isA && !withB) continue;
        if (isA && !withA) continue;
        const int part = isA ? (I >= 12) : (I >= 48);
        const int sub = isA ? (I - 12 * part) : (I - 24 - 24 * part);
        const _Float16* base = isA ? (part ? Al : Ah) + b * M * K + (k0 >> 5) * (M * 32)
                                   : (part ? Bl : Bh) + b * N * K + (k0 >> 5) * (N * 32);
        _Float16* dst = st + (isA ? part * APART : 2 * APART + part * BPART) + (16 * sub) * BK;
        __builtin_amdgcn_global_load_lds((const void*)(base + off[u]), (__attribute__((address_space(3))) void*)dst, 16,
                                         0, 0);
    }
}

template <int MODE>
__global__ __launch_bounds__(THREADS, 1) void probe_kernel(const _Float16* Ah, const _Float16* Al, const _Float16* Bh,
                                                           const _Float16* Bl, int64_t M, int64_t N, int64_t K,
                                                           int64_t tiles_n, float* C) {
    extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
    const int64_t b = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
    const int64_t n0 = tn * BN;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid & 1, wn = wid >> 1, l16 = lane & 15, lq = lane >> 4;
    uint32_t off[PER_WAVE];
#pragma unroll
    for (int u = 0; u < PER_WAVE; ++u) {
        const int I = wid * PER_WAVE + u;
        const bool isA = I < 24;
        const int part = isA ? (I >= 12) : (I >= 48);
        const int sub = isA ? (I - 12 * part) : (I - 24 - 24 * part);
        const int row = 16 * sub + (lane >> 2);
        const int c = (lane & 3) ^ swz(row);
        int64_t gr = (isA ? 0 : n0) + row;
        const int64_t lim = isA ? M : N;
        gr = gr < lim ? gr : lim - 1;
        off[u] = (uint32_t)(gr * 32 + c * 8);
    }
    f32x4v acc[6][4];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const int64_t nt = K / BK;
    issue(Ah, Al, Bh, Bl, b, M, N, K, wid, off, 0, smem, true);
    f16x8 bh3[4], bl3[4], a0h, a0l;   // mode 3: fragments read at the first step, reused
    // mode 7: this wave's X^T fragments (96 rows x 32, hi and lo) of the current and the next step
    f16x8 ra[6][2];
    auto load_a = [&](int64_t k0, int i) {
        const int64_t o = b * M * K + (k0 >> 5) * (M * 32) + (96 * wm + 16 * i + l16) * 32 + 8 * lq;
        ra[i][0] = *reinterpret_cast<const f16x8*>(Ah + o);
        ra[i][1] = *reinterpret_cast<const f16x8*>(Al + o);
    };
    if (MODE == 7)
#pragma unroll
        for (int i = 0; i < 6; ++i) load_a(0, i);
    for (int64_t t = 0; t < nt; ++t) {
        f16x8 bh[4], bl[4];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (t + 1 < nt && MODE != 2)
            issue(Ah, Al, Bh, Bl, b, M, N, K, wid, off, (t + 1) * BK, smem + ((t + 1) & 1) * STAGE,
                  (MODE != 1 || ((t + 1) & 1) == 0) && MODE != 6, MODE != 5 && MODE != 7);
        const _Float16* sA = smem + (t & 1) * STAGE;
        const _Float16* sB = sA + 2 * APART;
        if (MODE == 8) continue;
        if (MODE != 3) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                bh[j] = frag(sB, 64 * wn + 16 * j + l16, lq);
                bl[j] = frag(sB + BPART, 64 * wn + 16 * j + l16, lq);
            }
        } else {
            if (t == 0) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    bh3[j] = frag(sB, 64 * wn + 16 * j + l16, lq);
                    bl3[j] = frag(sB + BPART, 64 * wn + 16 * j + l16, lq);
                }
                a0h = frag(sA, 96 * wm + l16, lq);
                a0l = frag(sA + APART, 96 * wm + l16, lq);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) { bh[j] = bh3[j]; bl[j] = bl3[j]; }
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            f16x8 ah, al;
            if (MODE == 7) {
                ah = ra[i][0];
                al = ra[i][1];
            } else if (MODE != 3) {
                ah = frag(sA, 96 * wm + 16 * i + l16, lq);
                al = frag(sA + APART, 96 * wm + 16 * i + l16, lq);
            } else {
                ah = a0h;
                al = a0l;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (MODE != 4) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], al, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl[j], ah, acc[i][j], 0, 0, 0);
                }
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], ah, acc[i][j], 0, 0, 0);
            }
            if (MODE == 7 && t + 1 < nt) load_a((t + 1) * BK, i);
        }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = 96 * wm + 16 * i + l16, col = n0 + 64 * wn + 16 * j + 4 * lq;
            if (col < N)
                *reinterpret_cast<float4*>(C + (b * M + row) * N + col) =
                    make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        }
}


// mode 9 / 10: 192 x 192 tiles, 3-stage ring, two stages in flight
constexpr int BN3 = 192, BPART3 = BN3 * BK, STAGE3 = 2 * APART + 2 * BPART3;
constexpr size_t LDS3 = (size_t)3 * STAGE3 * 2;   // 144 KB
constexpr int PER_WAVE3 = 4;                      // 48 wave-instructions per stage / 12 waves

template <int MODE>
__global__ __launch_bounds__(THREADS, 1) void probe3_kernel(const _Float16* Ah, const _Float16* Al, const _Float16* Bh,
                                                            const _Float16* Bl, int64_t M, int64_t N, int64_t K,
                                                            int64_t tiles_n, float* C) {
    extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
    const int64_t b = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
    const int64_t n0 = tn * BN3;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid & 3, wn = wid >> 2, l16 = lane & 15, lq = lane >> 4;   // 4 x 48 rows, 3 x 64 columns
    uint32_t off[PER_WAVE3];
    const _Float16* src[PER_WAVE3];
    int dsto[PER_WAVE3];
#pragma unroll
    for (int u = 0; u < PER_WAVE3; ++u) {
        const int I = wid * PER_WAVE3 + u;   // 0..47: Ah 0-11, Al 12-23, Bh 24-35, Bl 36-47
        const bool isA = I < 24;
        const int part = isA ? (I >= 12) : (I >= 36);
        const int sub = isA ? (I - 12 * part) : (I - 24 - 12 * part);
        const int row = 16 * sub + (lane >> 2);
        const int c = (lane & 3) ^ swz(row);
        int64_t gr = (isA ? 0 : n0) + row;
        const int64_t lim = isA ? M : N;
        gr = gr < lim ? gr : lim - 1;
        off[u] = (uint32_t)(gr * 32 + c * 8);
        src[u] = isA ? (part ? Al : Ah) + b * M * K : (part ? Bl : Bh) + b * N * K;
        dsto[u] = (isA ? part * APART : 2 * APART + part * BPART3) + (16 * sub) * BK;
    }
    auto issue = [&](int64_t k0, _Float16* st) {
#pragma unroll
        for (int u = 0; u < PER_WAVE3; ++u) {
            const int64_t lda = (wid * PER_WAVE3 + u) < 24 ? M : N;   // A: instructions 0-23 (waves 0-5)
            __builtin_amdgcn_global_load_lds((const void*)(src[u] + (k0 >> 5) * (lda * 32) + off[u]),
                                             (__attribute__((address_space(3))) void*)(st + dsto[u]), 16, 0, 0);
        }
    };
    f32x4v acc[3][4];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const int64_t nt = K / BK;
    issue(0, smem);
    if (nt > 1) issue(BK, smem + STAGE3);
    for (int64_t t = 0; t < nt; ++t) {
        if (t + 1 < nt) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // stage t + 1 may still fly
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // stage t landed everywhere; slot of t - 1 fully read
        if (t + 2 < nt) issue((t + 2) * BK, smem + ((t + 2) % 3) * STAGE3);
        if (MODE == 10) continue;
        const _Float16* sA = smem + (t % 3) * STAGE3;
        const _Float16* sB = sA + 2 * APART;
        f16x8 bh[4], bl[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            bh[j] = frag(sB, 64 * wn + 16 * j + l16, lq);
            bl[j] = frag(sB + BPART3, 64 * wn + 16 * j + l16, lq);
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const f16x8 ah = frag(sA, 48 * wm + 16 * i + l16, lq);
            const f16x8 al = frag(sA + APART, 48 * wm + 16 * i + l16, lq);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], al, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl[j], ah, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], ah, acc[i][j], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = 48 * wm + 16 * i + l16, col = n0 + 64 * wn + 16 * j + 4 * lq;
            if (col < N)
                *reinterpret_cast<float4*>(C + (b * M + row) * N + col) =
                    make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        }
}

// mode 11 / 12: G two steps ahead in the 2-slot ring (a second barrier per step)
template <int MODE>
__global__ __launch_bounds__(THREADS, 1) void probe11_kernel(const _Float16* Ah, const _Float16* Al, const _Float16* Bh,
                                                             const _Float16* Bl, int64_t M, int64_t N, int64_t K,
                                                             int64_t tiles_n, float* C) {
    extern __shared__ __attribute__((aligned(16))) _Float16 smem[];
    const int64_t b = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
    const int64_t n0 = tn * BN;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wid & 1, wn = wid >> 1, l16 = lane & 15, lq = lane >> 4;
    const bool aw = wid < 4;   // waves 0-3 load X^T (instructions 0-23), waves 4-11 load G
    uint32_t off[PER_WAVE];
#pragma unroll
    for (int u = 0; u < PER_WAVE; ++u) {
        const int I = wid * PER_WAVE + u;
        const bool isA = I < 24;
        const int part = isA ? (I >= 12) : (I >= 48);
        const int sub = isA ? (I - 12 * part) : (I - 24 - 24 * part);
        const int row = 16 * sub + (lane >> 2);
        const int c = (lane & 3) ^ swz(row);
        int64_t gr = (isA ? 0 : n0) + row;
        const int64_t lim = isA ? M : N;
        gr = gr < lim ? gr : lim - 1;
        off[u] = (uint32_t)(gr * 32 + c * 8);
    }
    f32x4v acc[6][4];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const int64_t nt = K / BK;
    issue(Ah, Al, Bh, Bl, b, M, N, K, wid, off, 0, smem, true);
    if (nt > 1) issue(Ah, Al, Bh, Bl, b, M, N, K, wid, off, BK, smem + STAGE, true, false);   // G of step 1
    for (int64_t t = 0; t < nt; ++t) {
        if (!aw && t + 1 < nt) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // G of t + 1 may fly
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // stage t landed; X^T slot of t - 1 fully read
        if (t + 1 < nt) issue(Ah, Al, Bh, Bl, b, M, N, K, wid, off, (t + 1) * BK, smem + ((t + 1) & 1) * STAGE, false);
        const _Float16* sA = smem + (t & 1) * STAGE;
        const _Float16* sB = sA + 2 * APART;
        f16x8 bh[4], bl[4];
        if (MODE == 11) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                bh[j] = frag(sB, 64 * wn + 16 * j + l16, lq);
                bl[j] = frag(sB + BPART, 64 * wn + 16 * j + l16, lq);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();   // every wave holds its G fragments of step t: the G slot is free
        if (t + 2 < nt) issue(Ah, Al, Bh, Bl, b, M, N, K, wid, off, (t + 2) * BK, smem + (t & 1) * STAGE, true, false);
        if (MODE == 12) continue;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const f16x8 ah = frag(sA, 96 * wm + 16 * i + l16, lq);
            const f16x8 al = frag(sA + APART, 96 * wm + 16 * i + l16, lq);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], al, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bl[j], ah, acc[i][j], 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bh[j], ah, acc[i][j], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = 96 * wm + 16 * i + l16, col = n0 + 64 * wn + 16 * j + 4 * lq;
            if (col < N)
                *reinterpret_cast<float4*>(C + (b * M + row) * N + col) =
                    make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
        }
}

__global__ void fill_kernel(_Float16* p, int64_t n, uint32_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)i * 2654435761u ^ seed;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = (_Float16)(((float)(x & 0xffff) / 32768.f) - 1.f);
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
    const int64_t B = argc > 1 ? atoll(argv[1]) : 256, M = 192, N = 4096, K = 4096;
    const int64_t tiles_n = (N + BN - 1) / BN;
    _Float16 *Ah, *Al, *Bh, *Bl;
    float* C;
    CK(hipMalloc(&Ah, B * M * K * 2)); CK(hipMalloc(&Al, B * M * K * 2));
    CK(hipMalloc(&Bh, B * N * K * 2)); CK(hipMalloc(&Bl, B * N * K * 2));
    CK(hipMalloc(&C, B * M * N * 4));
    fill_kernel<<<4096, 256>>>(Ah, B * M * K, 1); fill_kernel<<<4096, 256>>>(Al, B * M * K, 2);
    fill_kernel<<<4096, 256>>>(Bh, B * N * K, 3); fill_kernel<<<4096, 256>>>(Bl, B * N * K, 4);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const unsigned grid = (unsigned)(B * tiles_n);
    const int64_t tiles3 = (N + BN3 - 1) / BN3;
    const char* names[13] = {"full split product", "G loads skipped on odd K steps (intake -1/3)",
                            "no loads after the first stage", "fragments read once (no per-step LDS reads)",
                            "one MFMA per block and step (loads + reads as full)",
                            "X^T loads skipped after the first stage (G every step)",
                            "G loads skipped after the first stage (X^T every step)",
                            "X^T fragments into registers one step ahead, G by LDS-DMA",
                            "loads and barriers only (2-stage ring intake floor)",
                            "192 x 192 tile, 3-stage ring, two stages in flight",
                            "192 x 192 tile, 3-stage ring: loads and barriers only",
                            "G two steps ahead (second barrier per step), X^T one step",
                            "G two steps ahead: loads and barriers only"};
    CK(hipFuncSetAttribute((const void*)probe3_kernel<9>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS3));
    CK(hipFuncSetAttribute((const void*)probe3_kernel<10>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS3));
    CK(hipFuncSetAttribute((const void*)probe_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_BYTES));
    const int first = argc > 2 ? atoi(argv[2]) : 0;
    for (int mode = first; mode < 13; ++mode) {
        auto launch = [&]() {
            switch (mode) {
                case 0: probe_kernel<0><<<grid, THREADS, LDS_BYTES>>>(Ah, Al, Bh, Bl, M, N, K, tiles_n, C); break;
                case 1: probe_kernel<1><<<grid, THREADS, LDS_BYTES>>>(Ah, Al, Bh, Bl, M, N, K, tiles_n, C); break;
                case 2: probe_kernel<2><<<grid, THREADS, LDS_BYTES>>>(Ah, Al, Bh, Bl, M, N, K, tiles_n, C); break;
                case 3: probe_kernel<3><<<grid, THREADS, LDS_BYTES>>>(Ah, Al, Bh, Bl, M, N, K, tiles_n, C); break;
                case 5: probe_kernel<5><<<grid, THREADS, LDS_BYTES>>>(Ah, Al, Bh, Bl, M, N, K, tiles_n, C); break;
                case 6: probe_kernel<6><<<grid, THREADS, LDS_BYTES>>>(Ah, Al, Bh, Bl, M, N, K, tiles_n, C); break;
                case 7: probe_kernel<7><<<grid, THREADS, LDS_BYTES>>>(Ah, Al, Bh, Bl, M, N, K, tiles_n, C); break;
                case 4: probe_kernel<4><<<grid, THREADS, LDS_BYTES>>>(Ah, Al, Bh, Bl, M, N, K, tiles_n, C); break;
                case 8: probe_kernel<8><<<grid, THREADS, LDS_BYTES>>>(Ah, Al, Bh, Bl, M, N, K, tiles_n, C); break;
                case 9: probe3_kernel<9><<<(unsigned)(B * tiles3), THREADS, LDS3>>>(Ah, Al, Bh, Bl, M, N, K, tiles3, C); break;
                case 10: probe3_kernel<10><<<(unsigned)(B * tiles3), THREADS, LDS3>>>(Ah, Al, Bh, Bl, M, N, K, tiles3, C); break;
                case 11: probe11_kernel<11><<<grid, THREADS, LDS_BYTES>>>(Ah, Al, Bh, Bl, M, N, K, tiles_n, C); break;
                case 12: probe11_kernel<12><<<grid, THREADS, LDS_BYTES>>>(Ah, Al, Bh, Bl, M, N, K, tiles_n, C); break;
                default: break;
            }
        };
        for (int w = 0; w < 3; ++w) launch();
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"mode\": %d, \"what\": \"%s\", \"batch\": %lld, \"ms_per_launch\": %.4f}\n", mode, names[mode],
               (long long)B, ms / reps);
        fflush(stdout);
    }
    return 0;
}
