// mlp.hip — per-point MLP (Conv1d k=1 + BatchNorm1d + ReLU) for MI355X / gfx950.
//
// Replaces the 1x1-conv chains of TargetEncoder (network/simple_encoder.py:52-107)
// and re_residual_net / FeedForwardNet_norm (network/deformation_net.py:96-107,
// attention_graph/attention_utils.py:62-86), forward and backward.
//
// Activations are point-major [M][C] (C contiguous), so a 1x1 conv is the GEMM
// Y = X W^T with M = points (up to 262,144 here), N = Cout, K = Cin. The GEMM
// runs on v_mfma_f32_32x32x2_f32 (fp32 in, fp32 accumulate, exact fma chains).
//
//  * block tile 128x128, BK = 32, 256 threads = 2x2 waves, each wave 64x64 =
//    2x2 MFMA 32x32 tiles (64 accumulator registers);
//  * LDS holds both operands reduction-major (As[k][m], Bs[k][n]) so every
//    MFMA operand is one conflict-free ds_read_b32 per lane; row-major global
//    operands are transposed on the LDS write (row pad 1 -> conflict-free
//    ds_write_b32), k-major ones are copied (pad 4 -> ds_write_b128);
//  * the next K-tile is prefetched into registers while the current one is
//    consumed (T14 split: issue early, write LDS after the barrier);
//  * fused prologue: the previous layer's BatchNorm + ReLU is applied while
//    staging the operand (relu(x*s+t) or relu(x)*s+t), so normalised
//    activations are never written to HBM;
//  * fused epilogues: bias / per-group row bias, BN batch-statistics partials
//    (per-block mean & M2, merged in fp64 by ured_bn_fwd_finalize — Chan's
//    parallel variance, order-fixed, deterministic), max-pool partials, the
//    BN-backward masks/partials of the previous layer, or split-K partials;
//  * XCD-aware tile order: blocks that share an A row-panel run on one XCD.
#include <cstdlib>
#define URED_DBG_FILE 1
#include "ured_common.h"
#include "../../include/ured_hip.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;

typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f2v __attribute__((ext_vector_type(2)));

struct Gemm {
    UredGemmDesc d;
};

__device__ __forceinline__ float pro_apply(int pro, float x, float s, float t) {
    if (pro == URED_PRO_ENC) return fmaxf(__builtin_fmaf(x, s, t), 0.f);
    if (pro == URED_PRO_RES) return __builtin_fmaf(fmaxf(x, 0.f), s, t);
    return x;
}

// XCD-aware bijective remap of a linear block id (blocks b and b+8 share an XCD).
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int q = nwg / 8, r = nwg % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// ---- operand staging -------------------------------------------------------
// Loads are branch-free: every lane loads from a clamped (always in-bounds) address and
// out-of-range elements are zeroed by a select afterwards, so hipcc keeps all loads of a
// tile in flight (a load under a per-lane branch gets its own vmcnt(0) wait).
// VEC: float4 loads (requires 16-B aligned rows and contiguous extents multiple of 4).
// A staged tile lives in registers between its loads (issued before the MFMAs of the
// previous tile) and its LDS write (after them). The prologue transform and the
// out-of-range zeroing are applied at write time so no wait sits in front of the MFMAs.
struct RowTile {
    float v[4][4];       // raw loaded values
    float s[4], t[4];    // prologue affine of the 4 channels this thread stages (per c)
    unsigned valid;      // bit 4*i+c
    unsigned raw;        // bit 4*i+c: element comes from the raw second operand (no prologue)
};

template <int PRO>
__device__ __forceinline__ float finish(const RowTile& r, int i, int c) {
    float y = r.v[i][c];
    if (PRO != URED_PRO_NONE) {
        const float z = pro_apply(PRO, y, r.s[c], r.t[c]);
        y = ((r.raw >> (4 * i + c)) & 1u) ? y : z;
    }
    return ((r.valid >> (4 * i + c)) & 1u) ? y : 0.f;
}

// "row-major" operand: rows (m or n) x BK (k) from G[row*ld + k]; k contiguous; staged
// transposed to S[k][row]. Thread t: k4 = t % 8 (4 consecutive k), rows t/8 + 32*i.
// k >= k1 reads the raw second operand A2[row*ld2 + k - k1] (concatenated input).
template <int PRO, bool VEC>
__device__ __forceinline__ void load_rowmajor(RowTile& r, const float* __restrict__ G, int ld, int rows, int row0,
                                              int K, int k0, const float* __restrict__ A2, int ld2, int k1,
                                              const float* __restrict__ ps, const float* __restrict__ pt) {
    const int t = threadIdx.x, k4 = t & 7;
    const int kb = k0 + 4 * k4;
    r.valid = 0u;
    r.raw = 0u;
    if constexpr (VEC) {
        const bool kv = kb < K;
        const int kc = kv ? kb : K - 4;
        const bool first = kc < k1;
        if (PRO != URED_PRO_NONE) {
            const int kp = first ? kc : k1 - 4;
            const float4 s = *reinterpret_cast<const float4*>(ps + kp);
            const float4 tt = *reinterpret_cast<const float4*>(pt + kp);
            r.s[0] = s.x; r.s[1] = s.y; r.s[2] = s.z; r.s[3] = s.w;
            r.t[0] = tt.x; r.t[1] = tt.y; r.t[2] = tt.z; r.t[3] = tt.w;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = row0 + (t >> 3) + 32 * i;
            const int rc = row < rows ? row : rows - 1;
            const float* src = first ? G + (size_t)rc * ld + kc : A2 + (size_t)rc * ld2 + (kc - k1);
            const float4 q = *reinterpret_cast<const float4*>(src);
            r.v[i][0] = q.x; r.v[i][1] = q.y; r.v[i][2] = q.z; r.v[i][3] = q.w;
            const unsigned m = (kv && row < rows) ? 0xFu : 0u;
            r.valid |= m << (4 * i);
            r.raw |= (first ? 0u : 0xFu) << (4 * i);
        }
    } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int k = kb + c;
            const int kc = k < K ? k : K - 1;
            const bool first = kc < k1;
            if (PRO != URED_PRO_NONE) {
                const int kp = first ? kc : 0;
                r.s[c] = ps[kp];
                r.t[c] = pt[kp];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = row0 + (t >> 3) + 32 * i;
                const int rc = row < rows ? row : rows - 1;
                const float* src = first ? G + (size_t)rc * ld + kc : A2 + (size_t)rc * ld2 + (kc - k1);
                r.v[i][c] = *src;
                r.valid |= (k < K && row < rows ? 1u : 0u) << (4 * i + c);
                r.raw |= (first ? 0u : 1u) << (4 * i + c);
            }
        }
    }
}

template <int LDP, int PRO>
__device__ __forceinline__ void store_rowmajor(const RowTile& r, float* S) {
    const int t = threadIdx.x, k4 = t & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = (t >> 3) + 32 * i;
#pragma unroll
        for (int c = 0; c < 4; ++c) S[(4 * k4 + c) * LDP + row] = finish<PRO>(r, i, c);
    }
}

// "k-major" operand: BK (k) x cols (m or n) from G[k*ld + col]; col contiguous; staged
// directly to S[k][col]. Thread t: col4 = t % 32, k = t/32 + 8*i. The prologue channel is col.
template <int PRO, bool VEC>
__device__ __forceinline__ void load_kmajor(RowTile& r, const float* __restrict__ G, int ld, int cols, int col0,
                                            int K, int k0, const float* __restrict__ ps,
                                            const float* __restrict__ pt) {
    const int t = threadIdx.x, c4 = t & 31;
    const int cb = col0 + 4 * c4;
    r.valid = 0u;
    r.raw = 0u;
    if constexpr (VEC) {
        const bool cv = cb < cols;
        const int cc = cv ? cb : cols - 4;
        if (PRO != URED_PRO_NONE) {
            const float4 s = *reinterpret_cast<const float4*>(ps + cc);
            const float4 tt = *reinterpret_cast<const float4*>(pt + cc);
            r.s[0] = s.x; r.s[1] = s.y; r.s[2] = s.z; r.s[3] = s.w;
            r.t[0] = tt.x; r.t[1] = tt.y; r.t[2] = tt.z; r.t[3] = tt.w;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = k0 + (t >> 5) + 8 * i;
            const int kc = k < K ? k : K - 1;
            const float4 q = *reinterpret_cast<const float4*>(G + (size_t)kc * ld + cc);
            r.v[i][0] = q.x; r.v[i][1] = q.y; r.v[i][2] = q.z; r.v[i][3] = q.w;
            r.valid |= ((cv && k < K) ? 0xFu : 0u) << (4 * i);
        }
    } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int col = cb + c;
            const int ccl = col < cols ? col : cols - 1;
            if (PRO != URED_PRO_NONE) { r.s[c] = ps[ccl]; r.t[c] = pt[ccl]; }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int k = k0 + (t >> 5) + 8 * i;
                const int kc = k < K ? k : K - 1;
                r.v[i][c] = G[(size_t)kc * ld + ccl];
                r.valid |= (col < cols && k < K ? 1u : 0u) << (4 * i + c);
            }
        }
    }
}

template <int LDP, int PRO>
__device__ __forceinline__ void store_kmajor(const RowTile& r, float* S) {
    const int t = threadIdx.x, c4 = t & 31;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = (t >> 5) + 8 * i;
        *reinterpret_cast<float4*>(S + k * LDP + 4 * c4) =
            make_float4(finish<PRO>(r, i, 0), finish<PRO>(r, i, 1), finish<PRO>(r, i, 2), finish<PRO>(r, i, 3));
    }
}

template <bool KM> struct Pad { static constexpr int v = KM ? BM + 4 : BM + 1; };

// streaming kernels for the K <= 4 edge layers (A/B switches, one per direction)
#ifndef URED_FWD_SMALL
#define URED_FWD_SMALL 1
#endif
#ifndef URED_DGRAD_SMALL
#define URED_DGRAD_SMALL 1
#endif
#ifndef URED_BNBWD_YALL
#define URED_BNBWD_YALL 1
#endif

// BN partials (EPI_FWD stat_ws {mean, M2}, EPI_BNBWD bwd_ws {sum g, sum g*xhat}): layout
// [2][N][nblk], nblk = ceil(M/128) — one column's block partials are contiguous, so the
// finalizes read them coalesced (the epilogues' few scattered 4-B writes per block are cheap)
__host__ __device__ __forceinline__ size_t part_idx(int q, int col, int blk, int N, int M) {
    const int nblk = (M + 127) / 128;
    return ((size_t)q * N + col) * nblk + blk;
}

// Debug build (-DURED_DEBUG_BOUNDS=1, ured_common.h): every LDS-DMA destination range and every
// epilogue buffer-store offset is checked against its allocation on the device.

// Phase timing build (-DURED_GEMM_TIMING=1 -DURED_TS_M=.. -DURED_TS_N=.. -DURED_TS_K=..): the
// BN-backward dgrad launches of that shape record, per workgroup, the real-time clock (100 MHz) at
// start, first operand step ready, K-loop end and epilogue end, plus HW_ID / XCC_ID
// (tools/gemm_phase.py reads them back through ured_debug_gemm_ts).
#ifndef URED_GEMM_TIMING
#define URED_GEMM_TIMING 0
#endif
#if URED_GEMM_TIMING
constexpr int TS_SLOTS = 8192;
__device__ unsigned long long ured_ts_buf[TS_SLOTS * 16];
// slots per block: 0 start, 1 first K-step ready, 2 K-loop issued, 3 epilogue end (stores done),
// 4 HW_ID, 5 XCC_ID, 6 tile, 7 valid, 8 Yp + column parameters landed, 9 G stores issued,
// 10 column sums through LDS, 11 block partials written (wave 0's view; the last K-step's MFMAs
// may still be executing at mark 2, so their drain shows up in the epilogue's first phases)
__device__ __forceinline__ bool ts_shape(const UredGemmDesc& d) {
    return d.M == URED_TS_M && d.N == URED_TS_N && d.K == URED_TS_K && blockIdx.x < TS_SLOTS;
}
#define URED_TS_MARK(d, k) do { if (ts_shape(d) && threadIdx.x == 0) \
    ured_ts_buf[(size_t)blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define URED_TS_MARK(d, k) do { } while (0)
#endif

// ---- shared epilogue ---------------------------------------------------------
// element (i, j, r): row = m0 + wm*64 + i*32 + (r&3) + 8*(r>>2) + 4*(lane>>5), col = n0 + wn*64 + j*32 + (lane&31)
#define RED(a, q, c) red_f[((a) * 2 + (q)) * BN + (c)]
#define REDI(a, q, c) red_i[((a) * 2 + (q)) * BN + (c)]
struct NoPre { __device__ void operator()() const {} };

// Workgroup barrier that orders LDS only. __syncthreads() also carries a release fence for
// global memory, i.e. a vmcnt(0) that waits for every outstanding store of the wave; the
// epilogue reductions and the K-loop only exchange data through LDS (the LDS-DMA landing
// is covered by an explicit vmcnt wait before the barrier).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Output writer. BUF (v2 kernel): every lane issues every store as a buffer store and an
// out-of-range element gets an offset past num_records (the hardware drops it), so a wave
// always issues exactly 64 stores per output tile, unconditionally: the persistent kernel
// relies on that count to wait for its prefetch DMA without waiting for the stores.
constexpr unsigned ST_OOB = 0x80000000u;
template <bool BUF>
struct OutTile {
    float* base; int ld;
    unsigned ld4;        // row pitch in bytes, laundered per tile (see below)
    unsigned nrec;       // num_records of the descriptor (bytes)
    __amdgpu_buffer_rsrc_t rsrc;
    __device__ OutTile(float* b, int ld_, int M, int N) : base(b), ld(ld_) {
        if constexpr (BUF) {
            nrec = (unsigned)(((long long)(M - 1) * ld_ + N) * 4);
            rsrc = __builtin_amdgcn_make_buffer_rsrc(b, (short)0, (int)nrec, 0x00020000);
            // opaque to the optimiser: keeps the 64 per-element row products from being
            // hoisted out of the persistent tile loop (and spilled)
            ld4 = (unsigned)ld_ * 4u;
            asm volatile("" : "+s"(ld4));
        }
    }
    __device__ __forceinline__ void put(bool ok, int row, int col, float v) {
        if constexpr (BUF) {
            // 32-bit byte offset (buf_ok guarantees M * ld * 4 < 2^31) and a select: no branch
            const unsigned off = (unsigned)row * ld4 + (unsigned)col * 4u;
#if URED_DEBUG_BOUNDS
            URED_DBG_CHECK(!(ok && (row < 0 || col < 0 || off + 4u > nrec)));
#endif
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rsrc, ok ? off : ST_OOB, 0, 0);
        } else if (ok) {
            base[(size_t)row * ld + col] = v;
        }
    }
};

// `pre` runs once all of the epilogue's own global loads are issued and before any of them
// is consumed: the persistent kernel issues the next tile's first LDS-DMA there, so it lands
// while this epilogue computes and stores (vmcnt counts in order, so a DMA issued earlier
// would make every epilogue load wait for it).
// Matching reader (BN-backward Yp). BUF: buffer loads at 32-bit offsets; rows/columns
// outside [M, N) read as 0 (their results are never stored). Otherwise clamped loads.
template <bool BUF>
struct InTile {
    const float* base; int ld, M, N;
    unsigned ld4;
    __amdgpu_buffer_rsrc_t rsrc;
    __device__ InTile(const float* b, int ld_, int M_, int N_) : base(b), ld(ld_), M(M_), N(N_) {
        if constexpr (BUF) {
            rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(b), (short)0,
                                                     (int)(((long long)(M_ - 1) * ld_ + N_) * 4), 0x00020000);
            ld4 = (unsigned)ld_ * 4u;
            asm volatile("" : "+s"(ld4));
        }
    }
    __device__ __forceinline__ float get(int row, int col) const {
        if constexpr (BUF) {
            const unsigned off = (unsigned)row * ld4 + (unsigned)col * 4u;
            return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, col < N ? off : ST_OOB, 0, 0));
        } else {
            row = row < M ? row : M - 1;
            col = col < N ? col : N - 1;
            return base[(size_t)row * ld + col];
        }
    }
};

// BN-backward epilogue of a full 128 x (64 TN) tile (every row < M, every column < N; no per-element
// residual gradient, pooled gradients only of 128-row-aligned groups): the general loop below
// without its per-element bounds selects, and with the Yp loads / G stores addressed as a per-lane
// buffer offset plus a scalar row offset (no per-element 32-bit multiplies). Same operations in the
// same order as the general loop, so the results are bitwise the same.
template <int ACT, bool POOL, int TN, class Pre>
__device__ __forceinline__ void bnbwd_full(const UredGemmDesc& d, f16v (&acc)[2][2], int m0, int n0, float (&s1)[2],
                                           float (&s2)[2], Pre pre) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w & 1, wn = w >> 1;
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(d.Yp), (short)0,
                                                                         (int)(((long long)(d.M - 1) * d.ldy + d.N) * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(d.C, (short)0,
                                                                         (int)(((long long)(d.M - 1) * d.ldc + d.N) * 4), 0x00020000);
    const unsigned ly = (unsigned)d.ldy * 4u, lc = (unsigned)d.ldc * 4u;
    const unsigned r0 = (unsigned)(m0 + wm * 64 + 4 * (lane >> 5));       // this lane's first row
    // rows of element (i, r): r0 + i*32 + (r&3) + 8*(r>>2) -> scalar offset (i*32 + (r&3) + 8*(r>>2)) * ld,
    // from an opaque copy of ld so that the products are s_muls at their use, not hoisted SGPRs
    auto roff = [&](int i, int r, unsigned ld) {
        asm volatile("" : "+s"(ld));
        return (unsigned)(i * 32 + (r & 3) + 8 * (r >> 2)) * ld;
    };
    float yh[2][2][16];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const unsigned vo = r0 * ly + (unsigned)(n0 + wn * (32 * TN) + j * 32 + (lane & 31)) * 4u;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                yh[j][i][r] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(yr, vo, roff(i, r, ly), 0));
    }
    float sc_[2], sh_[2], mu_[2], is_[2], pgr_[2];
    int pidx_[2];
    const int pg = POOL ? m0 / d.pool_group_rows : 0;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int col = n0 + wn * (32 * TN) + j * 32 + (lane & 31);
        sc_[j] = d.bn_scale[col]; sh_[j] = d.bn_shift[col]; mu_[j] = d.bn_mean[col]; is_[j] = d.bn_invstd[col];
        pidx_[j] = -1; pgr_[j] = 0.f;
        if (POOL) { pidx_[j] = d.pool_idx[(size_t)pg * d.N + col]; pgr_[j] = d.pool_grad[(size_t)pg * d.N + col]; }
    }
    pre();
#if URED_GEMM_TIMING
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    URED_TS_MARK(d, 8);
#endif
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const unsigned vo = r0 * lc + (unsigned)(n0 + wn * (32 * TN) + j * 32 + (lane & 31)) * 4u;
        const int prow = pidx_[j] - (int)r0;       // the pooled winner's row relative to this lane's first row
        float a1 = 0.f, a2 = 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const float a = acc[i][j][r];
                const float dh = (POOL && prow == i * 32 + (r & 3) + 8 * (r >> 2)) ? a + pgr_[j] : a;
                const float y = yh[j][i][r];
                float g, xh;
                if (ACT == URED_ACT_RES) {
                    g = dh;
                    xh = (fmaxf(y, 0.f) - mu_[j]) * is_[j];
                } else if (ACT == URED_ACT_BN) {
                    g = dh;
                    xh = (y - mu_[j]) * is_[j];
                } else {
                    g = (__builtin_fmaf(y, sc_[j], sh_[j]) > 0.f) ? dh : 0.f;
                    xh = (y - mu_[j]) * is_[j];
                }
#if URED_DEBUG_BOUNDS
                URED_DBG_CHECK(!((unsigned long long)vo + roff(i, r, lc) + 4u > (unsigned long long)(((long long)(d.M - 1) * d.ldc + d.N) * 4) ||
                                 r0 + (unsigned)(i * 32 + (r & 3) + 8 * (r >> 2)) >= (unsigned)d.M));
#endif
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, g), cr, vo, roff(i, r, lc), 0);
                a1 += g;
                a2 += g * xh;
            }
        a1 += __shfl_xor(a1, 32);
        a2 += __shfl_xor(a2, 32);
        s1[j] = a1; s2[j] = a2;
    }
    URED_TS_MARK(d, 9);
}

template <int EPI, bool BUFST = false, int TM = 2, int TN = 2, class Pre = NoPre>
__device__ __forceinline__ void epilogue(const UredGemmDesc& d, f16v (&acc)[2][2], int m0, int n0,
                                         float* red_f, int* red_i, Pre pre = Pre()) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w & 1, wn = w >> 1;
    // element (i, j, r): row = m0 + wm*64 + i*32 + (r&3) + 8*(r>>2) + 4*(lane>>5), col = n0 + wn*64 + j*32 + (lane&31)
    const int rbase = m0 + wm * (32 * TM) + 4 * (lane >> 5);
    auto row_of = [&](int i, int r) { return rbase + i * 32 + (r & 3) + 8 * (r >> 2); };

    if (EPI == URED_EPI_STORE || EPI == URED_EPI_SPLITK) {
        OutTile<BUFST> C(d.C + (EPI == URED_EPI_SPLITK ? (size_t)blockIdx.z * d.M * d.ldc : 0), d.ldc, d.M, d.N);
        float bsv[2];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn * (32 * TN) + j * 32 + (lane & 31);
            bsv[j] = (EPI == URED_EPI_STORE && d.bias && col < d.N) ? d.bias[col] : 0.f;
        }
        pre();
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn * (32 * TN) + j * 32 + (lane & 31);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = row_of(i, r);
                    C.put(row < d.M && col < d.N, row, col, acc[i][j][r] + bsv[j]);
                }
        }
        return;
    }

    const int blk = m0 / BM;
    const int nvalid = min(BM, d.M - m0);

    if (EPI == URED_EPI_FWD) {
        // value, store, per-column block stats (two-pass on registers: mean then M2).
        // Row bias of a block that lies inside one group (group_rows % BM == 0, no gidx):
        // one load per column, folded into the column bias.
        const bool rb_blk = d.rowbias && !d.gidx && d.group_rows % BM == 0;
        OutTile<BUFST> Cw(d.C, d.ldc, d.M, d.N);
        float bsv_[2];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn * (32 * TN) + j * 32 + (lane & 31);
            const bool cv = col < d.N;
            bsv_[j] = (cv && d.bias) ? d.bias[col] : 0.f;
            if (rb_blk && cv) bsv_[j] += d.rowbias[(size_t)(m0 / d.group_rows) * d.ldr + col];
        }
        pre();
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn * (32 * TN) + j * 32 + (lane & 31);
            const bool cv = col < d.N;
            const float bsv = bsv_[j];
            if (!d.rowbias || rb_blk) {   // common case: no per-element branch or load
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = row_of(i, r);
                        const float v = acc[i][j][r] + bsv;
                        Cw.put(cv && row < d.M, row, col, v);
                        acc[i][j][r] = v;
                    }
            } else {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = row_of(i, r);
                    float v = acc[i][j][r] + bsv;
                    if (cv && row < d.M) {
                        const int g = d.gidx ? d.gidx[row] : row / d.group_rows;
                        v += d.rowbias[(size_t)g * d.ldr + col];
                    }
                    Cw.put(cv && row < d.M, row, col, v);
                    acc[i][j][r] = v;
                }
            }
        }
        // the statistics are of relu(v) (stat_relu) or v: a clamp at 0 or at -inf
        const float plo = d.stat_relu ? 0.f : -__builtin_inff();
        // pass 1: column sums of p over valid rows
        float csum[2];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float p = fmaxf(acc[i][j][r], plo);
                    s += (row_of(i, r) < d.M) ? p : 0.f;
                }
            s += __shfl_xor(s, 32);
            csum[j] = s;
        }
        if (lane < 32) {
#pragma unroll
            for (int j = 0; j < TN; ++j) RED(wm, 0, wn * (32 * TN) + j * 32 + lane) = csum[j];
        }
        lds_barrier();
        float cmean[2];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int c = wn * (32 * TN) + j * 32 + (lane & 31);
            cmean[j] = (RED(0, 0, c) + RED(1, 0, c)) / (float)nvalid;
        }
        // pass 2: M2 about the block mean
        float cm2[2];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            float s = 0.f;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const float p = fmaxf(acc[i][j][r], plo);
                    const float e = p - cmean[j];
                    s += (row_of(i, r) < d.M) ? e * e : 0.f;
                }
            s += __shfl_xor(s, 32);
            cm2[j] = s;
        }
        if (lane < 32) {
#pragma unroll
            for (int j = 0; j < TN; ++j) RED(wm, 1, wn * (32 * TN) + j * 32 + lane) = cm2[j];
        }
        lds_barrier();
        if (wm == 0 && lane < 32) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int c = wn * (32 * TN) + j * 32 + lane;
                const int col = n0 + c;
                if (col < d.N) {
                    d.stat_ws[part_idx(0, col, blk, d.N, d.M)] = cmean[j];
                    d.stat_ws[part_idx(1, col, blk, d.N, d.M)] = RED(0, 1, c) + RED(1, 1, c);
                }
            }
        }
        if (d.pool_ws) {
            lds_barrier();
            // per column max/min of Y with lowest-row tie break
            float mx[2], mn[2];
            int ix[2], in_[2];
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                mx[j] = -__builtin_inff(); mn[j] = __builtin_inff(); ix[j] = 0x7fffffff; in_[j] = 0x7fffffff;
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = row_of(i, r);
                        if (row >= d.M) continue;
                        const float v = acc[i][j][r];
                        if (v > mx[j] || (v == mx[j] && row < ix[j])) { mx[j] = v; ix[j] = row; }
                        if (v < mn[j] || (v == mn[j] && row < in_[j])) { mn[j] = v; in_[j] = row; }
                    }
                const float omx = __shfl_xor(mx[j], 32), omn = __shfl_xor(mn[j], 32);
                const int oix = __shfl_xor(ix[j], 32), oin = __shfl_xor(in_[j], 32);
                if (omx > mx[j] || (omx == mx[j] && oix < ix[j])) { mx[j] = omx; ix[j] = oix; }
                if (omn < mn[j] || (omn == mn[j] && oin < in_[j])) { mn[j] = omn; in_[j] = oin; }
            }
            if (lane < 32) {
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int c = wn * (32 * TN) + j * 32 + lane;
                    RED(wm, 0, c) = mx[j]; REDI(wm, 0, c) = ix[j];
                    RED(wm, 1, c) = mn[j]; REDI(wm, 1, c) = in_[j];
                }
            }
            lds_barrier();
            if (wm == 0 && lane < 32) {
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int c = wn * (32 * TN) + j * 32 + lane;
                    const int col = n0 + c;
                    if (col >= d.N) continue;
                    float a = RED(0, 0, c); int ai = REDI(0, 0, c);
                    if (RED(1, 0, c) > a || (RED(1, 0, c) == a && REDI(1, 0, c) < ai)) { a = RED(1, 0, c); ai = REDI(1, 0, c); }
                    float b = RED(0, 1, c); int bi = REDI(0, 1, c);
                    if (RED(1, 1, c) < b || (RED(1, 1, c) == b && REDI(1, 1, c) < bi)) { b = RED(1, 1, c); bi = REDI(1, 1, c); }
                    float* pw = d.pool_ws + (size_t)blk * 4 * d.N;
                    pw[col] = a; reinterpret_cast<int*>(pw)[d.N + col] = ai;
                    pw[2 * d.N + col] = b; reinterpret_cast<int*>(pw)[3 * d.N + col] = bi;
                }
            }
        }
        return;
    }

    if (EPI == URED_EPI_BNBWD) {
        float s1[2], s2[2];
        const bool pool_al = d.pool_idx && (d.pool_group_rows % BM == 0);
        const bool full = BUFST && m0 + 64 * TM <= d.M && n0 + 64 * TN <= d.N && !d.gadd && (!d.pool_idx || pool_al);
        if (full) {
            if (pool_al) {
                if (d.bwd_res == URED_ACT_RES) bnbwd_full<URED_ACT_RES, true, TN>(d, acc, m0, n0, s1, s2, pre);
                else if (d.bwd_res == URED_ACT_BN) bnbwd_full<URED_ACT_BN, true, TN>(d, acc, m0, n0, s1, s2, pre);
                else bnbwd_full<URED_ACT_ENC, true, TN>(d, acc, m0, n0, s1, s2, pre);
            } else {
                if (d.bwd_res == URED_ACT_RES) bnbwd_full<URED_ACT_RES, false, TN>(d, acc, m0, n0, s1, s2, pre);
                else if (d.bwd_res == URED_ACT_BN) bnbwd_full<URED_ACT_BN, false, TN>(d, acc, m0, n0, s1, s2, pre);
                else bnbwd_full<URED_ACT_ENC, false, TN>(d, acc, m0, n0, s1, s2, pre);
            }
        } else {
        // Yp one column half (32 values) at a time: the j = 0 half and the per-column
        // parameters are issued before pre() (the persistent kernel's next-tile DMA), the j = 1
        // half after the j = 0 half is processed (registers: acc 64 + one half 32)
        // URED_BNBWD_YALL: both halves (64 values) are issued at once instead — after the K-loop
        // the fragment registers are dead, so the whole tile fits without raising the kernel's
        // VGPR peak, and the epilogue then waits for one HBM round trip instead of two (gfx9
        // vmcnt is in order: the second half's loads otherwise queue behind the first half's stores)
        f16v yh[URED_BNBWD_YALL ? 2 : 1][2];
        InTile<BUFST> Yr(d.Yp, d.ldy, d.M, d.N);
        auto load_y = [&](int j) {
            const int col = n0 + wn * (32 * TN) + j * 32 + (lane & 31);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) yh[URED_BNBWD_YALL ? j : 0][i][r] = Yr.get(row_of(i, r), col);
        };
        if (!URED_BNBWD_YALL) load_y(0);
        // max-pool backward: the pooled gradient lands on the winning row of each (group, column)
        const bool pool_blk = d.pool_idx && (d.pool_group_rows % BM == 0);
        const int pg = pool_blk ? m0 / d.pool_group_rows : 0;
        float sc_[2], sh_[2], mu_[2], is_[2], pgr_[2];
        int pidx_[2];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int col = n0 + wn * (32 * TN) + j * 32 + (lane & 31);
            const bool cv = col < d.N;
            const int cc = cv ? col : 0;
            sc_[j] = d.bn_scale[cc]; sh_[j] = d.bn_shift[cc]; mu_[j] = d.bn_mean[cc]; is_[j] = d.bn_invstd[cc];
            pidx_[j] = -1; pgr_[j] = 0.f;
            if (pool_blk && cv) { pidx_[j] = d.pool_idx[(size_t)pg * d.N + col]; pgr_[j] = d.pool_grad[(size_t)pg * d.N + col]; }
        }
        if (URED_BNBWD_YALL) { load_y(0); load_y(1); }   // behind the (L2-resident) per-column parameters
        pre();
        OutTile<BUFST> Gw(d.C, d.ldc, d.M, d.N);
        // per-element global reads (a residual gradient, or pooled gradients of groups that do
        // not align with the 128-row block) take the general loop below
        const bool slow = d.gadd || (d.pool_idx && !pool_blk);
        const bool relu_mask = d.bwd_res != URED_ACT_RES && d.bwd_res != URED_ACT_BN;
        const float ylo = d.bwd_res == URED_ACT_RES ? 0.f : -__builtin_inff();
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            if (!URED_BNBWD_YALL && j == 1) load_y(1);
            const int col = n0 + wn * (32 * TN) + j * 32 + (lane & 31);
            const bool cv = col < d.N;
            const float sc = sc_[j], sh = sh_[j], mu = mu_[j], is = is_[j];
            const int pidx = pidx_[j];
            const float pgr = pgr_[j];
            float a1 = 0.f, a2 = 0.f;
            if (!slow) {
                // common case, branch-free per element: the activation mode as a clamp and a mask
                // (ReLU mode: keep where y*sc+sh > 0; otherwise 0*y+1 > 0 keeps every element) and
                // the block's pooled gradient as a select (pidx = -1 matches no row)
                const float sck = relu_mask ? sc : 0.f, shk = relu_mask ? sh : 1.f;
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int row = row_of(i, r);
                        const bool ok = cv && row < d.M;
                        const float a = acc[i][j][r];
                        const float dh = (row == pidx) ? a + pgr : a;
                        const float y = yh[URED_BNBWD_YALL ? j : 0][i][r];
                        const float xh = (fmaxf(y, ylo) - mu) * is;
                        const float g = (__builtin_fmaf(y, sck, shk) > 0.f) ? dh : 0.f;
                        Gw.put(ok, row, col, g);
                        a1 += ok ? g : 0.f;
                        a2 += ok ? g * xh : 0.f;
                    }
            } else {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = row_of(i, r);
                    const bool ok = cv && row < d.M;
                    float dh = acc[i][j][r];
                    if (pool_blk) {
                        if (row == pidx) dh += pgr;
                    } else if (d.pool_idx && ok) {
                        const size_t ge = (size_t)(row / d.pool_group_rows) * d.N + col;
                        if (d.pool_idx[ge] == row) dh += d.pool_grad[ge];
                    }
                    if (d.gadd && ok) dh += d.gadd[(size_t)row * d.ldg + col];
                    const float y = yh[URED_BNBWD_YALL ? j : 0][i][r];
                    float g, xh;
                    if (d.bwd_res == URED_ACT_RES) {
                        g = dh;
                        xh = (fmaxf(y, 0.f) - mu) * is;
                    } else if (d.bwd_res == URED_ACT_BN) {
                        g = dh;
                        xh = (y - mu) * is;
                    } else {
                        g = (__builtin_fmaf(y, sc, sh) > 0.f) ? dh : 0.f;
                        xh = (y - mu) * is;
                    }
                    Gw.put(ok, row, col, g);
                    a1 += ok ? g : 0.f;
                    a2 += ok ? g * xh : 0.f;
                }
            }
            a1 += __shfl_xor(a1, 32);
            a2 += __shfl_xor(a2, 32);
            s1[j] = a1; s2[j] = a2;
        }
        }   // general loop
        if (lane < 32) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                RED(wm, 0, wn * (32 * TN) + j * 32 + lane) = s1[j];
                RED(wm, 1, wn * (32 * TN) + j * 32 + lane) = s2[j];
            }
        }
        lds_barrier();
        URED_TS_MARK(d, 10);
        if (wm == 0 && lane < 32) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int c = wn * (32 * TN) + j * 32 + lane;
                const int col = n0 + c;
                if (col < d.N) {
                    d.bwd_ws[part_idx(0, col, blk, d.N, d.M)] = RED(0, 0, c) + RED(1, 0, c);
                    d.bwd_ws[part_idx(1, col, blk, d.N, d.M)] = RED(0, 1, c) + RED(1, 1, c);
                }
            }
        }
        URED_TS_MARK(d, 11);
    }
}
#undef RED
#undef REDI

// ---- the kernel ---------------------------------------------------------------
// Double-buffered LDS: tile t+1 is loaded to registers before the MFMAs of tile t and
// written to the other buffer after them; one barrier per K-tile.
template <bool A_KM, bool B_KM, int PRO_A, int PRO_B, int EPI, bool VEC>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(const UredGemmDesc d) {
    constexpr int LDA = Pad<A_KM>::v, LDB = Pad<B_KM>::v;
    constexpr int SA = BK * LDA, SB = BK * LDB;
    __shared__ __attribute__((aligned(16))) float smem[2 * (SA + SB)];
    __shared__ float red_f[4 * BN];       // [wm][quantity][col] cross-wave reductions
    __shared__ int red_i[4 * BN];

    const int ntm = (d.M + BM - 1) / BM, ntn = (d.N + BN - 1) / BN;
    const int tile = xcd_remap(blockIdx.x, ntm * ntn);
    const int tm_ = tile / ntn, tn_ = tile % ntn;
    const int m0 = tm_ * BM, n0 = tn_ * BN;
    int kbeg = 0, kend = d.K;
    if (EPI == URED_EPI_SPLITK) {
        const int kps = ((d.K + d.splits - 1) / d.splits + BK - 1) / BK * BK;
        kbeg = blockIdx.z * kps;
        kend = min(d.K, kbeg + kps);
    }
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w & 1, wn = w >> 1;

    f16v acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    RowTile ra, rb;
    auto load = [&](int k0) {
        if constexpr (A_KM) load_kmajor<PRO_A, VEC>(ra, d.A, d.lda, d.M, m0, kend, k0, d.pro_s, d.pro_t);
        else load_rowmajor<PRO_A, VEC>(ra, d.A, d.lda, d.M, m0, kend, k0, d.A2, d.lda2, d.k1, d.pro_s, d.pro_t);
        if constexpr (B_KM) load_kmajor<PRO_B, VEC>(rb, d.B, d.ldb, d.N, n0, kend, k0, d.pro_s, d.pro_t);
        else load_rowmajor<URED_PRO_NONE, VEC>(rb, d.B, d.ldb, d.N, n0, kend, k0, d.B, 0, 0x7fffffff, nullptr, nullptr);
    };
    auto stage = [&](int buf) {
        float* As = smem + buf * (SA + SB);
        float* Bs = As + SA;
        if constexpr (A_KM) store_kmajor<LDA, PRO_A>(ra, As); else store_rowmajor<LDA, PRO_A>(ra, As);
        if constexpr (B_KM) store_kmajor<LDB, PRO_B>(rb, Bs); else store_rowmajor<LDB, URED_PRO_NONE>(rb, Bs);
    };

    if (kbeg < kend) {
        load(kbeg);
        stage(0);
        __syncthreads();
        int buf = 0;
        for (int k0 = kbeg; k0 < kend; k0 += BK) {
            const bool more = k0 + BK < kend;
            if (more) load(k0 + BK);   // global loads in flight under this tile's MFMAs
            const float* As = smem + buf * (SA + SB);
            const float* Bs = As + SA;
            const float* ap = As + (lane >> 5) * LDA + wm * 64 + (lane & 31);
            const float* bp = Bs + (lane >> 5) * LDB + wn * 64 + (lane & 31);
#pragma unroll
            for (int kk = 0; kk < BK / 2; ++kk) {
                const float a0 = ap[2 * kk * LDA], a1 = ap[2 * kk * LDA + 32];
                const float b0 = bp[2 * kk * LDB], b1 = bp[2 * kk * LDB + 32];
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
            }
            if (more) stage(buf ^ 1);   // the other buffer's last readers finished before the previous barrier
            __syncthreads();
            buf ^= 1;
        }
    }

    epilogue<EPI>(d, acc, m0, n0, red_f, red_i);
}


// ---- v2: LDS-DMA staged, persistent kernel (all-VEC shapes) ---------------------
// Both operands reach LDS by buffer_load_dwordx4 ... lds (no VGPR round trip, no staging
// registers): a row-major [rows][k] operand lands as a [128][32] image with its 16-B
// slots XOR-swizzled by ((row >> 1) & 7) and is read 4 consecutive k per ds_read_b128 (that
// swizzle keeps each of ds_read_b128's four 16-lane bank groups, lanes {0-3,12-15,20-27},
// {4-11,16-19,28-31} and their +32 twins, on 16 distinct 16-B slots: conflict-free; the
// plain (row & 7) swizzle put two lanes of a group on one slot); a k-major
// [k][cols] operand lands as a plain [32][128] image and is read with ds_read_b32.
// The MFMA k-order is permuted (k-step j of lane half h uses k = 16h + j) so both image
// kinds feed the same 32x32x2 sequence. The previous layer's BatchNorm+ReLU prologue is
// applied to the fragments after the LDS read (one fma+max per operand element, hidden
// under the 64-cycle MFMAs). Two LDS stages, the next K-step's DMA in flight during the
// current step's MFMAs, one barrier per K-step; one output tile per block (two resident per CU).
typedef __attribute__((address_space(3))) void lds_void_t;

// 1024 16-B chunks per 128x32 operand image; wave w issues chunks [w*256, w*256+256) as 4
// buffer-descriptor DMAs (operands < 2 GiB). Row-major: chunk c = (row r = c>>3, slot
// p = c&7) reads k = 4*(p ^ ((r>>1)&7)) (the XOR swizzle is on the source address, the LDS image
// stays lane-linear); k-major: chunk c = (k = c>>5, 4 columns at 4*(c&31)). The per-lane
// byte offsets are computed once per tile; a K-step only adds its k offset. Lanes whose row (row-major) or
// column (k-major) is outside the operand get an offset past num_records, and so does any
// k >= K row of a k-major operand: the hardware returns zeros for them.
constexpr unsigned BUF_OOB = 0x80000000u;
constexpr int PRO_LDS = 1024;            // max prologue channels staged in LDS by gemm2
// 64-wide block tiles for the narrow layers (gemm2_kernel TM / TN); 0 = 128 x 128 everywhere
#ifndef URED_GEMM_NARROW
#define URED_GEMM_NARROW 1
#endif
// Where a K-step issues the next step's LDS-DMA: 0 = before its fragment reads, 1 = in two
// halves between MFMA groups (rounds 3-4), 2 = right behind its fragment reads, ahead of every
// MFMA (round 5 default: DESIGN.md, "The multi-process fault"; 0.9 % of the step vs 1)
#ifndef URED_DMA_SPREAD
#define URED_DMA_SPREAD 2
#endif
constexpr int BUF_DWORD3 = 0x00020000;   // raw buffer, gfx9 family (gfx950)
#ifndef URED_EXP_DGRAD_PRO
#define URED_EXP_DGRAD_PRO 0
#endif

__host__ __device__ inline bool buf_ok(const UredGemmDesc& d) {
    // a concatenated second A source must start on a K-step boundary (one descriptor per step)
    const bool a2 = d.k1 >= d.K || (!d.a_kmajor && d.k1 % BK == 0 && d.A2 && (long long)d.M * d.lda2 * 4 < 0x7fffffffLL);
    return a2 && (long long)d.M * d.ldc * 4 < 0x7fffffffLL && (long long)d.M * d.ldy * 4 < 0x7fffffffLL &&
        (d.a_kmajor ? (long long)d.K * d.lda : (long long)d.M * d.lda) * 4 < 0x7fffffffLL &&
        (d.b_kmajor ? (long long)d.K * d.ldb : (long long)d.N * d.ldb) * 4 < 0x7fffffffLL;
}

struct BufOperand {
    __amdgpu_buffer_rsrc_t rs;   // raw buffer descriptor: base, stride 0, num_records (bytes)
    unsigned vo[4];              // per-lane byte offsets of the wave's pieces
};

// NP = EXT / 32: 16-B chunks per wave-lane of an EXT-wide operand image (EXT = 128 or 64 rows /
// columns), i.e. the number of 1-KB DMA pieces each of the 4 waves issues per image. Wave w
// issues chunks [w*NP*64, (w+1)*NP*64): row-major image chunk c = (row c>>3, slot c&7), k-major
// image chunk c = (k = c / (EXT/4), 4 columns at 4*(c % (EXT/4))).
template <bool KM, int EXT>
__device__ __forceinline__ void buf_setup(BufOperand& o, const float* G, int ld, int ext, int e0, int K, int w, int lane) {
    constexpr int NP = EXT / 32, CPR = EXT / 4;
    const long long bytes = KM ? ((long long)(K - 1) * ld + ext) * 4 : ((long long)(ext - 1) * ld + K) * 4;
    o.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(G), (short)0, (int)bytes, BUF_DWORD3);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
        const int c = (w * NP + i) * 64 + lane;
        if constexpr (!KM) {
            const int r = c >> 3, p = c & 7, sl = p ^ ((r >> 1) & 7);
            const int row = e0 + r;
            o.vo[i] = row < ext ? (unsigned)(((long long)row * ld + 4 * sl) * 4) : BUF_OOB;
        } else {
            const int kk = c / CPR, c4 = c % CPR;
            const int col = e0 + 4 * c4;
            o.vo[i] = col < ext ? (unsigned)(((long long)kk * ld + col) * 4) : BUF_OOB;
        }
    }
}

// The DMA is issued with the compiler's own LDS-DMA builtin (round 5): hipcc then sets M0
// itself, pads the SALU-M0-write -> LDS-DMA hazard, and counts every DMA in its vmcnt
// bookkeeping (cdna_hip_programming.md §5.7: "where a __builtin_amdgcn_* exists, prefer it").
// Rounds 2-4 issued it from inline asm that saved, advanced and restored M0 itself, invisible
// to the hazard recognizer and the waitcnt pass; that form was in every tree on which the
// 8-process config-5 test aborted with HSA_STATUS_ERROR_ILLEGAL_INSTRUCTION ("The
// multi-process fault"; its A/B numbers: profiles/r5a_dma_form_gemm_ab.log).
// Cross-wave completion is still ordered explicitly: each wave waits for its own DMA
// (vmcnt) before the K-loop's barrier; the compiler only sees this wave's reads.
constexpr unsigned GEMM2_SMEM_BYTES = 2u * 2u * (unsigned)(BM * BK) * 4u;   // both stages, A|B images

// One wave's NP 1-KB pieces of an operand image. smem: the stage images' LDS object; off:
// wave-uniform byte offset of this wave's first piece inside it.
template <bool KM, int NP>
__device__ __forceinline__ void buf_tile(const BufOperand& o, int ld, int k0, float* smem, unsigned off) {
    const unsigned toff = KM ? (unsigned)k0 * (unsigned)ld * 4u : (unsigned)k0 * 4u;
#if URED_DEBUG_BOUNDS
    URED_DBG_CHECK(!(off + NP * 1024u > GEMM2_SMEM_BYTES || (off & 1023u)));
#endif
    char* base = reinterpret_cast<char*>(smem) + off;
#pragma unroll
    for (int i = 0; i < NP; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(o.rs, (lds_void_t*)(base + i * 1024), 16, o.vo[i] + toff, 0, 0, 0);
}

template <int PRO>
__device__ __forceinline__ float pro_v(float x, float s, float t) {
    if (PRO == URED_PRO_ENC) return fmaxf(__builtin_fmaf(x, s, t), 0.f);
    if (PRO == URED_PRO_RES) return __builtin_fmaf(fmaxf(x, 0.f), s, t);
    return x;
}

// TM / TN: 32-row / 32-column MFMA tiles per wave (2 x 2 waves per block), so the block tile is
// (64 TM) x (64 TN): 128 x 128 for the wide layers; TN = 1 (128 x 64) for outputs of <= 64
// columns and TM = 1 (64 x ...) for split-K / store GEMMs of <= 64 output rows — the 32- and
// 64-channel layers, where a 128-wide tile spent half to three quarters of its MFMAs on zeros.
template <bool A_KM, bool B_KM, int PRO_A, int PRO_B, int EPI, int TM, int TN>
__global__ __launch_bounds__(NT, 2) void gemm2_kernel(const UredGemmDesc d) {
    static_assert(TM == 2 || EPI == URED_EPI_SPLITK || EPI == URED_EPI_STORE,
                  "64-row tiles only for epilogues without 128-row block partials");
    constexpr int TILE = BM * BK;                  // floats per (largest) operand image
    constexpr int BMT = 64 * TM, BNT = 64 * TN;    // this instance's block tile
    constexpr int NPA = BMT / 32, NPB = BNT / 32;  // 1-KB DMA pieces per wave and image
    // row-major A with a prologue: the per-channel scale/shift vectors (k < k1 <= PRO_LDS)
    // are staged in LDS once, so a tile reads them with broadcast ds_reads instead of
    // waiting on global (L2) latency every K-step
    constexpr bool PRO_IN_LDS = !A_KM && PRO_A != URED_PRO_NONE;
    // Separate __shared__ objects: the compiler can then prove the epilogue scratch and the
    // prologue vectors disjoint from the DMA stages (no vmcnt(0) in front of their ds_reads).
    __shared__ __attribute__((aligned(16))) float smem[2 * 2 * TILE];
    __shared__ float red_f[4 * BN];
    __shared__ int red_i[4 * BN];
    __shared__ __attribute__((aligned(16))) float pro_lds[PRO_IN_LDS ? 2 * PRO_LDS : 4];   // scale | shift

    const int ntm = (d.M + BMT - 1) / BMT, ntn = (d.N + BNT - 1) / BNT;
    const int ntiles = ntm * ntn;
    int kbeg = 0, kend = d.K;
    if (EPI == URED_EPI_SPLITK) {
        const int kps = ((d.K + d.splits - 1) / d.splits + BK - 1) / BK * BK;
        kbeg = blockIdx.z * kps;
        kend = min(d.K, kbeg + kps);
    }
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w & 1, wn = w >> 1;
    const int h = lane >> 5, li = lane & 31;

    // one output tile per block: tile blockIdx.x -> xcd_remap (blocks sharing an A panel on one XCD)
    if ((int)blockIdx.x >= ntiles) return;
#if URED_GEMM_TIMING
    const bool ts_on = EPI == URED_EPI_BNBWD && d.M == URED_TS_M && d.N == URED_TS_N && d.K == URED_TS_K &&
                       blockIdx.x < TS_SLOTS;
    unsigned long long ts_[4];
    ts_[0] = __builtin_amdgcn_s_memrealtime();
#endif
    int m0, n0;
    {
        const int tl = xcd_remap(blockIdx.x, ntiles);
        m0 = (tl / ntn) * BMT;
        n0 = (tl % ntn) * BNT;
    }

    // Operands reach LDS by buffer-descriptor DMA (launch() guarantees buf_ok): a
    // concatenated second A source [M][K-k1] (k1 % BK == 0) gets its own descriptor, chosen
    // per K-step.
    const bool has_a2 = !A_KM && d.k1 < d.K;
    BufOperand ba, ba2, bb;
    // a k-major operand's rows past kend must read as zero too (split-K: kend < K)
    buf_setup<A_KM, BMT>(ba, d.A, d.lda, d.M, m0, A_KM ? kend : min(kend, d.k1), w, lane);
    if (!A_KM && has_a2) buf_setup<false, BMT>(ba2, d.A2, d.lda2, d.M, m0, d.K - d.k1, w, lane);
    buf_setup<B_KM, BNT>(bb, d.B, d.ldb, d.N, n0, kend, w, lane);
    // this wave's first piece in the A / B images, wave-uniform (SGPR)
    const unsigned wu = (unsigned)__builtin_amdgcn_readfirstlane(w);
    const unsigned lds_a = wu * (NPA * 1024u), lds_b = TILE * 4u + wu * (NPB * 1024u);
    auto issue_a = [&](int stage, int k0) {
        const unsigned la = lds_a + (unsigned)stage * (2u * TILE * 4u);
        if (!A_KM && has_a2 && k0 >= d.k1) buf_tile<false, NPA>(ba2, d.lda2, k0 - d.k1, smem, la);
        else buf_tile<A_KM, NPA>(ba, d.lda, k0, smem, la);
    };
    auto issue_b = [&](int stage, int k0) {
        buf_tile<B_KM, NPB>(bb, d.ldb, k0, smem, lds_b + (unsigned)stage * (2u * TILE * 4u));
    };

    if constexpr (PRO_IN_LDS) {   // visible after the first loop barrier
        for (int i = t; i < d.k1; i += NT) { pro_lds[i] = d.pro_s[i]; pro_lds[PRO_LDS + i] = d.pro_t[i]; }
    }
    int stage = 0;
    // a reduction of exactly two K-steps (the 64-channel layers' K = 64) gets both stages'
    // DMA up front: one memory round trip in front of the MFMAs instead of two
    const bool both = kend - kbeg > BK && kend - kbeg <= 2 * BK;
    if (kbeg < kend) { issue_a(0, kbeg); issue_b(0, kbeg); }
    if (both) { issue_a(1, kbeg + BK); issue_b(1, kbeg + BK); }

    f16v acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    // k-major B with prologue (wgrad): the channel is this lane's output column, fixed
    float bs_[2] = {1.f, 1.f}, bt_[2] = {0.f, 0.f};
    if (PRO_B != URED_PRO_NONE) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            int c = n0 + wn * (32 * TN) + j * 32 + li;
            c = c < d.N ? c : d.N - 1;
            bs_[j] = d.pro_s[c]; bt_[j] = d.pro_t[c];
        }
        // Re-define the loaded values through an asm so the compiler's wait for these loads
        // sits here, once, and not inside the K-loop.
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(bs_[0]), "+v"(bs_[1]), "+v"(bt_[0]), "+v"(bt_[1]));
    }

    for (int k0 = kbeg; k0 < kend; k0 += BK) {
        // this wave's share of the step's DMA must have landed before the barrier (with both
        // stages in flight, the first step waits only for stage 0's pieces: vmcnt counts in order)
        if (both && k0 == kbeg) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NPA + NPB) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
#if URED_GEMM_TIMING
        if (k0 == kbeg) ts_[1] = __builtin_amdgcn_s_memrealtime();
#endif
        const float* As = smem + stage * 2 * TILE;
        const float* Bs = As + TILE;
        const bool tail = k0 + BK > kend;
        // next step's DMA goes into the other stage (its last readers passed the barrier
        // above); URED_DMA_SPREAD picks the issue point (see its definition)
        const bool next = k0 + BK < kend && !both;
        if (URED_DMA_SPREAD == 0 && next) { issue_a(stage ^ 1, k0 + BK); issue_b(stage ^ 1, k0 + BK); }

        // the prologue's scale/shift first: LDS reads complete in issue order, so the
        // prologue (and the MFMAs behind it) can start on the first A fragments
        float ss[16], tt[16];
        // k1 (start of the raw concatenated A2) is a multiple of BK when A2 is present
        // (buf_ok), so "this K-step needs the prologue" is wave-uniform: a scalar branch
        // instead of a per-element select
        const bool pro_step = PRO_IN_LDS && k0 < d.k1;
        if (pro_step) {
            const int kc = min(k0 + 16 * h, d.k1 - 16);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 sv = *reinterpret_cast<const float4*>(pro_lds + kc + 4 * q);
                const float4 tv = *reinterpret_cast<const float4*>(pro_lds + PRO_LDS + kc + 4 * q);
                ss[4 * q] = sv.x; ss[4 * q + 1] = sv.y; ss[4 * q + 2] = sv.z; ss[4 * q + 3] = sv.w;
                tt[4 * q] = tv.x; tt[4 * q + 1] = tv.y; tt[4 * q + 2] = tv.z; tt[4 * q + 3] = tv.w;
            }
        }
        // ---- fragments LDS -> VGPR: a[tm][j], b[tn][j] for k = k0 + 16h + j
        float a[2][16], b[2][16];
        if constexpr (!A_KM) {
#pragma unroll
            for (int tm = 0; tm < TM; ++tm) {
                const int r = wm * (32 * TM) + tm * 32 + li;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 v4 = *reinterpret_cast<const float4*>(As + r * 32 + 4 * ((4 * h + q) ^ ((r >> 1) & 7)));
                    a[tm][4 * q] = v4.x; a[tm][4 * q + 1] = v4.y; a[tm][4 * q + 2] = v4.z; a[tm][4 * q + 3] = v4.w;
                }
            }
        } else {
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int j = 0; j < 16; ++j) a[tm][j] = As[(16 * h + j) * BMT + wm * (32 * TM) + tm * 32 + li];
        }
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) {
            const int cidx = wn * (32 * TN) + tn * 32 + li;
            if constexpr (!B_KM) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 v4 = *reinterpret_cast<const float4*>(Bs + cidx * 32 + 4 * ((4 * h + q) ^ ((cidx >> 1) & 7)));
                    b[tn][4 * q] = v4.x; b[tn][4 * q + 1] = v4.y; b[tn][4 * q + 2] = v4.z; b[tn][4 * q + 3] = v4.w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 16; ++j) b[tn][j] = Bs[(16 * h + j) * BNT + cidx];
            }
        }

        // URED_DMA_SPREAD == 2: the next step's DMA right behind this step's fragment reads, in
        // front of every MFMA (the fence keeps the scheduler from sinking it among them)
        if (URED_DMA_SPREAD == 2 && next) {
            issue_a(stage ^ 1, k0 + BK);
            issue_b(stage ^ 1, k0 + BK);
            __builtin_amdgcn_sched_barrier(0);
        }
        // ---- prologues (previous layer's BN+ReLU) and the K tail, on the fragments
        if constexpr (!A_KM && PRO_A != URED_PRO_NONE) {
            if (pro_step) {
                // scalar v_fma_f32 + v_max_f32: beside MFMAs a packed v_pk_fma_f32 costs more
                // issue time than two plain fmas (MI355X_MICROARCH.md, filler prices)
#pragma unroll
                for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                    for (int j = 0; j < 16; ++j) a[tm][j] = pro_v<PRO_A>(a[tm][j], ss[j], tt[j]);
            }
        }
        if constexpr (B_KM && PRO_B != URED_PRO_NONE) {
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
#pragma unroll
                for (int j = 0; j < 16; ++j) b[tn][j] = pro_v<PRO_B>(b[tn][j], bs_[tn], bt_[tn]);
        }
        if (tail) {   // zero the k >= K part of the reduction (the images hold clamped copies)
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int j = 0; j < 16; ++j) a[tm][j] = (k0 + 16 * h + j < kend) ? a[tm][j] : 0.f;
        }
        // ---- MFMAs. s_setprio(1) around the cluster keeps hipcc from moving MFMAs out of it, in
        // among the next step's loads (cdna_hip_programming.md T5): forward, wgrad and store
        // variants +1-2 % isolated (tools/ab_libs_step.sh, same box, two rounds); the BN-backward
        // dgrad went -1..+1 %, so it keeps the plain schedule
        constexpr bool PRIO = EPI != URED_EPI_BNBWD;
        // URED_DMA_SPREAD == 1: MFMA group (of 16) behind which the next step's A / B halves are
        // issued: 6 / 11 with a k-major B, 1 / 5 with a row-major B (profiles/r4zh_*)
        constexpr int DMA_JA = B_KM ? 6 : 1, DMA_JB = B_KM ? 11 : 5;
        if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
#pragma unroll
            for (int tm = 0; tm < TM; ++tm)
#pragma unroll
                for (int tn = 0; tn < TN; ++tn)
                    acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[tm][j], b[tn][j], acc[tm][tn], 0, 0, 0);
            if (URED_DMA_SPREAD == 1 && next && j == DMA_JA) issue_a(stage ^ 1, k0 + BK);
            if (URED_DMA_SPREAD == 1 && next && j == DMA_JB) issue_b(stage ^ 1, k0 + BK);
        }
        if (PRIO) __builtin_amdgcn_s_setprio(0);
        stage ^= 1;
    }

#if URED_GEMM_TIMING
    ts_[2] = __builtin_amdgcn_s_memrealtime();
#endif
    epilogue<EPI, true, TM, TN>(d, acc, m0, n0, red_f, red_i);
#if URED_GEMM_TIMING
    if (ts_on) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ts_[3] = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) {
            unsigned long long* o = ured_ts_buf + (size_t)blockIdx.x * 16;
            o[0] = ts_[0]; o[1] = ts_[1]; o[2] = ts_[2]; o[3] = ts_[3];
            o[4] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
            o[5] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
            o[6] = (unsigned long long)m0 << 32 | (unsigned)n0;
            o[7] = 1;
        }
    }
#endif
}

// ---- small kernels -------------------------------------------------------------

// out[m][n] (+)= sum_z ws[z][m][n]. Block = 64 consecutive elements x nw waves (nw = blockDim/64,
// up to 16, chosen by the launcher from the split count); wave w sums splits w, w+nw, ... with
// eight loads in flight; fixed combine order (deterministic). Many of these reductions are
// short (a few thousand outputs over 8-128 splits): latency chains, hence the width.
__global__ __launch_bounds__(1024) void splitk_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N,
                                                             float* __restrict__ out, int ldo, int accumulate,
                                                             const float* __restrict__ bias) {
    __shared__ float part[16][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const size_t total = (size_t)M * N;
    const size_t e = (size_t)blockIdx.x * 64 + lane;
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (e < total) {
        int z = w;
        for (; z + 7 * nw < splits; z += 8 * nw) {
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = ws[(size_t)(z + i * nw) * total + e];
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] += v[i];
        }
        for (; z < splits; z += nw) a[0] += ws[(size_t)z * total + e];
    }
    part[w][lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    __syncthreads();
    if (w == 0 && e < total) {
        const int m = (int)(e / N), n = (int)(e % N);
        float sum = part[0][lane];
        for (int q = 1; q < nw; ++q) sum += part[q][lane];
        if (bias) sum += bias[n];
        float* o = out + (size_t)m * ldo + n;
        *o = accumulate ? *o + sum : sum;
    }
}

// ---- skinny weight gradient: out[co][ki] (+)= sum_m dY[m][co] * pro(X[m][ki]) for the edge layers
// where min(Cout, Kin) <= 4 (3-channel inputs / outputs): a 128x128 MFMA tile would be almost all
// padding, so this is a streaming reduction. The wide side D is spread over tpr = D/VEC threads
// (float4 loads when aligned), 256/tpr rows go at once, SK_UNROLL rows per thread in flight; each
// of <= SK_MAX_BLOCKS row blocks combines its lanes in LDS in a fixed order and writes one partial,
// then skinny_reduce_kernel sums the partials of each output in a fixed tree (deterministic).
constexpr int SK_MAX_BLOCKS = 256, SK_UNROLL = 4;

template <int PRO, bool SMALL_IS_OUT, int S, int VEC>
__global__ __launch_bounds__(256) void wgrad_skinny_kernel(const float* __restrict__ dY, int ldd,
        const float* __restrict__ X, int ldx, int D, int M, int rows_per_block, const float* __restrict__ ps,
        const float* __restrict__ pt, float* __restrict__ ws) {
    __shared__ float red[256 * VEC * S];
    const int tpr = D / VEC;
    const int t = threadIdx.x, jv = t % tpr, lane = t / tpr, lanes = 256 / tpr;
    const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
    float acc[VEC][S];
#pragma unroll
    for (int v = 0; v < VEC; ++v)
#pragma unroll
        for (int q = 0; q < S; ++q) acc[v][q] = 0.f;
    float bs[VEC], bt[VEC], ss[S], st[S];     // prologue scale/shift of the X side
#pragma unroll
    for (int v = 0; v < VEC; ++v) {
        bs[v] = (PRO != URED_PRO_NONE && SMALL_IS_OUT) ? ps[jv * VEC + v] : 0.f;
        bt[v] = (PRO != URED_PRO_NONE && SMALL_IS_OUT) ? pt[jv * VEC + v] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < S; ++q) {
        ss[q] = (PRO != URED_PRO_NONE && !SMALL_IS_OUT) ? ps[q] : 0.f;
        st[q] = (PRO != URED_PRO_NONE && !SMALL_IS_OUT) ? pt[q] : 0.f;
    }
    auto load = [&](int m, float (&big)[VEC], float (&small)[S]) {
        const float* bp = SMALL_IS_OUT ? X + (size_t)m * ldx + jv * VEC : dY + (size_t)m * ldd + jv * VEC;
        if constexpr (VEC == 4) {
            const float4 f = *reinterpret_cast<const float4*>(bp);
            big[0] = f.x; big[1] = f.y; big[2] = f.z; big[3] = f.w;
        } else {
            big[0] = bp[0];
        }
        const float* sp = SMALL_IS_OUT ? dY + (size_t)m * ldd : X + (size_t)m * ldx;
#pragma unroll
        for (int q = 0; q < S; ++q) small[q] = sp[q];
    };
    auto accum = [&](float (&big)[VEC], float (&small)[S]) {
#pragma unroll
        for (int v = 0; v < VEC; ++v) {
            const float bv = SMALL_IS_OUT ? pro_v<PRO>(big[v], bs[v], bt[v]) : big[v];
#pragma unroll
            for (int q = 0; q < S; ++q) {
                const float sv = SMALL_IS_OUT ? small[q] : pro_v<PRO>(small[q], ss[q], st[q]);
                acc[v][q] = __builtin_fmaf(sv, bv, acc[v][q]);
            }
        }
    };
    if (lane < lanes) {
        int m = r0 + lane;
        for (; m + (SK_UNROLL - 1) * lanes < r1; m += SK_UNROLL * lanes) {
            float big[SK_UNROLL][VEC], small[SK_UNROLL][S];
#pragma unroll
            for (int u = 0; u < SK_UNROLL; ++u) load(m + u * lanes, big[u], small[u]);
#pragma unroll
            for (int u = 0; u < SK_UNROLL; ++u) accum(big[u], small[u]);
        }
        for (; m < r1; m += lanes) {
            float big[VEC], small[S];
            load(m, big, small);
            accum(big, small);
        }
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v)
#pragma unroll
        for (int q = 0; q < S; ++q) red[(t * VEC + v) * S + q] = acc[v][q];
    __syncthreads();
    if (lane != 0) return;
    for (int l = 1; l < lanes; ++l)
#pragma unroll
        for (int v = 0; v < VEC; ++v)
#pragma unroll
            for (int q = 0; q < S; ++q) acc[v][q] += red[((l * tpr + jv) * VEC + v) * S + q];
    float* w = ws + (size_t)blockIdx.x * D * S;
#pragma unroll
    for (int v = 0; v < VEC; ++v)
#pragma unroll
        for (int q = 0; q < S; ++q) {
            const int j = jv * VEC + v;
            w[SMALL_IS_OUT ? q * D + j : j * S + q] = acc[v][q];       // [Cout][Kin] per block
        }
}

// one block per output element: the row-block partials in a fixed tree order
__global__ __launch_bounds__(256) void skinny_reduce_kernel(const float* __restrict__ ws, int nb, int total, int N,
                                                            float* __restrict__ out, int ldo, int accumulate) {
    __shared__ float red[256];
    const int e = blockIdx.x, t = threadIdx.x;
    float a = 0.f;
    for (int z = t; z < nb; z += 256) a += ws[(size_t)z * total + e];
    red[t] = a;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (t < h) red[t] += red[t + h];
        __syncthreads();
    }
    if (t == 0) {
        float* o = out + (size_t)(e / N) * ldo + e % N;
        *o = accumulate ? *o + red[0] : red[0];
    }
}

// one block (256 threads) per column; fp64 fixed-order tree reductions
// Row multiplicities (unique-row training, see DESIGN "unique source encoding"): when gw is
// non-null, every row of group g = row / grows stands for gw[g] identical rows of the full
// batch. grows is a multiple of BM, so a partial block has one weight: its count scales by w,
// its M2 by w, its mean is unchanged (Chan merge with weighted counts).
__device__ __forceinline__ double blk_weight(const float* gw, int grows, int b) {
    return gw ? (double)gw[(b * BM) / grows] : 1.0;
}

__global__ __launch_bounds__(256) void bn_fwd_finalize_kernel(const float* __restrict__ ws, int M, int N,
        const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
        float* running_mean, float* running_var, float* mean_o, float* invstd_o, float* scale_o, float* shift_o,
        const float* __restrict__ gw, int grows, long long* nbt) {
    __shared__ double sh[256], shc[256];
    const int n = blockIdx.x, t = threadIdx.x;
    if (nbt && n == 0 && t == 0) *nbt += 1;
    const int nblk = (M + BM - 1) / BM;
    double s = 0.0, c = 0.0;
    for (int b = t; b < nblk; b += 256) {
        const double cnt = (double)min(BM, M - b * BM) * blk_weight(gw, grows, b);
        s += cnt * (double)ws[part_idx(0, n, b, N, M)];
        c += cnt;
    }
    sh[t] = s;
    shc[t] = c;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) { if (t < o) { sh[t] += sh[t + o]; shc[t] += shc[t + o]; } __syncthreads(); }
    const double Mw = shc[0];
    const double mean = sh[0] / Mw;
    __syncthreads();
    double q = 0.0;
    for (int b = t; b < nblk; b += 256) {
        const double w = blk_weight(gw, grows, b);
        const double cnt = (double)min(BM, M - b * BM) * w;
        const double dm = (double)ws[part_idx(0, n, b, N, M)] - mean;
        q += w * (double)ws[part_idx(1, n, b, N, M)] + cnt * dm * dm;
    }
    sh[t] = q;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) { if (t < o) sh[t] += sh[t + o]; __syncthreads(); }
    if (t == 0) {
        const double m2 = sh[0];
        const double var = m2 / Mw;
        const float is = (float)(1.0 / sqrt(var + (double)eps));
        const float mf = (float)mean;
        mean_o[n] = mf;
        invstd_o[n] = is;
        const float sc = gamma ? gamma[n] * is : is;
        scale_o[n] = sc;
        shift_o[n] = (beta ? beta[n] : 0.f) - mf * sc;
        if (running_mean) running_mean[n] = (1.f - momentum) * running_mean[n] + momentum * mf;
        if (running_var) {
            const float uv = (float)(Mw > 1.0 ? m2 / (Mw - 1.0) : m2);
            running_var[n] = (1.f - momentum) * running_var[n] + momentum * uv;
        }
    }
}

__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ ws, int M, int N,
        const float* __restrict__ gamma, const float* __restrict__ invstd, float* dgamma, float* dbeta, int accumulate,
        float* ca, float* cb, float* cc, const float* __restrict__ gw, int grows) {
    // the partials are sums over stored rows of the (already multiplicity-summed) gradient, so
    // only the batch size M becomes the weighted row count
    __shared__ double s1[256], s2[256], s3[256];
    const int n = blockIdx.x, t = threadIdx.x;
    const int nblk = (M + BM - 1) / BM;
    double a = 0.0, b = 0.0, c = 0.0;
    for (int k = t; k < nblk; k += 256) {
        a += (double)ws[part_idx(0, n, k, N, M)];
        b += (double)ws[part_idx(1, n, k, N, M)];
        c += (double)min(BM, M - k * BM) * blk_weight(gw, grows, k);
    }
    s1[t] = a; s2[t] = b; s3[t] = c;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) { s1[t] += s1[t + o]; s2[t] += s2[t + o]; s3[t] += s3[t + o]; }
        __syncthreads();
    }
    if (t == 0) {
        const double db = s1[0], dg = s2[0];
        const double Mw = s3[0];
        if (dbeta) dbeta[n] = accumulate ? dbeta[n] + (float)db : (float)db;
        if (dgamma) dgamma[n] = accumulate ? dgamma[n] + (float)dg : (float)dg;
        const double is = invstd[n];
        const double k = (gamma ? (double)gamma[n] : 1.0) * is;
        ca[n] = (float)k;
        cb[n] = (float)(-k * is * dg / Mw);
        cc[n] = (float)(-k * db / Mw);
    }
}

// rows in blocks of 128 (matches the partial layout), 256 threads = columns
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const float* __restrict__ G, const float* __restrict__ Y,
        int M, int N, int ld, int res, const float* __restrict__ mean, const float* __restrict__ ca,
        const float* __restrict__ cb, const float* __restrict__ cc, float* __restrict__ dY, float* __restrict__ colsum,
        const float* __restrict__ gw, int grows) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    const int blk = blockIdx.y;
    if (n >= N) return;
    const int r0 = blk * BM, r1 = min(M, r0 + BM);
    // a stored row standing for w identical batch rows carries w times the batch-mean terms
    const float w = gw ? gw[r0 / grows] : 1.f;
    const float a = ca[n], b = cb[n] * w, c = cc[n] * w, mu = mean[n];
    float s = 0.f;
    for (int r = r0; r < r1; ++r) {
        const size_t e = (size_t)r * ld + n;
        const float y = Y[e];
        const float p = res ? fmaxf(y, 0.f) : y;
        float v = __builtin_fmaf(a, G[e], __builtin_fmaf(b, p - mu, c));
        if (res && !(y > 0.f)) v = 0.f;
        dY[e] = v;
        s += v;
    }
    if (colsum) colsum[(size_t)blk * N + n] = s;
}

// float4 form (N, ld multiples of 4, 16-B aligned bases): a block covers one 128-row partial
// block x 64 columns with 512 threads = 16 column quads x 32 row lanes, so each lane has its 4
// rows' loads in flight at once and narrow layers (N = 64) keep every lane busy; wave loads are
// 4 rows x 256 B contiguous. The 32 row lanes' column sums combine in LDS in a fixed order.
constexpr int BBA_CQ = 16, BBA_RL = 32;
__global__ __launch_bounds__(BBA_CQ * BBA_RL) void bn_bwd_apply4_kernel(const float* __restrict__ G,
        const float* __restrict__ Y, int M, int N, int ld, int res, const float* __restrict__ mean,
        const float* __restrict__ ca, const float* __restrict__ cb, const float* __restrict__ cc,
        float* __restrict__ dY, float* __restrict__ colsum, const float* __restrict__ gw, int grows) {
    __shared__ float4 part[BBA_RL][BBA_CQ];
    const int tx = threadIdx.x % BBA_CQ, ty = threadIdx.x / BBA_CQ;
    const int n = (blockIdx.x * BBA_CQ + tx) * 4;
    const int blk = blockIdx.y;
    const bool nv = n < N;
    const int nn = nv ? n : 0;
    const int r0 = blk * BM, r1 = min(M, r0 + BM);
    const float w = gw ? gw[r0 / grows] : 1.f;   // row multiplicity (see bn_bwd_apply_kernel)
    const float4 a = *reinterpret_cast<const float4*>(ca + nn);
    float4 b = *reinterpret_cast<const float4*>(cb + nn), c = *reinterpret_cast<const float4*>(cc + nn);
    b.x *= w; b.y *= w; b.z *= w; b.w *= w;
    c.x *= w; c.y *= w; c.z *= w; c.w *= w;
    const float4 mu = *reinterpret_cast<const float4*>(mean + nn);
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    auto one = [&](float y, float g, float av, float bv, float cv, float m) {
        const float p = res ? fmaxf(y, 0.f) : y;
        float v = __builtin_fmaf(av, g, __builtin_fmaf(bv, p - m, cv));
        return (res && !(y > 0.f)) ? 0.f : v;
    };
    if (nv) {
        constexpr int RPL = BM / BBA_RL;
        float4 y[RPL], g[RPL];
#pragma unroll
        for (int i = 0; i < RPL; ++i) {
            const int r = r0 + ty + i * BBA_RL;
            if (r < r1) {
                const size_t e = (size_t)r * ld + n;
                y[i] = *reinterpret_cast<const float4*>(Y + e);
                g[i] = *reinterpret_cast<const float4*>(G + e);
            }
        }
#pragma unroll
        for (int i = 0; i < RPL; ++i) {
            const int r = r0 + ty + i * BBA_RL;
            if (r < r1) {
                float4 v;
                v.x = one(y[i].x, g[i].x, a.x, b.x, c.x, mu.x);
                v.y = one(y[i].y, g[i].y, a.y, b.y, c.y, mu.y);
                v.z = one(y[i].z, g[i].z, a.z, b.z, c.z, mu.z);
                v.w = one(y[i].w, g[i].w, a.w, b.w, c.w, mu.w);
                *reinterpret_cast<float4*>(dY + (size_t)r * ld + n) = v;
                s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            }
        }
    }
    if (!colsum) return;
    part[ty][tx] = s;
    __syncthreads();
    if (ty == 0 && nv) {
        float4 t = part[0][tx];
        for (int q = 1; q < BBA_RL; ++q) {
            const float4 u = part[q][tx];
            t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
        }
        *reinterpret_cast<float4*>(colsum + (size_t)blk * N + n) = t;
    }
}

__global__ __launch_bounds__(256) void pool_finalize_kernel(const float* __restrict__ ws, int M, int N, int group_rows,
        const float* __restrict__ scale, const float* __restrict__ shift, int relu, float* pooled, int* argidx) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    const int g = blockIdx.y;
    if (n >= N) return;
    const int bpg = group_rows / BM;
    const float sc = scale[n], sh = shift[n];
    const bool up = sc >= 0.f;    // (relu of) sc*y+sh is non-decreasing in y iff sc >= 0
    float best = up ? -__builtin_inff() : __builtin_inff();
    int bi = 0x7fffffff;
    for (int b = g * bpg; b < (g + 1) * bpg && b * BM < M; ++b) {
        const float* pw = ws + (size_t)b * 4 * N;
        const float v = up ? pw[n] : pw[2 * N + n];
        const int vi = reinterpret_cast<const int*>(pw)[(up ? 1 : 3) * N + n];
        if ((up ? v > best : v < best) || (v == best && vi < bi)) { best = v; bi = vi; }
    }
    const float pv = __builtin_fmaf(best, sc, sh);
    pooled[(size_t)g * N + n] = relu ? fmaxf(pv, 0.f) : pv;
    argidx[(size_t)g * N + n] = bi;
}

// general max-pool (any group size): per (group, column) scan of the raw layer output
__global__ __launch_bounds__(256) void pool_rows_kernel(const float* __restrict__ Y, int N, int group_rows,
        const float* __restrict__ scale, const float* __restrict__ shift, int relu, float* pooled, int* argidx) {
    const int n = blockIdx.x * 256 + threadIdx.x;
    const int g = blockIdx.y;
    if (n >= N) return;
    const float sc = scale[n], sh = shift[n];
    const bool up = sc >= 0.f;
    float best = up ? -__builtin_inff() : __builtin_inff();
    int bi = g * group_rows;
    for (int r = g * group_rows; r < (g + 1) * group_rows; ++r) {
        const float v = Y[(size_t)r * N + n];
        if (up ? v > best : v < best) { best = v; bi = r; }
    }
    const float pv = __builtin_fmaf(best, sc, sh);
    pooled[(size_t)g * N + n] = relu ? fmaxf(pv, 0.f) : pv;
    argidx[(size_t)g * N + n] = bi;
}

// out[m][n] = act(Y[m][n]*scale[n] + shift[n]) (act = relu or identity): the BatchNorm
// (+ReLU) output materialised, where a caller needs the activation itself (PointNet's
// pointfeat / feature-transform input); float4 along n when N % 4 == 0.
__global__ __launch_bounds__(256) void bn_act_kernel(const float* __restrict__ Y, int M, int N, int ldy,
        const float* __restrict__ scale, const float* __restrict__ shift, int relu, float* __restrict__ out, int ldo,
        int vec) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (vec) {
        const int n4 = N >> 2;
        if (i >= (long long)M * n4) return;
        const int m = (int)(i / n4), n = (int)(i % n4) * 4;
        const float4 y = *reinterpret_cast<const float4*>(Y + (size_t)m * ldy + n);
        const float4 s = *reinterpret_cast<const float4*>(scale + n);
        const float4 t = *reinterpret_cast<const float4*>(shift + n);
        float4 o;
        o.x = __builtin_fmaf(y.x, s.x, t.x); o.y = __builtin_fmaf(y.y, s.y, t.y);
        o.z = __builtin_fmaf(y.z, s.z, t.z); o.w = __builtin_fmaf(y.w, s.w, t.w);
        if (relu) { o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f); }
        *reinterpret_cast<float4*>(out + (size_t)m * ldo + n) = o;
    } else {
        if (i >= (long long)M * N) return;
        const int m = (int)(i / N), n = (int)(i % N);
        const float v = __builtin_fmaf(Y[(size_t)m * ldy + n], scale[n], shift[n]);
        out[(size_t)m * ldo + n] = relu ? fmaxf(v, 0.f) : v;
    }
}

// out[g][n] = sum of rows [r0, r1) of column n. Block = 16 waves x 64 columns; wave w sums
// rows r0+w, r0+w+16, ... with eight independent accumulators (a wave reads 256 contiguous
// bytes per row, 8 rows in flight per lane, 128 per column), combined in a fixed order and
// across waves in LDS: deterministic. The short sums here (the per-128-row partials of a
// BN backward, 256-512 rows) are latency chains, hence the width. blockIdx.z = split s of S:
// the group's rows are cut into S equal ranges and split s writes ws[g][s][n] (S > 1) for a
// second pass over the S partials.
constexpr int GCS_WAVES = 16;
__global__ __launch_bounds__(GCS_WAVES * 64) void group_colsum_kernel(const float* __restrict__ X, int ldx, int N,
        const int* __restrict__ off, int group_rows, float* __restrict__ out, int ldo) {
    __shared__ float part[GCS_WAVES][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int n = blockIdx.x * 64 + lane;
    const int g = blockIdx.y, S = gridDim.z, sp = blockIdx.z;
    const int g0 = off ? off[g] : g * group_rows;
    const int g1 = off ? off[g + 1] : (g + 1) * group_rows;
    const long long len = g1 - g0;
    const int r0 = g0 + (int)(len * sp / S), r1 = g0 + (int)(len * (sp + 1) / S);
    float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (n < N) {
        const float* col = X + n;
        int r = r0 + w;
        for (; r + 7 * GCS_WAVES < r1; r += 8 * GCS_WAVES) {
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = col[(size_t)(r + i * GCS_WAVES) * ldx];
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] += v[i];
        }
        for (; r < r1; r += GCS_WAVES) a[0] += col[(size_t)r * ldx];
    }
    part[w][lane] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    __syncthreads();
    if (w == 0 && n < N) {
        float v = part[0][lane];
        for (int q = 1; q < GCS_WAVES; ++q) v += part[q][lane];
        if (S == 1) out[(size_t)g * ldo + n] = v;
        else out[((size_t)g * S + sp) * N + n] = v;
    }
}

// VEC (float4 staging) needs 16-B aligned rows and contiguous extents that are multiples of 4.
bool vec_ok(const UredGemmDesc& d) {
    const bool a = (d.lda % 4 == 0) && (d.a_kmajor ? d.M % 4 == 0 : (d.K % 4 == 0 && d.k1 % 4 == 0 &&
                   (d.k1 == d.K || d.lda2 % 4 == 0)));
    const bool b = (d.ldb % 4 == 0) && (d.b_kmajor ? d.N % 4 == 0 : d.K % 4 == 0);
    const bool p = !(d.pro_a || d.pro_b) || ((reinterpret_cast<uintptr_t>(d.pro_s) | reinterpret_cast<uintptr_t>(d.pro_t)) % 16 == 0);
    const bool al = (reinterpret_cast<uintptr_t>(d.A) % 16 == 0) && (reinterpret_cast<uintptr_t>(d.B) % 16 == 0) &&
                    (d.A2 == nullptr || reinterpret_cast<uintptr_t>(d.A2) % 16 == 0);
    return a && b && p && al;
}

// v2 additionally needs the A prologue channels to come in 16-aligned runs (k1 % 16 == 0) and
// rows/extents >= 4 so clamped 16-B sources stay in bounds.
bool v2_ok(const UredGemmDesc& d) {
    if (d.pro_a && (d.k1 % 16 != 0)) return false;
    if (d.pro_a && !d.a_kmajor && d.k1 > PRO_LDS) return false;
    if (d.K < 4 || (d.a_kmajor && d.M < 4) || (d.b_kmajor && d.N < 4)) return false;
    return true;
}

// 256 threads per 128-row block (1024 measured no faster and changes the summation order)
constexpr int SMALL_NT = 256;

// ---- edge-layer dgrad + BN-backward (K <= 4: the 3-channel output layers' input gradient) ----
// dh[m][c] = sum_k dY[m][k] W[k][c] (+ gadd), then the EPI_BNBWD arithmetic of epilogue()
// (ReLU/BN mask, G store, per-128-row-block partials {sum g, sum g*xhat} in bwd_ws), as a
// streaming kernel: a 128x128 MFMA tile is ~all padding at K = 3 and N = 32/64. One block per
// 128-row block (the partial layout the finalize expects); SMALL_NT / N row groups x N columns; each
// thread keeps its W column in registers and walks its rows; fixed-order LDS combine.
template <int KS>
__global__ __launch_bounds__(SMALL_NT) void dgrad_small_bnbwd_kernel(const UredGemmDesc d) {
    __shared__ float red[2][SMALL_NT];
    const int N = d.N, rg = SMALL_NT / N, t = threadIdx.x;
    const int c = t % N, g0 = t / N;
    const int m0 = blockIdx.x * BM;
    const int mend = min(m0 + BM, d.M);
    float a1 = 0.f, a2 = 0.f;
    if (g0 < rg) {
        float w[KS];
#pragma unroll
        for (int k = 0; k < KS; ++k) w[k] = d.B[(size_t)k * d.ldb + c];
        const float sc = d.bn_scale[c], sh = d.bn_shift[c], mu = d.bn_mean[c], is = d.bn_invstd[c];
#pragma unroll 4
        for (int m = m0 + g0; m < mend; m += rg) {
            const float* a = d.A + (size_t)m * d.lda;
            float dh = 0.f;
#pragma unroll
            for (int k = 0; k < KS; ++k) dh = __builtin_fmaf(a[k], w[k], dh);
            if (d.gadd) dh += d.gadd[(size_t)m * d.ldg + c];
            const float y = d.Yp[(size_t)m * d.ldy + c];
            float g, xh;
            if (d.bwd_res == URED_ACT_RES) {
                g = dh;
                xh = (fmaxf(y, 0.f) - mu) * is;
            } else if (d.bwd_res == URED_ACT_BN) {
                g = dh;
                xh = (y - mu) * is;
            } else {
                g = (__builtin_fmaf(y, sc, sh) > 0.f) ? dh : 0.f;
                xh = (y - mu) * is;
            }
            d.C[(size_t)m * d.ldc + c] = g;
            a1 += g;
            a2 += g * xh;
        }
    }
    red[0][t] = a1;
    red[1][t] = a2;
    __syncthreads();
    if (t < N) {
        float s1 = 0.f, s2 = 0.f;
        for (int q = 0; q < rg; ++q) { s1 += red[0][q * N + t]; s2 += red[1][q * N + t]; }
        d.bwd_ws[part_idx(0, t, blockIdx.x, N, d.M)] = s1;
        d.bwd_ws[part_idx(1, t, blockIdx.x, N, d.M)] = s2;
    }
}


// ---- edge-layer forward with BN statistics (K <= 4: the xyz input layers) ----------------
// Y[m][c] = sum_k X[m][k] W[c][k] + bias[c], stored, and the EPI_FWD per-128-row-block
// partials {block mean, M2 about it} of p = (stat_relu ? relu(Y) : Y) in stat_ws, two passes
// like epilogue() (the second recomputes Y from the 12-byte rows instead of re-reading it).
template <int KS>
__global__ __launch_bounds__(SMALL_NT) void fwd_small_stats_kernel(const UredGemmDesc d) {
    __shared__ float red[SMALL_NT];
    __shared__ float cmean[256];
    const int N = d.N, rg = SMALL_NT / N, t = threadIdx.x;
    const int c = t % N, g0 = t / N;
    const int m0 = blockIdx.x * BM;
    const int mend = min(m0 + BM, d.M);
    const bool act = g0 < rg;
    float w[KS];
    float bs = 0.f;
    if (act) {
#pragma unroll
        for (int k = 0; k < KS; ++k) w[k] = d.B[(size_t)c * d.ldb + k];
        if (d.bias) bs = d.bias[c];
    }
    auto yv = [&](int m) {
        const float* a = d.A + (size_t)m * d.lda;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < KS; ++k) acc = __builtin_fmaf(a[k], w[k], acc);
        return acc + bs;
    };
    float s1 = 0.f;
    if (act) {
#pragma unroll 4
        for (int m = m0 + g0; m < mend; m += rg) {
            const float v = yv(m);
            d.C[(size_t)m * d.ldc + c] = v;
            s1 += d.stat_relu ? fmaxf(v, 0.f) : v;
        }
    }
    red[t] = s1;
    __syncthreads();
    if (t < N) {
        float sum = 0.f;
        for (int q = 0; q < rg; ++q) sum += red[q * N + t];
        cmean[t] = sum / (float)(mend - m0);
    }
    __syncthreads();
    float s2 = 0.f;
    if (act) {
        const float mu = cmean[c];
#pragma unroll 4
        for (int m = m0 + g0; m < mend; m += rg) {
            const float v = yv(m);
            const float e = (d.stat_relu ? fmaxf(v, 0.f) : v) - mu;
            s2 += e * e;
        }
    }
    red[t] = s2;
    __syncthreads();
    if (t < N) {
        float sum = 0.f;
        for (int q = 0; q < rg; ++q) sum += red[q * N + t];
        d.stat_ws[part_idx(0, t, blockIdx.x, N, d.M)] = cmean[t];
        d.stat_ws[part_idx(1, t, blockIdx.x, N, d.M)] = sum;
    }
}

bool fwd_small_ok(const UredGemmDesc& d) {
    // the kernel reads A and B raw: no prologue on either operand
    return URED_FWD_SMALL && d.epi == URED_EPI_FWD && !d.a_kmajor && !d.b_kmajor && d.pro_a == URED_PRO_NONE &&
           d.pro_b == URED_PRO_NONE && d.K >= 1 && d.K <= 4 && d.N >= 1 && d.N <= 256 && !d.pool_ws && !d.rowbias &&
           d.k1 == d.K;
}

void launch_fwd_small(const UredGemmDesc& d, hipStream_t st) {
    const dim3 grid((d.M + BM - 1) / BM);
    switch (d.K) {
        case 1: hipLaunchKernelGGL(fwd_small_stats_kernel<1>, grid, dim3(SMALL_NT), 0, st, d); break;
        case 2: hipLaunchKernelGGL(fwd_small_stats_kernel<2>, grid, dim3(SMALL_NT), 0, st, d); break;
        case 3: hipLaunchKernelGGL(fwd_small_stats_kernel<3>, grid, dim3(SMALL_NT), 0, st, d); break;
        default: hipLaunchKernelGGL(fwd_small_stats_kernel<4>, grid, dim3(SMALL_NT), 0, st, d); break;
    }
}

bool dgrad_small_ok(const UredGemmDesc& d) {
    // the kernel reads A and B raw: no prologue on either operand
    return URED_DGRAD_SMALL && d.epi == URED_EPI_BNBWD && !d.a_kmajor && d.b_kmajor && d.pro_a == URED_PRO_NONE &&
           d.pro_b == URED_PRO_NONE && d.K >= 1 && d.K <= 4 && d.N >= 1 && d.N <= 256 && !d.pool_idx && d.k1 == d.K;
}

void launch_dgrad_small(const UredGemmDesc& d, hipStream_t st) {
    const dim3 grid((d.M + BM - 1) / BM);
    switch (d.K) {
        case 1: hipLaunchKernelGGL(dgrad_small_bnbwd_kernel<1>, grid, dim3(SMALL_NT), 0, st, d); break;
        case 2: hipLaunchKernelGGL(dgrad_small_bnbwd_kernel<2>, grid, dim3(SMALL_NT), 0, st, d); break;
        case 3: hipLaunchKernelGGL(dgrad_small_bnbwd_kernel<3>, grid, dim3(SMALL_NT), 0, st, d); break;
        default: hipLaunchKernelGGL(dgrad_small_bnbwd_kernel<4>, grid, dim3(SMALL_NT), 0, st, d); break;
    }
}

template <bool A_KM, bool B_KM, int PA, int PB, int EPI>
void launch(const UredGemmDesc& d, hipStream_t st) {
    if (EPI == URED_EPI_BNBWD && dgrad_small_ok(d)) { launch_dgrad_small(d, st); return; }
    if (EPI == URED_EPI_FWD && fwd_small_ok(d)) { launch_fwd_small(d, st); return; }
    const int ntm = (d.M + BM - 1) / BM, ntn = (d.N + BN - 1) / BN;
    dim3 grid(ntm * ntn, 1, EPI == URED_EPI_SPLITK ? d.splits : 1);
    if (vec_ok(d) && v2_ok(d) && buf_ok(d)) {
        // narrow tiles for outputs of <= 64 columns (and, split-K / store only, <= 64 rows)
        constexpr bool NARROW_M = EPI == URED_EPI_SPLITK || EPI == URED_EPI_STORE;
        const bool tn1 = URED_GEMM_NARROW && d.N <= 64;
        const bool tm1 = URED_GEMM_NARROW && NARROW_M && d.M <= 64;
        grid.x = ((d.M + (tm1 ? 63 : 127)) / (tm1 ? 64 : 128)) * ((d.N + (tn1 ? 63 : 127)) / (tn1 ? 64 : 128));
        if (tm1 && tn1) hipLaunchKernelGGL((gemm2_kernel<A_KM, B_KM, PA, PB, EPI, NARROW_M ? 1 : 2, 1>), grid, dim3(NT), 0, st, d);
        else if (tm1) hipLaunchKernelGGL((gemm2_kernel<A_KM, B_KM, PA, PB, EPI, NARROW_M ? 1 : 2, 2>), grid, dim3(NT), 0, st, d);
        else if (tn1) hipLaunchKernelGGL((gemm2_kernel<A_KM, B_KM, PA, PB, EPI, 2, 1>), grid, dim3(NT), 0, st, d);
        else hipLaunchKernelGGL((gemm2_kernel<A_KM, B_KM, PA, PB, EPI, 2, 2>), grid, dim3(NT), 0, st, d);
    }
    else if (vec_ok(d)) hipLaunchKernelGGL((gemm_kernel<A_KM, B_KM, PA, PB, EPI, true>), grid, dim3(NT), 0, st, d);
    else hipLaunchKernelGGL((gemm_kernel<A_KM, B_KM, PA, PB, EPI, false>), grid, dim3(NT), 0, st, d);
}

// The variants the MLP needs: forward (row-major A with prologue, row-major W),
// dgrad (row-major dY, k-major W), wgrad (k-major dY, k-major activations with prologue).
int dispatch(const UredGemmDesc& d, hipStream_t st) {
    const int key = (d.a_kmajor << 12) | (d.b_kmajor << 11) | (d.pro_a << 8) | (d.pro_b << 4) | d.epi;
#define URED_CASE(AK, BK_, PA, PB, E)                                          \
    case ((AK << 12) | (BK_ << 11) | (PA << 8) | (PB << 4) | E):              \
        launch<(bool)AK, (bool)BK_, PA, PB, E>(d, st);                        \
        return 0;
    switch (key) {
        // forward 1x1 conv
        URED_CASE(0, 0, URED_PRO_NONE, URED_PRO_NONE, URED_EPI_FWD)
        URED_CASE(0, 0, URED_PRO_ENC, URED_PRO_NONE, URED_EPI_FWD)
        URED_CASE(0, 0, URED_PRO_RES, URED_PRO_NONE, URED_EPI_FWD)
        URED_CASE(0, 0, URED_PRO_NONE, URED_PRO_NONE, URED_EPI_STORE)
        URED_CASE(0, 0, URED_PRO_ENC, URED_PRO_NONE, URED_EPI_STORE)
        URED_CASE(0, 0, URED_PRO_RES, URED_PRO_NONE, URED_EPI_STORE)
        // dgrad
        URED_CASE(0, 1, URED_PRO_NONE, URED_PRO_NONE, URED_EPI_BNBWD)
        URED_CASE(0, 1, URED_PRO_NONE, URED_PRO_NONE, URED_EPI_STORE)
#if URED_EXP_DGRAD_PRO
        // measurement build only (tools/gemm_bench.py dgrad_bnbwd_pro): the BN-backward dgrad with the
        // forward's one-input A prologue, the lower bound of folding the BN-backward apply into it
        URED_CASE(0, 1, URED_PRO_ENC, URED_PRO_NONE, URED_EPI_BNBWD)
#endif
        // few output tiles, long K (per-group codes, fc layers): split-K partials
        URED_CASE(0, 0, URED_PRO_NONE, URED_PRO_NONE, URED_EPI_SPLITK)
        URED_CASE(0, 1, URED_PRO_NONE, URED_PRO_NONE, URED_EPI_SPLITK)
        // wgrad (split-K over points)
        URED_CASE(1, 1, URED_PRO_NONE, URED_PRO_NONE, URED_EPI_SPLITK)
        URED_CASE(1, 1, URED_PRO_NONE, URED_PRO_ENC, URED_EPI_SPLITK)
        URED_CASE(1, 1, URED_PRO_NONE, URED_PRO_RES, URED_EPI_SPLITK)
        default:
            return ured::set_error(URED_EINVAL, "ured_gemm: unsupported variant a_kmajor=%d b_kmajor=%d pro_a=%d pro_b=%d epi=%d",
                                   d.a_kmajor, d.b_kmajor, d.pro_a, d.pro_b, d.epi);
    }
#undef URED_CASE
}

}  // namespace

extern "C" {

int ured_gemm(const UredGemmDesc* dp, void* stream) {
    ured::clear_error();
    URED_REQUIRE(dp, "ured_gemm: null descriptor");
    const UredGemmDesc& d = *dp;
    URED_REQUIRE(d.M >= 0 && d.N >= 0 && d.K >= 0, "ured_gemm: negative size");
    if (d.M == 0 || d.N == 0) return 0;
    URED_REQUIRE(d.A && d.B && d.C, "ured_gemm: null operand");
    URED_REQUIRE(d.k1 >= 0 && d.k1 <= d.K, "ured_gemm: k1 %d outside [0,K=%d]", d.k1, d.K);
    URED_REQUIRE(d.k1 == d.K || (!d.a_kmajor && d.A2), "ured_gemm: A2 split needs row-major A and A2");
    URED_REQUIRE(d.pro_a == URED_PRO_NONE || (d.pro_s && d.pro_t && !d.a_kmajor), "ured_gemm: bad A prologue");
    URED_REQUIRE(d.pro_b == URED_PRO_NONE || (d.pro_s && d.pro_t && d.b_kmajor), "ured_gemm: bad B prologue");
    URED_REQUIRE(!(d.pro_a && d.pro_b), "ured_gemm: one prologue per call");
    const long long tiles = (long long)((d.M + BM - 1) / BM) * ((d.N + BN - 1) / BN);
    URED_REQUIRE(tiles < (1LL << 31), "ured_gemm: too many tiles");
    if (d.epi == URED_EPI_FWD) {
        URED_REQUIRE(d.stat_ws, "ured_gemm: EPI_FWD needs stat_ws");
        URED_REQUIRE(!d.rowbias || d.gidx || d.group_rows > 0, "ured_gemm: rowbias needs gidx or group_rows");
        URED_REQUIRE(!d.pool_ws || (d.group_rows > 0 && d.group_rows % BM == 0),
                     "ured_gemm: pooling needs group_rows multiple of %d (got %d)", BM, d.group_rows);
    }
    if (d.epi == URED_EPI_BNBWD) {
        URED_REQUIRE(d.Yp && d.bn_mean && d.bn_invstd && d.bn_scale && d.bn_shift && d.bwd_ws, "ured_gemm: EPI_BNBWD inputs");
        URED_REQUIRE(!d.pool_idx || (d.pool_grad && d.pool_group_rows > 0), "ured_gemm: pool backward needs pool_grad, group rows");
    }
    if (d.epi == URED_EPI_SPLITK) URED_REQUIRE(d.splits >= 1 && d.splits <= 65535, "ured_gemm: splits %d", d.splits);
    int rc = dispatch(d, (hipStream_t)stream);
    if (rc) return rc;
    return ured::launch_status("ured_gemm");
}

int ured_wgrad_skinny(const float* dY, int ldd, const float* X, int ldx, int Cout, int Kin, int M, int pro,
                      const float* pro_s, const float* pro_t, float* out, int ldo, int accumulate, float* ws,
                      void* stream) {
    ured::clear_error();
    URED_REQUIRE(M >= 0 && Cout > 0 && Kin > 0 && ldo >= Kin, "ured_wgrad_skinny: bad sizes");
    const bool so = Cout <= 4;
    const int D = so ? Kin : Cout, S = so ? Cout : Kin;
    URED_REQUIRE((so || Kin <= 4) && D <= 256,
                 "ured_wgrad_skinny: needs min(Cout,Kin) <= 4 and max <= 256 (got %d x %d)", Cout, Kin);
    URED_REQUIRE(pro >= URED_PRO_NONE && pro <= URED_PRO_RES, "ured_wgrad_skinny: bad prologue %d", pro);
    URED_REQUIRE(pro == URED_PRO_NONE || (pro_s && pro_t), "ured_wgrad_skinny: prologue needs scale/shift");
    URED_REQUIRE(out && ws, "ured_wgrad_skinny: null pointer");
    hipStream_t st = (hipStream_t)stream;
    if (M == 0) {
        if (!accumulate)
            for (int r = 0; r < Cout; ++r)
                if (hipMemsetAsync(out + (size_t)r * ldo, 0, sizeof(float) * Kin, st) != hipSuccess)
                    return ured::launch_status("ured_wgrad_skinny");
        return ured::launch_status("ured_wgrad_skinny");
    }
    URED_REQUIRE(dY && X, "ured_wgrad_skinny: null pointer");
    const float* big = so ? X : dY;
    const int ldb = so ? ldx : ldd;
    const bool vec = D % 4 == 0 && ldb % 4 == 0 && ((uintptr_t)big & 15) == 0;
    const int nb = std::min(SK_MAX_BLOCKS, (M + 63) / 64), rpb = (M + nb - 1) / nb;
#define URED_SK(P, SO, SS, V) hipLaunchKernelGGL((wgrad_skinny_kernel<P, SO, SS, V>), dim3(nb), dim3(256), 0, st, \
                                                   dY, ldd, X, ldx, D, M, rpb, pro_s, pro_t, ws)
#define URED_SK_V(P, SO, SS) do { if (vec) URED_SK(P, SO, SS, 4); else URED_SK(P, SO, SS, 1); } while (0)
#define URED_SK_S(P, SO) do { switch (S) { case 1: URED_SK_V(P, SO, 1); break; case 2: URED_SK_V(P, SO, 2); break; \
                                           case 3: URED_SK_V(P, SO, 3); break; default: URED_SK_V(P, SO, 4); } } while (0)
#define URED_SK_P(SO) do { if (pro == URED_PRO_ENC) URED_SK_S(URED_PRO_ENC, SO); \
                           else if (pro == URED_PRO_RES) URED_SK_S(URED_PRO_RES, SO); else URED_SK_S(URED_PRO_NONE, SO); } while (0)
    if (so) URED_SK_P(true); else URED_SK_P(false);
#undef URED_SK_P
#undef URED_SK_S
#undef URED_SK_V
#undef URED_SK
    hipLaunchKernelGGL(skinny_reduce_kernel, dim3(Cout * Kin), dim3(256), 0, st, ws, nb, Cout * Kin, Kin, out, ldo,
                       accumulate);
    return ured::launch_status("ured_wgrad_skinny");
}

int ured_splitk_reduce(const float* ws, int splits, int M, int N, float* out, int ldo, int accumulate,
                       const float* bias, void* stream) {
    ured::clear_error();
    URED_REQUIRE(splits >= 1 && M >= 0 && N >= 0 && ldo >= N, "ured_splitk_reduce: bad sizes");
    if (M == 0 || N == 0) return 0;
    URED_REQUIRE(ws && out, "ured_splitk_reduce: null pointer");
    const size_t total = (size_t)M * N;
    URED_REQUIRE((total + 63) / 64 <= 0x7fffffff, "ured_splitk_reduce: too many elements");
    int nw = 1;
    while (nw < 16 && nw * 8 < splits) nw *= 2;      // about 8 splits per wave
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((total + 63) / 64)), dim3(64 * nw), 0, (hipStream_t)stream,
                       ws, splits, M, N, out, ldo, accumulate, bias);
    return ured::launch_status("ured_splitk_reduce");
}

int ured_bn_fwd_finalize(const float* stat_ws, int M, int N, const float* gamma, const float* beta,
                         float eps, float momentum, float* running_mean, float* running_var,
                         float* mean, float* invstd, float* scale, float* shift,
                         const float* group_w, int group_rows, long long* num_batches_tracked, void* stream) {
    ured::clear_error();
    URED_REQUIRE(M > 0 && N >= 0, "ured_bn_fwd_finalize: bad sizes M=%d N=%d", M, N);
    if (N == 0) return 0;
    URED_REQUIRE(stat_ws && mean && invstd && scale && shift, "ured_bn_fwd_finalize: null pointer");
    URED_REQUIRE(!group_w || (group_rows > 0 && group_rows % BM == 0),
                 "ured_bn_fwd_finalize: row weights need group_rows multiple of %d (got %d)", BM, group_rows);
    hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, stat_ws, M, N, gamma, beta,
                       eps, momentum, running_mean, running_var, mean, invstd, scale, shift, group_w, group_rows,
                       num_batches_tracked);
    return ured::launch_status("ured_bn_fwd_finalize");
}

int ured_bn_bwd_finalize(const float* bwd_ws, int M, int N, const float* gamma, const float* invstd,
                         float* dgamma, float* dbeta, int accumulate,
                         float* coef_a, float* coef_b, float* coef_c,
                         const float* group_w, int group_rows, void* stream) {
    ured::clear_error();
    URED_REQUIRE(M > 0 && N >= 0, "ured_bn_bwd_finalize: bad sizes");
    if (N == 0) return 0;
    URED_REQUIRE(bwd_ws && invstd && coef_a && coef_b && coef_c, "ured_bn_bwd_finalize: null pointer");
    URED_REQUIRE(!group_w || (group_rows > 0 && group_rows % BM == 0),
                 "ured_bn_bwd_finalize: row weights need group_rows multiple of %d (got %d)", BM, group_rows);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream, bwd_ws, M, N, gamma, invstd,
                       dgamma, dbeta, accumulate, coef_a, coef_b, coef_c, group_w, group_rows);
    return ured::launch_status("ured_bn_bwd_finalize");
}

int ured_bn_bwd_apply(const float* G, const float* Y, int M, int N, int ld, int res,
                      const float* mean, const float* coef_a, const float* coef_b, const float* coef_c,
                      float* dY, float* colsum_ws, const float* group_w, int group_rows, void* stream) {
    ured::clear_error();
    URED_REQUIRE(M >= 0 && N >= 0 && ld >= N, "ured_bn_bwd_apply: bad sizes");
    if (M == 0 || N == 0) return 0;
    URED_REQUIRE(G && Y && mean && coef_a && coef_b && coef_c && dY, "ured_bn_bwd_apply: null pointer");
    URED_REQUIRE(!group_w || (group_rows > 0 && group_rows % BM == 0),
                 "ured_bn_bwd_apply: row weights need group_rows multiple of %d (got %d)", BM, group_rows);
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (N % 4 == 0 && ld % 4 == 0 && al16(G) && al16(Y) && al16(dY) && al16(mean) && al16(coef_a) &&
        al16(coef_b) && al16(coef_c) && (!colsum_ws || al16(colsum_ws))) {
        dim3 grid((N / 4 + BBA_CQ - 1) / BBA_CQ, (M + BM - 1) / BM);
        hipLaunchKernelGGL(bn_bwd_apply4_kernel, grid, dim3(BBA_CQ * BBA_RL), 0, (hipStream_t)stream, G, Y, M, N, ld, res, mean,
                           coef_a, coef_b, coef_c, dY, colsum_ws, group_w, group_rows);
    } else {
        dim3 grid((N + 255) / 256, (M + BM - 1) / BM);
        hipLaunchKernelGGL(bn_bwd_apply_kernel, grid, dim3(256), 0, (hipStream_t)stream, G, Y, M, N, ld, res, mean,
                           coef_a, coef_b, coef_c, dY, colsum_ws, group_w, group_rows);
    }
    return ured::launch_status("ured_bn_bwd_apply");
}

int ured_pool_finalize(const float* pool_ws, int M, int N, int group_rows, const float* scale,
                       const float* shift, int relu, float* pooled, int* argidx, void* stream) {
    ured::clear_error();
    URED_REQUIRE(M > 0 && N > 0 && group_rows > 0 && group_rows % BM == 0 && M % group_rows == 0,
                 "ured_pool_finalize: M=%d must be a multiple of group_rows=%d (multiple of %d)", M, group_rows, BM);
    URED_REQUIRE(pool_ws && scale && shift && pooled && argidx, "ured_pool_finalize: null pointer");
    dim3 grid((N + 255) / 256, M / group_rows);
    hipLaunchKernelGGL(pool_finalize_kernel, grid, dim3(256), 0, (hipStream_t)stream, pool_ws, M, N, group_rows,
                       scale, shift, relu, pooled, argidx);
    return ured::launch_status("ured_pool_finalize");
}

int ured_pool_rows(const float* Y, int M, int N, int group_rows, const float* scale, const float* shift,
                   int relu, float* pooled, int* argidx, void* stream) {
    ured::clear_error();
    URED_REQUIRE(M > 0 && N > 0 && group_rows > 0 && M % group_rows == 0, "ured_pool_rows: bad sizes M=%d group_rows=%d", M, group_rows);
    URED_REQUIRE(M / group_rows <= 65535, "ured_pool_rows: too many groups");
    URED_REQUIRE(Y && scale && shift && pooled && argidx, "ured_pool_rows: null pointer");
    dim3 grid((N + 255) / 256, M / group_rows);
    hipLaunchKernelGGL(pool_rows_kernel, grid, dim3(256), 0, (hipStream_t)stream, Y, N, group_rows, scale, shift, relu, pooled, argidx);
    return ured::launch_status("ured_pool_rows");
}

int ured_bn_act(const float* Y, int M, int N, int ldy, const float* scale, const float* shift, int relu,
                float* out, int ldo, void* stream) {
    ured::clear_error();
    URED_REQUIRE(M >= 0 && N >= 0 && ldy >= N && ldo >= N, "ured_bn_act: bad sizes M=%d N=%d ldy=%d ldo=%d", M, N, ldy, ldo);
    if (M == 0 || N == 0) return 0;
    URED_REQUIRE(Y && scale && shift && out, "ured_bn_act: null pointer");
    const int v4 = (N & 3) == 0 && (ldy & 3) == 0 && (ldo & 3) == 0 &&
                   ((reinterpret_cast<uintptr_t>(Y) | reinterpret_cast<uintptr_t>(out) |
                     reinterpret_cast<uintptr_t>(scale) | reinterpret_cast<uintptr_t>(shift)) & 15) == 0;
    const long long items = (long long)M * (v4 ? N / 4 : N);
    hipLaunchKernelGGL(bn_act_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       Y, M, N, ldy, scale, shift, relu, out, ldo, v4);
    return ured::launch_status("ured_bn_act");
}

int ured_group_colsum(const float* X, int ldx, int N, const int* off, int group_rows, int G,
                      float* out, int ldo, void* stream) {
    return ured_group_colsum_split(X, ldx, N, off, group_rows, G, 1, nullptr, out, ldo, stream);
}

int ured_group_colsum_split(const float* X, int ldx, int N, const int* off, int group_rows, int G, int splits,
                            float* ws, float* out, int ldo, void* stream) {
    ured::clear_error();
    URED_REQUIRE(N >= 0 && G >= 0 && ldx >= N && ldo >= N, "ured_group_colsum: bad sizes");
    URED_REQUIRE(splits >= 1 && splits <= 1024, "ured_group_colsum: splits=%d outside [1, 1024]", splits);
    if (N == 0 || G == 0) return 0;
    URED_REQUIRE(X && out && (off || group_rows > 0), "ured_group_colsum: null pointer / no grouping");
    URED_REQUIRE(splits == 1 || ws, "ured_group_colsum: splits > 1 needs a workspace [G][splits][N]");
    URED_REQUIRE(G <= 65535, "ured_group_colsum: G=%d > 65535", G);
    dim3 grid((N + 63) / 64, G, splits);
    hipLaunchKernelGGL(group_colsum_kernel, grid, dim3(GCS_WAVES * 64), 0, (hipStream_t)stream, X, ldx, N, off, group_rows,
                       splits == 1 ? out : ws, ldo);
    if (splits > 1) {   // second pass: the S partials of each group, in split order
        dim3 grid2((N + 63) / 64, G, 1);
        hipLaunchKernelGGL(group_colsum_kernel, grid2, dim3(GCS_WAVES * 64), 0, (hipStream_t)stream, ws, N, N, nullptr, splits,
                           out, ldo);
    }
    return ured::launch_status("ured_group_colsum");
}

#if URED_GEMM_TIMING
// phase-timing build only: copy the recorded workgroup timestamps out (n slots of 16 u64)
int ured_debug_gemm_ts(unsigned long long* host, int n) {
    if (n > TS_SLOTS) n = TS_SLOTS;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(ured_ts_buf), (size_t)n * 128) == hipSuccess ? 0 : -1;
}
int ured_debug_gemm_ts_clear() {
    static unsigned long long z[TS_SLOTS * 16];
    return hipMemcpyToSymbol(HIP_SYMBOL(ured_ts_buf), z, sizeof z) == hipSuccess ? 0 : -1;
}
#endif
}  // extern "C"

URED_DBG_ACCESSOR(ured_dbg_mlp)
