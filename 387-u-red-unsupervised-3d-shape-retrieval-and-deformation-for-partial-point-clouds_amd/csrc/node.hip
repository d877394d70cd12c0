// node.hip — the graph-node layers of DeformNet_MatchingNet on MI355X (gfx950).
//
// Replaces, for the 2 + MAX_NUM_PARTS graph nodes per sample of the reference's
// GraphAttentionNet + param_decoder (network/deformation_net.py:61,74-93,
// attention_graph/attention_gnn.py:8-55, attention_graph/attention_utils.py:62-86):
//   * every Conv1d(k=1) over nodes (in_proj_q/k/v, out_proj, the FeedForwardNet_norm convs,
//     param_decoder) and its two backward GEMMs  -> node_gemm_kernel
//   * BatchNorm1d (train: batch statistics per node set, running stats; eval) after the ReLU
//     of FeedForwardNet_norm (Conv -> ReLU -> BN), forward and backward -> node_bn_*_kernel
//
// Shapes are small in M (B x nodes <= a few hundred rows) and moderate in N, K (<= 1536), so a
// 128x128-tile GEMM would leave most of the 256 CUs idle. node_gemm_kernel instead gives each
// workgroup one 32 x 32 output tile and splits its K over the workgroup's 8 waves (K chunks of
// 32 dealt round-robin): each wave loads its fragments straight from global/L2 into registers
// (the next chunk's loads issued before the current chunk's MFMAs), runs 16 x
// v_mfma_f32_32x32x2_f32 per chunk on two accumulators, and the 8 partial tiles are summed
// through LDS in fixed wave order (deterministic). Independent GEMMs (a layer's dgrad and
// wgrad, the q and k|v projections of a cross-attention) go in one launch as jobs. Operands are addressed by element strides, so A, A^T, W, W^T and the
// two-source concatenation of the FFN input (cat([x, message]) along K) are read in place.
// The epilogue fuses bias, a per-row-group bias (param_decoder's broadcast global half),
// ReLU, a ReLU gate (backward mask), a residual add and accumulation.
#include <hip/hip_runtime.h>
#define URED_DBG_FILE 4
#include "ured_common.h"
#include "../../include/ured_hip.h"

namespace {

typedef float f16v __attribute__((ext_vector_type(16)));

// Workgroup tile 32 x 32 (one MFMA tile), K split over the 8 waves in chunks of 32; the
// independent GEMMs of one layer (e.g. a backward's dgrad and wgrad) share one launch as jobs.
constexpr int NG_WAVES = 8, NG_NT = NG_WAVES * 64, NG_BM = 32, NG_BN = 32, NG_BK = 32, NG_JOBS = URED_NODE_MAX_JOBS;

struct NodeJob {
    UredNodeGemmDesc d;
    int akc, bkc;            // float4 fragment loads (k-contiguous, 16-B aligned operand)
    int ntn;                 // column tiles (kind 1: column blocks of 32)
};
struct NodeJobs {
    NodeJob job[NG_JOBS];
    int tile0[NG_JOBS + 1];  // first workgroup of each job
    int njobs;
};

// Per-lane operand streams. A lane's A row (m) and B column (n) are fixed for the whole tile,
// so each lane keeps one base pointer per source (rows past M / columns past N are clamped to a
// valid address: their products only reach outputs that are never stored) and walks k with a
// stride; only the last, partial chunk checks k < K (and zeroes A there: 0 * finite B = 0).
struct LaneSrc {
    const float* p1;   // element k (< k1) at p1 + k * s1
    const float* p2;   // element k (>= k1) at p2 + k * s2 (pre-offset by -k1 * s2)
    long long s1, s2;
    int k1;
};

__device__ __forceinline__ LaneSrc lane_a(const UredNodeGemmDesc& d, int m) {
    const long long mc = m < d.M ? m : 0;
    LaneSrc s;
    s.p1 = d.A + mc * d.sam;
    s.s1 = d.sak;
    s.k1 = d.k1;
    s.p2 = d.A2 ? d.A2 + mc * d.sam2 - (long long)d.k1 * d.sak2 : s.p1;
    s.s2 = d.A2 ? d.sak2 : d.sak;
    return s;
}

__device__ __forceinline__ LaneSrc lane_b(const UredNodeGemmDesc& d, int n) {
    const long long nc = n < d.N ? n : 0;
    const bool second = d.B2 && nc >= d.n1;
    LaneSrc s;
    if (second) { s.p1 = d.B2 + (nc - d.n1) * d.sbn2; s.s1 = d.sbk2; }
    else { s.p1 = d.B + nc * d.sbn; s.s1 = d.sbk; }
    s.p2 = s.p1; s.s2 = s.s1; s.k1 = 0x7fffffff;
    return s;
}

// 16 consecutive reduction indices kb..kb+15 of one lane (kb % 16 == 0, so the run lies in one
// source when k1 % 16 == 0). kc: unit k-stride and 16-B aligned -> four float4 loads.
__device__ __forceinline__ void ld16(const LaneSrc& s, bool kc, int kb, int K, bool zero_tail, float* out) {
    const float* base = kb < s.k1 ? s.p1 : s.p2;
    const long long st = kb < s.k1 ? s.s1 : s.s2;
    if (kb + 16 <= K) {
        if (kc) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float4 v = *reinterpret_cast<const float4*>(base + kb + 4 * q);
                out[4 * q] = v.x; out[4 * q + 1] = v.y; out[4 * q + 2] = v.z; out[4 * q + 3] = v.w;
            }
        } else {
            const float* p = base + (long long)kb * st;
#pragma unroll
            for (int j = 0; j < 16; ++j) { out[j] = *p; p += st; }
        }
    } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int k = kb + j;
            const bool ok = k < K;
            const float v = base[(long long)(ok ? k : K - 1) * st];
            out[j] = (ok || !zero_tail) ? v : 0.f;
        }
    }
}

// The MFMA k-order is permuted (instruction j of lane half h uses k = c0 + 16h + j) for both
// operands, so the sum is the same; each lane reads 16 consecutive k.
__device__ __forceinline__ void load_chunk(const LaneSrc& sa, const LaneSrc& sb, bool akc, bool bkc, int c0, int h,
                                           int K, float (&a)[16], float (&b)[16]) {
    const int kb = c0 + 16 * h;
    if (kb >= K) {            // this lane half's run is entirely past K: contributes nothing
#pragma unroll
        for (int j = 0; j < 16; ++j) { a[j] = 0.f; b[j] = 0.f; }
        return;
    }
    ld16(sa, akc, kb, K, true, a);
    ld16(sb, bkc, kb, K, false, b);
}

// partial tile -> LDS [wave][row][col]; element r: row (r&3) + 8(r>>2) + 4h, col li
__device__ __forceinline__ void node_partial(float* red, const f16v& acc, int w, int h, int li) {
    float* mine = red + w * NG_BM * NG_BN;
#pragma unroll
    for (int r = 0; r < 16; ++r) mine[((r & 3) + 8 * (r >> 2) + 4 * h) * NG_BN + li] = acc[r];
}

// 512 threads x 2 outputs: row t/16, columns 2(t%16), +1; the 8 waves' partial tiles summed in fixed
// order, then bias, row-group bias, ReLU, gate, residual and accumulation
__device__ __forceinline__ void node_combine(const UredNodeGemmDesc& d, const float* red, int m0, int n0) {
    const int t = threadIdx.x;
    const int row = t >> 4, cq = (t & 15) * 2;
    const int m = m0 + row;
    if (m >= d.M) return;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int col = cq + q, n = n0 + col;
        if (n >= d.N) break;
        float v = 0.f;
#pragma unroll
        for (int ww = 0; ww < NG_WAVES; ++ww) v += red[ww * NG_BM * NG_BN + row * NG_BN + col];
        if (d.bias) v += d.bias[n];
        if (d.rowbias) v += d.rowbias[(long long)(m / d.rdiv) * d.ldrb + n];
        if (d.relu_out) v = fmaxf(v, 0.f);
        if (d.gate) v = d.gate[(long long)m * d.ldgate + n] > 0.f ? v : 0.f;
        if (d.R && n < d.R_ncols) v += d.R[(long long)m * d.ldR + n];
        URED_DBG_CHECK(m < d.M && n < d.N && (!d.rowbias || m / d.rdiv >= 0));
        float* cp = d.C + (long long)m * d.ldc + n;
        if (d.accumulate) v += *cp;
        *cp = v;
    }
}

// bias gradient job: C[n] (+)= sum_m A(m, n)
__device__ __forceinline__ void node_colsum(const UredNodeGemmDesc& d, int tile) {
    __shared__ float part[16][33];
    const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5, n = tile * 32 + cl;
    float sacc = 0.f;
    if (n < d.N) {
        // unrolled so that eight loads are in flight per lane (the adds keep their order)
        const float* col = d.A + (long long)n * d.sak;
#pragma unroll 8
        for (int m = rl; m < d.M; m += 16) sacc += col[(long long)m * d.sam];
    }
    part[rl][cl] = sacc;
    __syncthreads();
    if (rl == 0 && n < d.N) {
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) v += part[q][cl];
        d.C[n] = d.accumulate ? d.C[n] + v : v;
    }
}

#ifndef URED_NODE_WG_PER_CU
#define URED_NODE_WG_PER_CU 2
#endif
// Phase timing build (-DURED_NODE_TIMING=1 -DURED_NTS_M=.. -DURED_NTS_N=.. -DURED_NTS_K=..): launches
// whose first job has that shape record per workgroup (wave 0) the real-time clock (100 MHz) at start,
// first chunk landed, MFMA loop end, partial tiles in LDS, stores done (tools/node_phase.py reads
// them through ured_debug_node_ts)
#ifndef URED_NODE_TIMING
#define URED_NODE_TIMING 0
#endif
#if URED_NODE_TIMING
constexpr int NTS_SLOTS = 4096;
__device__ unsigned long long ured_nts_buf[NTS_SLOTS * 8];
#define URED_NTS(k) do { if (nts_on && threadIdx.x == 0) nts_[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define URED_NTS(k) do { } while (0)
#endif
// two workgroups per CU (the second launch-bounds argument is waves per SIMD: 4 -> <= 128 VGPRs;
// one accumulator chain per wave, the four waves of a SIMD interleave their MFMAs), so a launch
// of a few hundred tiles runs in one round
__global__ __launch_bounds__(NG_NT, URED_NODE_WG_PER_CU * NG_WAVES / 4) void node_gemm_kernel(const NodeJobs jobs) {
    __shared__ float red[NG_WAVES * NG_BM * NG_BN];      // 32 KB: the 8 waves' partial tiles
    int ji = 0;
#pragma unroll
    for (int q = 1; q < NG_JOBS; ++q)
        if (q < jobs.njobs && (int)blockIdx.x >= jobs.tile0[q]) ji = q;
    const NodeJob& J = jobs.job[ji];
    const UredNodeGemmDesc& d = J.d;
    const int tile = blockIdx.x - jobs.tile0[ji];
    if (d.kind == URED_NODE_COLSUM) {
        node_colsum(d, tile);
        return;
    }
    const int m0 = (tile / J.ntn) * NG_BM, n0 = (tile % J.ntn) * NG_BN;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63, h = lane >> 5, li = lane & 31;
    const bool akc = J.akc, bkc = J.bkc;
#if URED_NODE_TIMING
    const UredNodeGemmDesc& d0 = jobs.job[0].d;
    const bool nts_on = d0.M == URED_NTS_M && d0.N == URED_NTS_N && d0.K == URED_NTS_K && blockIdx.x < NTS_SLOTS;
    unsigned long long nts_[5] = {0, 0, 0, 0, 0};
    URED_NTS(0);
#endif
    // URED_NODE_WG_PER_CU 1: two accumulators (even / odd k-steps), independent MFMA chains
    // summed at the end; 2: one chain (registers for the second resident workgroup)
    constexpr bool TWO_ACC = URED_NODE_WG_PER_CU == 1;
    f16v acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) { acc0[r] = 0.f; acc1[r] = 0.f; }

    const LaneSrc sa = lane_a(d, m0 + li);
    const LaneSrc sb = lane_b(d, n0 + li);
    const int nch = (d.K + NG_BK - 1) / NG_BK;
    float a[16], b[16], an[16], bn[16];
    int c = w;
    if (c < nch) load_chunk(sa, sb, akc, bkc, c * NG_BK, h, d.K, a, b);
#if URED_NODE_TIMING
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    URED_NTS(1);
#endif
    while (c < nch) {
        const int cn = c + NG_WAVES;
        // one chunk of prefetch with one resident workgroup; with two, the other waves of the
        // SIMD cover the load latency and the registers go to occupancy
        if (TWO_ACC && cn < nch) load_chunk(sa, sb, akc, bkc, cn * NG_BK, h, d.K, an, bn);
        if constexpr (TWO_ACC) {
#pragma unroll
            for (int j = 0; j < 16; j += 2) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[j], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j + 1], b[j + 1], acc1, 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[j], acc0, 0, 0, 0);
        }
        if (TWO_ACC && cn < nch) {
#pragma unroll
            for (int j = 0; j < 16; ++j) { a[j] = an[j]; b[j] = bn[j]; }
        } else if (!TWO_ACC && cn < nch) {
            load_chunk(sa, sb, akc, bkc, cn * NG_BK, h, d.K, a, b);
        }
        c = cn;
    }
    URED_NTS(2);
    f16v accs;
#pragma unroll
    for (int r = 0; r < 16; ++r) accs[r] = TWO_ACC ? acc0[r] + acc1[r] : acc0[r];
    node_partial(red, accs, w, h, li);
    __syncthreads();
    URED_NTS(3);
#if URED_NODE_TIMING
    if (nts_on && threadIdx.x == 0) {      // the end mark follows wave 0's stores
        unsigned long long* o = ured_nts_buf + (size_t)blockIdx.x * 8;
        o[0] = nts_[0]; o[1] = nts_[1]; o[2] = nts_[2]; o[3] = nts_[3];
        o[5] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        o[6] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
        o[7] = 1;
    }
#endif
    node_combine(d, red, m0, n0);
#if URED_NODE_TIMING
    if (nts_on && threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ured_nts_buf[(size_t)blockIdx.x * 8 + 4] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// ---- v4: two K half-chunks in flight per wave --------------------------------------------------
// v1 loads a wave's next K-chunk only after the current chunk's MFMAs, so a wave with c chunks
// waits c dependent L2 round trips (tools/node_phase.py: 2.8 us to the first chunk, 3.4 more for the
// second at 288 x 1536 x 512). v4 keeps URED_NODE_RING half-chunks (16 k per lane pair) in flight:
// the loads of half q + RING are issued behind the MFMAs of half q, in ring order (sched_barrier), and past
// the wave's last half it reloads chunk 0 (never consumed), so every iteration issues the same loads
// and hipcc's wait counts stay exact. Operands are read as raw buffer loads (per-lane byte offset in
// the VGPR offset, k * stride in the scalar offset); a k-contiguous operand (akc / bkc) as two 16-B
// loads per half, any other as eight 4-B loads — the four combinations are separate loop bodies, so
// each has a fixed load count. Same chunk -> wave assignment, MFMA order and fixed-order combine as
// v1: bitwise v1. Jobs need K, k1 (A2 split) and n1 (B2 split) multiples of 32 and every element
// below 2^29 of its operand base (node_v4_ok); other launches run v1.
#ifndef URED_NODE_V4
#define URED_NODE_V4 1
#endif
// half-chunks in flight per wave (3 at most for two strided operands: 16 loads per half). 2: DeformNet
// fwd+bwd 1.228 ms graph-replayed vs v1 1.276; 4: 1.352 (profiles/r5w_node_v4.log)
#ifndef URED_NODE_RING
#define URED_NODE_RING 2
#endif

struct Src4 {
    const float* base;   // operand base (uniform)
    unsigned vo;         // this lane's byte offset: row / column offset + its lane half's 16 k
    int sk4;             // k stride in bytes (4 for a k-contiguous operand)
#if URED_DEBUG_BOUNDS
    long long lim;       // bytes of the operand the job may read (node_v4_ok's extent)
#endif
};

typedef float f4v __attribute__((ext_vector_type(4)));

// k = kb .. kb + 7 of this lane (kb uniform)
template <bool KC>
__device__ __forceinline__ void ld8(const Src4& s, int kb, float* out) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(s.base), (short)0,
                                                                        0x7FFFFFFF, 0x00020000);
#if URED_DEBUG_BOUNDS
    // the eight elements' last byte lies inside the extent node_v4_ok admitted for this operand
    URED_DBG_CHECK(kb >= 0 && (long long)s.vo + (long long)(KC ? kb * 4 + 28 : (kb + 7) * (long long)s.sk4) + 4 <= s.lim);
#endif
    if constexpr (KC) {
        const f4v x = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, s.vo, kb * 4, 0));
        const f4v y = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rs, s.vo, kb * 4 + 16, 0));
        out[0] = x[0]; out[1] = x[1]; out[2] = x[2]; out[3] = x[3];
        out[4] = y[0]; out[5] = y[1]; out[6] = y[2]; out[7] = y[3];
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            out[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, s.vo, (kb + j) * s.sk4, 0));
    }
}

// DEPTH half-chunks in flight (slot s holds halves s, s + DEPTH, ...); the MFMAs of a slot past
// the wave's last half are skipped by a uniform branch with no loads inside (exact wait counts)
template <bool AKC, bool BKC, int DEPTH>
__device__ __forceinline__ void node_ring(const UredNodeGemmDesc& d, const Src4& a1, const Src4& a2, const Src4& bs,
                                          int w, f16v& acc) {
    const int nch = d.K / NG_BK;
    const int mine = w < nch ? (nch - w + NG_WAVES - 1) / NG_WAVES : 0;   // chunks w, w+8, ...
    const int halves = 2 * mine;
    float a[DEPTH][8], b[DEPTH][8];
    // half q: MFMAs j = 8(q & 1) .. +7 of chunk w + 8(q >> 1), i.e. k = c0 + 16h + 8(q & 1) + jj
    auto load = [&](int slot, int q) {
        const int c0 = (q < halves ? w + NG_WAVES * (q >> 1) : 0) * NG_BK, kh = 8 * (q & 1);
        const bool first = c0 < d.k1;          // k1 % 32 == 0: a chunk lies in one A source
        Src4 sa;
        sa.base = first ? a1.base : a2.base;
        sa.vo = first ? a1.vo : a2.vo;
        sa.sk4 = first ? a1.sk4 : a2.sk4;
#if URED_DEBUG_BOUNDS
        sa.lim = first ? a1.lim : a2.lim;
#endif
        ld8<AKC>(sa, (first ? c0 : c0 - d.k1) + kh, a[slot]);
        ld8<BKC>(bs, c0 + kh, b[slot]);
    };
#pragma unroll
    for (int sl = 0; sl < DEPTH; ++sl) {
        load(sl, sl);
        __builtin_amdgcn_sched_barrier(0);
    }
    for (int q = 0; q < halves; q += DEPTH) {
#pragma unroll
        for (int sl = 0; sl < DEPTH; ++sl) {
            __builtin_amdgcn_sched_barrier(0);
            if (sl == 0 || q + sl < halves) {
#pragma unroll
                for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[sl][j], b[sl][j], acc, 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            load(sl, q + sl + DEPTH);
        }
    }
}

__global__ __launch_bounds__(NG_NT, URED_NODE_WG_PER_CU * NG_WAVES / 4) void node_gemm4_kernel(const NodeJobs jobs) {
    __shared__ float red[NG_WAVES * NG_BM * NG_BN];
    int ji = 0;
#pragma unroll
    for (int q = 1; q < NG_JOBS; ++q)
        if (q < jobs.njobs && (int)blockIdx.x >= jobs.tile0[q]) ji = q;
    const NodeJob& J = jobs.job[ji];
    const UredNodeGemmDesc& d = J.d;
    const int tile = blockIdx.x - jobs.tile0[ji];
    if (d.kind == URED_NODE_COLSUM) {
        node_colsum(d, tile);
        return;
    }
    const int m0 = (tile / J.ntn) * NG_BM, n0 = (tile % J.ntn) * NG_BN;
    // the wave index as a provably uniform (SGPR) value: chunk counts and k offsets stay scalar
    const int t = threadIdx.x, w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63, h = lane >> 5, li = lane & 31;
    // rows / columns past M / N read the tile's first row / column (their outputs are never stored)
    const long long mc = m0 + li < d.M ? m0 + li : m0;
    const long long nc = n0 + li < d.N ? n0 + li : n0;
    Src4 a1, a2, bs;
    a1.base = d.A ? d.A : d.A2;                // k1 <= 0: every chunk reads A2
    a1.sk4 = (int)(d.sak * 4);
    a1.vo = (unsigned)((mc * d.sam + 16LL * h * d.sak) * 4);
    if (d.A2) {
        a2.base = d.A2; a2.sk4 = (int)(d.sak2 * 4);
        a2.vo = (unsigned)((mc * d.sam2 + 16LL * h * d.sak2) * 4);
    } else {
        a2 = a1;
    }
    const bool b2 = d.B2 && n0 >= d.n1;        // n1 % 32 == 0: a 32-column tile lies in one B source
    bs.base = b2 ? d.B2 : d.B;
    const long long sbk = b2 ? d.sbk2 : d.sbk;
    bs.sk4 = (int)(sbk * 4);
    bs.vo = (unsigned)(((b2 ? (nc - d.n1) * d.sbn2 : nc * d.sbn) + 16LL * h * sbk) * 4);
#if URED_DEBUG_BOUNDS
    {   // the extents node_v4_ok bounds: the last element a source holds, + 1, in bytes
        const int k1 = d.A2 ? d.k1 : d.K;
        a1.lim = 4 * ((long long)(d.M - 1) * d.sam + (long long)((k1 < d.K ? k1 : d.K) - 1) * d.sak + 1);
        if (d.A2) a2.lim = 4 * ((long long)(d.M - 1) * d.sam2 + (long long)(d.K - k1 - 1) * d.sak2 + 1);
        else a2.lim = a1.lim;
        if (!d.A || k1 <= 0) a1.lim = a2.lim;  // every chunk reads A2
        bs.lim = b2 ? 4 * ((long long)(d.N - d.n1 - 1) * d.sbn2 + (long long)(d.K - 1) * d.sbk2 + 1)
                    : 4 * ((long long)((d.B2 ? d.n1 : d.N) - 1) * d.sbn + (long long)(d.K - 1) * d.sbk + 1);
    }
#endif
#if URED_NODE_TIMING
    const UredNodeGemmDesc& d0 = jobs.job[0].d;
    const bool nts_on = d0.M == URED_NTS_M && d0.N == URED_NTS_N && d0.K == URED_NTS_K && blockIdx.x < NTS_SLOTS;
    unsigned long long nts_[5] = {0, 0, 0, 0, 0};
    URED_NTS(0);
    nts_[1] = nts_[0];                         // no separate first-chunk mark in the ring
#endif
    f16v acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // ring depth: at most ~48 loads in flight per wave (the vmcnt counter holds 63)
    switch (J.akc * 2 + J.bkc) {
        case 3: node_ring<true, true, URED_NODE_RING>(d, a1, a2, bs, w, acc); break;
        case 2: node_ring<true, false, URED_NODE_RING>(d, a1, a2, bs, w, acc); break;
        case 1: node_ring<false, true, URED_NODE_RING>(d, a1, a2, bs, w, acc); break;
        default: node_ring<false, false, (URED_NODE_RING < 3 ? URED_NODE_RING : 3)>(d, a1, a2, bs, w, acc); break;
    }
    URED_NTS(2);
    node_partial(red, acc, w, h, li);
    __syncthreads();
    URED_NTS(3);
#if URED_NODE_TIMING
    if (nts_on && threadIdx.x == 0) {
        unsigned long long* o = ured_nts_buf + (size_t)blockIdx.x * 8;
        o[0] = nts_[0]; o[1] = nts_[1]; o[2] = nts_[2]; o[3] = nts_[3];
        o[7] = 1;
    }
#endif
    node_combine(d, red, m0, n0);
#if URED_NODE_TIMING
    if (nts_on && threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ured_nts_buf[(size_t)blockIdx.x * 8 + 4] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// ---- BatchNorm1d over node sets (rows [off[s], off[s+1]) form one call of the module) -------
// One workgroup per 4 columns, 64 row lanes per column (a set of <= 288 node rows is a few
// dependent loads per lane; 16 columns x 16 lanes ran 1.2-1.5x longer, tools/node_bn_bench.py);
// sets processed in order, so the running statistics see the reference's sequence of module
// calls. fp64 sums, fixed order.
#ifndef URED_NODE_BN_COLS
#define URED_NODE_BN_COLS 4
#endif
constexpr int BN_COLS = URED_NODE_BN_COLS, BN_RL = 256 / BN_COLS, BN_NT = BN_COLS * BN_RL;

__device__ __forceinline__ float bn_in(const float* Y, int ldy, int m, int n, int relu_in) {
    const float y = Y[(long long)m * ldy + n];
    return relu_in ? fmaxf(y, 0.f) : y;
}

__global__ __launch_bounds__(BN_NT) void node_bn_fwd_kernel(const UredNodeBNDesc d) {
    __shared__ double part[BN_RL][BN_COLS];
    const int cl = threadIdx.x % BN_COLS, rl = threadIdx.x / BN_COLS;
    const int n = blockIdx.x * BN_COLS + cl;
    const bool cv = n < d.N;
    const int nc = cv ? n : 0;
    for (int s = 0; s < d.nsets; ++s) {
        const int r0 = d.off[s], r1 = d.off[s + 1], cnt = r1 - r0;
        float mean, invstd;
        if (d.training && d.stats_in) {          // SyncBN: the cross-rank merged statistics
            const double* st = d.stats_in + (size_t)s * 3 * d.N;
            const double c = st[nc], mu = st[d.N + nc], var = st[2 * d.N + nc] / fmax(c, 1.0);
            mean = (float)mu;
            invstd = (float)(1.0 / sqrt(var + (double)d.eps));
            if (rl == 0 && cv) {
                const double unb = c > 1.0 ? var * c / (c - 1.0) : var;
                d.running_mean[n] = (float)((1.0 - d.momentum) * d.running_mean[n] + d.momentum * mu);
                d.running_var[n] = (float)((1.0 - d.momentum) * d.running_var[n] + d.momentum * unb);
            }
        } else if (d.training) {
            double sum = 0.0;
            for (int m = r0 + rl; m < r1; m += BN_RL) sum += bn_in(d.Y, d.ldy, m, nc, d.relu_in);
            part[rl][cl] = sum;
            __syncthreads();
            double tot = 0.0;
#pragma unroll
            for (int q = 0; q < BN_RL; ++q) tot += part[q][cl];
            const double mu = tot / (double)max(cnt, 1);
            __syncthreads();
            double m2 = 0.0;
            for (int m = r0 + rl; m < r1; m += BN_RL) {
                const double e = (double)bn_in(d.Y, d.ldy, m, nc, d.relu_in) - mu;
                m2 += e * e;
            }
            part[rl][cl] = m2;
            __syncthreads();
            double m2t = 0.0;
#pragma unroll
            for (int q = 0; q < BN_RL; ++q) m2t += part[q][cl];
            const double var = m2t / (double)max(cnt, 1);
            __syncthreads();
            if (d.stats_out) {                   // SyncBN: this rank's per-set statistics only
                if (rl == 0 && cv) {
                    double* st = d.stats_out + (size_t)s * 3 * d.N;
                    st[n] = (double)cnt;
                    st[d.N + n] = mu;
                    st[2 * d.N + n] = m2t;
                }
                continue;
            }
            mean = (float)mu;
            invstd = (float)(1.0 / sqrt(var + (double)d.eps));
            if (rl == 0 && cv) {
                const double unb = cnt > 1 ? var * (double)cnt / (double)(cnt - 1) : var;
                d.running_mean[n] = (float)((1.0 - d.momentum) * d.running_mean[n] + d.momentum * mu);
                d.running_var[n] = (float)((1.0 - d.momentum) * d.running_var[n] + d.momentum * unb);
            }
        } else {
            mean = d.running_mean[nc];
            invstd = 1.f / sqrtf(d.running_var[nc] + d.eps);
        }
        const float scale = d.gamma[nc] * invstd, shift = d.beta[nc] - mean * scale;
        if (rl == 0 && cv) {
            d.mean[s * d.N + n] = mean;
            d.invstd[s * d.N + n] = invstd;
        }
        if (cv)
            for (int m = r0 + rl; m < r1; m += BN_RL)
                d.act[(long long)m * d.ld_act + n] = bn_in(d.Y, d.ldy, m, n, d.relu_in) * scale + shift;
        __syncthreads();
    }
    if (d.training && !d.stats_out && d.num_batches_tracked && blockIdx.x == 0 && threadIdx.x == 0)
        d.num_batches_tracked[0] += d.nsets;
}

// dY = d act / d Y: g (gradient of the BN output), per set: training dx = gamma*invstd*(g -
// mean(g) - xhat*mean(g*xhat)), eval dx = gamma*invstd*g; relu_in: masked by Y > 0.
// dgamma / dbeta summed over the sets (one module).
__global__ __launch_bounds__(BN_NT) void node_bn_bwd_kernel(const UredNodeBNBwdDesc d) {
    __shared__ double pg[BN_RL][BN_COLS], pgx[BN_RL][BN_COLS];
    const int cl = threadIdx.x % BN_COLS, rl = threadIdx.x / BN_COLS;
    const int n = blockIdx.x * BN_COLS + cl;
    const bool cv = n < d.N;
    const int nc = cv ? n : 0;
    const float gamma = d.gamma[nc];
    double dgam = 0.0, dbet = 0.0;
    for (int s = 0; s < d.nsets; ++s) {
        const int r0 = d.off[s], r1 = d.off[s + 1], cnt = r1 - r0;
        const float mean = d.mean[s * d.N + nc], invstd = d.invstd[s * d.N + nc];
        double sg = 0.0, sgx = 0.0;
        for (int m = r0 + rl; m < r1; m += BN_RL) {
            const float g = d.G[(long long)m * d.ldg + nc];
            const float xh = (bn_in(d.Y, d.ldy, m, nc, d.relu_in) - mean) * invstd;
            sg += g;
            sgx += (double)g * xh;
        }
        pg[rl][cl] = sg;
        pgx[rl][cl] = sgx;
        __syncthreads();
        sg = 0.0;
        sgx = 0.0;
#pragma unroll
        for (int q = 0; q < BN_RL; ++q) { sg += pg[q][cl]; sgx += pgx[q][cl]; }
        __syncthreads();
        if (d.sums_out) {                        // SyncBN: this rank's per-set sums only
            if (rl == 0 && cv) {
                double* so = d.sums_out + (size_t)s * 3 * d.N;
                so[n] = sg;
                so[d.N + n] = sgx;
                so[2 * d.N + n] = (double)cnt;
            }
            continue;
        }
        dgam += sgx;
        dbet += sg;
        const float k = gamma * invstd;
        double gsg = sg, gsgx = sgx, gcnt = (double)max(cnt, 1);
        if (d.sums_in) {                         // SyncBN: the cross-rank sums and count
            const double* si = d.sums_in + (size_t)s * 3 * d.N;
            gsg = si[nc];
            gsgx = si[d.N + nc];
            gcnt = fmax(si[2 * d.N + nc], 1.0);
        }
        const float mg = d.training ? (float)(gsg / gcnt) : 0.f;
        const float mgx = d.training ? (float)(gsgx / gcnt) : 0.f;
        if (cv)
            for (int m = r0 + rl; m < r1; m += BN_RL) {
                const float y = d.Y[(long long)m * d.ldy + n];
                const float x = d.relu_in ? fmaxf(y, 0.f) : y;
                const float xh = (x - mean) * invstd;
                float dx = k * (d.G[(long long)m * d.ldg + n] - mg - xh * mgx);
                if (d.relu_in && !(y > 0.f)) dx = 0.f;
                d.dY[(long long)m * d.lddy + n] = dx;
            }
    }
    if (rl == 0 && cv && !d.sums_out) {
        d.dgamma[n] = d.accumulate ? d.dgamma[n] + (float)dgam : (float)dgam;
        d.dbeta[n] = d.accumulate ? d.dbeta[n] + (float)dbet : (float)dbet;
    }
}

}  // namespace

extern "C" {

static int check_node_job(const UredNodeGemmDesc& d, NodeJob& J) {
    URED_REQUIRE(d.M >= 0 && d.N >= 0 && d.K >= 0, "ured_node_gemm: bad sizes %d x %d x %d", d.M, d.N, d.K);
    if (d.kind == URED_NODE_COLSUM) {
        URED_REQUIRE(d.A && d.C, "ured_node_gemm: colsum job needs A and C");
        J.d = d;
        J.akc = J.bkc = 0;
        J.ntn = (d.N + 31) / 32;
        return 0;
    }
    URED_REQUIRE(d.kind == URED_NODE_GEMM, "ured_node_gemm: unknown job kind %d", d.kind);
    URED_REQUIRE(d.C && d.B && (d.A || d.k1 <= 0) && (d.A2 || d.k1 >= d.K), "ured_node_gemm: null operand");
    URED_REQUIRE(!d.rowbias || d.rdiv > 0, "ured_node_gemm: rowbias needs rdiv > 0");
    URED_REQUIRE(d.k1 >= d.K || d.k1 % 16 == 0, "ured_node_gemm: the A2 split k1 = %d must be a multiple of 16", d.k1);
    URED_REQUIRE(!d.B2 || (d.n1 > 0 && d.n1 <= d.N), "ured_node_gemm: B2 needs 0 < n1 <= N");
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    // float4 fragment loads: k-contiguous operand(s) with 16-B aligned rows
    J.akc = d.sak == 1 && al16(d.A) && d.sam % 4 == 0 && (d.k1 >= d.K || (d.sak2 == 1 && al16(d.A2) && d.sam2 % 4 == 0));
    J.bkc = d.sbk == 1 && al16(d.B) && d.sbn % 4 == 0 && (!d.B2 || (d.sbk2 == 1 && al16(d.B2) && d.sbn2 % 4 == 0));
    J.d = d;
    J.ntn = (d.N + NG_BN - 1) / NG_BN;
    return 0;
}

// v4 takes a job when its K, k1 (A2 split) and n1 (B2 split) are multiples of the 32-wide chunk /
// tile and every element it reads lies below 2^29 elements of its operand base (31-bit byte
// offsets in the buffer descriptors)
static bool node_v4_ok(const UredNodeGemmDesc& d) {
    if (d.kind == URED_NODE_COLSUM) return true;
    const auto fits = [](long long v) { return v >= 0 && v < (1LL << 29); };
    // v4 reads A2 at element (k - k1): a negative k1 would read past the bound checked below
    if (d.A2 && d.k1 < 0) return false;
    const int k1 = d.A2 ? d.k1 : d.K;
    return d.K > 0 && d.K % NG_BK == 0 && (k1 >= d.K || k1 % NG_BK == 0) && (!d.B2 || d.n1 % NG_BN == 0) &&
           (k1 == 0 || fits((long long)(d.M - 1) * d.sam + (long long)(k1 - 1) * d.sak)) &&
           (!d.A2 || k1 >= d.K || fits((long long)(d.M - 1) * d.sam2 + (long long)(d.K - k1 - 1) * d.sak2)) &&
           fits((long long)((d.B2 ? d.n1 : d.N) - 1) * d.sbn + (long long)(d.K - 1) * d.sbk) &&
           (!d.B2 || fits((long long)(d.N - d.n1 - 1) * d.sbn2 + (long long)(d.K - 1) * d.sbk2));
}

int ured_node_gemm_batch(const UredNodeGemmDesc* const* ds, int n, void* stream) {
    ured::clear_error();
    URED_REQUIRE(ds && n >= 1 && n <= URED_NODE_MAX_JOBS, "ured_node_gemm_batch: 1..%d jobs", URED_NODE_MAX_JOBS);
    NodeJobs jobs;
    jobs.njobs = 0;
    int tiles = 0;
    for (int i = 0; i < n; ++i) {
        URED_REQUIRE(ds[i], "ured_node_gemm_batch: null descriptor");
        const UredNodeGemmDesc& d = *ds[i];
        if (d.M == 0 || d.N == 0) continue;
        NodeJob& J = jobs.job[jobs.njobs];
        const int rc = check_node_job(d, J);
        if (rc) return rc;
        jobs.tile0[jobs.njobs] = tiles;
        tiles += d.kind == URED_NODE_COLSUM ? J.ntn : ((d.M + NG_BM - 1) / NG_BM) * J.ntn;
        ++jobs.njobs;
    }
    if (jobs.njobs == 0) return 0;
    for (int q = jobs.njobs; q <= NG_JOBS; ++q) jobs.tile0[q] = tiles;
    bool v4 = URED_NODE_V4;
    for (int q = 0; q < jobs.njobs; ++q) v4 = v4 && node_v4_ok(jobs.job[q].d);
    if (v4) hipLaunchKernelGGL(node_gemm4_kernel, dim3(tiles), dim3(NG_NT), 0, (hipStream_t)stream, jobs);
    else hipLaunchKernelGGL(node_gemm_kernel, dim3(tiles), dim3(NG_NT), 0, (hipStream_t)stream, jobs);
    return ured::launch_status("ured_node_gemm");
}

int ured_node_gemm(const UredNodeGemmDesc* dp, void* stream) {
    ured::clear_error();
    URED_REQUIRE(dp, "ured_node_gemm: null descriptor");
    const UredNodeGemmDesc* one[1] = {dp};
    return ured_node_gemm_batch(one, 1, stream);
}

int ured_node_bn_fwd(const UredNodeBNDesc* dp, void* stream) {
    ured::clear_error();
    URED_REQUIRE(dp, "ured_node_bn_fwd: null descriptor");
    const UredNodeBNDesc& d = *dp;
    URED_REQUIRE(d.nsets >= 1 && d.nsets <= URED_NODE_MAX_SETS && d.N >= 1, "ured_node_bn_fwd: bad sizes");
    URED_REQUIRE(d.Y && d.gamma && d.beta && d.running_mean && d.running_var &&
                 (d.stats_out || (d.mean && d.invstd && d.act)), "ured_node_bn_fwd: null pointer");
    URED_REQUIRE(!(d.stats_out && d.stats_in), "ured_node_bn_fwd: stats_out and stats_in are exclusive");
    URED_REQUIRE(d.training || !(d.stats_out || d.stats_in), "ured_node_bn_fwd: SyncBN statistics in eval mode");
    for (int s = 0; s < d.nsets; ++s)
        URED_REQUIRE(d.off[s] <= d.off[s + 1], "ured_node_bn_fwd: set offsets must be non-decreasing");
    hipLaunchKernelGGL(node_bn_fwd_kernel, dim3((d.N + BN_COLS - 1) / BN_COLS), dim3(BN_NT), 0, (hipStream_t)stream, d);
    return ured::launch_status("ured_node_bn_fwd");
}

int ured_node_bn_bwd(const UredNodeBNBwdDesc* dp, void* stream) {
    ured::clear_error();
    URED_REQUIRE(dp, "ured_node_bn_bwd: null descriptor");
    const UredNodeBNBwdDesc& d = *dp;
    URED_REQUIRE(d.nsets >= 1 && d.nsets <= URED_NODE_MAX_SETS && d.N >= 1, "ured_node_bn_bwd: bad sizes");
    URED_REQUIRE(d.G && d.Y && d.gamma && d.mean && d.invstd && (d.sums_out || (d.dY && d.dgamma && d.dbeta)),
                 "ured_node_bn_bwd: null pointer");
    URED_REQUIRE(!(d.sums_out && d.sums_in), "ured_node_bn_bwd: sums_out and sums_in are exclusive");
    hipLaunchKernelGGL(node_bn_bwd_kernel, dim3((d.N + BN_COLS - 1) / BN_COLS), dim3(BN_NT), 0, (hipStream_t)stream, d);
    return ured::launch_status("ured_node_bn_bwd");
}

#if URED_NODE_TIMING
// phase-timing build only: copy the recorded node-GEMM workgroup timestamps out (n slots of 8 u64)
int ured_debug_node_ts(unsigned long long* host, int n) {
    if (n > NTS_SLOTS) n = NTS_SLOTS;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(ured_nts_buf), (size_t)n * 64) == hipSuccess ? 0 : -1;
}
#endif
}  // extern "C"

URED_DBG_ACCESSOR(ured_dbg_node)
