// nn.hip — nearest-neighbour (chamfer) kernels for MI355X / gfx950.
//
// Replaces the DCD chamfer3D extension
//   Density_aware_Chamfer_Distance/utils_v2/metrics/CD/chamfer3D/chamfer3D.cu:12-195
// and batches the per-sample Shape_Measure / pytorch3d calls of
//   loss/chamfer_loss.py:13-30 and loss/basic_loss.py:249-265
// into ragged "segment pair" launches (no host sync, one launch per family).
//
// Forward design (FP32-VALU bound, ~51 pairs per HBM byte):
//   * one workgroup = 256 threads = a block of queries x all refs of its pair;
//     refs staged through LDS in SoA tiles of NN_TILE points (broadcast reads,
//     every lane of a wave reads the same address -> no bank conflicts);
//   * refs processed two at a time with packed fp32 math (v_pk_add/mul/fma_f32)
//     on exactly the contract formula d = fma(dz,dz, fma(dy,dy, dx*dx));
//   * the hot loop keeps only a running min (v_min3_f32) per 16-ref chunk and
//     remembers the first chunk that lowered the best value; the argmin is
//     recovered at the end by rescanning that one chunk for the first d == best.
//     Strict '<' across chunks + first-equal within the chunk = lowest index on
//     ties, exactly the reference rule (chamfer3D.cu:36-69,126);
//   * QPT queries per thread amortise the LDS reads; RS groups of waves split
//     the ref range when there are too few queries to fill 256 CUs, merged in
//     LDS by (value, chunk) lexicographic min (order-independent result).
// Backward: gather form, deterministic (no float atomics): each point owns its
//   output; the contributions of the other direction are found by streaming the
//   other side's idx array through LDS in ascending order, each wave compacting
//   the entries that target its own 64 points (O(n + m) work per pair).
#define URED_DBG_FILE 2
#include "ured_common.h"
#include "../../include/ured_hip.h"

namespace {

constexpr int NN_THREADS = 256;
constexpr int NN_TILE = 1024;   // refs per LDS tile (12 KiB SoA)
constexpr int NN_CHUNK = 16;    // refs per min-tracking chunk
constexpr float NN_PAD = 1.0e30f;  // padding coordinate: distance overflows to +inf
#ifndef URED_NN_TILE_ALL
#define URED_NN_TILE_ALL 1
#endif

typedef float f2 __attribute__((ext_vector_type(2)));

struct NNFwdArgs {
    const float* a;      // [*,3]
    const float* b;      // [*,3]
    const int4* segs;    // nullptr -> dense mode
    int n, m;            // dense: points per batch in a / b
    int dirs;            // bit0: a->b, bit1: b->a
    float* dist_a; int* idx_a;
    float* dist_b; int* idx_b;
};

__device__ __forceinline__ float sqd(float qx, float qy, float qz, float rx, float ry, float rz) {
    float dx = rx - qx, dy = ry - qy, dz = rz - qz;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

__device__ __forceinline__ void resolve_pair(const NNFwdArgs& A, int dir, int s,
                                             const float*& Q, const float*& R, int& q_off, int& q_len,
                                             int& r_off, int& r_len, float*& dist, int*& idx) {
    int ao, al, bo, bl;
    if (A.segs) {
        int4 sg = A.segs[s];
        ao = sg.x; al = sg.y; bo = sg.z; bl = sg.w;
    } else {
        ao = s * A.n; al = A.n; bo = s * A.m; bl = A.m;
    }
    if (dir == 0) { Q = A.a; R = A.b; q_off = ao; q_len = al; r_off = bo; r_len = bl; dist = A.dist_a; idx = A.idx_a; }
    else          { Q = A.b; R = A.a; q_off = bo; q_len = bl; r_off = ao; r_len = al; dist = A.dist_b; idx = A.idx_b; }
}

// TILE: refs per LDS fill. The whole-set variant (TILE = NN_TILE_ALL, used when every segment's
// refs fit) fills LDS once and takes the argmin rescan of the winning chunk from LDS too, so a
// small launch pays one fill and no dependent global reads at the end.
constexpr int NN_TILE_ALL = 4096;   // 48 KiB SoA
template <int QPT, int RS, int TILE = NN_TILE>
__global__ __launch_bounds__(NN_THREADS) void nn_fwd_kernel(NNFwdArgs args) {
    constexpr int G = NN_THREADS / RS;      // threads per ref-split group
    constexpr int QB = G * QPT;             // queries per block
    constexpr int SUB = TILE / RS;          // refs per group per tile
    constexpr bool ALL = TILE == NN_TILE_ALL;
    __shared__ __attribute__((aligned(16))) float sx[TILE];
    __shared__ __attribute__((aligned(16))) float sy[TILE];
    __shared__ __attribute__((aligned(16))) float sz[TILE];
    __shared__ float mbest[RS > 1 ? RS * QB : 1];
    __shared__ int mchunk[RS > 1 ? RS * QB : 1];

    const int dir = (args.dirs == 2) ? 1 : (int)blockIdx.z;
    const float *Q, *R; int q_off, q_len, r_off, r_len; float* dist; int* idx;
    resolve_pair(args, dir, blockIdx.y, Q, R, q_off, q_len, r_off, r_len, dist, idx);
    // a segment table entry must be non-negative and fit the launch's bounds (the grid covers
    // max_q queries per segment; a longer segment would leave queries unwritten)
    URED_DBG_CHECK(q_off >= 0 && r_off >= 0 && q_len >= 0 && r_len >= 0 && q_len <= (int)gridDim.x * QB);
    const int q0 = blockIdx.x * QB;
    if (q0 >= q_len) return;                 // uniform per block
    const int t = threadIdx.x, g = t / G, u = t % G;

    if (r_len <= 0) {
        for (int i = t; i < QB; i += NN_THREADS)
            if (q0 + i < q_len) { dist[q_off + q0 + i] = 0.f; idx[q_off + q0 + i] = 0; }
        return;
    }

    float qx[QPT], qy[QPT], qz[QPT], best[QPT];
    int bchunk[QPT];
#pragma unroll
    for (int i = 0; i < QPT; ++i) {
        int qi = q0 + u + i * G;
        qi = qi < q_len ? qi : q_len - 1;    // clamp: duplicate work, result discarded
        const float* p = Q + 3 * (size_t)(q_off + qi);
        qx[i] = p[0]; qy[i] = p[1]; qz[i] = p[2];
        best[i] = __builtin_inff();
        bchunk[i] = 0;
    }

    for (int t0 = 0; t0 < r_len; t0 += TILE) {
        const int tn = min(TILE, r_len - t0);
        // refs per group: SUB, or (whole-set tile) the fill split evenly over the RS groups in
        // whole chunks (RS * sub <= TILE, since TILE is a multiple of RS * NN_CHUNK)
        const int sub = ALL ? ((tn + RS - 1) / RS + NN_CHUNK - 1) / NN_CHUNK * NN_CHUNK : SUB;
        __syncthreads();
        const int fill = ALL ? RS * sub : TILE;
        const float* rp = R + 3 * (size_t)(r_off + t0);
        if ((((uintptr_t)rp) & 15) == 0) {
            // four points (three float4) per thread and step, the steps unrolled so their loads
            // are in flight together; SoA rows written as float4
            const int full = min(tn, fill) >> 2;             // whole groups of 4 points
            const int part = (tn < fill && (tn & 3)) ? full : -1;   // the group holding the last point
#pragma unroll 4
            for (int i4 = t; i4 < (fill >> 2); i4 += NN_THREADS) {
                if (i4 == part) continue;
                float4 v0 = make_float4(NN_PAD, NN_PAD, NN_PAD, NN_PAD), v1 = v0, v2 = v0;
                if (i4 < full) {
                    const float4* q4 = reinterpret_cast<const float4*>(rp) + 3 * i4;
                    v0 = q4[0]; v1 = q4[1]; v2 = q4[2];
                }
                *reinterpret_cast<float4*>(sx + 4 * i4) = make_float4(v0.x, v0.w, v1.z, v2.y);
                *reinterpret_cast<float4*>(sy + 4 * i4) = make_float4(v0.y, v1.x, v1.w, v2.z);
                *reinterpret_cast<float4*>(sz + 4 * i4) = make_float4(v0.z, v1.y, v2.x, v2.w);
            }
            // the partial group, point by point
            if (part >= 0 && t < 4) {
                const int i = 4 * part + t;
                float x = NN_PAD, y = NN_PAD, z = NN_PAD;
                if (i < tn) { x = rp[3 * i]; y = rp[3 * i + 1]; z = rp[3 * i + 2]; }
                sx[i] = x; sy[i] = y; sz[i] = z;
            }
        } else {
            for (int i = t; i < fill; i += NN_THREADS) {
                float x = NN_PAD, y = NN_PAD, z = NN_PAD;
                if (i < tn) {
                    const float* p = rp + 3 * (size_t)i;
                    x = p[0]; y = p[1]; z = p[2];
                }
                sx[i] = x; sy[i] = y; sz[i] = z;
            }
        }
        __syncthreads();
        // this group's sub-range of the tile, in chunks of NN_CHUNK
        const int base = g * sub;
        const int sub_n = min(sub, max(0, tn - base));
        const int nch = (sub_n + NN_CHUNK - 1) / NN_CHUNK;
        const int chunk0 = (t0 + base) / NN_CHUNK;
        for (int c = 0; c < nch; ++c) {
            const f2* px = reinterpret_cast<const f2*>(sx + base + c * NN_CHUNK);
            const f2* py = reinterpret_cast<const f2*>(sy + base + c * NN_CHUNK);
            const f2* pz = reinterpret_cast<const f2*>(sz + base + c * NN_CHUNK);
            float mn[QPT];
#pragma unroll
            for (int i = 0; i < QPT; ++i) mn[i] = __builtin_inff();
#pragma unroll
            for (int r = 0; r < NN_CHUNK / 2; ++r) {
                const f2 rx = px[r], ry = py[r], rz = pz[r];
#pragma unroll
                for (int i = 0; i < QPT; ++i) {
                    const f2 dx = rx - qx[i];
                    const f2 dy = ry - qy[i];
                    const f2 dz = rz - qz[i];
                    f2 d = dx * dx;
                    d = __builtin_elementwise_fma(dy, dy, d);
                    d = __builtin_elementwise_fma(dz, dz, d);
                    mn[i] = __builtin_fminf(__builtin_fminf(mn[i], d.x), d.y);
                }
            }
#pragma unroll
            for (int i = 0; i < QPT; ++i)
                if (mn[i] < best[i]) { best[i] = mn[i]; bchunk[i] = chunk0 + c; }
        }
    }

    if constexpr (RS > 1) {
        __syncthreads();
#pragma unroll
        for (int i = 0; i < QPT; ++i) {
            mbest[g * QB + u + i * G] = best[i];
            mchunk[g * QB + u + i * G] = bchunk[i];
        }
        __syncthreads();
        if (g != 0) return;
#pragma unroll
        for (int i = 0; i < QPT; ++i) {
            for (int h = 1; h < RS; ++h) {
                float v = mbest[h * QB + u + i * G];
                int c = mchunk[h * QB + u + i * G];
                if (v < best[i] || (v == best[i] && c < bchunk[i])) { best[i] = v; bchunk[i] = c; }
            }
        }
    }

    // argmin recovery: first ref of the winning chunk whose distance equals best
#pragma unroll
    for (int i = 0; i < QPT; ++i) {
        const int qi = q0 + u + i * G;
        if (qi >= q_len) continue;
        const int k0 = bchunk[i] * NN_CHUNK;
        const int kn = min(NN_CHUNK, r_len - k0);
        URED_DBG_CHECK(k0 >= 0 && k0 < r_len);
        int bi = k0;
        for (int k = 0; k < kn; ++k) {
            float rx, ry, rz;
            if constexpr (ALL) { rx = sx[k0 + k]; ry = sy[k0 + k]; rz = sz[k0 + k]; }
            else {
                const float* p = R + 3 * (size_t)(r_off + k0 + k);
                rx = p[0]; ry = p[1]; rz = p[2];
            }
            if (sqd(qx[i], qy[i], qz[i], rx, ry, rz) == best[i]) { bi = k0 + k; break; }
        }
        dist[q_off + qi] = best[i];
        idx[q_off + qi] = bi;
    }
}

struct NNBwdArgs {
    const float* a; const float* b; const int4* segs; int n, m;
    const float* gd_a; const float* gd_b; const int* idx_a; const int* idx_b;
    float* ga; float* gb;
    int accumulate;      // 1: ga/gb += (the reference contract); 0: ga/gb = (no zero fill needed)
};

// Gradient for the points of one side of a pair (dir 0: a-points, dir 1: b-points).
__global__ __launch_bounds__(NN_THREADS) void nn_bwd_kernel(NNBwdArgs args) {
    __shared__ __attribute__((aligned(16))) int sidx[NN_TILE];
    __shared__ float sg[NN_TILE], sx[NN_TILE], sy[NN_TILE], sz[NN_TILE];
    __shared__ int slist[(NN_THREADS / 64) * NN_TILE];   // per-wave compacted entry lists
    const int dir = blockIdx.z, s = blockIdx.y;
    int ao, al, bo, bl;
    if (args.segs) { int4 q = args.segs[s]; ao = q.x; al = q.y; bo = q.z; bl = q.w; }
    else { ao = s * args.n; al = args.n; bo = s * args.m; bl = args.m; }
    const float *P, *O, *gdP, *gdO; const int *idxP, *idxO; float* gP; int p_off, p_len, o_off, o_len;
    if (dir == 0) { P = args.a; O = args.b; gdP = args.gd_a; gdO = args.gd_b; idxP = args.idx_a; idxO = args.idx_b; gP = args.ga;
                    p_off = ao; p_len = al; o_off = bo; o_len = bl; }
    else          { P = args.b; O = args.a; gdP = args.gd_b; gdO = args.gd_a; idxP = args.idx_b; idxO = args.idx_a; gP = args.gb;
                    p_off = bo; p_len = bl; o_off = ao; o_len = al; }
    const int j0 = blockIdx.x * NN_THREADS;
    if (j0 >= p_len) return;
    const int j = j0 + threadIdx.x;
    const bool valid = j < p_len;
    const int jc = valid ? j : p_len - 1;
    const float* pj = P + 3 * (size_t)(p_off + jc);
    const float px = pj[0], py = pj[1], pz = pj[2];
    float ax = 0.f, ay = 0.f, az = 0.f;
    URED_DBG_CHECK(p_off >= 0 && o_off >= 0 && p_len >= 0 && o_len >= 0);
    if (o_len > 0 && gdP) {
        URED_DBG_CHECK((unsigned)idxP[p_off + jc] < (unsigned)o_len);   // the NN index lies in the other side
        const float* r = O + 3 * (size_t)(o_off + idxP[p_off + jc]);
        const float g = gdP[p_off + jc] * 2.f;
        ax = g * (px - r[0]); ay = g * (py - r[1]); az = g * (pz - r[2]);
    }
    if (gdO) {
        for (int t0 = 0; t0 < o_len; t0 += NN_TILE) {
            const int tn = min(NN_TILE, o_len - t0);
            __syncthreads();
            for (int i = threadIdx.x; i < NN_TILE; i += NN_THREADS) {
                int id = -1; float gg = 0.f, x = 0.f, y = 0.f, z = 0.f;
                if (i < tn) {
                    const int k = o_off + t0 + i;
                    id = idxO[k]; gg = gdO[k];
                    x = O[3 * (size_t)k]; y = O[3 * (size_t)k + 1]; z = O[3 * (size_t)k + 2];
                }
                sidx[i] = id; sg[i] = gg; sx[i] = x; sy[i] = y; sz[i] = z;
            }
            __syncthreads();
            // Each wave compacts, in ascending k, the tile entries whose NN lands in its own 64
            // points (ballot + prefix popcount), then walks only that list; the owner lane
            // accumulates. Same summation order as a full ascending scan (own term first, then
            // k ascending), so the result is bit-identical to it — without every lane paying
            // for every entry.
            const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
            const int jw0 = j0 + wv * 64;
            int* lst = slist + wv * NN_TILE;
            int cnt = 0;
            for (int c = 0; c < tn; c += 64) {
                const int k = c + ln;
                const int id = k < tn ? sidx[k] : -1;
                const bool pred = (unsigned)(id - jw0) < 64u;
                const unsigned long long mask = __ballot(pred);
                if (pred) lst[cnt + __popcll(mask & ((1ull << ln) - 1ull))] = k;
                cnt += __popcll(mask);
            }
            for (int e = 0; e < cnt; ++e) {
                const int k = lst[e];
                const bool own = sidx[k] == j;
                const float g = sg[k] * 2.f;
                const float nx = ax - g * (sx[k] - px);
                const float ny = ay - g * (sy[k] - py);
                const float nz = az - g * (sz[k] - pz);
                ax = own ? nx : ax; ay = own ? ny : ay; az = own ? nz : az;
            }
        }
    }
    if (valid) {
        float* o = gP + 3 * (size_t)(p_off + j);
        if (args.accumulate) { ax += o[0]; ay += o[1]; az += o[2]; }
        o[0] = ax; o[1] = ay; o[2] = az;
    }
}

template <int QPT, int RS>
void launch_fwd(const NNFwdArgs& a, int max_q, int max_r, int nseg, int ndirs, hipStream_t st) {
    constexpr int QB = (NN_THREADS / RS) * QPT;
    dim3 grid((max_q + QB - 1) / QB, nseg, ndirs);
    if (URED_NN_TILE_ALL && max_r <= NN_TILE_ALL)
        hipLaunchKernelGGL((nn_fwd_kernel<QPT, RS, NN_TILE_ALL>), grid, dim3(NN_THREADS), 0, st, a);
    else
        hipLaunchKernelGGL((nn_fwd_kernel<QPT, RS>), grid, dim3(NN_THREADS), 0, st, a);
}

// Pick queries-per-thread / ref-split so that the launch has enough waves for 256 CUs.
int fwd_dispatch(const NNFwdArgs& a, int nseg, int max_a, int max_b, hipStream_t st) {
    const int ndirs = (a.dirs == 3) ? 2 : 1;
    int max_q = 0, max_r = 0;
    long long total_q = 0;
    if (a.dirs & 1) { max_q = max(max_q, max_a); max_r = max(max_r, max_b); total_q += (long long)nseg * max_a; }
    if (a.dirs & 2) { max_q = max(max_q, max_b); max_r = max(max_r, max_a); total_q += (long long)nseg * max_b; }
    if (max_q <= 0 || nseg <= 0) return 0;
    // waves launched with QPT=2, RS=1: 4 waves per 512 queries
    const long long waves1 = (total_q + 511) / 512 * 4;
    // about 2048 waves (two per SIMD) or as close as the splits allow; with the whole-set tile
    // a small ref set splits evenly too. Measured (graph-replayed, tools/chamfer_rates.py):
    // 16x2048x2048 <2,4> 26.1 us (<1,4> 26.9, <1,8> 30.8); 32x2000x1000 <2,4> 32.7 (<1,8> 33.4);
    // 2x512x512 <1,8> 5.4 (<2,4> 8.3, <2,1> 15.6)
    // With the whole-set tile the split is at least 4 ref groups: a ragged launch (the loss head's
    // part family: 512 segments, a quarter of them non-empty) is sized by its bounds, so waves1
    // overstates its work; 4 groups cost one small LDS combine where the bound is tight.
    const bool all = URED_NN_TILE_ALL && max_r <= NN_TILE_ALL;
    if (!all && (waves1 >= 4096 || max_r < NN_TILE)) launch_fwd<2, 1>(a, max_q, max_r, nseg, ndirs, st);
    else if (!all && waves1 >= 2048) launch_fwd<2, 2>(a, max_q, max_r, nseg, ndirs, st);
    // whole-set tile over 2048 refs: eight ref groups (512 refs each); 32 x 4096 x 2048 both
    // directions <2,8> 77 us vs <2,4> 99 (at 2048 refs <2,4> stays ahead: 44 vs 46)
    else if (all && waves1 >= 512 && max_r > 2048) launch_fwd<2, 8>(a, max_q, max_r, nseg, ndirs, st);
    else if (waves1 >= 512 || !all) launch_fwd<2, 4>(a, max_q, max_r, nseg, ndirs, st);
    else if (waves1 >= 256) launch_fwd<1, 4>(a, max_q, max_r, nseg, ndirs, st);
    else launch_fwd<1, 8>(a, max_q, max_r, nseg, ndirs, st);
    return 0;
}

// ---- fused forward: both directions from ONE evaluation of every distance -----------------
// The two-pass kernel above evaluates each pair twice (once per direction). Here a wave holds
// QPT queries (a-points) per lane in registers (64*QPT per wave, contiguous per lane) and
// streams a range of refs (b-points) through its own LDS tile; each distance feeds
//   * the query's running row minimum (in-lane v_min3, chunk-of-16 tracking as above), and
//   * the ref's column minimum: in-lane over the lane's QPT queries, then across the wave
//     (4 DPP steps + 4 readlanes on the float bits — distances are >= 0, so the unsigned
//     order is the float order), and the FIRST lane holding that minimum by a ballot.
// Each wave stores, per ref / per query, a 64-bit key (value bits << 32 | tag) into a
// workspace slab (one slot per (q-tile, ref) and per (ref-range, query); plain stores, no
// atomics); nn_fused_finalize takes the lexicographic minimum over the slab (lowest tag
// on equal values = lowest chunk / lowest query group) and rescans that one chunk (16 refs)
// or query group (QPT queries) for the first index with d == min: the reference's
// lowest-index tie rule, exactly, with every distance evaluated by the contract formula.
constexpr int NF_TILE = 512;    // refs per LDS fill (per wave, 6 KiB SoA)
#ifndef URED_NF_TARGET_WAVES
#define URED_NF_TARGET_WAVES 4096
#endif
#ifndef URED_NF_QPT16_PAIRS
#define URED_NF_QPT16_PAIRS (1ll << 28)
#endif
constexpr int NF_TARGET_WAVES = URED_NF_TARGET_WAVES;

struct NNFusedArgs {
    const float* a; const float* b; const int4* segs;
    int n, m;                    // dense mode sizes
    int qtiles, rsplit, rr;      // grid.x = qtiles * rsplit; rr refs per range (multiple of 16)
    int a_total, b_total;        // slab strides
    unsigned long long* rowslab; // [rsplit][a_total]
    unsigned long long* colslab; // [qtiles][b_total]
    float* dist_a; int* idx_a; float* dist_b; int* idx_b;
};

__device__ __forceinline__ void seg_of(const NNFusedArgs& A, int s, int& ao, int& al, int& bo, int& bl) {
    if (A.segs) { const int4 q = A.segs[s]; ao = q.x; al = q.y; bo = q.z; bl = q.w; }
    else { ao = s * A.n; al = A.n; bo = s * A.m; bl = A.m; }
}

template <int CTRL, int ROW_MASK>
__device__ __forceinline__ unsigned dpp_min(unsigned v) {
    // full-row patterns: every lane has a source (foldable into v_min_u32_dpp);
    // row_bcast with a row mask: rows outside the mask keep v (old = v)
    const unsigned o = ROW_MASK == 0xF
        ? (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true)
        : (unsigned)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, ROW_MASK, 0xF, false);
    return v < o ? v : o;
}

// s_min_u32 on wave-uniform values (hipcc otherwise moves them to VGPRs for a v_min3_u32).
__device__ __forceinline__ unsigned smin(unsigned a, unsigned b) {
    unsigned r;
    asm("s_min_u32 %0, %1, %2" : "=s"(r) : "s"(a), "s"(b));
    return r;
}

// Minimum over the 64 lanes of each of four values, as wave-uniform (SGPR) results. Four
// independent DPP chains interleaved (no hazard nops) make each value uniform within its row
// of 16 lanes; four readlanes and scalar mins finish the reduction.
__device__ __forceinline__ void wave_min4(unsigned (&v)[4], unsigned (&w)[4]) {
#define URED_STEP(C) _Pragma("unroll") for (int k = 0; k < 4; ++k) v[k] = dpp_min<C, 0xF>(v[k]);
    URED_STEP(0xB1)    // quad_perm [1,0,3,2]
    URED_STEP(0x4E)    // quad_perm [2,3,0,1]
    URED_STEP(0x141)   // row_half_mirror
    URED_STEP(0x140)   // row_mirror
#undef URED_STEP
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const unsigned r0 = (unsigned)__builtin_amdgcn_readlane((int)v[k], 0);
        const unsigned r1 = (unsigned)__builtin_amdgcn_readlane((int)v[k], 16);
        const unsigned r2 = (unsigned)__builtin_amdgcn_readlane((int)v[k], 32);
        const unsigned r3 = (unsigned)__builtin_amdgcn_readlane((int)v[k], 48);
        w[k] = smin(smin(r0, r1), smin(r2, r3));
    }
}

// v_writelane_b32 (lane `sel` of `old` := src, both wave-uniform): the LLVM intrinsic under its
// IR name (this toolchain has no clang builtin for it); the compiler routes `sel` through m0.
__device__ int ured_writelane(int src, int sel, int old) __asm("llvm.amdgcn.writelane.i32");

template <int QPT>
__global__ __launch_bounds__(64) void nn_fused_kernel(NNFusedArgs A) {
    // refs stored replicated ({x,x}) so one LDS read feeds both halves of a packed op whose
    // other operand is a pair of queries: queries then need no replicated registers.
    __shared__ __attribute__((aligned(16))) f2 sx[NF_TILE];
    __shared__ __attribute__((aligned(16))) f2 sy[NF_TILE];
    __shared__ __attribute__((aligned(16))) f2 sz[NF_TILE];
    constexpr int QP = QPT / 2;
    const int s = blockIdx.y;
    const int qt = blockIdx.x % A.qtiles, rs = blockIdx.x / A.qtiles;
    int ao, al, bo, bl;
    seg_of(A, s, ao, al, bo, bl);
    URED_DBG_CHECK(ao >= 0 && bo >= 0 && al >= 0 && bl >= 0 && ao + al <= A.a_total && bo + bl <= A.b_total);
    const int q0 = qt * 64 * QPT;
    const int r_begin = rs * A.rr;
    if (q0 >= al || r_begin >= bl) return;   // wave-uniform
    const int r_end = min(bl, r_begin + A.rr);
    const int lane = threadIdx.x;

    f2 qx[QP], qy[QP], qz[QP];               // queries 2j, 2j+1 of this lane
    float best[QPT];
    int bchunk[QPT];
#pragma unroll
    for (int i = 0; i < QPT; ++i) {
        const int qi = q0 + lane * QPT + i;
        float x = NN_PAD, y = NN_PAD, z = NN_PAD;   // padded queries: d = +inf to every ref
        if (qi < al) {
            const float* p = A.a + 3 * (size_t)(ao + qi);
            x = p[0]; y = p[1]; z = p[2];
        }
        if (i & 1) { qx[i >> 1].y = x; qy[i >> 1].y = y; qz[i >> 1].y = z; }
        else       { qx[i >> 1].x = x; qy[i >> 1].x = y; qz[i >> 1].x = z; }
        best[i] = __builtin_inff();
        bchunk[i] = 0;
    }
    unsigned long long* colslab = A.colslab + (size_t)qt * A.b_total + bo;
    const int qgroup0 = q0 / QPT;

    for (int t0 = r_begin; t0 < r_end; t0 += NF_TILE) {
        const int tn = min(NF_TILE, r_end - t0);
        __syncthreads();
        for (int k = lane; k < ((tn + 15) & ~15); k += 64) {
            float x = NN_PAD, y = NN_PAD, z = NN_PAD;
            if (k < tn) {
                const float* p = A.b + 3 * (size_t)(bo + t0 + k);
                x = p[0]; y = p[1]; z = p[2];
            }
            sx[k] = f2{x, x}; sy[k] = f2{y, y}; sz[k] = f2{z, z};
        }
        __syncthreads();
        const int nch = (tn + 15) >> 4;
        for (int c = 0; c < nch; ++c) {
            float mn[QPT];
#pragma unroll
            for (int i = 0; i < QPT; ++i) mn[i] = __builtin_inff();
            int klo = 0, khi = 0;        // lane k < 16: column key (tag, value bits) of ref k of this chunk
#pragma unroll 1
            for (int p = 0; p < 16; p += 4) {
                f2 rx[4], ry[4], rz[4];
#pragma unroll
                for (int h = 0; h < 4; ++h) { rx[h] = sx[c * 16 + p + h]; ry[h] = sy[c * 16 + p + h]; rz[h] = sz[c * 16 + p + h]; }
                float cm[4] = {__builtin_inff(), __builtin_inff(), __builtin_inff(), __builtin_inff()};
#pragma unroll
                for (int j = 0; j < QP; ++j) {
                    f2 d[4];
#pragma unroll
                    for (int h = 0; h < 4; ++h) {
                        const f2 dx = rx[h] - qx[j], dy = ry[h] - qy[j], dz = rz[h] - qz[j];
                        f2 e = dx * dx;
                        e = __builtin_elementwise_fma(dy, dy, e);
                        d[h] = __builtin_elementwise_fma(dz, dz, e);
                    }
                    mn[2 * j] = __builtin_fminf(__builtin_fminf(mn[2 * j], d[0].x), d[1].x);
                    mn[2 * j] = __builtin_fminf(__builtin_fminf(mn[2 * j], d[2].x), d[3].x);
                    mn[2 * j + 1] = __builtin_fminf(__builtin_fminf(mn[2 * j + 1], d[0].y), d[1].y);
                    mn[2 * j + 1] = __builtin_fminf(__builtin_fminf(mn[2 * j + 1], d[2].y), d[3].y);
#pragma unroll
                    for (int h = 0; h < 4; ++h) cm[h] = __builtin_fminf(__builtin_fminf(cm[h], d[h].x), d[h].y);
                }
                // column keys of refs p .. p+3: wave minimum + first lane holding it
                const unsigned v[4] = {__float_as_uint(cm[0]), __float_as_uint(cm[1]),
                                       __float_as_uint(cm[2]), __float_as_uint(cm[3])};
                unsigned t[4] = {v[0], v[1], v[2], v[3]}, w[4];
                wave_min4(t, w);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const unsigned tag = (unsigned)qgroup0 + (unsigned)__builtin_ctzll(__ballot(v[k] == w[k]));
                    klo = ured_writelane((int)tag, p + k, klo);
                    khi = ured_writelane((int)w[k], p + k, khi);
                }
            }
            const int gc = (t0 + c * 16) >> 4;       // chunk index within the segment's refs
#pragma unroll
            for (int i = 0; i < QPT; ++i)
                if (mn[i] < best[i]) { best[i] = mn[i]; bchunk[i] = gc; }
            const int r = t0 + c * 16 + lane;
            if (lane < 16 && r < r_end)
                colslab[r] = ((unsigned long long)(unsigned)khi << 32) | (unsigned)klo;
        }
    }
    unsigned long long* rowslab = A.rowslab + (size_t)rs * A.a_total + ao;
#pragma unroll
    for (int i = 0; i < QPT; ++i) {
        const int qi = q0 + lane * QPT + i;
        if (qi < al) rowslab[qi] = ((unsigned long long)__float_as_uint(best[i]) << 32) | (unsigned)bchunk[i];
    }
}

// One thread per point of either side: lexicographic min over the slab, then the exact rescan.
template <int QPT>
__global__ __launch_bounds__(256) void nn_fused_finalize(NNFusedArgs A) {
    const int s = blockIdx.y, dir = blockIdx.z;
    int ao, al, bo, bl;
    seg_of(A, s, ao, al, bo, bl);
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (dir == 0) {
        if (j >= al) return;
        if (bl <= 0) { A.dist_a[ao + j] = 0.f; A.idx_a[ao + j] = 0; return; }
        const int nrs = (bl + A.rr - 1) / A.rr;
        unsigned long long key = ~0ull;
        for (int r = 0; r < nrs; ++r) {
            const unsigned long long k = A.rowslab[(size_t)r * A.a_total + ao + j];
            key = k < key ? k : key;
        }
        const float v = __uint_as_float((unsigned)(key >> 32));
        const int k0 = (int)(unsigned)key * 16, kn = min(16, bl - k0);
        URED_DBG_CHECK(ao + al <= A.a_total && k0 >= 0 && k0 < bl);
        const float* q = A.a + 3 * (size_t)(ao + j);
        int bi = k0;
        for (int k = 0; k < kn; ++k) {
            const float* p = A.b + 3 * (size_t)(bo + k0 + k);
            if (sqd(q[0], q[1], q[2], p[0], p[1], p[2]) == v) { bi = k0 + k; break; }
        }
        A.dist_a[ao + j] = v;
        A.idx_a[ao + j] = bi;
    } else {
        if (j >= bl) return;
        if (al <= 0) { A.dist_b[bo + j] = 0.f; A.idx_b[bo + j] = 0; return; }
        const int nqt = (al + 64 * QPT - 1) / (64 * QPT);
        unsigned long long key = ~0ull;
        for (int t = 0; t < nqt; ++t) {
            const unsigned long long k = A.colslab[(size_t)t * A.b_total + bo + j];
            key = k < key ? k : key;
        }
        const float v = __uint_as_float((unsigned)(key >> 32));
        const int k0 = (int)(unsigned)key * QPT, kn = min(QPT, al - k0);
        URED_DBG_CHECK(bo + bl <= A.b_total && k0 >= 0 && k0 < al);
        const float* p = A.b + 3 * (size_t)(bo + j);
        int bi = k0;
        for (int k = 0; k < kn; ++k) {
            const float* q = A.a + 3 * (size_t)(ao + k0 + k);
            if (sqd(q[0], q[1], q[2], p[0], p[1], p[2]) == v) { bi = k0 + k; break; }
        }
        A.dist_b[bo + j] = v;
        A.idx_b[bo + j] = bi;
    }
}

// Grid plan of the fused path (host-only arithmetic; also sizes the workspace).
struct FusedPlan { int qpt, qtiles, rsplit, rr; size_t ws_bytes; };

FusedPlan fused_plan(int nseg, int max_a, int max_b, int a_total, int b_total) {
    FusedPlan p{};
    if (nseg <= 0 || max_a <= 0 || max_b <= 0) return p;
    const long long pairs = (long long)nseg * max_a * max_b;
    p.qpt = (pairs >= URED_NF_QPT16_PAIRS && max_a >= 1024) ? 16 : 8;
    const int qtile = 64 * p.qpt;
    p.qtiles = (max_a + qtile - 1) / qtile;
    const long long base = (long long)nseg * p.qtiles;
    // The grid is sized by the host-side bounds; ragged tables usually hold far less work (the
    // step's part family: 64 of 256 pairs non-empty, refs ~1/4 of the bound). With the buffers
    // partitioned by the segments, a_total * b_total / nseg estimates the real pair count; plan
    // proportionally more waves so that about NF_TARGET_WAVES of them do work (at most 4x).
    const double est = (double)a_total * (double)b_total / (double)nseg;
    const double ratio = est > 0.0 ? (double)pairs / est : 1.0;
    const long long target = (long long)(NF_TARGET_WAVES * (ratio < 1.0 ? 1.0 : (ratio > 4.0 ? 4.0 : ratio)));
    long long rs = (target + base - 1) / base;
    const long long rs_max = (max_b + 63) / 64;         // at least 64 refs per wave
    rs = rs < 1 ? 1 : (rs > rs_max ? rs_max : rs);
    int rr = (int)((max_b + rs - 1) / rs);
    rr = (rr + 15) & ~15;
    p.rr = rr;
    p.rsplit = (max_b + rr - 1) / rr;
    p.ws_bytes = 8ull * ((size_t)p.rsplit * (size_t)a_total + (size_t)p.qtiles * (size_t)b_total);
    return p;
}

int fused_dispatch(NNFusedArgs a, int nseg, int max_a, int max_b, void* ws, size_t ws_bytes, hipStream_t st) {
    const FusedPlan p = fused_plan(nseg, max_a, max_b, a.a_total, a.b_total);
    if (p.qpt == 0) return -1;   // not applicable: the caller runs the two-pass kernel
    URED_REQUIRE(ws && ws_bytes >= p.ws_bytes, "nn fused: workspace of %zu bytes needed (got %zu)", p.ws_bytes, ws_bytes);
    URED_REQUIRE((long long)p.qtiles * p.rsplit < (1ll << 31), "nn fused: grid too large");
    a.qtiles = p.qtiles; a.rsplit = p.rsplit; a.rr = p.rr;
    a.rowslab = reinterpret_cast<unsigned long long*>(ws);
    a.colslab = a.rowslab + (size_t)p.rsplit * a.a_total;
    const dim3 grid(p.qtiles * p.rsplit, nseg), fgrid((max(max_a, max_b) + 255) / 256, nseg, 2);
    if (p.qpt == 16) {
        hipLaunchKernelGGL(nn_fused_kernel<16>, grid, dim3(64), 0, st, a);
        hipLaunchKernelGGL(nn_fused_finalize<16>, fgrid, dim3(256), 0, st, a);
    } else {
        hipLaunchKernelGGL(nn_fused_kernel<8>, grid, dim3(64), 0, st, a);
        hipLaunchKernelGGL(nn_fused_finalize<8>, fgrid, dim3(256), 0, st, a);
    }
    return 0;
}

// sides = 2: a and b points; 1: the a points only (blockIdx.z = 0)
int bwd_dispatch(const NNBwdArgs& a, int nseg, int max_a, int max_b, hipStream_t st, int sides = 2) {
    const int max_p = sides == 2 ? max(max_a, max_b) : max_a;
    if (max_p <= 0 || nseg <= 0) return 0;
    dim3 grid((max_p + NN_THREADS - 1) / NN_THREADS, nseg, sides);
    hipLaunchKernelGGL(nn_bwd_kernel, grid, dim3(NN_THREADS), 0, st, a);
    return 0;
}


// ---- density-aware chamfer reduction (calc_dcd, utils_v2/model_utils.py:13-51) --------
// One workgroup per batch item. NN visit counts live in LDS (integer atomics: exact), the
// six per-item sums are strided per thread then tree-reduced in a fixed order.
constexpr int DCD_THREADS = 256;
constexpr int DCD_MAX_POINTS = 16384;   // n1 + n2 per item (64 KiB of LDS counts)

__global__ __launch_bounds__(DCD_THREADS) void dcd_kernel(const float* __restrict__ d1, const int* __restrict__ i1,
        const float* __restrict__ d2, const int* __restrict__ i2, int n1, int n2, float alpha, int lam,
        float frac12, float frac21, float* __restrict__ loss, float* __restrict__ cdp, float* __restrict__ cdt) {
    extern __shared__ int cnt[];            // [n2] visits of x points by gt NNs, then [n1] vice versa
    __shared__ float red[6][DCD_THREADS];
    int* c1 = cnt;                           // indexed by idx1 (an x point)
    int* c2 = cnt + n2;                      // indexed by idx2 (a gt point)
    const int b = blockIdx.x, t = threadIdx.x;
    const float* D1 = d1 + (size_t)b * n1; const int* I1 = i1 + (size_t)b * n1;
    const float* D2 = d2 + (size_t)b * n2; const int* I2 = i2 + (size_t)b * n2;
    for (int k = t; k < n1 + n2; k += DCD_THREADS) cnt[k] = 0;
    __syncthreads();
    for (int k = t; k < n1; k += DCD_THREADS) {
        URED_DBG_CHECK((unsigned)I1[k] < (unsigned)n2);     // LDS counter index
        atomicAdd(&c1[I1[k]], 1);
    }
    for (int k = t; k < n2; k += DCD_THREADS) {
        URED_DBG_CHECK((unsigned)I2[k] < (unsigned)n1);
        atomicAdd(&c2[I2[k]], 1);
    }
    __syncthreads();
    auto wpow = [&](int c) {
        const float f = (float)c;
        return lam == 1 ? f : (lam == 2 ? f * f : powf(f, (float)lam));
    };
    float l1 = 0.f, l2 = 0.f, s1 = 0.f, s2 = 0.f, t1 = 0.f, t2 = 0.f;
    for (int k = t; k < n1; k += DCD_THREADS) {
        const float d = D1[k];
        const float w = (1.0f / (wpow(c1[I1[k]]) + 1e-6f)) * frac21;
        l1 += 1.0f - expf(-d * alpha) * w;
        s1 += sqrtf(d);
        t1 += d;
    }
    for (int k = t; k < n2; k += DCD_THREADS) {
        const float d = D2[k];
        const float w = (1.0f / (wpow(c2[I2[k]]) + 1e-6f)) * frac12;
        l2 += 1.0f - expf(-d * alpha) * w;
        s2 += sqrtf(d);
        t2 += d;
    }
    red[0][t] = l1; red[1][t] = l2; red[2][t] = s1; red[3][t] = s2; red[4][t] = t1; red[5][t] = t2;
    __syncthreads();
    for (int h = DCD_THREADS / 2; h > 0; h >>= 1) {
        if (t < h) {
#pragma unroll
            for (int q = 0; q < 6; ++q) red[q][t] += red[q][t + h];
        }
        __syncthreads();
    }
    if (t == 0) {
        const float fn1 = (float)n1, fn2 = (float)n2;
        loss[b] = (red[0][0] / fn1 + red[1][0] / fn2) / 2.0f;
        cdp[b] = (red[2][0] / fn1 + red[3][0] / fn2) / 2.0f;
        cdt[b] = red[4][0] / fn1 + red[5][0] / fn2;
    }
}

// ---- get_part regrouping backward (ured_part_rows_bwd) ---------------------------------------
// Row-wise gather: each block covers rows_per_block output rows (C/V vector lanes per row), reads
// the sorted-row gradient and the part-sum gradient of the row's sorted position once each (V
// floats per lane) and writes the sum. HBM-bound: 2 reads + 1 write of R x C floats. `add`
// (nullable, may be `out` itself) is another consumer's gradient of the same tensor, added last:
// out = (ds + dsum) + add, the sum autograd would have formed.
template <int V>
__global__ __launch_bounds__(256) void part_rows_bwd_kernel(const float* __restrict__ ds, const float* __restrict__ dsum,
                                                            const long long* __restrict__ inv,
                                                            const int* __restrict__ gid, int N, int C, long long rows,
                                                            int rows_per_block, const float* add, float* out) {
    const int per_row = C / V;
    const int lr = threadIdx.x / (per_row < 256 ? per_row : 256);
    if (lr >= rows_per_block) return;
    const long long r = (long long)blockIdx.x * rows_per_block + lr;
    if (r >= rows) return;
    const long long b = r / N;
    URED_DBG_CHECK(inv[r] >= 0 && inv[r] < N);
    const long long s = b * N + inv[r];
    const long long g = gid[s];
    URED_DBG_CHECK(g >= 0);
    for (int c = threadIdx.x - lr * (per_row < 256 ? per_row : 256); c < per_row; c += 256) {
        if constexpr (V == 4) {
            float4 v = ds ? reinterpret_cast<const float4*>(ds + s * C)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
            if (dsum) {
                const float4 u = reinterpret_cast<const float4*>(dsum + g * C)[c];
                v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
            }
            if (add) {
                const float4 a = reinterpret_cast<const float4*>(add + r * C)[c];
                v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
            }
            reinterpret_cast<float4*>(out + r * C)[c] = v;
        } else {
            float v = ds ? ds[s * C + c] : 0.f;
            if (dsum) v += dsum[g * C + c];
            if (add) v += add[r * C + c];
            out[r * C + c] = v;
        }
    }
}

// ---- per-part axis-aligned boxes (compute_aabbox, dataset/dataset_utils.py:77-85) ---------
// One workgroup per segment of the label-sorted points: min / max of each coordinate (exact,
// order-independent), then (center, half extent) = ((lo+hi)/2, (hi-lo)/2). Empty segments
// give zeros, as the torch scatter_reduce(include_self=False) over a zero tensor did.
__global__ __launch_bounds__(256) void seg_aabb_kernel(const float* __restrict__ x, const int* __restrict__ off,
                                                       float* __restrict__ out) {
    __shared__ float red[6][4];
    const int g = blockIdx.x, t = threadIdx.x;
    const int r0 = off[g], r1 = off[g + 1];
    URED_DBG_CHECK(r0 >= 0 && r1 >= r0);
    float lo[3] = {__builtin_inff(), __builtin_inff(), __builtin_inff()};
    float hi[3] = {-__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
    for (int r = r0 + t; r < r1; r += 256) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float v = x[3 * (size_t)r + c];
            lo[c] = fminf(lo[c], v);
            hi[c] = fmaxf(hi[c], v);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            lo[c] = fminf(lo[c], __shfl_xor(lo[c], o));
            hi[c] = fmaxf(hi[c], __shfl_xor(hi[c], o));
        }
    }
    if ((t & 63) == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { red[c][t >> 6] = lo[c]; red[3 + c][t >> 6] = hi[c]; }
    }
    __syncthreads();
    if (t < 3) {
        const float l = fminf(fminf(red[t][0], red[t][1]), fminf(red[t][2], red[t][3]));
        const float h = fmaxf(fmaxf(red[3 + t][0], red[3 + t][1]), fmaxf(red[3 + t][2], red[3 + t][3]));
        const bool empty = r1 <= r0;
        out[6 * (size_t)g + t] = empty ? 0.f : (l + h) / 2.0f;
        out[6 * (size_t)g + 3 + t] = empty ? 0.f : (h - l) / 2.0f;
    }
}

// ---- get_shape (dataset/dataset_utils.py:691-726): per part slot, A [R, 6] @ p [6] ---------
// A batched GEMV — HBM-bound (18.9 MB of A at config 2) — that the BLAS libraries run as tile
// GEMMs (130-140 us on MI355X). Forward: one thread per output row, the 6-term fma chain in
// order k = 0..5. Backward (grad of p; A is data): one workgroup per part slot, fixed-order
// shuffle + LDS reduction of the 6 column sums (deterministic).
__global__ __launch_bounds__(256) void get_shape_fwd_kernel(const float* __restrict__ A, const float* __restrict__ p,
                                                            int R, long long total, float* __restrict__ out) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const long long bp = i / R;
    const float2* a = reinterpret_cast<const float2*>(A + 6 * i);
    const float* pp = p + 6 * bp;
    const float2 a0 = a[0], a1 = a[1], a2 = a[2];
    float v = a0.x * pp[0];
    v = __builtin_fmaf(a0.y, pp[1], v);
    v = __builtin_fmaf(a1.x, pp[2], v);
    v = __builtin_fmaf(a1.y, pp[3], v);
    v = __builtin_fmaf(a2.x, pp[4], v);
    v = __builtin_fmaf(a2.y, pp[5], v);
    out[i] = v;
}

__global__ __launch_bounds__(256) void get_shape_bwd_kernel(const float* __restrict__ A, const float* __restrict__ g,
                                                            int R, float* __restrict__ gp) {
    __shared__ float red[4][6];
    const int bp = blockIdx.x, t = threadIdx.x;
    const float* a = A + (size_t)bp * R * 6;
    const float* gg = g + (size_t)bp * R;
    float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = t; r < R; r += 256) {
        const float2* ar = reinterpret_cast<const float2*>(a + 6 * (size_t)r);
        const float2 a0 = ar[0], a1 = ar[1], a2 = ar[2];
        const float gv = gg[r];
        acc[0] = __builtin_fmaf(a0.x, gv, acc[0]); acc[1] = __builtin_fmaf(a0.y, gv, acc[1]);
        acc[2] = __builtin_fmaf(a1.x, gv, acc[2]); acc[3] = __builtin_fmaf(a1.y, gv, acc[3]);
        acc[4] = __builtin_fmaf(a2.x, gv, acc[4]); acc[5] = __builtin_fmaf(a2.y, gv, acc[5]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < 6; ++k) acc[k] += __shfl_xor(acc[k], o);
    if ((t & 63) == 0)
#pragma unroll
        for (int k = 0; k < 6; ++k) red[t >> 6][k] = acc[k];
    __syncthreads();
    if (t < 6) gp[6 * (size_t)bp + t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
}

// get_shape straight from the source database (the training step's form): part slot j reads
// mats[src_j] with src_j = labels[j] (+ nsrc when negative: python indexing,
// dataset_utils.py:800-805) instead of a gathered [nparts, rows, 6] copy, and builds its six
// parameters as weight * param + default in-kernel (the mul and the add of get_shape, in that
// order, rounded separately: bitwise the composed form). The backward returns
// weight * sum_r A grad_out (MulBackward's product after the same fixed-order reduction).
__device__ __forceinline__ long long src_row(const long long* labels, int nsrc, long long j) {
    long long s = labels[j];
    s = s < 0 ? s + nsrc : s;
    URED_DBG_CHECK(s >= 0 && s < nsrc);
    return s < 0 ? 0 : (s >= nsrc ? nsrc - 1 : s);   // out-of-range labels read a valid row
}

__global__ __launch_bounds__(256) void get_shape_src_fwd_kernel(const float* __restrict__ mats,
        const long long* __restrict__ labels, int nsrc, const float* __restrict__ param,
        const float* __restrict__ dflt, float weight, int R, long long total, float* __restrict__ out) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    const long long bp = i / R, r = i - bp * R;
    const float2* a = reinterpret_cast<const float2*>(mats + 6 * (src_row(labels, nsrc, bp) * R + r));
    float pp[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const float w = weight * param[6 * bp + k];
        pp[k] = dflt ? w + dflt[6 * bp + k] : w;
    }
    const float2 a0 = a[0], a1 = a[1], a2 = a[2];
    float v = a0.x * pp[0];
    v = __builtin_fmaf(a0.y, pp[1], v);
    v = __builtin_fmaf(a1.x, pp[2], v);
    v = __builtin_fmaf(a1.y, pp[3], v);
    v = __builtin_fmaf(a2.x, pp[4], v);
    v = __builtin_fmaf(a2.y, pp[5], v);
    out[i] = v;
}

__global__ __launch_bounds__(256) void get_shape_src_bwd_kernel(const float* __restrict__ mats,
        const long long* __restrict__ labels, int nsrc, const float* __restrict__ g, float weight, int R,
        float* __restrict__ gparam) {
    __shared__ float red[4][6];
    const int bp = blockIdx.x, t = threadIdx.x;
    const float* a = mats + (size_t)src_row(labels, nsrc, bp) * R * 6;
    const float* gg = g + (size_t)bp * R;
    float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = t; r < R; r += 256) {
        const float2* ar = reinterpret_cast<const float2*>(a + 6 * (size_t)r);
        const float2 a0 = ar[0], a1 = ar[1], a2 = ar[2];
        const float gv = gg[r];
        acc[0] = __builtin_fmaf(a0.x, gv, acc[0]); acc[1] = __builtin_fmaf(a0.y, gv, acc[1]);
        acc[2] = __builtin_fmaf(a1.x, gv, acc[2]); acc[3] = __builtin_fmaf(a1.y, gv, acc[3]);
        acc[4] = __builtin_fmaf(a2.x, gv, acc[4]); acc[5] = __builtin_fmaf(a2.y, gv, acc[5]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int k = 0; k < 6; ++k) acc[k] += __shfl_xor(acc[k], o);
    if ((t & 63) == 0)
#pragma unroll
        for (int k = 0; k < 6; ++k) red[t >> 6][k] = acc[k];
    __syncthreads();
    if (t < 6) gparam[6 * (size_t)bp + t] = weight * ((red[0][t] + red[1][t]) + (red[2][t] + red[3][t]));
}

}  // namespace

extern "C" {

int ured_abi_version(void) { return URED_ABI_VERSION; }
const char* ured_last_error(void) { return ured::err_buf(); }

int ured_nn_fwd(const float* xyz1, const float* xyz2, int b, int n, int m, int dirs,
                float* dist1, int* idx1, float* dist2, int* idx2, void* stream) {
    ured::clear_error();
    URED_REQUIRE(b >= 0 && n >= 0 && m >= 0, "ured_nn_fwd: negative size (b=%d n=%d m=%d)", b, n, m);
    URED_REQUIRE(dirs >= 1 && dirs <= 3, "ured_nn_fwd: dirs must be 1, 2 or 3 (got %d)", dirs);
    if (b == 0) return 0;
    URED_REQUIRE(xyz1 && xyz2, "ured_nn_fwd: null point buffer");
    URED_REQUIRE(!(dirs & 1) || (dist1 && idx1), "ured_nn_fwd: null dist1/idx1");
    URED_REQUIRE(!(dirs & 2) || (dist2 && idx2), "ured_nn_fwd: null dist2/idx2");
    NNFwdArgs a{xyz1, xyz2, nullptr, n, m, dirs, dist1, idx1, dist2, idx2};
    fwd_dispatch(a, b, n, m, (hipStream_t)stream);
    return ured::launch_status("ured_nn_fwd");
}

size_t ured_nn_fwd_workspace(int nseg, int max_a_len, int max_b_len, int a_total, int b_total, int dirs) {
    if (dirs != 3 || nseg <= 0 || max_a_len <= 0 || max_b_len <= 0 || a_total < 0 || b_total < 0) return 0;
    return fused_plan(nseg, max_a_len, max_b_len, a_total, b_total).ws_bytes;
}

int ured_nn_fwd_ws(const float* xyz1, const float* xyz2, int b, int n, int m, int dirs,
                   float* dist1, int* idx1, float* dist2, int* idx2, void* workspace, size_t ws_bytes,
                   void* stream) {
    if (dirs != 3 || !workspace)
        return ured_nn_fwd(xyz1, xyz2, b, n, m, dirs, dist1, idx1, dist2, idx2, stream);
    ured::clear_error();
    URED_REQUIRE(b >= 0 && n >= 0 && m >= 0, "ured_nn_fwd_ws: negative size (b=%d n=%d m=%d)", b, n, m);
    URED_REQUIRE(b <= 65535, "ured_nn_fwd_ws: b %d exceeds 65535", b);
    if (b == 0 || n == 0 || m == 0)
        return ured_nn_fwd(xyz1, xyz2, b, n, m, dirs, dist1, idx1, dist2, idx2, stream);
    URED_REQUIRE(xyz1 && xyz2 && dist1 && idx1 && dist2 && idx2, "ured_nn_fwd_ws: null pointer");
    URED_REQUIRE((long long)b * n < (1ll << 31) && (long long)b * m < (1ll << 31), "ured_nn_fwd_ws: too many points");
    NNFusedArgs a{xyz1, xyz2, nullptr, n, m, 0, 0, 0, b * n, b * m, nullptr, nullptr, dist1, idx1, dist2, idx2};
    const int rc = fused_dispatch(a, b, n, m, workspace, ws_bytes, (hipStream_t)stream);
    if (rc == -1) return ured_nn_fwd(xyz1, xyz2, b, n, m, dirs, dist1, idx1, dist2, idx2, stream);
    if (rc) return rc;
    return ured::launch_status("ured_nn_fwd_ws");
}

int ured_nn_seg_fwd_ws(const float* a, const float* b, const int* segs, int nseg,
                       int max_a_len, int max_b_len, int dirs, int a_total, int b_total,
                       float* dist_a, int* idx_a, float* dist_b, int* idx_b,
                       void* workspace, size_t ws_bytes, void* stream) {
    if (dirs != 3 || !workspace)
        return ured_nn_seg_fwd(a, b, segs, nseg, max_a_len, max_b_len, dirs, dist_a, idx_a, dist_b, idx_b, stream);
    ured::clear_error();
    URED_REQUIRE(nseg >= 0 && max_a_len >= 0 && max_b_len >= 0 && a_total >= 0 && b_total >= 0,
                 "ured_nn_seg_fwd_ws: negative size");
    URED_REQUIRE(nseg <= 65535, "ured_nn_seg_fwd_ws: nseg %d exceeds 65535", nseg);
    if (nseg == 0) return 0;
    URED_REQUIRE(a && b && segs && dist_a && idx_a && dist_b && idx_b, "ured_nn_seg_fwd_ws: null pointer");
    if (max_a_len == 0 || max_b_len == 0)   // only "empty other side" pairs: the two-pass path writes them
        return ured_nn_seg_fwd(a, b, segs, nseg, max_a_len, max_b_len, dirs, dist_a, idx_a, dist_b, idx_b, stream);
    NNFusedArgs A{a, b, reinterpret_cast<const int4*>(segs), 0, 0, 0, 0, 0, a_total, b_total, nullptr, nullptr,
                  dist_a, idx_a, dist_b, idx_b};
    const int rc = fused_dispatch(A, nseg, max_a_len, max_b_len, workspace, ws_bytes, (hipStream_t)stream);
    if (rc == -1)
        return ured_nn_seg_fwd(a, b, segs, nseg, max_a_len, max_b_len, dirs, dist_a, idx_a, dist_b, idx_b, stream);
    if (rc) return rc;
    return ured::launch_status("ured_nn_seg_fwd_ws");
}

int ured_nn_bwd(const float* xyz1, const float* xyz2, int b, int n, int m,
                const float* gd1, const float* gd2, const int* idx1, const int* idx2,
                float* gxyz1, float* gxyz2, void* stream) {
    ured::clear_error();
    URED_REQUIRE(b >= 0 && n >= 0 && m >= 0, "ured_nn_bwd: negative size");
    if (b == 0) return 0;
    URED_REQUIRE(xyz1 && xyz2 && idx1 && idx2 && gxyz1 && gxyz2, "ured_nn_bwd: null pointer");
    NNBwdArgs a{xyz1, xyz2, nullptr, n, m, gd1, gd2, idx1, idx2, gxyz1, gxyz2, 1};
    bwd_dispatch(a, b, n, m, (hipStream_t)stream);
    return ured::launch_status("ured_nn_bwd");
}

int ured_nn_bwd_set(const float* xyz1, const float* xyz2, int b, int n, int m,
                    const float* gd1, const float* gd2, const int* idx1, const int* idx2,
                    float* gxyz1, float* gxyz2, void* stream) {
    ured::clear_error();
    URED_REQUIRE(b >= 0 && n >= 0 && m >= 0, "ured_nn_bwd_set: negative size");
    if (b == 0) return 0;
    URED_REQUIRE(xyz1 && xyz2 && idx1 && idx2 && gxyz1 && gxyz2, "ured_nn_bwd_set: null pointer");
    URED_REQUIRE(n > 0 && m > 0, "ured_nn_bwd_set: empty point set (the caller zero-fills instead)");
    NNBwdArgs a{xyz1, xyz2, nullptr, n, m, gd1, gd2, idx1, idx2, gxyz1, gxyz2, 0};
    bwd_dispatch(a, b, n, m, (hipStream_t)stream);
    return ured::launch_status("ured_nn_bwd_set");
}

int ured_nn_seg_fwd(const float* a, const float* b, const int* segs, int nseg,
                    int max_a_len, int max_b_len, int dirs,
                    float* dist_a, int* idx_a, float* dist_b, int* idx_b, void* stream) {
    ured::clear_error();
    URED_REQUIRE(nseg >= 0 && max_a_len >= 0 && max_b_len >= 0, "ured_nn_seg_fwd: negative size");
    URED_REQUIRE(dirs >= 1 && dirs <= 3, "ured_nn_seg_fwd: dirs must be 1, 2 or 3 (got %d)", dirs);
    URED_REQUIRE(nseg <= 65535, "ured_nn_seg_fwd: nseg %d exceeds 65535", nseg);
    if (nseg == 0) return 0;
    URED_REQUIRE(a && b && segs, "ured_nn_seg_fwd: null pointer");
    URED_REQUIRE(!(dirs & 1) || (dist_a && idx_a), "ured_nn_seg_fwd: null dist_a/idx_a");
    URED_REQUIRE(!(dirs & 2) || (dist_b && idx_b), "ured_nn_seg_fwd: null dist_b/idx_b");
    NNFwdArgs A{a, b, reinterpret_cast<const int4*>(segs), 0, 0, dirs, dist_a, idx_a, dist_b, idx_b};
    fwd_dispatch(A, nseg, max_a_len, max_b_len, (hipStream_t)stream);
    return ured::launch_status("ured_nn_seg_fwd");
}

int ured_nn_seg_bwd(const float* a, const float* b, const int* segs, int nseg,
                    int max_a_len, int max_b_len,
                    const float* gd_a, const float* gd_b, const int* idx_a, const int* idx_b,
                    float* ga, float* gb, void* stream) {
    ured::clear_error();
    URED_REQUIRE(nseg >= 0 && max_a_len >= 0 && max_b_len >= 0, "ured_nn_seg_bwd: negative size");
    URED_REQUIRE(nseg <= 65535, "ured_nn_seg_bwd: nseg %d exceeds 65535", nseg);
    if (nseg == 0) return 0;
    URED_REQUIRE(a && b && segs && idx_a && idx_b && ga, "ured_nn_seg_bwd: null pointer");
    NNBwdArgs A{a, b, reinterpret_cast<const int4*>(segs), 0, 0, gd_a, gd_b, idx_a, idx_b, ga, gb, 1};
    bwd_dispatch(A, nseg, max_a_len, max_b_len, (hipStream_t)stream, gb ? 2 : 1);
    return ured::launch_status("ured_nn_seg_bwd");
}

int ured_get_shape_fwd(const float* A, const float* p, int nparts, int rows, float* out, void* stream) {
    ured::clear_error();
    URED_REQUIRE(nparts >= 0 && rows >= 0, "ured_get_shape_fwd: negative size");
    if (nparts == 0 || rows == 0) return 0;
    URED_REQUIRE(A && p && out, "ured_get_shape_fwd: null pointer");
    URED_REQUIRE(((uintptr_t)A & 7) == 0, "ured_get_shape_fwd: A must be 8-byte aligned");
    const long long total = (long long)nparts * rows;
    hipLaunchKernelGGL(get_shape_fwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       A, p, rows, total, out);
    return ured::launch_status("ured_get_shape_fwd");
}

int ured_get_shape_bwd(const float* A, const float* grad_out, int nparts, int rows, float* grad_p, void* stream) {
    ured::clear_error();
    URED_REQUIRE(nparts >= 0 && rows >= 0, "ured_get_shape_bwd: negative size");
    if (nparts == 0) return 0;
    URED_REQUIRE(A && grad_out && grad_p, "ured_get_shape_bwd: null pointer");
    URED_REQUIRE(((uintptr_t)A & 7) == 0, "ured_get_shape_bwd: A must be 8-byte aligned");
    hipLaunchKernelGGL(get_shape_bwd_kernel, dim3(nparts), dim3(256), 0, (hipStream_t)stream, A, grad_out, rows, grad_p);
    return ured::launch_status("ured_get_shape_bwd");
}

int ured_get_shape_src_fwd(const float* mats, const long long* labels, int nsrc, const float* param,
                           const float* dflt, float weight, int nparts, int rows, float* out, void* stream) {
    ured::clear_error();
    URED_REQUIRE(nparts >= 0 && rows >= 0 && nsrc >= 0, "ured_get_shape_src_fwd: negative size");
    if (nparts == 0 || rows == 0) return 0;
    URED_REQUIRE(nsrc > 0, "ured_get_shape_src_fwd: empty source database");
    URED_REQUIRE(mats && labels && param && out, "ured_get_shape_src_fwd: null pointer");
    URED_REQUIRE(((uintptr_t)mats & 7) == 0, "ured_get_shape_src_fwd: mats must be 8-byte aligned");
    const long long total = (long long)nparts * rows;
    hipLaunchKernelGGL(get_shape_src_fwd_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, mats, labels, nsrc, param, dflt, weight, rows, total, out);
    return ured::launch_status("ured_get_shape_src_fwd");
}

int ured_get_shape_src_bwd(const float* mats, const long long* labels, int nsrc, const float* grad_out, float weight,
                           int nparts, int rows, float* grad_param, void* stream) {
    ured::clear_error();
    URED_REQUIRE(nparts >= 0 && rows >= 0 && nsrc >= 0, "ured_get_shape_src_bwd: negative size");
    if (nparts == 0) return 0;
    URED_REQUIRE(nsrc > 0, "ured_get_shape_src_bwd: empty source database");
    URED_REQUIRE(mats && labels && grad_out && grad_param, "ured_get_shape_src_bwd: null pointer");
    URED_REQUIRE(((uintptr_t)mats & 7) == 0, "ured_get_shape_src_bwd: mats must be 8-byte aligned");
    hipLaunchKernelGGL(get_shape_src_bwd_kernel, dim3(nparts), dim3(256), 0, (hipStream_t)stream, mats, labels, nsrc,
                       grad_out, weight, rows, grad_param);
    return ured::launch_status("ured_get_shape_src_bwd");
}

int ured_seg_aabb(const float* x, const int* off, int G, float* out, void* stream) {
    ured::clear_error();
    URED_REQUIRE(G >= 0, "ured_seg_aabb: negative segment count");
    if (G == 0) return 0;
    URED_REQUIRE(x && off && out, "ured_seg_aabb: null pointer");
    URED_REQUIRE(G <= (1 << 30), "ured_seg_aabb: too many segments");
    hipLaunchKernelGGL(seg_aabb_kernel, dim3(G), dim3(256), 0, (hipStream_t)stream, x, off, out);
    return ured::launch_status("ured_seg_aabb");
}

int ured_part_rows_bwd(const float* d_sorted, const float* d_sums, const long long* inv, const int* gid, int B, int N,
                       int C, float* out, void* stream) {
    return ured_part_rows_bwd_add(d_sorted, d_sums, inv, gid, B, N, C, nullptr, out, stream);
}

int ured_part_rows_bwd_add(const float* d_sorted, const float* d_sums, const long long* inv, const int* gid, int B,
                           int N, int C, const float* add, float* out, void* stream) {
    ured::clear_error();
    URED_REQUIRE(B >= 0 && N >= 0 && C >= 0, "ured_part_rows_bwd: negative size");
    if (B == 0 || N == 0 || C == 0) return 0;
    URED_REQUIRE(inv && gid && out, "ured_part_rows_bwd: null pointer");
    URED_REQUIRE((long long)B * N * C < (1LL << 40), "ured_part_rows_bwd: too large");
    const bool vec = C % 4 == 0 && (((uintptr_t)out | (uintptr_t)d_sorted | (uintptr_t)d_sums | (uintptr_t)add) & 15) == 0;
    const long long rows = (long long)B * N;
    const int per_row = vec ? C / 4 : C;
    const int rows_per_block = per_row >= 256 ? 1 : 256 / per_row;
    const unsigned grid = (unsigned)((rows + rows_per_block - 1) / rows_per_block);
    if (vec)
        hipLaunchKernelGGL(part_rows_bwd_kernel<4>, dim3(grid), dim3(256), 0, (hipStream_t)stream, d_sorted, d_sums, inv,
                           gid, N, C, rows, rows_per_block, add, out);
    else
        hipLaunchKernelGGL(part_rows_bwd_kernel<1>, dim3(grid), dim3(256), 0, (hipStream_t)stream, d_sorted, d_sums, inv,
                           gid, N, C, rows, rows_per_block, add, out);
    return ured::launch_status("ured_part_rows_bwd");
}

int ured_dcd(const float* dist1, const int* idx1, const float* dist2, const int* idx2, int b, int n1, int n2,
             float alpha, int n_lambda, float frac_12, float frac_21, float* loss, float* cd_p, float* cd_t,
             void* stream) {
    ured::clear_error();
    URED_REQUIRE(b >= 0 && n1 > 0 && n2 > 0, "ured_dcd: bad sizes b=%d n1=%d n2=%d", b, n1, n2);
    URED_REQUIRE(n1 + n2 <= DCD_MAX_POINTS, "ured_dcd: n1+n2=%d exceeds %d", n1 + n2, DCD_MAX_POINTS);
    URED_REQUIRE(n_lambda >= 0, "ured_dcd: n_lambda must be >= 0");
    if (b == 0) return 0;
    URED_REQUIRE(dist1 && idx1 && dist2 && idx2 && loss && cd_p && cd_t, "ured_dcd: null pointer");
    hipLaunchKernelGGL(dcd_kernel, dim3(b), dim3(DCD_THREADS), (size_t)(n1 + n2) * sizeof(int), (hipStream_t)stream,
                       dist1, idx1, dist2, idx2, n1, n2, alpha, n_lambda, frac_12, frac_21, loss, cd_p, cd_t);
    return ured::launch_status("ured_dcd");
}

}  // extern "C"

URED_DBG_ACCESSOR(ured_dbg_nn)
