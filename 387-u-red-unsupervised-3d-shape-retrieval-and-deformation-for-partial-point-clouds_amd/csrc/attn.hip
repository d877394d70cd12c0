// attn.hip — multi-head softmax attention over graph nodes (DeformNet_MatchingNet's
// GraphAttentionNet), forward and backward, one workgroup per (sample, head).
//
// Replaces, per ResidualAttentionMessagePropagation call, the reference's
//   view(B, H, d, n) -> transpose/contiguous -> matmul -> * d^-0.5 -> softmax -> matmul
//   -> transpose/contiguous chain (attention_graph/attention.py:8-19,
//   attention_gnn.py:20-32) and its autograd (~20 small launches with copies) by two
//   launches. Node features stay node-major [B, nodes, C] with C = H*d (channel h*d + j
//   is head h, component j — the reference's view(B, H, d, n) split), so q / k / v are
//   read in place from the fused projection outputs (any row stride, e.g. [B, n, 3C]).
//
// Sizes are tiny (n, m <= 32 nodes, d <= 128): the whole (b, h) problem lives in LDS,
// rows padded to d+1 floats so the per-(i, j) dot products (consecutive threads on
// consecutive key rows) are bank-conflict free. fp32 throughout, fixed summation order
// (deterministic).
#define URED_DBG_FILE 6
#include "ured_common.h"
#include "ured_hip.h"

namespace {

constexpr int ATT_THREADS = 256;

struct AttnArgs {
    const float* q; int ldq;
    const float* k; int ldk;
    const float* v; int ldv;
    int n, m, d, H;
    float scale;
    float* out; int ldo;       // fwd output / bwd: unused
    float* w;                  // softmax weights [B][H][n][m] (fwd writes, bwd reads)
    const float* dout; int lddo;
    float* dq; int lddq;
    float* dk; int lddk;
    float* dv; int lddv;
};

// Up to URED_ATTN_MAX_SETS independent calls per launch: set si owns workgroups
// [first[si], first[si + 1]), one per (sample, head) of that call, so each block computes exactly what
// a separate launch's block would.
struct AttnSets {
    AttnArgs s[URED_ATTN_MAX_SETS];
    int first[URED_ATTN_MAX_SETS + 1];
    int nsets;
};

__device__ __forceinline__ const AttnArgs& pick_set(const AttnSets& S, int& bx) {
    int si = 0;
#pragma unroll
    for (int q = 1; q < URED_ATTN_MAX_SETS; ++q)
        if (q < S.nsets && (int)blockIdx.x >= S.first[q]) si = q;
    bx = (int)blockIdx.x - S.first[si];
    return S.s[si];
}

// Load rows x (row stride ld, head offset h*d) of `rows` nodes into LDS [rows][d+1]: 16-B global
// loads when the head slice is 16-B aligned (the fused projection outputs are), else 4-B loads.
__device__ inline void load_rows(float* dst, const float* src, int ld, int rows, int d, int hoff, int b) {
    const int dp = d + 1;
    if (((d | ld | hoff) & 3) == 0 && ((uintptr_t)src & 15) == 0) {
        const int d4 = d >> 2;
        for (int e = threadIdx.x; e < rows * d4; e += ATT_THREADS) {
            const int r = e / d4, c = (e - r * d4) * 4;
            const float4 v = *reinterpret_cast<const float4*>(src + (size_t)(b * rows + r) * ld + hoff + c);
            float* o = dst + r * dp + c;
            o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
        }
        return;
    }
    for (int e = threadIdx.x; e < rows * d; e += ATT_THREADS) {
        const int r = e / d, c = e - r * d;
        dst[r * dp + c] = src[(size_t)(b * rows + r) * ld + hoff + c];
    }
}

__global__ __launch_bounds__(ATT_THREADS) void attn_fwd_kernel(const AttnSets sets) {
    extern __shared__ float sm[];
    int bx;
    const AttnArgs& a = pick_set(sets, bx);
    const int b = bx / a.H, h = bx - b * a.H;
    const int n = a.n, m = a.m, d = a.d, dp = d + 1, hoff = h * d;
    float* Q = sm;
    float* Kt = Q + n * dp;
    float* V = Kt + m * dp;
    float* S = V + m * dp;     // [n][m]
    load_rows(Q, a.q, a.ldq, n, d, hoff, b);
    load_rows(Kt, a.k, a.ldk, m, d, hoff, b);
    load_rows(V, a.v, a.ldv, m, d, hoff, b);
    __syncthreads();
    for (int e = threadIdx.x; e < n * m; e += ATT_THREADS) {
        const int i = e / m, j = e - i * m;
        float s = 0.f;
        for (int c = 0; c < d; ++c) s = __builtin_fmaf(Q[i * dp + c], Kt[j * dp + c], s);
        S[e] = s * a.scale;
    }
    __syncthreads();
    float* W = a.w + (size_t)bx * n * m;
    for (int i = threadIdx.x; i < n; i += ATT_THREADS) {
        float mx = -__builtin_inff();
        for (int j = 0; j < m; ++j) mx = fmaxf(mx, S[i * m + j]);
        float sum = 0.f;
        for (int j = 0; j < m; ++j) {
            const float p = expf(S[i * m + j] - mx);
            S[i * m + j] = p;
            sum += p;
        }
        const float inv = 1.f / sum;
        for (int j = 0; j < m; ++j) {
            const float p = S[i * m + j] * inv;
            S[i * m + j] = p;
            W[i * m + j] = p;
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < n * d; e += ATT_THREADS) {
        const int i = e / d, c = e - i * d;
        float o = 0.f;
        for (int j = 0; j < m; ++j) o = __builtin_fmaf(S[i * m + j], V[j * dp + c], o);
        a.out[(size_t)(b * n + i) * a.ldo + hoff + c] = o;
    }
}

__global__ __launch_bounds__(ATT_THREADS) void attn_bwd_kernel(const AttnSets sets) {
    extern __shared__ float sm[];
    int bx;
    const AttnArgs& a = pick_set(sets, bx);
    const int b = bx / a.H, h = bx - b * a.H;
    const int n = a.n, m = a.m, d = a.d, dp = d + 1, hoff = h * d;
    float* Q = sm;
    float* Kt = Q + n * dp;
    float* V = Kt + m * dp;
    float* dO = V + m * dp;
    float* P = dO + n * dp;     // softmax weights [n][m]
    float* dS = P + n * m;      // [n][m]
    load_rows(Q, a.q, a.ldq, n, d, hoff, b);
    load_rows(Kt, a.k, a.ldk, m, d, hoff, b);
    load_rows(V, a.v, a.ldv, m, d, hoff, b);
    load_rows(dO, a.dout, a.lddo, n, d, hoff, b);
    const float* W = a.w + (size_t)bx * n * m;
    for (int e = threadIdx.x; e < n * m; e += ATT_THREADS) P[e] = W[e];
    __syncthreads();
    // dV[j][c] = sum_i P[i][j] dO[i][c]
    for (int e = threadIdx.x; e < m * d; e += ATT_THREADS) {
        const int j = e / d, c = e - j * d;
        float s = 0.f;
        for (int i = 0; i < n; ++i) s = __builtin_fmaf(P[i * m + j], dO[i * dp + c], s);
        a.dv[(size_t)(b * m + j) * a.lddv + hoff + c] = s;
    }
    // dP[i][j] = sum_c dO[i][c] V[j][c]
    for (int e = threadIdx.x; e < n * m; e += ATT_THREADS) {
        const int i = e / m, j = e - i * m;
        float s = 0.f;
        for (int c = 0; c < d; ++c) s = __builtin_fmaf(dO[i * dp + c], V[j * dp + c], s);
        dS[e] = s;
    }
    __syncthreads();
    // softmax backward: dS = P * (dP - sum_j P dP), times the score scale
    for (int i = threadIdx.x; i < n; i += ATT_THREADS) {
        float t = 0.f;
        for (int j = 0; j < m; ++j) t = __builtin_fmaf(P[i * m + j], dS[i * m + j], t);
        for (int j = 0; j < m; ++j) dS[i * m + j] = P[i * m + j] * (dS[i * m + j] - t) * a.scale;
    }
    __syncthreads();
    // dQ[i][c] = sum_j dS[i][j] K[j][c];  dK[j][c] = sum_i dS[i][j] Q[i][c]
    for (int e = threadIdx.x; e < n * d; e += ATT_THREADS) {
        const int i = e / d, c = e - i * d;
        float s = 0.f;
        for (int j = 0; j < m; ++j) s = __builtin_fmaf(dS[i * m + j], Kt[j * dp + c], s);
        a.dq[(size_t)(b * n + i) * a.lddq + hoff + c] = s;
    }
    for (int e = threadIdx.x; e < m * d; e += ATT_THREADS) {
        const int j = e / d, c = e - j * d;
        float s = 0.f;
        for (int i = 0; i < n; ++i) s = __builtin_fmaf(dS[i * m + j], Q[i * dp + c], s);
        a.dk[(size_t)(b * m + j) * a.lddk + hoff + c] = s;
    }
}

int check_sizes(const char* who, int B, int H, int n, int m, int d) {
    URED_REQUIRE(B >= 0 && H > 0 && n > 0 && m > 0 && d > 0, "%s: bad sizes B=%d H=%d n=%d m=%d d=%d", who, B, H, n, m, d);
    URED_REQUIRE(n <= URED_ATTN_MAX_NODES && m <= URED_ATTN_MAX_NODES, "%s: n=%d m=%d exceed %d nodes", who, n, m,
                 URED_ATTN_MAX_NODES);
    URED_REQUIRE(d <= URED_ATTN_MAX_HEAD_DIM, "%s: head dim %d exceeds %d", who, d, URED_ATTN_MAX_HEAD_DIM);
    URED_REQUIRE((long)B * H <= 0x7fffffffL, "%s: too many (sample, head) pairs", who);
    return 0;
}

size_t fwd_lds(int n, int m, int d) { return sizeof(float) * ((size_t)(n + 2 * m) * (d + 1) + (size_t)n * m); }
size_t bwd_lds(int n, int m, int d) { return sizeof(float) * ((size_t)(2 * n + 2 * m) * (d + 1) + 2 * (size_t)n * m); }


// Validate one set and add it to the launch table (B == 0 sets add no workgroups).
int add_set(const char* who, bool bwd, const UredAttnSet& x, AttnSets& S, size_t& lds) {
    if (int rc = check_sizes(who, x.B, x.H, x.n, x.m, x.d)) return rc;
    const size_t need = bwd ? bwd_lds(x.n, x.m, x.d) : fwd_lds(x.n, x.m, x.d);
    URED_REQUIRE(need <= 65536, "%s: n=%d m=%d d=%d needs more than 64 KB of LDS", who, x.n, x.m, x.d);
    if (x.B == 0) return 0;
    const int hd = x.H * x.d;
    URED_REQUIRE(x.q && x.k && x.v && x.weights, "%s: null pointer", who);
    URED_REQUIRE(x.ldq >= hd && x.ldk >= hd && x.ldv >= hd, "%s: row stride < H*d", who);
    if (bwd) {
        URED_REQUIRE(x.dout && x.dq && x.dk && x.dv, "%s: null pointer", who);
        URED_REQUIRE(x.lddo >= hd && x.lddq >= hd && x.lddk >= hd && x.lddv >= hd, "%s: row stride < H*d", who);
    } else {
        URED_REQUIRE(x.out, "%s: null pointer", who);
        URED_REQUIRE(x.ldo >= hd, "%s: row stride < H*d", who);
    }
    const long long end = (long long)S.first[S.nsets] + (long long)x.B * x.H;
    URED_REQUIRE(end <= 0x7fffffffLL, "%s: too many (sample, head) pairs", who);
    S.s[S.nsets] = AttnArgs{x.q, x.ldq, x.k, x.ldk, x.v, x.ldv, x.n, x.m, x.d, x.H, x.scale,
                            bwd ? nullptr : x.out, bwd ? 0 : x.ldo, x.weights, bwd ? x.dout : nullptr,
                            bwd ? x.lddo : 0, bwd ? x.dq : nullptr, bwd ? x.lddq : 0, bwd ? x.dk : nullptr,
                            bwd ? x.lddk : 0, bwd ? x.dv : nullptr, bwd ? x.lddv : 0};
    S.first[S.nsets + 1] = (int)end;
    ++S.nsets;
    lds = need > lds ? need : lds;
    return 0;
}

int launch_sets(const char* who, bool bwd, int nsets, const UredAttnSet* sets, void* stream) {
    URED_REQUIRE(nsets >= 1 && nsets <= URED_ATTN_MAX_SETS && sets, "%s: nsets=%d (1..%d)", who, nsets,
                 URED_ATTN_MAX_SETS);
    AttnSets S{};
    size_t lds = 0;
    for (int i = 0; i < nsets; ++i)
        if (int rc = add_set(who, bwd, sets[i], S, lds)) return rc;
    const int blocks = S.first[S.nsets];
    if (blocks == 0) return 0;
    if (bwd) hipLaunchKernelGGL(attn_bwd_kernel, dim3(blocks), dim3(ATT_THREADS), lds, (hipStream_t)stream, S);
    else hipLaunchKernelGGL(attn_fwd_kernel, dim3(blocks), dim3(ATT_THREADS), lds, (hipStream_t)stream, S);
    return ured::launch_status(who);
}

}  // namespace

extern "C" {

int ured_attn_fwd(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv,
                  int B, int H, int n, int m, int d, float scale, float* out, int ldo, float* weights,
                  void* stream) {
    ured::clear_error();
    const UredAttnSet x{q, ldq, k, ldk, v, ldv, B, H, n, m, d, scale, out, ldo, weights, nullptr, 0,
                        nullptr, 0, nullptr, 0, nullptr, 0};
    return launch_sets("ured_attn_fwd", false, 1, &x, stream);
}

int ured_attn_bwd(const float* q, int ldq, const float* k, int ldk, const float* v, int ldv, const float* weights,
                  const float* dout, int lddo, int B, int H, int n, int m, int d, float scale,
                  float* dq, int lddq, float* dk, int lddk, float* dv, int lddv, void* stream) {
    ured::clear_error();
    const UredAttnSet x{q, ldq, k, ldk, v, ldv, B, H, n, m, d, scale, nullptr, 0, const_cast<float*>(weights),
                        dout, lddo, dq, lddq, dk, lddk, dv, lddv};
    return launch_sets("ured_attn_bwd", true, 1, &x, stream);
}

int ured_attn_fwd_sets(int nsets, const UredAttnSet* sets, void* stream) {
    ured::clear_error();
    return launch_sets("ured_attn_fwd_sets", false, nsets, sets, stream);
}

int ured_attn_bwd_sets(int nsets, const UredAttnSet* sets, void* stream) {
    ured::clear_error();
    return launch_sets("ured_attn_bwd_sets", true, nsets, sets, stream);
}

}  // extern "C"

URED_DBG_ACCESSOR(ured_dbg_attn)
