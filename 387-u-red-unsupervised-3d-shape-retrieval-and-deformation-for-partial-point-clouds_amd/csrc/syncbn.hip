// syncbn.hip — cross-rank batch statistics for the per-point MLP BatchNorms (optional SyncBN,
// cfg["sync_bn"]; the reference trains on one GPU and has no distributed path, README.md:25).
//
// Without SyncBN each rank normalises with its own batch statistics (what DDP does). With it,
// every BN layer of the encoders (network/simple_encoder.py:52-85) and residual nets
// (attention_utils.py:62-86) uses the statistics of the GLOBAL batch, as torch's SyncBatchNorm:
//   forward : per rank, the fp64 (count, mean, M2) of each column from the GEMM epilogue's
//             per-block partials (ured_bn_stats: the Chan merge of ured_bn_fwd_finalize) ->
//             all-gathered and merged in rank order (host side, fp64) -> ured_bn_finalize_stats
//             (mean / invstd / scale / shift, running statistics with the global count);
//   backward: per rank, the fp64 sums of g and g * xhat and the count (ured_bn_bwd_sums) ->
//             all-reduced -> ured_bn_bwd_finalize_sums: the input-gradient coefficients from the
//             GLOBAL sums, dgamma / dbeta from the rank's LOCAL sums (averaged later by the
//             gradient all-reduce, exactly as SyncBatchNorm + DDP).
// Partial layout (mlp.hip part_idx): [q][column][row block], row blocks of 128 rows; group_w
// (nullable) gives the row multiplicity of a unique-row batch per group of group_rows rows.
#include <hip/hip_runtime.h>
#define URED_DBG_FILE 10
#include "ured_common.h"
#include "../../include/ured_hip.h"

namespace {

constexpr int SB_BM = 128, SB_T = 256;

__device__ __forceinline__ size_t pidx(int q, int col, int blk, int N, int nblk) {
    return ((size_t)q * N + col) * nblk + blk;
}

__device__ __forceinline__ double bweight(const float* gw, int grows, int b) {
    return gw ? (double)gw[(b * SB_BM) / grows] : 1.0;
}

__device__ __forceinline__ double bsum(double v, double* sh) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int o = SB_T / 2; o > 0; o >>= 1) {
        if (t < o) sh[t] += sh[t + o];
        __syncthreads();
    }
    const double r = sh[0];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(SB_T) void bn_stats_kernel(const float* __restrict__ ws, int M, int N,
        const float* __restrict__ gw, int grows, double* __restrict__ out) {
    __shared__ double sh[SB_T];
    const int n = blockIdx.x, t = threadIdx.x;
    const int nblk = (M + SB_BM - 1) / SB_BM;
    double s = 0.0, c = 0.0;
    for (int b = t; b < nblk; b += SB_T) {
        const double cnt = (double)min(SB_BM, M - b * SB_BM) * bweight(gw, grows, b);
        s += cnt * (double)ws[pidx(0, n, b, N, nblk)];
        c += cnt;
    }
    const double Mw = bsum(c, sh);
    const double mean = bsum(s, sh) / Mw;
    double q = 0.0;
    for (int b = t; b < nblk; b += SB_T) {
        const double w = bweight(gw, grows, b);
        const double cnt = (double)min(SB_BM, M - b * SB_BM) * w;
        const double dm = (double)ws[pidx(0, n, b, N, nblk)] - mean;
        q += w * (double)ws[pidx(1, n, b, N, nblk)] + cnt * dm * dm;
    }
    const double m2 = bsum(q, sh);
    if (t == 0) { out[n] = Mw; out[N + n] = mean; out[2 * N + n] = m2; }
}

__global__ __launch_bounds__(SB_T) void bn_finalize_stats_kernel(const double* __restrict__ st, int N,
        const float* __restrict__ gamma, const float* __restrict__ beta, float eps, float momentum,
        float* running_mean, float* running_var, float* mean_o, float* invstd_o, float* scale_o, float* shift_o,
        long long* nbt) {
    const int n = blockIdx.x * SB_T + threadIdx.x;
    if (nbt && n == 0) *nbt += 1;
    if (n >= N) return;
    const double Mw = st[n], mean = st[N + n], m2 = st[2 * N + n];
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

__global__ __launch_bounds__(SB_T) void bn_bwd_sums_kernel(const float* __restrict__ ws, int M, int N,
        const float* __restrict__ gw, int grows, double* __restrict__ out) {
    __shared__ double sh[SB_T];
    const int n = blockIdx.x, t = threadIdx.x;
    const int nblk = (M + SB_BM - 1) / SB_BM;
    double a = 0.0, b2 = 0.0, c = 0.0;
    for (int k = t; k < nblk; k += SB_T) {
        a += (double)ws[pidx(0, n, k, N, nblk)];
        b2 += (double)ws[pidx(1, n, k, N, nblk)];
        c += (double)min(SB_BM, M - k * SB_BM) * bweight(gw, grows, k);
    }
    a = bsum(a, sh); b2 = bsum(b2, sh); c = bsum(c, sh);
    if (t == 0) { out[n] = a; out[N + n] = b2; out[2 * N + n] = c; }
}

__global__ __launch_bounds__(SB_T) void bn_bwd_finalize_sums_kernel(const double* __restrict__ loc,
        const double* __restrict__ glob, int N, const float* __restrict__ gamma, const float* __restrict__ invstd,
        float* dgamma, float* dbeta, int accumulate, float* ca, float* cb, float* cc) {
    const int n = blockIdx.x * SB_T + threadIdx.x;
    if (n >= N) return;
    if (dbeta) dbeta[n] = accumulate ? dbeta[n] + (float)loc[n] : (float)loc[n];
    if (dgamma) dgamma[n] = accumulate ? dgamma[n] + (float)loc[N + n] : (float)loc[N + n];
    const double is = invstd[n];
    const double k = (gamma ? (double)gamma[n] : 1.0) * is;
    const double Mw = glob[2 * N + n];
    ca[n] = (float)k;
    cb[n] = (float)(-k * is * glob[N + n] / Mw);
    cc[n] = (float)(-k * glob[n] / Mw);
}

}  // namespace

extern "C" {

int ured_bn_stats(const float* stat_ws, int M, int N, const float* group_w, int group_rows, double* out,
                  void* stream) {
    ured::clear_error();
    URED_REQUIRE(M > 0 && N >= 0, "ured_bn_stats: bad sizes M=%d N=%d", M, N);
    if (N == 0) return 0;
    URED_REQUIRE(stat_ws && out, "ured_bn_stats: null pointer");
    URED_REQUIRE(!group_w || (group_rows > 0 && group_rows % SB_BM == 0), "ured_bn_stats: bad group_rows");
    hipLaunchKernelGGL(bn_stats_kernel, dim3(N), dim3(SB_T), 0, (hipStream_t)stream, stat_ws, M, N, group_w, group_rows,
                       out);
    return ured::launch_status("ured_bn_stats");
}

int ured_bn_finalize_stats(const double* stats, int N, const float* gamma, const float* beta, float eps,
                           float momentum, float* running_mean, float* running_var, float* mean, float* invstd,
                           float* scale, float* shift, long long* num_batches_tracked, void* stream) {
    ured::clear_error();
    URED_REQUIRE(N >= 0, "ured_bn_finalize_stats: bad size");
    if (N == 0) return 0;
    URED_REQUIRE(stats && mean && invstd && scale && shift, "ured_bn_finalize_stats: null pointer");
    hipLaunchKernelGGL(bn_finalize_stats_kernel, dim3((N + SB_T - 1) / SB_T), dim3(SB_T), 0, (hipStream_t)stream,
                       stats, N, gamma, beta, eps, momentum, running_mean, running_var, mean, invstd, scale, shift,
                       num_batches_tracked);
    return ured::launch_status("ured_bn_finalize_stats");
}

int ured_bn_bwd_sums(const float* bwd_ws, int M, int N, const float* group_w, int group_rows, double* out,
                     void* stream) {
    ured::clear_error();
    URED_REQUIRE(M > 0 && N >= 0, "ured_bn_bwd_sums: bad sizes");
    if (N == 0) return 0;
    URED_REQUIRE(bwd_ws && out, "ured_bn_bwd_sums: null pointer");
    URED_REQUIRE(!group_w || (group_rows > 0 && group_rows % SB_BM == 0), "ured_bn_bwd_sums: bad group_rows");
    hipLaunchKernelGGL(bn_bwd_sums_kernel, dim3(N), dim3(SB_T), 0, (hipStream_t)stream, bwd_ws, M, N, group_w,
                       group_rows, out);
    return ured::launch_status("ured_bn_bwd_sums");
}

int ured_bn_bwd_finalize_sums(const double* local, const double* global, int N, const float* gamma,
                              const float* invstd, float* dgamma, float* dbeta, int accumulate, float* coef_a,
                              float* coef_b, float* coef_c, void* stream) {
    ured::clear_error();
    URED_REQUIRE(N >= 0, "ured_bn_bwd_finalize_sums: bad size");
    if (N == 0) return 0;
    URED_REQUIRE(local && global && invstd && coef_a && coef_b && coef_c, "ured_bn_bwd_finalize_sums: null pointer");
    hipLaunchKernelGGL(bn_bwd_finalize_sums_kernel, dim3((N + SB_T - 1) / SB_T), dim3(SB_T), 0, (hipStream_t)stream,
                       local, global, N, gamma, invstd, dgamma, dbeta, accumulate, coef_a, coef_b, coef_c);
    return ured::launch_status("ured_bn_bwd_finalize_sums");
}

}  // extern "C"

URED_DBG_ACCESSOR(ured_dbg_syncbn)
