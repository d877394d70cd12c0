// parts.hip — get_part's per-sample part bookkeeping (engine/train.py:103-136, with
// compute_aabbox, dataset/dataset_utils.py:77-85) as ONE launch, one workgroup per sample.
//
// The reference loops over torch.unique(labels[w]) with boolean masks (a host sync per part);
// the composed device form took ~20 small kernels (scatter_add counts, cumsums, a radix sort,
// scatters, gathers, an AABB segment kernel, the param_def gather). Here, per sample:
//   * label histogram (LDS, integer), present / rank_of_label / k;
//   * a STABLE counting sort by label: every thread owns a contiguous run of points, per-label
//     exclusive scans over the threads give each point its position — the order torch.sort(stable)
//     and the reference's per-label boolean masks produce;
//   * per part slot: counts, row offsets, the mask, the axis-aligned box (min / max are
//     order-independent, so the box is exact) and param_def indexed by label value
//     (engine/train.py:120: param_def[w, int(sem)] = compute_aabbox(part points)).
#include <hip/hip_runtime.h>
#define URED_DBG_FILE 9
#include "ured_common.h"
#include "../../include/ured_hip.h"

namespace {

constexpr int BP_T = 256;
constexpr int BP_MAXP = 32;

__device__ __forceinline__ int f2o(float f) {        // order-preserving float -> int
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float o2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

__global__ __launch_bounds__(BP_T) void build_parts_kernel(const long long* __restrict__ labels,
        const float* __restrict__ x, int B, int N, int P, float* __restrict__ x_sorted, long long* __restrict__ perm,
        long long* __restrict__ inv_perm, int* __restrict__ gid, int* __restrict__ off, long long* __restrict__ counts,
        long long* __restrict__ kout, float* __restrict__ mask, long long* __restrict__ rank_of_label,
        unsigned char* __restrict__ present, float* __restrict__ aabb, float* __restrict__ param_def) {
    __shared__ int hist[BP_T][BP_MAXP + 1];          // per-thread label counts, then their exclusive scans
    __shared__ int lab_cnt[BP_MAXP], lab_start[BP_MAXP], lab_rank[BP_MAXP];
    __shared__ int lo[BP_MAXP][3], hi[BP_MAXP][3];
    const int b = blockIdx.x, t = threadIdx.x;
    const long long* L = labels + (size_t)b * N;
    const float* X = x + (size_t)b * N * 3;
    const int per = (N + BP_T - 1) / BP_T, n0 = min(N, t * per), n1 = min(N, n0 + per);
    for (int l = 0; l < P; ++l) hist[t][l] = 0;
    if (t < P) {
#pragma unroll
        for (int c = 0; c < 3; ++c) { lo[t][c] = 0x7fffffff; hi[t][c] = (int)0x80000000; }
    }
    __syncthreads();
    // labels are part ids in [0, P) (the reference indexes param_def[w, int(sem)] with them);
    // an out-of-range id is clamped so that it cannot address outside the sample's tables
    auto lab = [&](int n) { return min(max((int)L[n], 0), P - 1); };
    for (int n = n0; n < n1; ++n) {
        const int l = lab(n);
        hist[t][l] += 1;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const int v = f2o(X[3 * n + c]);
            atomicMin(&lo[l][c], v);
            atomicMax(&hi[l][c], v);
        }
    }
    __syncthreads();
    if (t < P) {                                      // exclusive scan of label t over the threads
        int s = 0;
        for (int q = 0; q < BP_T; ++q) { const int h = hist[q][t]; hist[q][t] = s; s += h; }
        lab_cnt[t] = s;
    }
    __syncthreads();
    if (t == 0) {
        int r = -1, st = 0;
        for (int l = 0; l < P; ++l) {
            const bool pr = lab_cnt[l] > 0;
            r += pr ? 1 : 0;
            lab_rank[l] = r;                          // cumsum(present) - 1 (as the composed form)
            lab_start[l] = st;
            st += lab_cnt[l];
        }
        kout[b] = r + 1;
        if (b == 0) off[B * P] = B * N;
    }
    __syncthreads();
    for (int n = n0; n < n1; ++n) {                   // stable: a thread's run in order
        const int l = lab(n);
        const int pos = lab_start[l] + hist[t][l]++;
        perm[(size_t)b * N + pos] = n;
        inv_perm[(size_t)b * N + n] = pos;
        gid[(size_t)b * N + pos] = b * P + lab_rank[l];
#pragma unroll
        for (int c = 0; c < 3; ++c) x_sorted[((size_t)b * N + pos) * 3 + c] = X[3 * n + c];
    }
    if (t < P) {
        const int l = t;
        const bool pr = lab_cnt[l] > 0;
        rank_of_label[(size_t)b * P + l] = lab_rank[l];
        present[(size_t)b * P + l] = pr ? 1 : 0;
        // part slot i = rank: the i-th present label (slots past k are empty, placed at the end)
        const int k = lab_rank[P - 1] + 1;
        const int i = t;
        int li = -1;
        for (int q = 0; q < P; ++q) if (lab_cnt[q] > 0 && lab_rank[q] == i) li = q;
        const int cnt = li >= 0 ? lab_cnt[li] : 0;
        counts[(size_t)b * P + i] = cnt;
        off[b * P + i] = b * N + (li >= 0 ? lab_start[li] : N);
        mask[(size_t)b * P + i] = i < k ? 1.f : 0.f;
        float box[6];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float a = li >= 0 ? o2f(lo[li][c]) : 0.f, z = li >= 0 ? o2f(hi[li][c]) : 0.f;
            box[c] = li >= 0 ? (a + z) / 2.0f : 0.f;
            box[3 + c] = li >= 0 ? (z - a) / 2.0f : 0.f;
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) aabb[((size_t)b * P + i) * 6 + c] = box[c];
        // param_def by label value: the label's own box if present, else 0
        float pb[6];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float a = o2f(lo[l][c]), z = o2f(hi[l][c]);
            pb[c] = pr ? (a + z) / 2.0f : 0.f;
            pb[3 + c] = pr ? (z - a) / 2.0f : 0.f;
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) param_def[((size_t)b * P + l) * 6 + c] = pb[c];
    }
}

}  // namespace

extern "C" int ured_build_parts(const long long* labels, const float* x, int B, int N, int P, float* x_sorted,
                                long long* perm, long long* inv_perm, int* gid, int* off, long long* counts,
                                long long* k, float* mask, long long* rank_of_label, unsigned char* present,
                                float* aabb, float* param_def, void* stream) {
    ured::clear_error();
    URED_REQUIRE(B >= 0 && N > 0 && P > 0 && P <= BP_MAXP, "ured_build_parts: bad sizes (N %d, P %d <= %d)", N, P,
                 BP_MAXP);
    if (B == 0) return 0;
    URED_REQUIRE((long long)B * N < (1LL << 31), "ured_build_parts: too many points");
    URED_REQUIRE(labels && x && x_sorted && perm && inv_perm && gid && off && counts && k && mask && rank_of_label &&
                 present && aabb && param_def, "ured_build_parts: null pointer");
    hipLaunchKernelGGL(build_parts_kernel, dim3(B), dim3(BP_T), 0, (hipStream_t)stream, labels, x, B, N, P, x_sorted,
                       perm, inv_perm, gid, off, counts, k, mask, rank_of_label, present, aabb, param_def);
    return ured::launch_status("ured_build_parts");
}

URED_DBG_ACCESSOR(ured_dbg_parts)
