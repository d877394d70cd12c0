// emd.hip — auction-algorithm EMD approximation for MI355X / gfx950.
//
// Replaces the EMD extension of the reference
//   Density_aware_Chamfer_Distance/utils_v2/metrics/EMD/emd_cuda.cu:23-307 (emd_cuda_forward /
//   emd_cuda_backward) behind emdModule / calc_emd (emd_module.py:36-92, utils_v2/model_utils.py:72-76).
//
// Same auction as the reference, per batch item and iteration:
//   bid    : every unassigned point i of xyz1 evaluates every point k of xyz2,
//            value = (float)((3.0 - (double)sqrtf(|x2_k - x1_i|^2)) - (double)price[k])
//            (the reference's double-promoted expression, emd_cuda.cu:145), keeps the best and
//            second-best value (strict '>' scan) and bids best - better + eps on the best k;
//   assign : every object takes its highest bid (the bidder's previous owner is evicted,
//            price += increment); in the last iteration every bidder is assigned to its bid;
//   dist   : squared distance to the assigned point.
// Made deterministic (the reference decides with float atomicMax + a +-1e-6 window, where
// the last racing writer wins): bids are 64-bit keys (increment bits << 32 | ~bidder) under
// one integer atomicMax, so an object goes to the highest increment and, on equal increments,
// to the lowest bidder index; equal values during the scan go to the lowest object index.
// The same rules are restated in oracle/emd_oracle.c, which the GPU result matches bit for bit.
//
// Layout / work: a workgroup = 64 bidders x 4 waves; wave q scans the contiguous quarter q of
// xyz2 (so the in-thread strict '>' and the in-order merge give the lowest index on ties),
// objects staged through LDS as SoA + price (broadcast reads). Workgroups whose 64 bidders are
// all assigned leave at once, so late iterations cost little. Backward is a gather (each point
// owns its gradient): no atomics.
#define URED_DBG_FILE 5
#include "ured_common.h"
#include "../../include/ured_hip.h"

namespace {

constexpr int EMD_BIDDERS = 64;       // bidders per workgroup (one per lane)
constexpr int EMD_QUARTERS = 4;       // waves per workgroup, each a quarter of the objects
constexpr int EMD_SUB = 256;          // objects per wave per LDS step

__device__ __forceinline__ float sqd(float x1, float y1, float z1, float x2, float y2, float z2) {
    const float dx = x2 - x1, dy = y2 - y1, dz = z2 - z1;
    return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
}

struct EmdWs {
    float* price; int* inv; int* bid; float* inc; unsigned long long* key;
};

__host__ __device__ inline EmdWs carve(void* ws, size_t total) {
    EmdWs w;
    char* p = reinterpret_cast<char*>(ws);
    w.key = reinterpret_cast<unsigned long long*>(p); p += 8 * total;
    w.price = reinterpret_cast<float*>(p); p += 4 * total;
    w.inc = reinterpret_cast<float*>(p); p += 4 * total;
    w.inv = reinterpret_cast<int*>(p); p += 4 * total;
    w.bid = reinterpret_cast<int*>(p);
    return w;
}

__global__ __launch_bounds__(256) void emd_init_kernel(EmdWs w, int* assignment, size_t total) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    w.price[i] = 0.f; w.inv[i] = -1; w.bid[i] = -1; w.inc[i] = 0.f; w.key[i] = 0ull;
    assignment[i] = -1;
}

__global__ __launch_bounds__(256) void emd_bid_kernel(const float* __restrict__ xyz1, const float* __restrict__ xyz2,
                                                      int n, float eps, const int* __restrict__ assignment, EmdWs w) {
    __shared__ float ox[EMD_QUARTERS][EMD_SUB], oy[EMD_QUARTERS][EMD_SUB], oz[EMD_QUARTERS][EMD_SUB],
        op[EMD_QUARTERS][EMD_SUB];
    __shared__ float mb[EMD_QUARTERS][EMD_BIDDERS], mr[EMD_QUARTERS][EMD_BIDDERS];
    __shared__ int mi[EMD_QUARTERS][EMD_BIDDERS];
    const int b = blockIdx.y;
    const int s = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int i = blockIdx.x * EMD_BIDDERS + s;
    const size_t base = (size_t)b * n;
    const bool active = i < n && assignment[base + i] == -1;
    if (!__syncthreads_or(active)) return;            // all 64 bidders assigned: nothing to bid
    float x1 = 0.f, y1 = 0.f, z1 = 0.f;
    if (active) {
        const float* p = xyz1 + 3 * (base + i);
        x1 = p[0]; y1 = p[1]; z1 = p[2];
    }
    float best = -1e9f, better = -1e9f;
    int best_i = -1;
    const int n4 = (n + EMD_QUARTERS - 1) / EMD_QUARTERS;   // objects of quarter q: [q*n4, min(n, (q+1)*n4))
    const int q0 = q * n4, q1 = min(n, q0 + n4);
    for (int t0 = 0; t0 < n4; t0 += EMD_SUB) {
        __syncthreads();
        for (int k = s; k < EMD_SUB; k += 64) {
            const int o = q0 + t0 + k;
            float x = 0.f, y = 0.f, z = 0.f, pr = __builtin_inff();   // padding: value -inf, never taken
            if (t0 + k < n4 && o < q1) {
                const float* p = xyz2 + 3 * (base + o);
                x = p[0]; y = p[1]; z = p[2]; pr = w.price[base + o];
            }
            ox[q][k] = x; oy[q][k] = y; oz[q][k] = z; op[q][k] = pr;
        }
        __syncthreads();
        if (active) {
            const int kn = min(EMD_SUB, n4 - t0);
            for (int k = 0; k < kn; ++k) {
                const float dd = sqd(x1, y1, z1, ox[q][k], oy[q][k], oz[q][k]);
                const float d = (float)((3.0 - (double)__builtin_sqrtf(dd)) - (double)op[q][k]);
                if (d > best) { better = best; best = d; best_i = q0 + t0 + k; }
                else if (d > better) better = d;
            }
        }
    }
    mb[q][s] = best; mr[q][s] = better; mi[q][s] = best_i;
    __syncthreads();
    if (q != 0 || !active) return;
    // merge the quarters in object order (the reference's in-order merge, emd_cuda.cu:168-176)
    for (int h = 1; h < EMD_QUARTERS; ++h) {
        const float bh = mb[h][s];
        if (bh > best) { better = fmaxf(best, mr[h][s]); best = bh; best_i = mi[h][s]; }
        else better = fmaxf(better, bh);
    }
    if (best_i < 0) { w.bid[base + i] = -1; return; }   // no finite value (cannot happen for finite inputs)
    const float incr = best - better + eps;
    URED_DBG_CHECK(best_i < n);
    w.bid[base + i] = best_i;
    w.inc[base + i] = incr;
    const unsigned long long key = ((unsigned long long)__float_as_uint(incr) << 32) | (0xFFFFFFFFu - (unsigned)i);
    atomicMax(&w.key[base + best_i], key);
}

__global__ __launch_bounds__(256) void emd_assign_kernel(int n, int* assignment, EmdWs w, int last) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const size_t base = (size_t)b * n;
    if (assignment[base + i] != -1) return;
    const int j = w.bid[base + i];
    if (j < 0) return;
    URED_DBG_CHECK(j < n);
    const unsigned long long key = w.key[base + j];
    const bool won = last || (0xFFFFFFFFu - (unsigned)(key & 0xFFFFFFFFull)) == (unsigned)i;
    if (!won) return;
    if (!last) {
        const int prev = w.inv[base + j];
        URED_DBG_CHECK(prev >= -1 && prev < n);
        if (prev != -1) assignment[base + prev] = -1;
        w.key[base + j] = 0ull;
    }
    w.inv[base + j] = i;
    assignment[base + i] = j;
    w.price[base + j] += w.inc[base + i];
}

__global__ __launch_bounds__(256) void emd_dist_kernel(const float* __restrict__ xyz1, const float* __restrict__ xyz2,
                                                       int n, const int* __restrict__ assignment, float* __restrict__ dist) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const size_t base = (size_t)b * n;
    const int k = assignment[base + i];
    URED_DBG_CHECK(k >= -1 && k < n);
    const float* p = xyz1 + 3 * (base + i);
    const float* r = xyz2 + 3 * (base + (k < 0 ? 0 : k));
    dist[base + i] = sqd(r[0], r[1], r[2], p[0], p[1], p[2]);   // (x1 - x2)^2 terms, emd_cuda.cu:247-250
}

__global__ __launch_bounds__(256) void emd_bwd_kernel(const float* __restrict__ xyz1, const float* __restrict__ xyz2,
                                                      int n, const float* __restrict__ gd, const int* __restrict__ assignment,
                                                      float* __restrict__ g1) {
    const int b = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const size_t base = (size_t)b * n;
    const int k = assignment[base + i];
    URED_DBG_CHECK(k >= -1 && k < n);
    const float* p = xyz1 + 3 * (base + i);
    const float* r = xyz2 + 3 * (base + (k < 0 ? 0 : k));
    const float g = gd[base + i] * 2.f;
    float* o = g1 + 3 * (base + i);
    o[0] += g * (p[0] - r[0]);
    o[1] += g * (p[1] - r[1]);
    o[2] += g * (p[2] - r[2]);
}

}  // namespace

extern "C" {

size_t ured_emd_workspace(int b, int n) {
    if (b <= 0 || n <= 0) return 0;
    return (size_t)24 * (size_t)b * (size_t)n;
}

int ured_emd_fwd(const float* xyz1, const float* xyz2, int b, int n, float eps, int iters,
                 float* dist, int* assignment, void* workspace, size_t ws_bytes, void* stream) {
    ured::clear_error();
    URED_REQUIRE(b >= 0 && n >= 0 && iters >= 0, "ured_emd_fwd: negative size / iterations");
    URED_REQUIRE(b <= 65535, "ured_emd_fwd: b=%d exceeds 65535", b);
    if (b == 0 || n == 0) return 0;
    URED_REQUIRE(xyz1 && xyz2 && dist && assignment && workspace, "ured_emd_fwd: null pointer");
    const size_t total = (size_t)b * n;
    URED_REQUIRE(ws_bytes >= ured_emd_workspace(b, n), "ured_emd_fwd: workspace of %zu bytes needed",
                 ured_emd_workspace(b, n));
    hipStream_t st = (hipStream_t)stream;
    const EmdWs w = carve(workspace, total);
    hipLaunchKernelGGL(emd_init_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, w, assignment, total);
    const dim3 gb((n + EMD_BIDDERS - 1) / EMD_BIDDERS, b), ga((n + 255) / 256, b);
    for (int it = 0; it < iters; ++it) {
        hipLaunchKernelGGL(emd_bid_kernel, gb, dim3(256), 0, st, xyz1, xyz2, n, eps, assignment, w);
        hipLaunchKernelGGL(emd_assign_kernel, ga, dim3(256), 0, st, n, assignment, w, (int)(it == iters - 1));
    }
    hipLaunchKernelGGL(emd_dist_kernel, ga, dim3(256), 0, st, xyz1, xyz2, n, assignment, dist);
    return ured::launch_status("ured_emd_fwd");
}

int ured_emd_bwd(const float* xyz1, const float* xyz2, int b, int n, const float* graddist, const int* assignment,
                 float* gradxyz1, void* stream) {
    ured::clear_error();
    URED_REQUIRE(b >= 0 && n >= 0, "ured_emd_bwd: negative size");
    URED_REQUIRE(b <= 65535, "ured_emd_bwd: b=%d exceeds 65535", b);
    if (b == 0 || n == 0) return 0;
    URED_REQUIRE(xyz1 && xyz2 && graddist && assignment && gradxyz1, "ured_emd_bwd: null pointer");
    hipLaunchKernelGGL(emd_bwd_kernel, dim3((n + 255) / 256, b), dim3(256), 0, (hipStream_t)stream,
                       xyz1, xyz2, n, graddist, assignment, gradxyz1);
    return ured::launch_status("ured_emd_bwd");
}

}  // extern "C"

URED_DBG_ACCESSOR(ured_dbg_emd)
