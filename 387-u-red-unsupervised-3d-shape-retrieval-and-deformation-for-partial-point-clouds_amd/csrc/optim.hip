// optim.hip — the optimizer tail of the training step (engine/train.py:331-346,
// clip_grad_norm_(module.parameters(), 5.0) for each of six modules, then Adam with L2 weight
// decay, train_utils/optimizer_dm.py:68-104) over ONE flat HBM buffer per state tensor.
//
// torch's fused Adam walks ~500 parameter tensors in multi-tensor-apply chunks (≈1.9 TB/s at
// this model's mix of 64-element BN vectors and 1024x1152 weights), and the clip adds a
// per-tensor norm launch and a per-module scale launch. Here the parameters, gradients and the
// two moments live in flat buffers (each tensor's slice 16-float aligned, padding zero), cut
// into chunks that never straddle a parameter; only the chunks of parameters that have a
// gradient this step are listed (torch's clip_grad_norm_ and Adam skip the others, and Adam
// keeps a step count per parameter): pass 1 writes one fp64 sum of squares per chunk, pass 2 (a
// workgroup per module) sums its chunks in a fixed tree -> norm -> clip factor and advances the
// listed parameters' device step counters, pass 3 streams p, g, m, v once (float4): clipped
// gradient written back (the gradient after the step is the clipped one, as with
// clip_grad_norm_), moments and parameter updated. Fixed partition and order: deterministic.
// Arithmetic per element follows torch's fused Adam (ADAM_MODE::ORIGINAL, no amsgrad; its
// hyper-parameters are doubles, so each update expression is evaluated in double and rounded
// to float on assignment, and the bias corrections are floats):
//   g += wd * p;  m = b1*m + (1-b1)*g;  v = b2*v + (1-b2)*g*g;
//   step_size = lr / (1 - b1^t);  denom = sqrt(v) / sqrt(1 - b2^t) + eps;  p -= step_size * m / denom
#include <hip/hip_runtime.h>
#define URED_DBG_FILE 8
#include "ured_common.h"
#include "../../include/ured_hip.h"

namespace {

__global__ __launch_bounds__(256) void chunk_sumsq_kernel(const float* __restrict__ g,
        const long long* __restrict__ cbeg, const long long* __restrict__ cend, double* __restrict__ partial) {
    __shared__ double red[256];
    const int c = blockIdx.x, t = threadIdx.x;
    const long long b = cbeg[c], e = cend[c];
    float a0 = 0.f, a1 = 0.f;
    for (long long i = b + 4ll * t; i < e; i += 4ll * 256) {
        const float4 v = *reinterpret_cast<const float4*>(g + i);
        a0 += v.x * v.x + v.y * v.y;
        a1 += v.z * v.z + v.w * v.w;
    }
    red[t] = (double)a0 + (double)a1;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (t < h) red[t] += red[t + h];
        __syncthreads();
    }
    if (t == 0) partial[c] = red[0];
}

// one workgroup per segment: its chunk partials strided over 256 threads, then a fixed tree.
// Workgroup 0 also advances the step counter of every parameter that takes this step (torch's
// Adam keeps one step count per parameter and skips parameters without a gradient).
__global__ __launch_bounds__(256) void seg_coef_kernel(const double* __restrict__ partial, const int* __restrict__ seg_chunk0,
        float max_norm, float* __restrict__ coef, float* __restrict__ param_step,
        const int* __restrict__ active_params, int n_active) {
    __shared__ double red[256];
    const int s = blockIdx.x, t = threadIdx.x;
    double a = 0.0;
    if (max_norm > 0.f)
        for (int c = seg_chunk0[s] + t; c < seg_chunk0[s + 1]; c += 256) a += partial[c];
    red[t] = a;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if (t < h) red[t] += red[t + h];
        __syncthreads();
    }
    if (t == 0) {
        const float norm = (float)sqrt(red[0]);
        coef[s] = max_norm > 0.f ? fminf(max_norm / (norm + 1e-6f), 1.f) : 1.f;
    }
    if (s == 0)
        for (int i = t; i < n_active; i += 256) param_step[active_params[i]] += 1.f;
}

__global__ __launch_bounds__(256) void adam_flat_kernel(float* __restrict__ p, float* __restrict__ g,
        float* __restrict__ m, float* __restrict__ v, const long long* __restrict__ cbeg,
        const long long* __restrict__ cend, const int* __restrict__ cseg, const int* __restrict__ cparam,
        const float* __restrict__ coef, const float* __restrict__ lr_p, const float* __restrict__ param_step,
        double b1, double b2, double eps, double wd, int write_grad) {
    const int c = blockIdx.x, t = threadIdx.x;
    const long long b = cbeg[c], e = cend[c];
    const float cf = coef[cseg[c]];
    // the hyper-parameters are doubles and the bias corrections floats, as in torch's fused Adam
    const double lr = (double)lr_p[0];
    const float st = param_step[cparam[c]];
    const float bc1 = (float)(1.0 - pow(b1, (double)st));
    const float bc2s = sqrtf((float)(1.0 - pow(b2, (double)st)));
    const double step_size = lr / (double)bc1;
    for (long long i = b + 4ll * t; i < e; i += 4ll * 256) {
        float4 pp = *reinterpret_cast<const float4*>(p + i);
        float4 gg = *reinterpret_cast<const float4*>(g + i);
        float4 mm = *reinterpret_cast<const float4*>(m + i);
        float4 vv = *reinterpret_cast<const float4*>(v + i);
        float* pe = &pp.x; float* ge = &gg.x; float* me = &mm.x; float* ve = &vv.x;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float gc = ge[q] * cf;                               // clip_grad_norm_'s in-place scale
            ge[q] = gc;
            const float gw = (float)((double)gc + (double)pe[q] * wd); // L2 weight decay (Adam, not AdamW)
            me[q] = (float)(b1 * (double)me[q] + (1.0 - b1) * (double)gw);
            ve[q] = (float)(b2 * (double)ve[q] + (1.0 - b2) * (double)gw * (double)gw);
            const float denom = (float)((double)(sqrtf(ve[q]) / bc2s) + eps);
            pe[q] = (float)((double)pe[q] - step_size * (double)me[q] / (double)denom);
        }
        *reinterpret_cast<float4*>(p + i) = pp;
        *reinterpret_cast<float4*>(m + i) = mm;
        *reinterpret_cast<float4*>(v + i) = vv;
        if (write_grad) *reinterpret_cast<float4*>(g + i) = gg;
    }
}

}  // namespace

extern "C" {

int ured_adam_clip_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq,
                        const long long* chunk_beg, const long long* chunk_end, const int* chunk_seg,
                        const int* chunk_param, int nchunks, const int* seg_chunk0, int nseg, float max_norm,
                        const float* lr, float* param_step, const int* active_params, int n_active,
                        double beta1, double beta2, double eps, double weight_decay, double* partial, float* coef,
                        void* stream) {
    ured::clear_error();
    URED_REQUIRE(nchunks >= 0 && nseg >= 1 && nseg <= 64 && n_active >= 0,
                 "ured_adam_clip_step: bad sizes (%d chunks, %d segments, %d parameters)", nchunks, nseg, n_active);
    URED_REQUIRE(param && grad && exp_avg && exp_avg_sq && chunk_beg && chunk_end && chunk_seg && chunk_param &&
                 seg_chunk0 && lr && param_step && (active_params || n_active == 0) && partial && coef,
                 "ured_adam_clip_step: null pointer");
    auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
    URED_REQUIRE(al16(param) && al16(grad) && al16(exp_avg) && al16(exp_avg_sq),
                 "ured_adam_clip_step: flat buffers must be 16-B aligned");
    hipStream_t st = (hipStream_t)stream;
    if (nchunks > 0 && max_norm > 0.f)
        hipLaunchKernelGGL(chunk_sumsq_kernel, dim3(nchunks), dim3(256), 0, st, grad, chunk_beg, chunk_end, partial);
    hipLaunchKernelGGL(seg_coef_kernel, dim3(nseg), dim3(256), 0, st, partial, seg_chunk0, max_norm, coef, param_step,
                       active_params, n_active);
    if (nchunks > 0)
        hipLaunchKernelGGL(adam_flat_kernel, dim3(nchunks), dim3(256), 0, st, param, grad, exp_avg, exp_avg_sq,
                           chunk_beg, chunk_end, chunk_seg, chunk_param, coef, lr, param_step, beta1, beta2, eps,
                           weight_decay, max_norm > 0.f ? 1 : 0);
    return ured::launch_status("ured_adam_clip_step");
}

}  // extern "C"

URED_DBG_ACCESSOR(ured_dbg_optim)
