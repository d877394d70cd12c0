// Probe: does a bf16-MFMA kernel running concurrently (another stream) change the results of a
// packed-fp32 (v_pk_fma_f32) or scalar-fp32 VALU kernel? The victims are pure functions of their
// inputs; each is re-run many times beside an aggressor and compared bitwise with its result on
// an idle GPU.
//
//   hipcc --offload-arch=gfx950 -O3 tools/mfma_interference.hip -o tools/mfma_interference
//   ./mfma_interference [seconds per case]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef __bf16 bf8v __attribute__((ext_vector_type(8)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int VN = 1 << 20;   // victim elements (float2 pairs)

// packed fp32: a chain of v_pk_fma_f32 per pair, plus an LDS round trip (like the skinny kernel)
__global__ __launch_bounds__(256) void victim_pk(const f2* __restrict__ in, f2* __restrict__ out, int iters) {
    __shared__ f2 red[256];
    const int i = blockIdx.x * 256 + threadIdx.x;
    f2 x = in[i], acc = {0.f, 0.f};
    const f2 m = {1.0001f, 0.9999f}, c = {0.5f, -0.25f};
    for (int k = 0; k < iters; ++k) {
        acc = x * m + acc;          // v_pk_fma_f32
        x = x * m + c;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    out[i] = red[threadIdx.x ^ 1] + acc;
}

// scalar fp32 FMA chain
__global__ __launch_bounds__(256) void victim_scalar(const float* __restrict__ in, float* __restrict__ out, int iters) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    float x = in[i], acc = 0.f;
    for (int k = 0; k < iters; ++k) {
        acc = __builtin_fmaf(x, 1.0001f, acc);
        x = __builtin_fmaf(x, 0.9999f, 0.5f);
    }
    out[i] = acc;
}

// aggressors: long MFMA chains on register operands (BF16: 32x32x16 bf16; F32: 32x32x2 f32)
template <bool BF16>
__global__ __launch_bounds__(256, 2) void aggressor(float* __restrict__ sink, int iters) {
    f16v acc;
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if constexpr (BF16) {
        bf8v a, b;
        for (int e = 0; e < 8; ++e) { a[e] = (__bf16)(0.001f * (threadIdx.x + e)); b[e] = (__bf16)(0.002f * e); }
        for (int k = 0; k < iters; ++k) {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, acc, 0, 0, 0);
        }
    } else {
        const float a = 0.001f * threadIdx.x, b = 0.002f;
        for (int k = 0; k < iters; ++k) {
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, acc, 0, 0, 0);
        }
    }
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += acc[r];
    sink[blockIdx.x * 256 + threadIdx.x] = s;
}

int run_case(const char* name, int aggr, bool pk, double seconds) {
    hipStream_t sa, sv;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sv, hipStreamNonBlocking));
    std::vector<float> h(2 * VN);
    for (int i = 0; i < 2 * VN; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
    float *in, *out, *sink;
    CK(hipMalloc(&in, 8 * VN));
    CK(hipMalloc(&out, 8 * VN));
    CK(hipMalloc(&sink, 4 * 1024 * 256));
    CK(hipMemcpy(in, h.data(), 8 * VN, hipMemcpyHostToDevice));
    const int iters = 200, n = pk ? VN : 2 * VN;
    auto victim = [&]() {
        if (pk) hipLaunchKernelGGL(victim_pk, dim3(VN / 256), dim3(256), 0, sv, (const f2*)in, (f2*)out, iters);
        else hipLaunchKernelGGL(victim_scalar, dim3(2 * VN / 256), dim3(256), 0, sv, in, out, iters);
    };
    victim();
    CK(hipStreamSynchronize(sv));
    std::vector<float> ref(n), got(n);
    CK(hipMemcpy(ref.data(), out, 4 * n, hipMemcpyDeviceToHost));
    int runs = 0, bad = 0;
    auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < seconds) {
        if (aggr == 1) hipLaunchKernelGGL(aggressor<true>, dim3(1024), dim3(256), 0, sa, sink, 100000);
        if (aggr == 2) hipLaunchKernelGGL(aggressor<false>, dim3(1024), dim3(256), 0, sa, sink, 25000);
        for (int r = 0; r < 4; ++r) {
            victim();
            CK(hipStreamSynchronize(sv));
            CK(hipMemcpy(got.data(), out, 4 * n, hipMemcpyDeviceToHost));
            ++runs;
            bad += memcmp(got.data(), ref.data(), 4 * n) != 0;
        }
        CK(hipStreamSynchronize(sa));
    }
    printf("%-40s runs %5d differing %5d\n", name, runs, bad);
    fflush(stdout);
    CK(hipFree(in)); CK(hipFree(out)); CK(hipFree(sink));
    CK(hipStreamDestroy(sa)); CK(hipStreamDestroy(sv));
    return 0;
}

int main(int argc, char** argv) {
    const double sec = argc > 1 ? atof(argv[1]) : 8.0;
    if (run_case("pk victim, no aggressor", 0, true, sec)) return 1;
    if (run_case("pk victim, bf16 MFMA aggressor", 1, true, sec)) return 1;
    if (run_case("pk victim, f32 MFMA aggressor", 2, true, sec)) return 1;
    if (run_case("scalar victim, bf16 MFMA aggressor", 1, false, sec)) return 1;
    return 0;
}
