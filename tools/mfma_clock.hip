// mfma_clock.hip — does the fp32 16x16x4 MFMA sustain more FLOP/s than 32x32x2 under load?
// (MI355X_MICROARCH.md "DVFS give-back" item 7 measured this for bf16 only.)
// Each wave keeps a 64x64 fp32 accumulator tile (64 VGPRs either way) and re-reads its
// fragments from LDS every K-step exactly like gemm2_kernel's main loop (16 ds_read_b128
// per wave per 32-deep step), random operands. Launch: 2 blocks of 256 per CU (as gemm2).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_clock tools/mfma_clock.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

typedef int i32x4 __attribute__((ext_vector_type(4)));

// one wave's four 1-KB LDS-DMA pieces (as gemm2_kernel's dma4)
__device__ __forceinline__ void dma4(const i32x4& rsrc, unsigned v0, unsigned lds) {
    unsigned saved;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, 0 offen offset:1024 lds\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, 0 offen offset:2048 lds\n\t"
        "s_add_u32 m0, m0, 0x400\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %2, %3, 0 offen offset:3072 lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(saved) : "s"(lds), "v"(v0), "s"(rsrc) : "memory", "scc");
}

// SHAPE 33: the 32x32x2 loop plus gemm2's per-step operand DMA (8 x 1 KB per wave into the other
// LDS stage, vmcnt(0) before the barrier) from a buffer of `span` bytes (L2-hot when small)
template <int SHAPE>
__global__ __launch_bounds__(256, 2) void loop_kernel(const float* __restrict__ src, float* __restrict__ out, int steps,
                                                       unsigned span) {
    __shared__ __attribute__((aligned(16))) float lds[(SHAPE >= 33 ? 4 : 2) * 128 * 32];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w & 1, wn = w >> 1;
    for (int i = t; i < (SHAPE >= 33 ? 4 : 2) * 128 * 32; i += 256) lds[i] = src[(blockIdx.x * 977 + i) & ((1 << 20) - 1)];
    __syncthreads();
    if constexpr (SHAPE == 32 || SHAPE >= 33) {
        i32x4 rsrc;
        {
            const unsigned long long b = (unsigned long long)(uintptr_t)src;
            rsrc.x = (int)(unsigned)(b & 0xffffffffull);
            rsrc.y = (int)(unsigned)((b >> 32) & 0xffffull);
            rsrc.z = (int)span;
            rsrc.w = 0x00020000;
        }
        const unsigned lds_w = __builtin_amdgcn_readfirstlane(
            (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)lds + (unsigned)w * 4096u);
        unsigned goff = ((blockIdx.x * 64u + (unsigned)w) * 4096u + (unsigned)lane * 16u) % span;
        f16v acc[2][2];
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j)
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
        const int h = lane >> 5, li = lane & 31;
        for (int s = 0; s < steps; ++s) {
            const float* As = lds + (SHAPE >= 33 ? (s & 1) * 2 * 128 * 32 : 0);
            const float* Bs = As + 128 * 32;
            const unsigned st = lds_w + (unsigned)((s & 1) ^ 1) * (2u * 128 * 32 * 4);
            if (SHAPE >= 33) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                goff = (goff + 8192u * 64u) % span;
            }
            if (SHAPE == 33) {
                dma4(rsrc, goff, st);
                dma4(rsrc, (goff + 16384u) % span, st + 16384u);
            }
            float a[2][16], b[2][16];
#pragma unroll
            for (int tm = 0; tm < 2; ++tm) {
                const int r = wm * 64 + tm * 32 + li;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 v = *reinterpret_cast<const float4*>(As + r * 32 + 4 * ((4 * h + q) ^ ((r >> 1) & 7)));
                    a[tm][4 * q] = v.x; a[tm][4 * q + 1] = v.y; a[tm][4 * q + 2] = v.z; a[tm][4 * q + 3] = v.w;
                }
                const int c = wn * 64 + tm * 32 + li;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 v = *reinterpret_cast<const float4*>(Bs + c * 32 + 4 * ((4 * h + q) ^ ((c >> 1) & 7)));
                    b[tm][4 * q] = v.x; b[tm][4 * q + 1] = v.y; b[tm][4 * q + 2] = v.z; b[tm][4 * q + 3] = v.w;
                }
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0][j], b[0][j], acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0][j], b[1][j], acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1][j], b[0][j], acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[1][j], b[1][j], acc[1][1], 0, 0, 0);
                if (SHAPE == 34 && j == 1) dma4(rsrc, goff, st);
                if (SHAPE == 34 && j == 5) dma4(rsrc, (goff + 16384u) % span, st + 16384u);
            }
            if (SHAPE == 32) __builtin_amdgcn_s_barrier();
        }
        float s = 0.f;
        for (int i = 0; i < 2; ++i)
            for (int j = 0; j < 2; ++j)
                for (int r = 0; r < 16; ++r) s += acc[i][j][r];
        out[blockIdx.x * 256 + t] = s;
    } else {
        f4v acc[4][4];
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;
        const float* As = lds;
        const float* Bs = lds + 128 * 32;
        const int g = lane >> 4, li = lane & 15;
        for (int s = 0; s < steps; ++s) {
            float a[4][8], b[4][8];   // lane group g holds k = 8g .. 8g+7
#pragma unroll
            for (int tm = 0; tm < 4; ++tm) {
                const int r = wm * 64 + tm * 16 + li;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const float4 v = *reinterpret_cast<const float4*>(As + r * 32 + 4 * ((2 * g + q) ^ ((r >> 1) & 7)));
                    a[tm][4 * q] = v.x; a[tm][4 * q + 1] = v.y; a[tm][4 * q + 2] = v.z; a[tm][4 * q + 3] = v.w;
                }
                const int c = wn * 64 + tm * 16 + li;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const float4 v = *reinterpret_cast<const float4*>(Bs + c * 32 + 4 * ((2 * g + q) ^ ((c >> 1) & 7)));
                    b[tm][4 * q] = v.x; b[tm][4 * q + 1] = v.y; b[tm][4 * q + 2] = v.z; b[tm][4 * q + 3] = v.w;
                }
            }
#pragma unroll
            for (int kk = 0; kk < 8; ++kk)
#pragma unroll
                for (int tm = 0; tm < 4; ++tm)
#pragma unroll
                    for (int tn = 0; tn < 4; ++tn)
                        acc[tm][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[tm][kk], b[tn][kk], acc[tm][tn], 0, 0, 0);
            __builtin_amdgcn_s_barrier();
        }
        float s = 0.f;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                for (int r = 0; r < 4; ++r) s += acc[i][j][r];
        out[blockIdx.x * 256 + t] = s;
    }
}

template <int SHAPE>
static double run(const float* src, float* out, int blocks, int steps, int launches, unsigned span = 1u << 20) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) loop_kernel<SHAPE><<<blocks, 256>>>(src, out, steps, span);
    hipEventRecord(e0);
    for (int i = 0; i < launches; ++i) loop_kernel<SHAPE><<<blocks, 256>>>(src, out, steps, span);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const double flop = 2.0 * 128 * 128 * 32 * (double)steps * blocks * launches;
    return flop / (ms * 1e-3) / 1e12;
}

int main(int argc, char** argv) {
    const int zero = argc > 1 && atoi(argv[1]) == 1;
    const int n = 1 << 28;   // 1 GiB: the DMA variant streams from it (HBM) or from its first 1 MiB (L2)
    std::vector<float> h(n);
    unsigned s = 12345u;
    for (int i = 0; i < n; ++i) {
        s = s * 1664525u + 1013904223u;
        h[i] = zero ? 0.f : ((s >> 8) * (1.0f / 16777216.0f) - 0.5f);
    }
    float *src, *out;
    hipMalloc(&src, n * 4);
    hipMalloc(&out, 4096 * 256 * 4);
    hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice);
    const int blocks = 512, steps = 2000, launches = argc > 2 ? atoi(argv[2]) : 400;   // ~2.8 s per shape at peak
    for (int rep = 0; rep < 2; ++rep) {
        const double t32 = run<32>(src, out, blocks, steps, launches);
        const double t16 = run<16>(src, out, blocks, steps, launches);
        const double d2 = run<33>(src, out, blocks, steps, launches, 1u << 20);
        const double dh = run<33>(src, out, blocks, steps, launches, 0x3fff0000u);
        const double s2 = run<34>(src, out, blocks, steps, launches, 1u << 20);
        const double sh = run<34>(src, out, blocks, steps, launches, 0x3fff0000u);
        printf("%s rep %d: 32x32x2 %.1f TF/s  16x16x4 %.1f TF/s  ratio %.3f | 32x32x2 + operand DMA: L2-hot %.1f, HBM stream %.1f | DMA among the MFMAs: L2-hot %.1f, HBM %.1f\n",
               zero ? "zero" : "random", rep, t32, t16, t16 / t32, d2, dh, s2, sh);
    }
    hipFree(src);
    hipFree(out);
    return 0;
}
