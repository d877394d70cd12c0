// copy.hip — several device-to-device copies in one launch (ured_copy_batch, include/ured_hip.h).
//
// The HIP-graph training step copies each new batch into the captured graph's static input
// tensors before the replay (engine/graph.py); one launch of this kernel replaces one runtime
// blit per tensor (9 per config-2 step). Each item moves in 16-, 4- or 1-byte units (the widest
// its two addresses and size allow); the launch's threads stride over the concatenated unit
// ranges, so a large item and many small ones share the grid.
#include <hip/hip_runtime.h>
#define URED_DBG_FILE 7
#include "ured_common.h"
#include "../../include/ured_hip.h"

namespace {

struct CopyArgs {
    UredCopyItem it[URED_COPY_MAX];
    long long start[URED_COPY_MAX + 1];   // first unit index of each item (exclusive prefix sum)
    int unit[URED_COPY_MAX];
    int n;
};

__global__ __launch_bounds__(256) void copy_batch_kernel(const CopyArgs a) {
    const long long total = a.start[a.n];
    for (long long u = (long long)blockIdx.x * 256 + threadIdx.x; u < total; u += (long long)gridDim.x * 256) {
        int i = 0;
#pragma unroll
        for (int q = 1; q < URED_COPY_MAX; ++q)
            if (q < a.n && u >= a.start[q]) i = q;
        const long long k = u - a.start[i];
        const UredCopyItem& c = a.it[i];
        if (a.unit[i] == 16) reinterpret_cast<float4*>(c.dst)[k] = reinterpret_cast<const float4*>(c.src)[k];
        else if (a.unit[i] == 4) reinterpret_cast<unsigned*>(c.dst)[k] = reinterpret_cast<const unsigned*>(c.src)[k];
        else reinterpret_cast<unsigned char*>(c.dst)[k] = reinterpret_cast<const unsigned char*>(c.src)[k];
    }
}

}  // namespace

extern "C" int ured_copy_batch(const UredCopyItem* items, int n, void* stream) {
    ured::clear_error();
    URED_REQUIRE(n >= 0 && n <= URED_COPY_MAX && (n == 0 || items), "ured_copy_batch: 0..%d items", URED_COPY_MAX);
    CopyArgs a;
    a.n = 0;
    a.start[0] = 0;
    for (int i = 0; i < n; ++i) {
        const UredCopyItem& c = items[i];
        URED_REQUIRE(c.bytes >= 0, "ured_copy_batch: negative size");
        if (c.bytes == 0) continue;
        URED_REQUIRE(c.dst && c.src, "ured_copy_batch: null pointer");
        const unsigned long long al = (unsigned long long)(uintptr_t)c.dst | (unsigned long long)(uintptr_t)c.src |
                                      (unsigned long long)c.bytes;
        const int unit = (al % 16 == 0) ? 16 : (al % 4 == 0) ? 4 : 1;
        a.it[a.n] = c;
        a.unit[a.n] = unit;
        a.start[a.n + 1] = a.start[a.n] + c.bytes / unit;
        ++a.n;
    }
    for (int q = a.n + 1; q <= URED_COPY_MAX; ++q) a.start[q] = a.start[a.n];
    if (a.n == 0) return 0;
    const long long units = a.start[a.n];
    const int blocks = (int)std::min<long long>((units + 255) / 256, 2048);
    hipLaunchKernelGGL(copy_batch_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
    return ured::launch_status("ured_copy_batch");
}

URED_DBG_ACCESSOR(ured_dbg_copy)
