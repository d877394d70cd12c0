// ured_common.h — shared helpers for the libured_hip.so C-ABI (error state, checks).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdarg>

namespace ured {

// Thread-local message for ured_last_error().
inline char* err_buf() {
    static thread_local char buf[512];
    return buf;
}

inline int set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(err_buf(), 512, fmt, ap);
    va_end(ap);
    return code;
}

inline void clear_error() { err_buf()[0] = 0; }

// Check the launch status of the kernels just enqueued.
inline int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error((int)e, "%s: %s", what, hipGetErrorString(e));
    return 0;
}

}  // namespace ured

// Debug build (-DURED_DEBUG_BOUNDS=1): device-side bounds checks of the indices a kernel derives
// from its arguments or reads from device tables (segment tables, NN indices, labels), of the raw
// buffer offsets and LDS-DMA ranges of the MFMA kernels, and of their epilogue stores. A violation
// does not trap: the first one of each source file is recorded as (file id << 32 | line) in that
// file's device word, which the host reads (and clears) through ured_debug_violation(file id)
// (tests/conftest.py checks it after every test when the debug library is loaded). Compiled out
// (no code) in the default build.
#ifndef URED_DEBUG_BOUNDS
#define URED_DEBUG_BOUNDS 0
#endif
#if URED_DEBUG_BOUNDS
#ifndef URED_DBG_FILE
#error "define URED_DBG_FILE (the source file's id) before including ured_common.h"
#endif
__device__ unsigned long long ured_dbg_first;   // one per source file (each .hip is its own code object)
#define URED_DBG_CHECK(cond)                                                                             \
    do {                                                                                                 \
        if (!(cond))                                                                                     \
            atomicCAS(&ured_dbg_first, 0ull, ((unsigned long long)URED_DBG_FILE << 32) | (unsigned)__LINE__); \
    } while (0)
// host accessor of this file's word (one extern "C" function per source file)
#define URED_DBG_ACCESSOR(NAME)                                                                          \
    extern "C" unsigned long long NAME(int reset) {                                                      \
        unsigned long long v = 0;                                                                        \
        if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(ured_dbg_first), sizeof v) != hipSuccess) return ~0ull;   \
        if (reset) {                                                                                     \
            const unsigned long long z = 0;                                                              \
            if (hipMemcpyToSymbol(HIP_SYMBOL(ured_dbg_first), &z, sizeof z) != hipSuccess) return ~0ull; \
        }                                                                                                \
        return v;                                                                                        \
    }
#else
#define URED_DBG_CHECK(cond) do { } while (0)
#define URED_DBG_ACCESSOR(NAME)
#endif

#define URED_REQUIRE(cond, ...)                                  \
    do {                                                         \
        if (!(cond)) return ured::set_error(URED_EINVAL, __VA_ARGS__); \
    } while (0)
