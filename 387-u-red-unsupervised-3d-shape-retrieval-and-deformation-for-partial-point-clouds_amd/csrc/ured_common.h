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
// from its arguments or reads from device tables (segment tables, NN indices, labels), and of the
// raw buffer offsets of the MFMA kernels; a violation traps (the launch fails with a fault that
// names the kernel). Compiled out (no code) in the default build.
#ifndef URED_DEBUG_BOUNDS
#define URED_DEBUG_BOUNDS 0
#endif
#define URED_DBG_CHECK(cond)                                     \
    do {                                                         \
        if (URED_DEBUG_BOUNDS && !(cond)) __builtin_trap();      \
    } while (0)

#define URED_REQUIRE(cond, ...)                                  \
    do {                                                         \
        if (!(cond)) return ured::set_error(URED_EINVAL, __VA_ARGS__); \
    } while (0)
