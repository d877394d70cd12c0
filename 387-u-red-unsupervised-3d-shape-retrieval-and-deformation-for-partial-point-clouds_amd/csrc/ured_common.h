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

#define URED_REQUIRE(cond, ...)                                  \
    do {                                                         \
        if (!(cond)) return ured::set_error(URED_EINVAL, __VA_ARGS__); \
    } while (0)
