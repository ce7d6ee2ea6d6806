// et_common.h — shared helpers of libembtab_hip.so (gfx950 / CDNA4 only).
//
// Error reporting for the C ABI (thread-local message + int status), the
// device-side out-of-range counter, 16-byte vector helpers and the
// counter-based hash shared with oracle/embtab_oracle.c.
#pragma once

#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "embtab.h"

namespace et {

// ---------------------------------------------------------------------------
// Host-side error plumbing
// ---------------------------------------------------------------------------
inline char* err_buf() {
    static thread_local char buf[512] = {0};
    return buf;
}

inline int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(err_buf(), 512, fmt, ap);
    va_end(ap);
    return code;
}

inline void clear_err() { err_buf()[0] = 0; }

#define ET_HIP_CHECK(call)                                                              \
    do {                                                                                \
        hipError_t e_ = (call);                                                         \
        if (e_ != hipSuccess)                                                           \
            return ::et::fail(ET_ERR_HIP, "%s failed: %s", #call, hipGetErrorString(e_)); \
    } while (0)

#define ET_LAUNCH_CHECK(what)                                                          \
    do {                                                                                \
        hipError_t e_ = hipGetLastError();                                              \
        if (e_ != hipSuccess)                                                           \
            return ::et::fail(ET_ERR_HIP, "launch of %s failed: %s", what,              \
                              hipGetErrorString(e_));                                   \
    } while (0)

inline int elsize(int dtype) {
    switch (dtype) {
        case ET_F32: return 4;
        case ET_F16: return 2;
        case ET_BF16: return 2;
        case ET_F64: return 8;
        case ET_I32: return 4;
        case ET_I64: return 8;
        default: return 0;
    }
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// ---------------------------------------------------------------------------
// Device-side helpers
// ---------------------------------------------------------------------------

// Out-of-range index counter (read + cleared by et_check_errors).
__device__ unsigned long long g_oob_count;

__device__ __forceinline__ void note_oob(int n = 1) { atomicAdd(&g_oob_count, (unsigned long long)n); }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void store16(void* p, u32x4 v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    else
        *reinterpret_cast<u32x4*>(p) = v;
}

template <bool NT, typename T>
__device__ __forceinline__ void store_scalar(T* p, T v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// splitmix64 finaliser — identical to oracle/embtab_oracle.c:hash64.
__host__ __device__ __forceinline__ uint64_t hash64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__host__ __device__ __forceinline__ uint64_t fill_hash(uint64_t seed, uint64_t i) {
    return hash64(seed * 0xD1B54A32D192ED03ull + i);
}

}  // namespace et
