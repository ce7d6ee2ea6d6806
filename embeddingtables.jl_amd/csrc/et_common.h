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
#include <stdlib.h>
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

// Tuning knobs.  The shipped library reads NO environment variable: ET_KNOB(name, dflt) is
// the tuned default, a compile-time constant.  An experiment build (-DET_EXPERIMENTS,
// tools/exp_build.sh, never the library the package loads) reads `name` from the
// environment instead (an integer; unset = dflt), so a sweep needs no source edit.  Every
// knob selects between correct variants only (schedules, grids, thresholds): results are
// bit-identical whatever its value.  tests/test_knobs.py checks that the shipped library
// carries no knob name.
#ifdef ET_EXPERIMENTS
inline long long env_knob(const char* name, long long dflt) {
    const char* e = getenv(name);
    return e && *e ? atoll(e) : dflt;
}
#define ET_KNOB(name, dflt) ((decltype(dflt))::et::env_knob(name, (long long)(dflt)))
#else
#define ET_KNOB(name, dflt) (dflt)
#endif

// ---------------------------------------------------------------------------
// Device-side helpers
// ---------------------------------------------------------------------------

// Out-of-range index counter, one per translation unit (internal linkage, so the
// kernels of each TU need no relocatable device code); each TU exports its reader
// through ET_OOB_READER and et_check_errors sums them.
static __device__ unsigned long long g_oob_count;

// Opens the device's exact-update side queues at the first library call (et_update.hip,
// SideStreams: the order in which a process opens hardware queues decides their pipes).
void open_side_streams(hipStream_t caller);

int oob_take_lookup(uint64_t* v);
int oob_take_update(uint64_t* v);
int oob_take_misc(uint64_t* v);

// Read and clear this TU's counter (the device is synchronised by the caller).
#define ET_OOB_READER(name)                                                              \
    namespace et {                                                                       \
    int oob_take_##name(uint64_t* v) {                                                   \
        unsigned long long x = 0, zero = 0;                                              \
        ET_HIP_CHECK(hipMemcpyFromSymbol(&x, HIP_SYMBOL(g_oob_count), sizeof(x), 0,      \
                                         hipMemcpyDeviceToHost));                        \
        ET_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_oob_count), &zero, sizeof(zero), 0,  \
                                       hipMemcpyHostToDevice));                          \
        *v = x;                                                                          \
        return ET_OK;                                                                    \
    }                                                                                    \
    }

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

// ---------------------------------------------------------------------------
// Shared by the lookup and update translation units
// ---------------------------------------------------------------------------
// Address of column `row` (0-based) of a contiguous or paged (SplitEmbedding) table.
template <typename T>
__device__ __forceinline__ T* col_ptr(const void* table, int64_t ld, int64_t cols_per_page,
                                      uint64_t row) {
    if (cols_per_page > 0) {
        T* const* pages = reinterpret_cast<T* const*>(table);
        return pages[row / (uint64_t)cols_per_page] + (row % (uint64_t)cols_per_page) * ld;
    }
    return (T*)table + row * (uint64_t)ld;
}

constexpr int kVecDims[] = {16, 32, 64, 128, 256, 512};

inline bool vec_dim_ok(int D) {
    for (int x : kVecDims)
        if (x == D) return true;
    return false;
}

// Dims that are a multiple of 16 bytes but not a power-of-two vector width: the masked
// vector kernel at the next power-of-two capacity (up to 2048 elements).
inline int masked_capacity(int D) {
    int c = 16;
    while (c < D) c <<= 1;
    return c;
}

}  // namespace et
