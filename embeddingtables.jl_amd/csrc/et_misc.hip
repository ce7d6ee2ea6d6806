// et_misc.hip — ABI housekeeping, synthetic-data fills and the multi-GPU concat
// assembly (its own translation unit).
#include "et_common.h"

namespace et {

// Same arithmetic as oracle/embtab_oracle.c:fill_range (fma in double, then one
// rounding to the element type) so CPU and GPU fills are bit-identical.
template <typename T>
__global__ __launch_bounds__(256) void k_fill_uniform(T* __restrict__ dst, int64_t n,
                                                      uint64_t seed, uint64_t offset, double lo,
                                                      double span) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * 256) {
        const uint64_t h = fill_hash(seed, offset + (uint64_t)i);
        const double u = (double)(h >> 40) * (1.0 / 16777216.0);
        const double v = __fma_rn(span, u, lo);
        if constexpr (sizeof(T) == 2)
            dst[i] = (T)(float)v;  // double -> float -> half / bf16, as the oracle does
        else if constexpr (__is_same(T, int32_t) || __is_same(T, int64_t))
            dst[i] = (T)floor(v);
        else
            dst[i] = (T)v;
    }
}

__global__ __launch_bounds__(256) void k_fill_index(int64_t* __restrict__ idx, int64_t n,
                                                    uint64_t nrows, uint64_t seed,
                                                    uint64_t offset) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * 256) {
        const uint64_t h = fill_hash(seed, offset + (uint64_t)i);
        idx[i] = 1 + (int64_t)__umul64hi(h, nrows);
    }
}

// dst[off_r + f, j] = slab_r[f, j] for f < rows_r (concat), or the reverse (split):
// one wave per (rank, bag) row segment.
struct ConcatPack {
    int32_t rows[64];
    int64_t off[64];
};

template <bool SPLIT>
__global__ __launch_bounds__(256) void k_slab_copy(char* __restrict__ slabs, int nranks,
                                                   int64_t slab_ld_b, int64_t batch,
                                                   ConcatPack pack, char* __restrict__ dst,
                                                   int64_t ld_dst_b, int es) {
    const int64_t w = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    const int r = (int)(w % nranks);
    const int64_t j = w / nranks;
    if (j >= batch) return;
    const int64_t nb = (int64_t)pack.rows[r] * es;
    char* slab = slabs + ((int64_t)r * batch + j) * slab_ld_b;
    char* mat = dst + j * ld_dst_b + pack.off[r] * es;
    const char* src = SPLIT ? mat : slab;
    char* out = SPLIT ? slab : mat;
    if (((uintptr_t)src & 15) == 0 && ((uintptr_t)out & 15) == 0 && (nb & 15) == 0) {
        for (int64_t b = (int64_t)lane * 16; b < nb; b += 64 * 16)
            *reinterpret_cast<u32x4*>(out + b) = *reinterpret_cast<const u32x4*>(src + b);
    } else {
        for (int64_t b = lane; b < nb; b += 64) out[b] = src[b];
    }
}

template <bool SPLIT>
int slab_copy(int dtype, void* slabs, int32_t nranks, int64_t slab_ld, int64_t batch,
              const int32_t* rows, const int64_t* off, void* mat, int64_t ld, void* stream) {
    const int es = elsize(dtype);
    if (!es) return fail(ET_ERR_UNSUPPORTED, "dtype %d", dtype);
    if (nranks <= 0 || nranks > 64) return fail(ET_ERR_ARG, "nranks must be in 1..64");
    if (batch <= 0) return ET_OK;
    if (!slabs || !mat || !rows || !off) return fail(ET_ERR_ARG, "NULL argument");
    ConcatPack pack;
    for (int r = 0; r < nranks; ++r) {
        if (rows[r] < 0 || rows[r] > slab_ld) return fail(ET_ERR_ARG, "rank %d rows", r);
        if (rows[r] > 0 && (off[r] < 0 || off[r] + rows[r] > ld))
            return fail(ET_ERR_ARG, "rank %d rows outside the matrix", r);
        pack.rows[r] = rows[r];
        pack.off[r] = off[r];
    }
    const int64_t waves = (int64_t)nranks * batch;
    const int64_t blocks = (waves + 3) / 4;
    if (blocks > 0x7fffffffll) return fail(ET_ERR_ARG, "grid too large");
    hipLaunchKernelGGL(k_slab_copy<SPLIT>, dim3((unsigned)blocks), dim3(256), 0,
                       static_cast<hipStream_t>(stream), static_cast<char*>(slabs), nranks,
                       slab_ld * es, batch, pack, static_cast<char*>(mat), ld * es, es);
    ET_LAUNCH_CHECK("k_slab_copy");
    return ET_OK;
}

// One-sided exchange of a sharded step ("fused P2P xGMI
// writes"): every 16-byte vector of this rank's destination columns is read once
// and stored straight into the same columns of each peer's destination (mapped
// with et_ipc_open).  One thread per vector; the system-scope fence makes the
// remote stores visible before the kernel retires, so a stream-ordered barrier
// after the launch (a one-element RCCL all-reduce) publishes them.
struct PeerPack {
    char* p[ET_MAX_PEERS];
};

template <bool VEC>
__global__ __launch_bounds__(256) void k_push_cols(const char* __restrict__ src, int64_t ld_b,
                                                   int64_t batch, int64_t nb, PeerPack peers,
                                                   int npeers) {
    const int64_t per_row = VEC ? nb >> 4 : nb;
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t < batch * per_row) {
        const int64_t j = t / per_row;
        const int64_t o = j * ld_b + (t - j * per_row) * (VEC ? 16 : 1);
        if constexpr (VEC) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(src + o);
            for (int q = 0; q < npeers; ++q) *reinterpret_cast<u32x4*>(peers.p[q] + o) = v;
        } else {
            const char v = src[o];
            for (int q = 0; q < npeers; ++q) peers.p[q][o] = v;
        }
    }
    __threadfence_system();
}

}  // namespace et

extern "C" int et_push_cols(int dtype, const void* src, int64_t ld, int64_t batch, int64_t col,
                            int64_t ncols, void* const* peers, int32_t npeers, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    const int es = et::elsize(dtype);
    if (!es) return et::fail(ET_ERR_UNSUPPORTED, "dtype %d", dtype);
    if (npeers < 0 || npeers > ET_MAX_PEERS)
        return et::fail(ET_ERR_ARG, "npeers must be in 0..%d", ET_MAX_PEERS);
    if (batch < 0 || ncols < 0 || col < 0 || col + ncols > ld)
        return et::fail(ET_ERR_ARG, "columns [%lld, %lld) outside ld %lld", (long long)col,
                        (long long)(col + ncols), (long long)ld);
    if (batch == 0 || ncols == 0 || npeers == 0) return ET_OK;
    if (!src || !peers) return et::fail(ET_ERR_ARG, "NULL argument");
    et::PeerPack pack = {};
    bool vec = ((uintptr_t)src & 15) == 0 && ((ld * es) & 15) == 0 && ((col * es) & 15) == 0 &&
               ((ncols * es) & 15) == 0;
    for (int q = 0; q < npeers; ++q) {
        if (!peers[q]) return et::fail(ET_ERR_ARG, "peer %d is NULL", q);
        pack.p[q] = static_cast<char*>(peers[q]) + col * es;
        vec = vec && ((uintptr_t)peers[q] & 15) == 0;
    }
    const char* s = static_cast<const char*>(src) + col * es;
    const int64_t nb = ncols * es;
    const int64_t threads = batch * (vec ? nb / 16 : nb);
    const int64_t blocks = (threads + 255) / 256;
    if (blocks > 0x7fffffffll) return et::fail(ET_ERR_ARG, "grid too large");
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (vec)
        hipLaunchKernelGGL(et::k_push_cols<true>, dim3((unsigned)blocks), dim3(256), 0, st, s,
                           ld * es, batch, nb, pack, npeers);
    else
        hipLaunchKernelGGL(et::k_push_cols<false>, dim3((unsigned)blocks), dim3(256), 0, st, s,
                           ld * es, batch, nb, pack, npeers);
    ET_LAUNCH_CHECK("k_push_cols");
    return ET_OK;
}

extern "C" int et_ipc_handle(const void* ptr, void* handle, int64_t* offset) {
    et::clear_err();
    if (!ptr || !handle || !offset) return et::fail(ET_ERR_ARG, "NULL argument");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    ET_HIP_CHECK(hipMemGetAddressRange(&base, &size, const_cast<void*>(ptr)));
    hipIpcMemHandle_t h;
    ET_HIP_CHECK(hipIpcGetMemHandle(&h, base));
    memcpy(handle, &h, sizeof(h));
    *offset = static_cast<const char*>(ptr) - static_cast<const char*>(base);
    return ET_OK;
}

extern "C" int et_ipc_open(const void* handle, int64_t offset, void** ptr) {
    et::clear_err();
    if (!handle || !ptr || offset < 0) return et::fail(ET_ERR_ARG, "bad argument");
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    void* base = nullptr;
    ET_HIP_CHECK(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess));
    *ptr = static_cast<char*>(base) + offset;
    return ET_OK;
}

extern "C" int et_ipc_close(void* ptr, int64_t offset) {
    et::clear_err();
    if (!ptr || offset < 0) return et::fail(ET_ERR_ARG, "bad argument");
    ET_HIP_CHECK(hipIpcCloseMemHandle(static_cast<char*>(ptr) - offset));
    return ET_OK;
}

extern "C" int et_abi_version(void) { return ET_ABI_VERSION; }

extern "C" const char* et_last_error(void) { return et::err_buf(); }

extern "C" int et_fill_uniform(int dtype, void* dst, int64_t n, uint64_t seed, uint64_t offset,
                               double lo, double hi, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    if (n < 0) return et::fail(ET_ERR_ARG, "negative n");
    if (n == 0) return ET_OK;
    if (!dst) return et::fail(ET_ERR_ARG, "dst is NULL");
    hipStream_t s = static_cast<hipStream_t>(stream);
    int64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    const double span = hi - lo;
    switch (dtype) {
        case ET_F32:
            hipLaunchKernelGGL(et::k_fill_uniform<float>, dim3(blocks), dim3(256), 0, s,
                               (float*)dst, n, seed, offset, lo, span);
            break;
        case ET_F64:
            hipLaunchKernelGGL(et::k_fill_uniform<double>, dim3(blocks), dim3(256), 0, s,
                               (double*)dst, n, seed, offset, lo, span);
            break;
        case ET_F16:
            hipLaunchKernelGGL(et::k_fill_uniform<_Float16>, dim3(blocks), dim3(256), 0, s,
                               (_Float16*)dst, n, seed, offset, lo, span);
            break;
        case ET_BF16:
            hipLaunchKernelGGL(et::k_fill_uniform<__bf16>, dim3(blocks), dim3(256), 0, s,
                               (__bf16*)dst, n, seed, offset, lo, span);
            break;
        case ET_I32:
            hipLaunchKernelGGL(et::k_fill_uniform<int32_t>, dim3(blocks), dim3(256), 0, s,
                               (int32_t*)dst, n, seed, offset, lo, span);
            break;
        case ET_I64:
            hipLaunchKernelGGL(et::k_fill_uniform<int64_t>, dim3(blocks), dim3(256), 0, s,
                               (int64_t*)dst, n, seed, offset, lo, span);
            break;
        default: return et::fail(ET_ERR_UNSUPPORTED, "dtype %d", dtype);
    }
    ET_LAUNCH_CHECK("k_fill_uniform");
    return ET_OK;
}

extern "C" int et_fill_index_uniform(int64_t* idx, int64_t n, int64_t nrows, uint64_t seed,
                                     uint64_t offset, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    if (n < 0 || nrows <= 0) return et::fail(ET_ERR_ARG, "need n >= 0 and nrows > 0");
    if (n == 0) return ET_OK;
    if (!idx) return et::fail(ET_ERR_ARG, "idx is NULL");
    int64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(et::k_fill_index, dim3(blocks), dim3(256), 0,
                       static_cast<hipStream_t>(stream), idx, n, (uint64_t)nrows, seed, offset);
    ET_LAUNCH_CHECK("k_fill_index");
    return ET_OK;
}

extern "C" int et_concat_slabs(int dtype, const void* slabs, int32_t nranks, int64_t slab_ld,
                               int64_t batch, const int32_t* rows, const int64_t* dst_row_off,
                               void* dst, int64_t ld_dst, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    return et::slab_copy<false>(dtype, const_cast<void*>(slabs), nranks, slab_ld, batch, rows,
                                dst_row_off, dst, ld_dst, stream);
}

extern "C" int et_split_slabs(int dtype, const void* src, int64_t ld_src, int64_t batch,
                              int32_t nranks, const int32_t* rows, const int64_t* src_row_off,
                              void* slabs, int64_t slab_ld, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    return et::slab_copy<true>(dtype, slabs, nranks, slab_ld, batch, rows, src_row_off,
                               const_cast<void*>(src), ld_src, stream);
}

ET_OOB_READER(misc)

extern "C" int et_check_errors(uint64_t* oob_count) {
    et::clear_err();
    ET_HIP_CHECK(hipDeviceSynchronize());
    uint64_t a = 0, b = 0, c = 0;
    int st;
    if ((st = et::oob_take_lookup(&a)) != ET_OK) return st;
    if ((st = et::oob_take_update(&b)) != ET_OK) return st;
    if ((st = et::oob_take_misc(&c)) != ET_OK) return st;
    if (oob_count) *oob_count = a + b + c;
    return ET_OK;
}
