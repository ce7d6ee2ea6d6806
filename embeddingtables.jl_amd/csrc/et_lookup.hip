// et_lookup.hip — forward gather kernels for gfx950.
//
// Replaces the reference's CPU kernels (darchr/EmbeddingTables.jl):
//   lookup_generic! / lookup_static!        src/lookup.jl:51-182
//   maplookup!(::PreallocationStrategy)     src/lookup.jl:316-371
//
// Design:
//   * one lane GROUP per output bag; a group is the LPR = min(64, row_bytes/16) lanes
//     that together hold one embedding row as 16-byte vectors, so D = 128 fp32
//     (512 B) is a half-wave and one wave-instruction moves two rows (1 KiB);
//   * the bag's index list is read once, coalesced, by the group's lanes and
//     broadcast with a lane shuffle (ds_bpermute), so row addresses never wait on a
//     second global load;
//   * U rows per group are issued before any is consumed (U * 1 KiB per wave in
//     flight), then accumulated strictly in pool order starting from the first
//     row — the reference's summation order, so fp32 results are bit-identical;
//   * a workgroup (4 waves) owns a chunk of consecutive bags of ONE table; the
//     grid enumerates (table, chunk) items table-fastest, like the reference's
//     `_divrem_index(k, ntables)` work queue (src/lookup.jl:351-355);
//   * descriptors travel by value in the kernel-argument segment (no device
//     allocation, hipGraph-capturable).
#include <type_traits>
#include "et_common.h"

#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <utility>
#include <vector>

namespace et {

struct XcdQueue;
struct LookupPack {
    et_lookup_desc d[ET_MAX_TABLES_PER_LAUNCH];
    // the caller's queue block (et_maplookup_prealloc_q), or null: the static stripe schedule
    XcdQueue* queue = nullptr;
};

// Geometry of the vector path for element type T and feature size D.
template <typename T, int D>
struct VecGeom {
    static constexpr int N = 16 / (int)sizeof(T);     // elements per 16-B vector
    static constexpr int VPR = D / N;                 // vectors per row
    static constexpr int LPR = VPR < 64 ? VPR : 64;   // lanes per group (one row)
    static constexpr int NV = VPR / LPR;              // vectors per lane per row
    static constexpr int GPW = 64 / LPR;              // groups (bags) per wave
    static constexpr int U = NV >= 8 ? 1 : 8 / NV;    // default rows in flight per group
    static_assert(D % N == 0, "row must be whole vectors");
    static_assert(VPR <= 64 ? (64 % VPR == 0) : (VPR % 64 == 0), "unsupported row size");
};

template <typename T, int N>
__device__ __forceinline__ void unpack16(u32x4 v, T (&x)[N]) {
    static_assert(N * sizeof(T) == 16, "");
    __builtin_memcpy(x, &v, 16);
}

template <typename T, int N>
__device__ __forceinline__ u32x4 pack16(const T (&x)[N]) {
    u32x4 v;
    __builtin_memcpy(&v, x, 16);
    return v;
}

// Broadcast the 64-bit value held by lane (g*LPR + i) to every lane of group g; i is
// wave-uniform.  With <= ET_BCAST_READLANE_MAX_GPW groups per wave this is 2*GPW
// v_readlane + selects (no LDS round trip, nothing for the waitcnt pass to serialise);
// wider waves use ds_bpermute.  Round 4: 2 (four groups — 256-byte rows, the Float16
// config-3 leg — take ds_bpermute: 14 VALU per row were the issue bound of its
// L2-resident tables); -DET_BCAST_READLANE_MAX_GPW=4 restores the round-3 choice.
#ifndef ET_BCAST_READLANE_MAX_GPW
#define ET_BCAST_READLANE_MAX_GPW 2
#endif
template <int LPR>
__device__ __forceinline__ long long group_bcast(long long v, int i, int g) {
    constexpr int GPW = 64 / LPR;
    if constexpr (GPW <= ET_BCAST_READLANE_MAX_GPW) {
        const int lo = (int)v, hi = (int)(v >> 32);
        int rlo = __builtin_amdgcn_readlane(lo, i), rhi = __builtin_amdgcn_readlane(hi, i);
#pragma unroll
        for (int gg = 1; gg < GPW; ++gg) {
            const int tlo = __builtin_amdgcn_readlane(lo, gg * LPR + i);
            const int thi = __builtin_amdgcn_readlane(hi, gg * LPR + i);
            rlo = g == gg ? tlo : rlo;
            rhi = g == gg ? thi : rhi;
        }
        return (long long)(((unsigned long long)(unsigned)rhi << 32) | (unsigned)rlo);
    } else {
        return __shfl(v, g * LPR + i, 64);
    }
}

// The same for a 32-bit value (one readlane per group, or one ds_bpermute).
template <int LPR>
__device__ __forceinline__ uint32_t group_bcast32(uint32_t v, int i, int g) {
    constexpr int GPW = 64 / LPR;
    if constexpr (GPW <= ET_BCAST_READLANE_MAX_GPW) {
        int r = __builtin_amdgcn_readlane((int)v, i);
#pragma unroll
        for (int gg = 1; gg < GPW; ++gg) {
            const int t = __builtin_amdgcn_readlane((int)v, gg * LPR + i);
            r = g == gg ? t : r;
        }
        return (uint32_t)r;
    } else {
        return (uint32_t)__shfl((int)v, g * LPR + i, 64);
    }
}

// A lane's 1-based index as its 0-based row, or ~0 when out of range (checked once per
// index, before the broadcast, instead of once per row in every lane of its group).
__device__ __forceinline__ uint32_t idx_row32(long long v, uint32_t nrows) {
    const uint64_t row = (uint64_t)(v - 1);
    return row < (uint64_t)nrows ? (uint32_t)row : ~0u;
}

// The first (up to) LPR indices of a bag, one per lane of the group; lanes past the
// end re-read the last one so that no lane is masked off.
template <int LPR, bool NTI = false>
__device__ __forceinline__ long long load_idx_chunk(const int64_t* __restrict__ ip, int cnt,
                                                    int sub) {
    const int64_t* p = ip + (sub < cnt ? sub : cnt - 1);
    if constexpr (NTI)
        return (long long)__builtin_nontemporal_load(p);
    else
        return (long long)*p;
}

// Issue UU row loads of one bag (slots i0 .. i0+UU-1 of the current index chunk, all
// valid), then add them to the accumulator in slot order.  Straight-line code: every
// load is issued before the first add waits, so UU rows per group are in flight (the
// waitcnt pass counts vmcnt down through the adds).  Row offsets use one 32x32->64
// multiply (the host guarantees nrows and ld_table below 2^32).
//
// PG (paged table, SplitEmbedding): `table` is the device array of page pointers and
// column r lives in page r / cpp at column r % cpp; the UU page-pointer loads are
// issued together before the row loads.
//
// MK (masked geometry): D is a power-of-two CAPACITY and the table's rows have only
// `vpr` 16-byte vectors (any dim that is a multiple of 16 bytes); lanes beyond the row
// re-read its last vector (same cache line, never out of bounds) and never store.
template <typename T, typename A, int D, int UU, bool NTL, bool PG = false, bool MK = false>
__device__ __forceinline__ void load_add(const T* __restrict__ table, uint32_t ld_table,
                                         uint32_t nrows, uint32_t cpp, uint32_t myr, int g,
                                         int sub, int i0, bool first_batch,
                                         A (&acc)[VecGeom<T, D>::NV][VecGeom<T, D>::N],
                                         int& bad, int vpr) {
    using G = VecGeom<T, D>;
    constexpr int N = G::N, LPR = G::LPR, NV = G::NV;
    uint64_t off[UU];
    bool ok[UU];
    const T* base[UU];
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        const uint32_t r = group_bcast32<LPR>(myr, i0 + u, g);  // idx_row32 of the index
        ok[u] = r != ~0u;
        const uint32_t row32 = ok[u] ? r : 0u;
        if constexpr (PG) {
            const uint32_t page = row32 / cpp;
            off[u] = (uint64_t)(row32 - page * cpp) * ld_table;
            base[u] = reinterpret_cast<const T* const*>(table)[page];
        } else {
            off[u] = (uint64_t)row32 * ld_table;
            base[u] = table;
        }
    }
    int vix[NV];  // this lane's vector of the row for each v
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        vix[v] = sub + v * LPR;
        if constexpr (MK) vix[v] = vix[v] < vpr ? vix[v] : vpr - 1;
    }
    u32x4 buf[UU][NV];
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        const u32x4* src = reinterpret_cast<const u32x4*>(base[u] + off[u]);
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            if constexpr (NTL)
                buf[u][v] = __builtin_nontemporal_load(src + vix[v]);
            else
                buf[u][v] = src[vix[v]];
        }
    }
    // Out-of-range rows (loaded from row 0) add zeros.  They are rare, so the wave tests
    // the batch once and only a batch holding one pays the per-row zero selects (round 4:
    // four selects per 16-byte vector and row were a tenth of the L2-resident tables' VALU).
    int anybad = 0;
#pragma unroll
    for (int u = 0; u < UU; ++u) anybad |= ok[u] ? 0 : 1;
    auto add_rows = [&](auto checked) {
#pragma unroll
        for (int u = 0; u < UU; ++u) {
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                T x[N];
                if constexpr (decltype(checked)::value)
                    unpack16<T, N>(ok[u] ? buf[u][v] : u32x4{0u, 0u, 0u, 0u}, x);
                else
                    unpack16<T, N>(buf[u][v], x);
#pragma unroll
                for (int k = 0; k < N; ++k) {
                    if (u == 0)
                        acc[v][k] = first_batch ? A(x[k]) : A(acc[v][k] + A(x[k]));
                    else
                        acc[v][k] = A(acc[v][k] + A(x[k]));
                }
            }
        }
    };
    if (__builtin_expect(__any(anybad), 0)) {
#pragma unroll
        for (int u = 0; u < UU; ++u) bad += ok[u] ? 0 : 1;
        add_rows(std::true_type{});
    } else {
        add_rows(std::false_type{});
    }
}

// Pooled sum of one bag by one lane group (vector path).
//   ip  : the bag's index list (1-based), `pool` >= 1 entries
//   my0 : its first index chunk, already loaded (load_idx_chunk)
//   out : the bag's output column
// Accumulation is acc = row(I[1]); acc += row(I[i]) for i = 2..P, element-wise and in
// order (src/lookup.jl:139-146), so fp32/fp64/int results equal the reference bit
// for bit; F16 rounds after every add (Julia Float16 `+`) unless A = float.
template <typename T, typename A, int D, int U, bool NT, bool NTL, bool PG = false,
          bool MK = false>
__device__ __forceinline__ void bag_sum_vec(const T* __restrict__ table, uint32_t ld_table,
                                            uint32_t nrows, uint32_t cpp,
                                            const int64_t* __restrict__ ip,
                                            int pool, long long my0, T* __restrict__ out, int g,
                                            int sub, int vpr) {
    using G = VecGeom<T, D>;
    constexpr int N = G::N, LPR = G::LPR, NV = G::NV;
    A acc[NV][N];
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
        for (int k = 0; k < N; ++k) acc[v][k] = A(0);
    int bad = 0;  // out-of-range indices of this bag (same in every lane of the group)

    for (int c0 = 0; c0 < pool; c0 += LPR) {
        const int cnt = pool - c0 < LPR ? pool - c0 : LPR;
        const long long my = c0 == 0 ? my0 : load_idx_chunk<LPR>(ip + c0, cnt, sub);
        const uint32_t myr = idx_row32(my, nrows);
        int i0 = 0;
#define ET_LOAD_ADD(UU) \
    load_add<T, A, D, UU, NTL, PG, MK>(table, ld_table, nrows, cpp, myr, g, sub, i0,       \
                                       c0 + i0 == 0, acc, bad, vpr)
        for (; i0 + U <= cnt; i0 += U) ET_LOAD_ADD(U);
        if constexpr (U > 8) {
            if (cnt - i0 >= 8) {
                ET_LOAD_ADD(8);
                i0 += 8;
            }
        }
        if constexpr (U > 4) {
            if (cnt - i0 >= 4) {
                ET_LOAD_ADD(4);
                i0 += 4;
            }
        }
        if constexpr (U > 2) {
            if (cnt - i0 >= 2) {
                ET_LOAD_ADD(2);
                i0 += 2;
            }
        }
        if (cnt - i0 >= 1) ET_LOAD_ADD(1);
#undef ET_LOAD_ADD
    }
    if (bad && sub == 0) note_oob(bad);
    u32x4* o = reinterpret_cast<u32x4*>(out) + sub;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        T y[N];
#pragma unroll
        for (int k = 0; k < N; ++k) y[k] = T(acc[v][k]);
        if (!MK || sub + v * LPR < vpr) store16<NT>(o + v * LPR, pack16<T, N>(y));
    }
}

// `rounds` bags of one table per lane group, the next bag's first index chunk loaded
// while the current bag's rows are in flight.
template <typename T, typename A, int D, int U, bool NT, bool NTL, bool NTI = false,
          bool PG = false, bool MK = false>
__device__ __forceinline__ void run_bags(const et_lookup_desc& d, int64_t batch,
                                         T* __restrict__ dst, int64_t ld_dst, int64_t chunk,
                                         int rounds) {
    using G = VecGeom<T, D>;
    const T* table = reinterpret_cast<const T*>(d.table);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane / G::LPR, sub = lane % G::LPR;
    const int64_t per_round = 4 * G::GPW;
    const int pool = d.pool;
    const int cnt0 = pool < G::LPR ? pool : G::LPR;
    const uint32_t ldt = (uint32_t)d.ld_table, nr = (uint32_t)d.nrows;
    const int vpr = MK ? d.dim / G::N : G::VPR;  // vectors per row
    int64_t bag = chunk * per_round * rounds + wave * G::GPW + g;
    long long my_next = load_idx_chunk<G::LPR, NTI>(
        d.idx + (bag < batch ? bag : batch - 1) * d.ld_idx, cnt0, sub);
    for (int r = 0; r < rounds; ++r) {
        if (bag >= batch) break;
        const long long my = my_next;
        const int64_t nbag = bag + per_round;
        if (r + 1 < rounds)
            my_next = load_idx_chunk<G::LPR, NTI>(
                d.idx + (nbag < batch ? nbag : batch - 1) * d.ld_idx, cnt0, sub);
        bag_sum_vec<T, A, D, U, NT, NTL, PG, MK>(table, ldt, nr, (uint32_t)d.cols_per_page,
                                                 d.idx + bag * d.ld_idx, pool, my,
                                                 dst + bag * ld_dst + d.dst_row_off, g, sub, vpr);
        bag = nbag;
    }
}

// A feature slice of a bag range (the feature-split tables of the striped schedule): the
// bags [bag0, bag1) of table d, features [fofs, fofs + DS) only — DS-feature rows at the
// table's row stride, so each lane group reads DS * sizeof(T) bytes per row.  Sums are per
// feature in pool order, exactly as run_bags, so the output is bit-identical however the
// features are cut.
template <typename T, typename A, int DS, bool NT>
__device__ __forceinline__ void run_bags_slice(const et_lookup_desc& d, int64_t batch,
                                               T* __restrict__ dst, int64_t ld_dst, int64_t bag0,
                                               int64_t bag1, int fofs) {
    using G = VecGeom<T, DS>;
    const T* table = reinterpret_cast<const T*>(d.table) + fofs;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane / G::LPR, sub = lane % G::LPR;
    const int64_t per_round = 4 * G::GPW;
    const int pool = d.pool;
    const int cnt0 = pool < G::LPR ? pool : G::LPR;
    const uint32_t ldt = (uint32_t)d.ld_table, nr = (uint32_t)d.nrows;
    const int64_t end = bag1 < batch ? bag1 : batch;
    int64_t bag = bag0 + wave * G::GPW + g;
    long long my_next = load_idx_chunk<G::LPR>(d.idx + (bag < end ? bag : end - 1) * d.ld_idx,
                                                cnt0, sub);
    while (bag < end) {
        const long long my = my_next;
        const int64_t nbag = bag + per_round;
        if (nbag < end) my_next = load_idx_chunk<G::LPR>(d.idx + nbag * d.ld_idx, cnt0, sub);
        bag_sum_vec<T, A, DS, G::U, NT, false>(table, ldt, nr, 0u, d.idx + bag * d.ld_idx, pool,
                                               my, dst + bag * ld_dst + d.dst_row_off + fofs, g,
                                               sub, G::VPR);
        bag = nbag;
    }
}

// ---------------------------------------------------------------------------
// Scalar-addressed bag loop for 512-byte rows (D = 128 fp32, 256 f16 / bf16, 64 f64 /
// i64): LPR = 32, so a wave holds two bags — A in lanes 0-31, B in lanes 32-63 — and
// both are wave-uniform.  Their index lists are therefore read with SCALAR loads
// (through the constant address space) and the 64-bit row addresses are formed on the
// scalar ALU; per row pair the vector ALU only picks one of the two addresses for its
// half and adds the lane's 16-byte offset.  load_add instead broadcasts every index
// lane by lane (v_readlane), selects per group, multiplies in 64 bits and selects the
// zero row per lane — about 20 vector instructions per 1 KiB wave-load that made the
// L2-resident tables issue-bound.  The summation order is unchanged (pool order from
// the first row), so results stay bit-identical.  A batch holding an out-of-range
// index is detected before its rows are loaded and the bag pair is redone by
// bag_pair_checked (rare; undefined behaviour in the reference).  Tried and dropped:
// touching the next round's index lines with a vector load behind the first batch
// (so its scalar loads hit L2) — 4% slower on the Criteo mix, 15% on L2-resident
// tables (in-order vmcnt: the next batch's waits include the prefetch).  Also dropped:
// pairing a heavy table's stripe with a light one in the two halves of each wave (light
// rows riding on the heavy rows' latency) — +11% on the Criteo mix: a wave then keeps
// half as many heavy-table bytes in flight, and the heavy tables are concurrency-bound.
// The same scheme for 256-byte rows (four bags per wave, three masked differences: 10
// instead of ~30 VALU per KiB) measured slower than load_add (D = 64 fp32, 8 tables,
// B = 65536: L2-resident 0.248 vs 0.227 ms, HBM 0.539 vs 0.462 ms) — four bags' scalar
// index loads stall each batch, where load_add prefetches the next bag's indices — so
// only 512-byte rows take this loop.
typedef const __attribute__((address_space(4))) int64_t* cidx_ptr;

// Bytes per lane of the scalar-addressed loop: 16 for 512-byte rows, 8 for 256-byte rows
// (D = 128 fp16 / bf16, 64 fp32): two bags per wave either way — half a wave per row —
// so both bags stay wave-uniform and their indices scalar.  (Round 2 tried 256-byte rows
// as FOUR bags per wave with 16-byte lanes: the four scalar index streams stalled each
// batch, and it was slower than load_add.)
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <int BPL> struct SgVec { typedef u32x4 type; };
template <> struct SgVec<8> { typedef u32x2 type; };
template <typename T> constexpr int sg_bpl(int D) { return D * (int)sizeof(T) / 32; }

template <bool NT, typename V>
__device__ __forceinline__ void store_v(V* p, V v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

__device__ __forceinline__ cidx_ptr as_scalar_idx(const int64_t* p) {
    return (cidx_ptr)(uintptr_t)p;
}

typedef const __attribute__((address_space(1))) u32x4 gvec16;

// Row offset of a 1-based index v (wave-uniform) in bytes: 32-bit scalar ops only
// (gfx950's scalar ALU has no 64-bit multiply or ordered 64-bit compare); `bad` gets
// a nonzero bit unless 1 <= v <= nrows.
__device__ __forceinline__ uint64_t row_off_s(int64_t v, uint32_t ldb, uint32_t nrows,
                                              uint32_t& bad) {
    const uint32_t lo = (uint32_t)v - 1u;
    // lo < nrows  <=>  the 64-bit difference lo - nrows borrows (all-ones high word);
    // arithmetic instead of a compare keeps the check on the scalar ALU
    const uint32_t borrow = (uint32_t)(((uint64_t)lo - (uint64_t)nrows) >> 32);
    bad |= (uint32_t)((uint64_t)v >> 32) | ~borrow;
    return (((uint64_t)__umulhi(lo, ldb)) << 32) | (uint64_t)(lo * ldb);
}

// One batch of UU rows of both bags.  Returns false — before issuing any row load —
// if an index of the batch is out of range; the caller then redoes the bag pair with
// bag_pair_checked.
// NA (experiment builds only, ET_HEAD_NOADD): the same loads, waits and stores with the adds
// replaced by an empty consumer (each loaded vector is an input of an empty asm, so its
// load must complete there; the result is the bag's first row, not its sum) — the ceiling of
// this schedule's byte mix without the arithmetic.
template <typename T, typename A, int UU, bool NTL, int BPL = 16, int NA = 0>
__device__ __forceinline__ bool load_add_s(uintptr_t tb, uint32_t ldb, uint32_t nrows,
                                           cidx_ptr ia, cidx_ptr ib, uint64_t hmask,
                                           uint64_t lane_off, bool first_batch,
                                           A (&acc)[BPL / sizeof(T)]) {
    constexpr int N = BPL / (int)sizeof(T);
    typedef typename SgVec<BPL>::type V;
    typedef const __attribute__((address_space(1))) V gvec;
    // lane address = table + row_off(A) + (hi ? row_off(B) - row_off(A) : 0) + 16*sub:
    // the difference is masked per lane (hmask = ~0 in lanes 32-63), so a row pair costs
    // two v_and and two 64-bit adds — no 64-bit selects between scalar operands
    uint64_t oa[UU], dd[UU];
    uint32_t bad = 0u;
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        oa[u] = row_off_s(ia[u], ldb, nrows, bad);
        dd[u] = row_off_s(ib[u], ldb, nrows, bad) - oa[u];
    }
    if (bad) return false;
    V buf[UU];
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        const uint64_t a = ((dd[u] & hmask) + lane_off) + (tb + oa[u]);
        const gvec* src = reinterpret_cast<const gvec*>(a);
        if constexpr (NTL)
            buf[u] = __builtin_nontemporal_load(src);
        else
            buf[u] = *src;
    }
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        T x[N];
        __builtin_memcpy(x, &buf[u], BPL);
        if constexpr (NA != 0) {
            if (u == 0 && first_batch) {
#pragma unroll
                for (int k = 0; k < N; ++k) acc[k] = A(x[k]);
            } else {
                asm volatile("" ::"v"(buf[u]));
            }
            continue;
        }
#pragma unroll
        for (int k = 0; k < N; ++k) {
            if (u == 0)
                acc[k] = first_batch ? A(x[k]) : A(acc[k] + A(x[k]));
            else
                acc[k] = A(acc[k] + A(x[k]));
        }
    }
    return true;
}

// The bag pair again, one row at a time with per-lane range checks: an out-of-range
// index contributes a zero row and is counted (the reference leaves it undefined).
template <typename T, typename A, int BPL = 16>
__device__ __forceinline__ void bag_pair_checked(uintptr_t tb, uint32_t ldb, uint32_t nrows,
                                                 const int64_t* ia, const int64_t* ib, bool hi,
                                                 int sub, int pool, A* acc, int* bad) {
    constexpr int N = BPL / (int)sizeof(T);
    typedef typename SgVec<BPL>::type V;
    const int64_t* ip = hi ? ib : ia;
#pragma unroll 1
    for (int i = 0; i < pool; ++i) {
        const uint64_t r = (uint64_t)(ip[i] - 1);
        const bool ok = r < (uint64_t)nrows;
        *bad += ok ? 0 : 1;
        const V v = *(reinterpret_cast<const V*>(
                          tb + (uint64_t)(ok ? (uint32_t)r : 0u) * ldb) + sub);
        T x[N];
        const V z = ok ? v : V(0u);
        __builtin_memcpy(x, &z, BPL);
        for (int k = 0; k < N; ++k) acc[k] = i == 0 ? A(x[k]) : A(acc[k] + A(x[k]));
    }
}

// `rounds` rounds of 8 bags per workgroup (bag mapping identical to run_bags: wave w
// of round r holds bags chunk*8*rounds + r*8 + 2w + {0, 1}).
template <typename T, typename A, int U, bool NT, bool NTL, int BPL = 16, int NA = 0>
__device__ __forceinline__ void run_bags_s(const et_lookup_desc& d, int64_t batch,
                                           T* __restrict__ dst, int64_t ld_dst, int64_t chunk,
                                           int rounds) {
    constexpr int N = BPL / (int)sizeof(T);
    typedef typename SgVec<BPL>::type V;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool hi = lane >= 32;
    const int sub = lane & 31;
    uint32_t hm = hi ? ~0u : 0u;
    asm volatile("" : "+v"(hm));  // opaque: keep `dd & hmask` two v_and, not selects
    const uint64_t hmask = ((uint64_t)hm << 32) | hm, lane_off = (uint64_t)sub * (uint64_t)BPL;
    const uintptr_t tb = reinterpret_cast<uintptr_t>(d.table);
    const uint32_t ldb = (uint32_t)(d.ld_table * (int64_t)sizeof(T)), nr = (uint32_t)d.nrows;
    const int pool = d.pool;
    int64_t bag = chunk * 8 * rounds + 2 * wave;
    for (int r = 0; r < rounds; ++r, bag += 8) {
        if (bag >= batch) break;
        const bool has_b = bag + 1 < batch;
        const cidx_ptr ia = as_scalar_idx(d.idx + bag * d.ld_idx);
        const cidx_ptr ib = has_b ? as_scalar_idx(d.idx + (bag + 1) * d.ld_idx) : ia;
        A acc[N];
#pragma unroll
        for (int k = 0; k < N; ++k) acc[k] = A(0);
        bool ok = true;
        int i0 = 0;
#define ET_LOAD_ADD_S(UU) \
    load_add_s<T, A, UU, NTL, BPL, NA>(tb, ldb, nr, ia + i0, ib + i0, hmask, lane_off, i0 == 0, acc)
        for (; ok && i0 + U <= pool; i0 += U) ok = ET_LOAD_ADD_S(U);
        if constexpr (U > 4) {
            if (ok && pool - i0 >= 4) {
                ok = ET_LOAD_ADD_S(4);
                i0 += 4;
            }
        }
        if constexpr (U > 2) {
            if (ok && pool - i0 >= 2) {
                ok = ET_LOAD_ADD_S(2);
                i0 += 2;
            }
        }
        if (ok && pool - i0 >= 1) ok = ET_LOAD_ADD_S(1);
#undef ET_LOAD_ADD_S
        int bad = 0;
        if (!ok)
            bag_pair_checked<T, A, BPL>(tb, ldb, nr, d.idx + bag * d.ld_idx,
                                   d.idx + (has_b ? bag + 1 : bag) * d.ld_idx, hi, sub, pool, acc,
                                   &bad);
        if (hi && !has_b) bad = 0;  // the upper half re-ran bag A: counted by the lower
        if (bad && sub == 0) note_oob(bad);
        if (!hi || has_b) {
            T y[N];
#pragma unroll
            for (int k = 0; k < N; ++k) y[k] = T(acc[k]);
            V* o = reinterpret_cast<V*>(dst + (bag + (hi ? 1 : 0)) * ld_dst + d.dst_row_off) + sub;
            V yv;
            __builtin_memcpy(&yv, y, BPL);
            store_v<NT>(o, yv);
        }
    }
}

// Pooled-sum kernel, vector path: grid = ntables * nchunks workgroups of 256.
// SG: the scalar-addressed loop (512-byte rows, contiguous tables, no masking).
template <typename T, typename A, int D, int U, bool NT, bool PG = false, bool MK = false,
          bool SG = false>
__global__ __launch_bounds__(256) void k_pooled_vec(LookupPack pack, int ntables, int64_t batch,
                                                    T* __restrict__ dst, int64_t ld_dst,
                                                    int rounds) {
    const int64_t item = blockIdx.x;
    const int t = (int)(item % ntables);
    const int64_t chunk = item / ntables;
    if constexpr (SG)
        run_bags_s<T, A, U, NT, false, sg_bpl<T>(D)>(pack.d[t], batch, dst, ld_dst, chunk, rounds);
    else
        run_bags<T, A, D, U, NT, false, false, PG, MK>(pack.d[t], batch, dst, ld_dst, chunk,
                                                       rounds);
}

// XCD-aware stripe schedule for multi-table launches.  Every table's chunks are cut
// into kXcds stripes; XCD x owns `ntables` stripes: one stripe of every HEAVY table
// (too big for an L2, so its rows come from HBM / the Infinity Cache whoever reads
// them) and whole runs of the LIGHT tables' stripes, so each XCD's 4 MiB L2 only
// ever holds a couple of light tables.  Workgroup b runs on XCD b % 8 (the observed
// round-robin dispatch; a different placement changes speed only, never results),
// and consecutive workgroups of one XCD cycle through its stripes, mixing HBM-bound
// and L2-bound work in time.
constexpr int kXcds = 8;

// 32-bit entries (table | stripe << 8) so the map is read with scalar loads (gfx950
// has no scalar byte loads).
constexpr int kMaxStripeEntries = 40;  // per XCD (kernel-argument size bound)
struct StripeMap {
    // entry[x][k]: table (bits 0-7), stripe (8-15), feature group + 1 (16-23; 0: whole
    // rows); every XCD has nent entries (the feature-split tables take fsplit_g each)
    uint32_t entry[kXcds][kMaxStripeEntries];
    int nent;
    int fsplit_g;          // feature groups of a split table (2, 4 or 8)
    uint32_t ntload_mask;  // bit t: non-temporal row loads for table t
    uint32_t prio_mask;    // bit t: table t's waves run at raised issue priority
    int prio;
    int nheavy;            // entry[x][0, nheavy): the heavy tables (> light_bytes)
    int qorder;            // queued schedule: 1 = every heavy item before the light ones
};

template <typename T, typename A, int D, int U, bool NT, bool NTI, bool SG = false, int NA = 0>
__device__ __forceinline__ void striped_body(const LookupPack& pack, const StripeMap& sm,
                                             int ntables, int64_t batch, T* __restrict__ dst,
                                             int64_t ld_dst, int rounds, int64_t stripe_chunks,
                                             int64_t nchunks, int x = blockIdx.x % kXcds,
                                             int64_t slot = blockIdx.x / kXcds) {
    const int k = (int)(slot % ntables);
    const int64_t j = slot / ntables;
    const uint32_t e = sm.entry[x][k];
    const int t = (int)(e & 0xff);
    const int64_t chunk = (int64_t)((e >> 8) & 0xff) * stripe_chunks + j;
    if (j >= stripe_chunks || chunk >= nchunks) return;
    if ((sm.prio_mask >> t) & 1u) __builtin_amdgcn_s_setprio(2);
#ifdef ET_FSPLIT
    // Feature-split tables (experiment build only, -DET_FSPLIT: measured slower, and the
    // slice loop's registers cost the default kernel 1.6% of the headline when compiled in)
    if constexpr (D == 128 && sizeof(T) == 4) {
        const uint32_t fg = e >> 16;
        if (fg != 0u) {  // a feature slice of a split table (build_stripe_map)
            if constexpr (SG) {
                // G = 2: 256-byte half rows through the scalar-addressed loop with 8-byte lanes
                // (round 4's 256-byte row loop, run_bags_s BPL = 8): the table and output
                // columns start fofs features on, the row stride is the table's
                if (sm.fsplit_g == 2) {
                    et_lookup_desc h = pack.d[t];
                    const int fofs = (int)(fg - 1u) * (D / 2);
                    h.table = reinterpret_cast<const T*>(h.table) + fofs;
                    h.dst_row_off += fofs;
                    run_bags_s<T, A, U, NT, false, 8>(h, batch, dst, ld_dst, chunk, rounds);
                    return;
                }
            }
            const int64_t per_round = SG ? 8 : 4 * VecGeom<T, D>::GPW;
            const int64_t b0 = chunk * per_round * rounds, b1 = b0 + per_round * rounds;
            const int fofs = (int)(fg - 1u) * (D / sm.fsplit_g);
            switch (sm.fsplit_g) {
                case 2: run_bags_slice<T, A, D / 2, NT>(pack.d[t], batch, dst, ld_dst, b0, b1, fofs); break;
                case 8: run_bags_slice<T, A, D / 8, NT>(pack.d[t], batch, dst, ld_dst, b0, b1, fofs); break;
                default: run_bags_slice<T, A, D / 4, NT>(pack.d[t], batch, dst, ld_dst, b0, b1, fofs); break;
            }
            return;
        }
    }
#endif
    if constexpr (SG) {
        if ((sm.ntload_mask >> t) & 1u)
            run_bags_s<T, A, U, NT, true, sg_bpl<T>(D), NA>(pack.d[t], batch, dst, ld_dst, chunk,
                                                             rounds);
        else
            run_bags_s<T, A, U, NT, false, sg_bpl<T>(D), NA>(pack.d[t], batch, dst, ld_dst, chunk,
                                                              rounds);
    } else {
        if ((sm.ntload_mask >> t) & 1u)
            run_bags<T, A, D, U, NT, true, NTI>(pack.d[t], batch, dst, ld_dst, chunk, rounds);
        else
            run_bags<T, A, D, U, NT, false, NTI>(pack.d[t], batch, dst, ld_dst, chunk, rounds);
    }
}

#ifdef ET_WG_TIMELINE
// Profiling build only (tools/wg_timeline.sh; never in the library the package loads):
// every workgroup of the striped launch records its start / end on the 100 MHz
// constant clock, its table, XCC and hardware slot, read back by et_debug_timeline.
constexpr uint32_t kTlCap = 1u << 17;
__device__ uint4 g_tl[kTlCap][2];
#endif

template <typename T, typename A, int D, int U, bool NT, bool NTI = false, bool SG = false>
__global__ __launch_bounds__(256) void k_pooled_vec_striped(LookupPack pack, StripeMap sm,
                                                            int ntables, int64_t batch,
                                                            T* __restrict__ dst, int64_t ld_dst,
                                                            int rounds, int64_t stripe_chunks,
                                                            int64_t nchunks) {
#ifdef ET_WG_TIMELINE
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#endif
    striped_body<T, A, D, U, NT, NTI, SG>(pack, sm, ntables, batch, dst, ld_dst, rounds,
                                          stripe_chunks, nchunks);
#ifdef ET_WG_TIMELINE
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < kTlCap) {
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        uint32_t xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        const int x = blockIdx.x % kXcds;
        const int64_t slot = blockIdx.x / kXcds;
        const int64_t j = slot / ntables;
        const uint32_t e = sm.entry[x][slot % ntables];
        const int64_t chunk = (int64_t)(e >> 8) * stripe_chunks + j;
        const uint32_t t = j >= stripe_chunks || chunk >= nchunks ? 0xffu : (e & 0xffu);
        g_tl[blockIdx.x][0] = make_uint4((uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)t1,
                                         (uint32_t)(t1 >> 32));
        g_tl[blockIdx.x][1] = make_uint4(t, xcc, hw, gridDim.x);
    }
#endif
}

// Per-XCD work queues: the same stripe map, but a workgroup takes its
// item from the queue of the XCD it actually runs on (one atomic head per XCD, items in the
// static schedule's order) and, once that queue is empty, from the other XCDs' queues, so an
// XCD whose stripes run faster (the static schedule's XCDs finished between 1184 and 1266 us,
// profiles/r03/b/wg_timeline.json) takes over the tail of the slower ones.  The grid has
// exactly as many workgroups as items, so every workgroup finds one.  The heads live in a
// queue block the CALLER owns (et_maplookup_prealloc_q, ET_LOOKUP_QUEUE_BYTES, zero before its
// first use) and the last workgroup to finish resets them, so the block is zero again when
// the launch completes: stream order makes the block safe for every later launch on the same
// stream (a HIP graph replay included), and a block is never shared by launches the library
// could not order (round 4 kept one block per (device, stream handle) in the library —
// a per-thread default stream, a re-created stream handle or another device's
// stream could share one).  Which workgroup sums which bags never changes a result:
// bit-identical to the static schedule.
struct XcdQueue {
    uint32_t head[kXcds];
    uint32_t done;
    uint32_t pad[32 - kXcds - 1];  // one 128-byte line
};
static_assert(sizeof(XcdQueue) == ET_LOOKUP_QUEUE_BYTES, "queue block size (include/embtab.h)");

template <typename T, typename A, int D, int U, bool NT, bool SG, int NA = 0>
__global__ __launch_bounds__(256) void k_pooled_vec_queued(LookupPack pack, StripeMap sm,
                                                           int ntables, int64_t batch,
                                                           T* __restrict__ dst, int64_t ld_dst,
                                                           int rounds, int64_t stripe_chunks,
                                                           int64_t nchunks) {
    __shared__ uint32_t s_item;
    XcdQueue& q = *pack.queue;
    const uint32_t per = (uint32_t)(ntables * stripe_chunks);  // items per XCD
    if (threadIdx.x == 0) {
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        uint32_t it = ~0u;
        for (uint32_t k = 0; k < (uint32_t)kXcds; ++k) {
            const uint32_t x = (xcc + k) & (uint32_t)(kXcds - 1);
            const uint32_t h = atomicAdd(&q.head[x], 1u);
            if (h < per) {
                it = x * per + h;
                break;
            }
        }
        s_item = it;
    }
    __syncthreads();
    const uint32_t it = s_item;
    if (it != ~0u) {
        int64_t slot = (int64_t)(it % per);
#ifdef ET_EXPERIMENTS
        if (sm.qorder == 1 && sm.nheavy > 0 && sm.nheavy < ntables) {
            // heavy-first: the queue's first nheavy * stripe_chunks items are the heavy
            // tables' chunks, then the light ones (slot = j * ntables + k, as the static order)
            const int64_t hn = (int64_t)sm.nheavy * stripe_chunks;
            const int nl = ntables - sm.nheavy;
            slot = slot < hn ? (slot / sm.nheavy) * ntables + slot % sm.nheavy
                             : ((slot - hn) / nl) * ntables + sm.nheavy + (slot - hn) % nl;
        } else if (sm.qorder == 2 && sm.nheavy > 0 && sm.nheavy < ntables) {  // light first
            const int nl = ntables - sm.nheavy;
            const int64_t ln = (int64_t)nl * stripe_chunks;
            slot = slot < ln ? (slot / nl) * ntables + sm.nheavy + slot % nl
                             : ((slot - ln) / sm.nheavy) * ntables + (slot - ln) % sm.nheavy;
        }
#endif
        striped_body<T, A, D, U, NT, false, SG, NA>(pack, sm, ntables, batch, dst, ld_dst, rounds,
                                                    stripe_chunks, nchunks, (int)(it / per), slot);
    }
    if (threadIdx.x == 0 && atomicAdd(&q.done, 1u) == gridDim.x - 1u) {  // the last one
        for (int x = 0; x < kXcds; ++x) atomicExch(&q.head[x], 0u);
        atomicExch(&q.done, 0u);
    }
}

#ifdef ET_EXPERIMENTS
// The same kernel held to 64 VGPRs (8 waves per SIMD instead of 7): ET_W8=1 experiment.
template <typename T, typename A, int D, int U, bool NT, bool NTI = false, bool SG = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void
k_pooled_vec_striped_w8(LookupPack pack, StripeMap sm, int ntables, int64_t batch,
                        T* __restrict__ dst, int64_t ld_dst, int rounds, int64_t stripe_chunks,
                        int64_t nchunks) {
    striped_body<T, A, D, U, NT, NTI, SG>(pack, sm, ntables, batch, dst, ld_dst, rounds,
                                          stripe_chunks, nchunks);
}
#endif

// Non-reducing gather (bit copy) of RB-byte rows: each group moves U rows at once.
template <int RB, bool NT>
__global__ __launch_bounds__(256) void k_gather_vec(LookupPack pack, int ntables, int64_t batch,
                                                    char* __restrict__ dst, int64_t ld_dst_b,
                                                    int es, int rounds) {
    constexpr int VPR = RB / 16;
    constexpr int LPR = VPR < 64 ? VPR : 64;
    constexpr int NV = VPR / LPR;
    constexpr int GPW = 64 / LPR;
    constexpr int U = NV >= 8 ? 1 : 8 / NV;
    static_assert(VPR <= 64 ? (64 % VPR == 0) : (VPR % 64 == 0), "unsupported row size");

    const int64_t item = blockIdx.x;
    const int t = (int)(item % ntables);
    const int64_t chunk = item / ntables;
    const et_lookup_desc& d = pack.d[t];
    const char* table = reinterpret_cast<const char*>(d.table);
    const int64_t ld_b = d.ld_table * es;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane / LPR, sub = lane % LPR;
    const int64_t per_round = 4 * GPW;
    const int64_t per_block = per_round * U * rounds;
    int64_t bag0 = chunk * per_block + wave * GPW + g;
    for (int r = 0; r < rounds; ++r, bag0 += per_round * U) {
        if (bag0 >= batch) break;
        uint64_t off[U];
        bool okv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int64_t bag = bag0 + u * per_round;
            bag = bag < batch ? bag : batch - 1;  // keep every lane active
            const uint64_t row = (uint64_t)(d.idx[bag * d.ld_idx] - 1);
            okv[u] = row < (uint64_t)d.nrows;
            off[u] = okv[u] ? row * (uint64_t)ld_b : 0;
        }
        u32x4 buf[U][NV];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u32x4* src = reinterpret_cast<const u32x4*>(table + off[u]) + sub;
#pragma unroll
            for (int v = 0; v < NV; ++v) buf[u][v] = src[v * LPR];
        }
        int bad = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t bag = bag0 + u * per_round;
            if (bag < batch) {
                bad += okv[u] ? 0 : 1;
                u32x4* o =
                    reinterpret_cast<u32x4*>(dst + bag * ld_dst_b + d.dst_row_off * es) + sub;
#pragma unroll
                for (int v = 0; v < NV; ++v)
                    store16<NT>(o + v * LPR, okv[u] ? buf[u][v] : u32x4{0u, 0u, 0u, 0u});
            }
        }
        if (bad && sub == 0) note_oob(bad);
    }
}

// Non-reducing gather (config 2, round 6): one round per workgroup of W waves, each lane group
// (RB / 16 lanes, one 16-byte vector each) holding its U rows in flight at once and storing each
// as it arrives (vector loads return in order, so the store of row u waits for rows 0..u only).
// U = 8, W = 4 — 1,024 workgroups at B = 65,536 — measured 14.32-14.40 us per graph-replayed
// launch against 15.25 for round 5's k_gather_pipe (two rounds of 8 in 512 workgroups), U = 16
// 15.6-15.8, U = 4 / W = 8 14.9, U = 6 / 12 15.6-15.9, W = 2 / 8 / 1 14.48-14.58 / 14.40-14.43 /
// 14.87 (profiles/r06/cfg2_variants.txt; ET_GATHER_ONE / ET_GATHER_W in experiment builds).
template <int RB, bool NT, bool NTL, int U, int W = 4>
__global__ __launch_bounds__(64 * W) void k_gather_one(LookupPack pack, int ntables, int64_t batch,
                                                       char* __restrict__ dst, int64_t ld_dst_b,
                                                       int es) {
#ifdef ET_WG_TIMELINE
    const uint64_t tl0 = __builtin_amdgcn_s_memrealtime();
#endif
    constexpr int VPR = RB / 16;
    static_assert(VPR <= 64 && 64 % VPR == 0, "one vector per lane");
    constexpr int GPW = 64 / VPR;
    const int64_t item = blockIdx.x;
    const int t = (int)(item % ntables);
    const int64_t chunk = item / ntables;
    const et_lookup_desc& d = pack.d[t];
    const char* table = reinterpret_cast<const char*>(d.table);
    const int64_t ld_b = d.ld_table * es;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane / VPR, sub = lane % VPR;
    const int64_t per_round = W * GPW;
    const int64_t bag0 = chunk * per_round * U + wave * GPW + g;
    int64_t iv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        int64_t b = bag0 + u * per_round;
        b = b < batch ? b : batch - 1;
        iv[u] = d.idx[b * d.ld_idx];
    }
    u32x4 cur[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t row = (uint64_t)(iv[u] - 1);
        ok[u] = row < (uint64_t)d.nrows;
        const u32x4* src = reinterpret_cast<const u32x4*>(table + (ok[u] ? row * (uint64_t)ld_b : 0)) + sub;
        if constexpr (NTL) cur[u] = __builtin_nontemporal_load(src);
        else cur[u] = *src;
    }
#ifdef ET_WG_TIMELINE
    asm volatile("" ::: "memory");
    const uint64_t tl1 = __builtin_amdgcn_s_memrealtime();  // indices in, rows issued
#endif
    int bad = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t bag = bag0 + u * per_round;
        if (bag < batch) {
            bad += ok[u] ? 0 : 1;
            u32x4* o = reinterpret_cast<u32x4*>(dst + bag * ld_dst_b + d.dst_row_off * es) + sub;
            store16<NT>(o, ok[u] ? cur[u] : u32x4{0u, 0u, 0u, 0u});
        }
    }
    if (bad && sub == 0) note_oob(bad);
#ifdef ET_WG_TIMELINE
    // Profiling build only (tools/gather_timeline.py): wave 0's start, the moment its row
    // loads are issued (its indices have arrived), and the workgroup's end with every store
    // complete, on the 100 MHz constant clock
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < kTlCap) {
        const uint64_t tl2 = __builtin_amdgcn_s_memrealtime();
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_tl[blockIdx.x][0] = make_uint4((uint32_t)tl0, (uint32_t)(tl0 >> 32), (uint32_t)tl1,
                                         (uint32_t)(tl1 >> 32));
        g_tl[blockIdx.x][1] = make_uint4((uint32_t)tl2, (uint32_t)(tl2 >> 32), xcc, gridDim.x);
    }
#endif
}

#ifdef ET_EXPERIMENTS
// Experiment (ET_GATHER_S=1, config 2): 512-byte rows with the indices read through the SCALAR
// cache — each wave's 16 contiguous bags' indices by scalar loads (vector indices, ld_idx = 1),
// so the index reads do not queue behind the row reads in the CU's vector memory path (the
// gather timeline shows wave 0's index loads returning after 1-8 us) — then k_gather_one's
// round: 8 rows per half-wave in flight, each stored as it arrives.
template <bool NT, bool NTL>
__global__ __launch_bounds__(256) void k_gather_s512(LookupPack pack, int ntables, int64_t batch,
                                                     char* __restrict__ dst, int64_t ld_dst_b,
                                                     int es) {
    const int64_t item = blockIdx.x;
    const int t = (int)(item % ntables);
    const int64_t chunk = item / ntables;
    const et_lookup_desc& d = pack.d[t];
    const char* table = reinterpret_cast<const char*>(d.table);
    const uint64_t ld_b = (uint64_t)(d.ld_table * es);
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int hi = lane >= 32 ? 1 : 0;
    const int sub = lane & 31;
    const int64_t base = chunk * 64 + wave * 16;
    if (base >= batch) return;  // wave-uniform
    const cidx_ptr ip = as_scalar_idx(d.idx + base);
    int64_t iv[16];
    if (base + 16 <= batch) {
#pragma unroll
        for (int k = 0; k < 16; ++k) iv[k] = ip[k];
    } else {
        const int64_t last = batch - 1 - base;
#pragma unroll
        for (int k = 0; k < 16; ++k) iv[k] = ip[k < last ? k : last];
    }
    u32x4 cur[8];
    bool ok[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const uint64_t row = (uint64_t)((hi ? iv[2 * u + 1] : iv[2 * u]) - 1);
        ok[u] = row < (uint64_t)d.nrows;
        const u32x4* src = reinterpret_cast<const u32x4*>(table + (ok[u] ? row * ld_b : 0)) + sub;
        if constexpr (NTL) cur[u] = __builtin_nontemporal_load(src);
        else cur[u] = *src;
    }
    int bad = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int64_t bag = base + 2 * u + hi;
        if (bag < batch) {
            bad += ok[u] ? 0 : 1;
            u32x4* o = reinterpret_cast<u32x4*>(dst + bag * ld_dst_b + d.dst_row_off * es) + sub;
            store16<NT>(o, ok[u] ? cur[u] : u32x4{0u, 0u, 0u, 0u});
        }
    }
    if (bad && sub == 0) note_oob(bad);
}
#endif

#ifdef ET_EXPERIMENTS
// The same gather, software-pipelined over `rounds` rounds per workgroup: round r + 1's rows
// are loaded before round r's are stored, and round r + 2's indices before those, so each
// wave keeps a round of rows in flight while it writes the previous one.  The one-round
// kernel loads every row of the launch, then stores them all: reads and writes never overlap
// (config 2: 18.5 us per kernel for 67.6 MB, compulsory traffic only by PMC; pipelined: 15.5,
// profiles/r05/cfg2/).  Vector memory counters retire in issue order, so the issue order is
// indices(r + 2), store(r), rows(r + 1): the store waits only for round r's rows, the row
// addresses of round r + 1 only for indices issued before them.  Rows of 16 * LPR bytes, one
// vector per lane (NV = 1).  Bit copies, so any schedule gives the same bytes.
template <int RB, bool NT, bool NTL = false>
__global__ __launch_bounds__(256) void k_gather_pipe(LookupPack pack, int ntables, int64_t batch,
                                                     char* __restrict__ dst, int64_t ld_dst_b,
                                                     int es, int rounds) {
    constexpr int VPR = RB / 16;
    static_assert(VPR <= 64 && 64 % VPR == 0, "one vector per lane");
    constexpr int LPR = VPR;
    constexpr int GPW = 64 / LPR;
    constexpr int U = 8;
    const int64_t item = blockIdx.x;
    const int t = (int)(item % ntables);
    const int64_t chunk = item / ntables;
    const et_lookup_desc& d = pack.d[t];
    const char* table = reinterpret_cast<const char*>(d.table);
    const int64_t ld_b = d.ld_table * es;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane / LPR, sub = lane % LPR;
    const int64_t per_round = 4 * GPW;
    const int64_t step = per_round * U;  // bags per round
    const int64_t bag_base = chunk * step * rounds + wave * GPW + g;
    auto bag_of = [&](int r, int u) { return bag_base + r * step + u * per_round; };
    auto idx_of = [&](int r, int u) {
        int64_t b = bag_of(r, u);
        b = b < batch ? b : batch - 1;  // keep every lane active
        return d.idx[b * d.ld_idx];
    };
    int64_t iv[U];    // indices of round r + 1 (then r + 2)
    u32x4 cur[U];     // rows of round r
    bool okc[U];
    int bad = 0;
    // prologue: round 0's indices and rows, round 1's indices
#pragma unroll
    for (int u = 0; u < U; ++u) iv[u] = idx_of(0, u);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t row = (uint64_t)(iv[u] - 1);
        okc[u] = row < (uint64_t)d.nrows;
        const u32x4* src = reinterpret_cast<const u32x4*>(table + (okc[u] ? row * (uint64_t)ld_b : 0)) + sub;
        if constexpr (NTL) cur[u] = __builtin_nontemporal_load(src);
        else cur[u] = *src;
    }
    if (rounds > 1)
#pragma unroll
        for (int u = 0; u < U; ++u) iv[u] = idx_of(1, u);
    for (int r = 0; r < rounds; ++r) {
        if (bag_of(r, 0) >= batch) break;  // uniform per group: later rounds are past too
        int64_t nx[U];
        if (r + 2 < rounds)
#pragma unroll
            for (int u = 0; u < U; ++u) nx[u] = idx_of(r + 2, u);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t bag = bag_of(r, u);
            if (bag < batch) {
                bad += okc[u] ? 0 : 1;
                u32x4* o = reinterpret_cast<u32x4*>(dst + bag * ld_dst_b + d.dst_row_off * es) + sub;
                store16<NT>(o, okc[u] ? cur[u] : u32x4{0u, 0u, 0u, 0u});
            }
        }
        if (r + 1 < rounds) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t row = (uint64_t)(iv[u] - 1);
                okc[u] = row < (uint64_t)d.nrows;
                const u32x4* src =
                    reinterpret_cast<const u32x4*>(table + (okc[u] ? row * (uint64_t)ld_b : 0)) + sub;
                if constexpr (NTL) cur[u] = __builtin_nontemporal_load(src);
                else cur[u] = *src;
            }
        }
        if (r + 2 < rounds)
#pragma unroll
            for (int u = 0; u < U; ++u) iv[u] = nx[u];
    }
    if (bad && sub == 0) note_oob(bad);
}
#endif  // ET_EXPERIMENTS: round 5's two-round gather (ET_GATHER_PIPE=2..)


// Generic path: any feature size / alignment / per-table dims / paged tables.  One wave
// per bag, lanes stride over the features, pool order sequential per feature.
// Store conversion T -> O; bfloat16 converts through float (exact for 16-bit types).
template <typename O, typename T>
__device__ __forceinline__ O convert_elt(T x) {
    if constexpr ((__is_same(T, __bf16) || __is_same(O, __bf16)) && !__is_same(T, float) &&
                  !__is_same(O, float))
        return O((float)x);
    else
        return O(x);
}

// O: the destination element type (PreallocationStrategy{U}, src/lookup.jl:284-315: the
// sum is formed in the table's type T, then converted to U on the store).
template <typename T, typename A, bool NT, typename O = T>
__global__ __launch_bounds__(256) void k_pooled_generic(LookupPack pack, int ntables,
                                                        int64_t batch, O* __restrict__ dst,
                                                        int64_t ld_dst) {
    constexpr int K = 4;
    const int64_t item = blockIdx.x;
    const int t = (int)(item % ntables);
    const int64_t chunk = item / ntables;
    const et_lookup_desc& d = pack.d[t];
    const T* table = reinterpret_cast<const T*>(d.table);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t bag = chunk * 4 + wave;
    if (bag >= batch) return;
    const int64_t* ip = d.idx + bag * d.ld_idx;
    O* out = dst + bag * ld_dst + d.dst_row_off;
    const int dim = d.dim, pool = d.pool;
    for (int f0 = 0; f0 < dim; f0 += 64 * K) {
        A acc[K];
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = A(0);
        for (int i = 0; i < pool; ++i) {
            uint64_t row = (uint64_t)(ip[i] - 1);
            const bool ok = row < (uint64_t)d.nrows;
            if (!ok && lane == 0 && f0 == 0) note_oob();
            row = ok ? row : 0;
            const T* src = col_ptr<const T>(d.table, d.ld_table, d.cols_per_page, row);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int f = f0 + lane + 64 * k;
                if (f < dim) {
                    const T x = ok ? src[f] : T(0);
                    acc[k] = i == 0 ? A(x) : A(acc[k] + A(x));
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int f = f0 + lane + 64 * k;
            if (f < dim) store_scalar<NT>(out + f, convert_elt<O>(T(acc[k])));
        }
    }
}

// ---------------------------------------------------------------------------
// Host dispatch
// ---------------------------------------------------------------------------

inline bool gather_rb_ok(int64_t rb) {
    return rb == 32 || rb == 64 || rb == 128 || rb == 256 || rb == 512 || rb == 1024 ||
           rb == 2048 || rb == 4096;
}

// Bags per workgroup round for the vector path.
int max_rounds();

inline int rounds_for(int64_t batch, int64_t bags_per_round, int ntables) {
    // Aim for >= ~8 workgroups per CU (2048) before making workgroups longer.
    int64_t blocks1 = (batch + bags_per_round - 1) / bags_per_round * ntables;
    int rounds = 1;
    const int mr = max_rounds();
    while (rounds < mr && blocks1 / (rounds * 2) >= 4096) rounds *= 2;
    return rounds;
}

// Scheduling knobs: the defaults are the tuned choice; an experiment build (-DET_EXPERIMENTS)
// reads them from the environment once (et_common.h, ET_KNOB).  Every setting is bit-identical.
struct LookupTuning {
    int striped = 1;               // ET_SCHED=linear disables the XCD stripe schedule
    // per-XCD work queues (k_pooled_vec_queued) wherever the caller passes a queue block:
    // headline 1.261-1.262 vs 1.270-1.271 ms for the static stripe schedule (A/B twice on one
    // box, round 4, profiles/r04/queue_ab.txt); ET_SCHED=stripe keeps the static schedule
    int queued = 1;
    // Tables larger than the 256 MiB Infinity Cache cannot stay cache resident: their
    // rows are loaded non-temporally so they do not evict the light tables from L2
    // (measured -5% on the Criteo mix; nt on the cache-resident mid-size tables hurts).
    int ntload = 1;                          // ET_NTLOAD=0 disables
    int64_t ntload_bytes = 256ll << 20;      // ET_NTLOAD_BYTES
    int ntidx = 0;                           // ET_NTIDX=1: non-temporal index loads
    int max_rounds = 8;                      // ET_ROUNDS: max bag rounds per workgroup
    int64_t light_bytes = 4 << 20; // tables up to one XCD L2 (4 MiB) are "light"
    int rows_in_flight = 0;        // ET_U=4|8|16: rows per group in flight (fp32 D=128)
    int w8 = 0;                    // ET_W8=1: the striped kernel held to 8 waves per SIMD
    int sgpr = 1;                  // ET_SGPR=0: 512-byte rows use the per-lane loop too
    int sg256 = 0;                 // ET_SG256=1: 256-byte rows take the scalar loop too
    int heavy_prio = 0;            // ET_HEAVY_PRIO=1: heavy tables' waves at priority 2
    int qorder = 0;                // ET_QORDER=1: queued schedule, heavy items first
    int noadd = 0;                 // ET_HEAD_NOADD=1: the scalar loop without its adds
    // Tables of (light_bytes, fsplit_bytes] cut into fsplit_g feature groups, group g on XCDs
    // [g * 8 / G, (g + 1) * 8 / G), so each XCD's L2 holds 1/G of the table (ET_FSPLIT_*)
    int64_t fsplit_bytes = 0;
    int fsplit_g = 4;
};

inline const LookupTuning& tuning() {
    static LookupTuning t = [] {
        LookupTuning v;
#ifdef ET_EXPERIMENTS
        if (const char* e = getenv("ET_SCHED")) {
            v.striped = strcmp(e, "linear") != 0;
            v.queued = v.striped && strcmp(e, "stripe") != 0;
        }
        v.ntload = (int)ET_KNOB("ET_NTLOAD", v.ntload);
        v.ntload_bytes = ET_KNOB("ET_NTLOAD_BYTES", v.ntload_bytes);
        v.ntidx = (int)ET_KNOB("ET_NTIDX", v.ntidx);
        v.max_rounds = (int)ET_KNOB("ET_ROUNDS", v.max_rounds);
        if (v.max_rounds < 1) v.max_rounds = 1;
        v.light_bytes = ET_KNOB("ET_LIGHT_BYTES", v.light_bytes);
        v.rows_in_flight = (int)ET_KNOB("ET_U", v.rows_in_flight);
        v.w8 = (int)ET_KNOB("ET_W8", v.w8);
        v.noadd = (int)ET_KNOB("ET_HEAD_NOADD", v.noadd);
        v.sgpr = (int)ET_KNOB("ET_SGPR", v.sgpr);
        v.sg256 = (int)ET_KNOB("ET_SG256", v.sg256);
        v.heavy_prio = (int)ET_KNOB("ET_HEAVY_PRIO", v.heavy_prio);
        v.qorder = (int)ET_KNOB("ET_QORDER", v.qorder);
        v.fsplit_bytes = ET_KNOB("ET_FSPLIT_BYTES", v.fsplit_bytes);
        const int g = (int)ET_KNOB("ET_FSPLIT_G", 4);
        v.fsplit_g = g == 2 || g == 8 ? g : 4;
#endif
        return v;
    }();
    return t;
}

int max_rounds() { return tuning().max_rounds; }

// Stripe assignment: heavy tables -> stripe x on XCD x; light tables' stripes laid out
// table after table (alternating large and small tables) and cut into kXcds equal runs.
inline void build_stripe_map(const LookupPack& pack, int n, int es, StripeMap& sm,
                             bool can_split = false) {
    const LookupTuning& tu = tuning();
    int heavy[ET_MAX_TABLES_PER_LAUNCH], light[ET_MAX_TABLES_PER_LAUNCH];
    int split[ET_MAX_TABLES_PER_LAUNCH];
    int nh = 0, nl = 0, nsp = 0;
    int64_t bytes[ET_MAX_TABLES_PER_LAUNCH];
    sm.ntload_mask = 0;
    sm.prio_mask = 0;
    sm.qorder = tu.qorder;
    sm.fsplit_g = tu.fsplit_g;
    for (int t = 0; t < n; ++t) {
        bytes[t] = pack.d[t].nrows * pack.d[t].ld_table * es;
#ifndef ET_FSPLIT
        can_split = false;  // the slice loop is not compiled in (striped_body)
#endif
        if (can_split && bytes[t] > tu.light_bytes && bytes[t] <= tu.fsplit_bytes &&
            pack.d[t].cols_per_page == 0 && pack.d[t].dim == 128 &&
            n + (nsp + 1) * (tu.fsplit_g - 1) <= kMaxStripeEntries) {
            split[nsp++] = t;
        } else if (bytes[t] > tu.light_bytes) {
            heavy[nh++] = t;
            if (tu.heavy_prio) sm.prio_mask |= 1u << t;
            if (tu.ntload && bytes[t] > tu.ntload_bytes) sm.ntload_mask |= 1u << t;
        } else {
            light[nl++] = t;
        }
    }
    // light tables by size, then interleave large / small
    for (int a = 0; a < nl; ++a)
        for (int b = a + 1; b < nl; ++b)
            if (bytes[light[b]] > bytes[light[a]]) {
                int tmp = light[a];
                light[a] = light[b];
                light[b] = tmp;
            }
    int order[ET_MAX_TABLES_PER_LAUNCH];
    for (int i = 0, lo = 0, hi = nl - 1; i < nl; ++i) order[i] = (i & 1) ? light[hi--] : light[lo++];
    int cnt[kXcds] = {0};
    for (int x = 0; x < kXcds; ++x)
        for (int h = 0; h < nh; ++h) sm.entry[x][cnt[x]++] = (uint32_t)heavy[h] | ((uint32_t)x << 8);
    // split tables: XCD x serves feature group g = x / P (P = 8 / G XCDs per group) over the
    // stripes G * (x % P) .. G * (x % P) + G - 1, so every group covers all 8 stripes
    const int G = sm.fsplit_g, P = kXcds / G;
    for (int x = 0; x < kXcds; ++x)
        for (int q = 0; q < nsp; ++q)
            for (int m = 0; m < G; ++m)
                sm.entry[x][cnt[x]++] = (uint32_t)split[q] |
                                        ((uint32_t)(G * (x % P) + m) << 8) |
                                        ((uint32_t)(x / P + 1) << 16);
    sm.nheavy = nh + nsp * G;
    // linear list of light stripes (order[i], st), st < kXcds; XCD x takes [x*nl, (x+1)*nl)
    for (int q = 0; q < nl * kXcds; ++q) {
        const int x = q / (nl > 0 ? nl : 1);
        sm.entry[x][cnt[x]++] = (uint32_t)order[q / kXcds] | ((uint32_t)(q % kXcds) << 8);
    }
    sm.nent = cnt[0];
}

template <typename T, typename A, int D, int U, bool NT, bool PG = false, bool MK = false>
int launch_pooled_vec_u(const LookupPack& pack, int n, int64_t batch, void* dst, int64_t ld_dst,
                        hipStream_t s);

template <typename T, typename A, int D, bool NT, bool PG = false>
int launch_pooled_vec(const LookupPack& pack, int n, int64_t batch, void* dst, int64_t ld_dst,
                      hipStream_t s) {
    if constexpr (PG)  // paged tables: one schedule, the default rows in flight
        return launch_pooled_vec_u<T, A, D, VecGeom<T, D>::U, NT, true>(pack, n, batch, dst,
                                                                         ld_dst, s);
#ifdef ET_EXPERIMENTS
    if constexpr (D == 128 && __is_same(T, float)) {
        switch (tuning().rows_in_flight) {
            case 4: return launch_pooled_vec_u<T, A, D, 4, NT>(pack, n, batch, dst, ld_dst, s);
            case 16: return launch_pooled_vec_u<T, A, D, 16, NT>(pack, n, batch, dst, ld_dst, s);
            default: break;
        }
    }
#endif
    return launch_pooled_vec_u<T, A, D, VecGeom<T, D>::U, NT>(pack, n, batch, dst, ld_dst, s);
}

template <typename T, typename A, int D, int U, bool NT, bool PG, bool MK>
int launch_pooled_vec_u(const LookupPack& pack, int n, int64_t batch, void* dst, int64_t ld_dst,
                        hipStream_t s) {
    using G = VecGeom<T, D>;
    // the scalar-addressed loop: 512-byte rows, and 256-byte rows with 8-byte lanes (ET_SG256)
    constexpr bool kSG = !PG && !MK && (D * (int)sizeof(T) == 512 || D * (int)sizeof(T) == 256);
    bool sg = kSG && tuning().sgpr &&
              (D * (int)sizeof(T) == 512 || tuning().sg256);  // row strides must fit 32 bits
    for (int t = 0; t < n && sg; ++t) sg = pack.d[t].ld_table * (int64_t)sizeof(T) < (1ll << 32);
    const int64_t per_round = sg ? 8 : 4 * G::GPW;  // the scalar loop: two bags per wave
    const int rounds = rounds_for(batch, per_round, n);
    const int64_t nchunks = (batch + per_round * rounds - 1) / (per_round * rounds);
    if (nchunks <= 0) return ET_OK;
    if (!PG && !MK && n > 1 && tuning().striped) {
        StripeMap sm;
        build_stripe_map(pack, n, (int)sizeof(T), sm, D == 128 && sizeof(T) == 4);
        const int ne = sm.nent;  // entries per XCD (n, plus fsplit_g - 1 per split table)
        const int64_t stripe_chunks = (nchunks + kXcds - 1) / kXcds;
        const int64_t grid = (int64_t)kXcds * ne * stripe_chunks;
        if (grid > 0x7fffffffll) return fail(ET_ERR_ARG, "grid too large");
        if (pack.queue && tuning().queued && grid < 0xffffffffll) {
            if constexpr (kSG) {
#ifdef ET_EXPERIMENTS
                if (sg && tuning().noadd) {  // ET_HEAD_NOADD: the adds-free ceiling variant
                    hipLaunchKernelGGL((k_pooled_vec_queued<T, A, D, U, NT, true, 1>),
                                       dim3((unsigned)grid), dim3(256), 0, s, pack, sm, ne, batch,
                                       reinterpret_cast<T*>(dst), ld_dst, rounds, stripe_chunks,
                                       nchunks);
                    ET_LAUNCH_CHECK("k_pooled_vec_queued<noadd>");
                    return ET_OK;
                }
#endif
                if (sg) {
                    hipLaunchKernelGGL((k_pooled_vec_queued<T, A, D, U, NT, true>),
                                       dim3((unsigned)grid), dim3(256), 0, s, pack, sm, ne, batch,
                                       reinterpret_cast<T*>(dst), ld_dst, rounds, stripe_chunks,
                                       nchunks);
                    ET_LAUNCH_CHECK("k_pooled_vec_queued");
                    return ET_OK;
                }
            }
            hipLaunchKernelGGL((k_pooled_vec_queued<T, A, D, U, NT, false>), dim3((unsigned)grid),
                               dim3(256), 0, s, pack, sm, ne, batch, reinterpret_cast<T*>(dst),
                               ld_dst, rounds, stripe_chunks, nchunks);
            ET_LAUNCH_CHECK("k_pooled_vec_queued");
            return ET_OK;
        }
#ifdef ET_EXPERIMENTS
        if constexpr (kSG) {
            if (sg && tuning().w8) {
                hipLaunchKernelGGL((k_pooled_vec_striped_w8<T, A, D, U, NT, false, true>),
                                   dim3((unsigned)grid), dim3(256), 0, s, pack, sm, ne, batch,
                                   reinterpret_cast<T*>(dst), ld_dst, rounds, stripe_chunks,
                                   nchunks);
                ET_LAUNCH_CHECK("k_pooled_vec_striped");
                return ET_OK;
            }
        }
#endif
        if constexpr (kSG) {
            if (sg) {
                hipLaunchKernelGGL((k_pooled_vec_striped<T, A, D, U, NT, false, true>),
                                   dim3((unsigned)grid), dim3(256), 0, s, pack, sm, ne, batch,
                                   reinterpret_cast<T*>(dst), ld_dst, rounds, stripe_chunks,
                                   nchunks);
                ET_LAUNCH_CHECK("k_pooled_vec_striped");
                return ET_OK;
            }
        }
#ifdef ET_EXPERIMENTS
        if (tuning().w8 && D == 128 && __is_same(T, float))
            hipLaunchKernelGGL((k_pooled_vec_striped_w8<T, A, D, U, NT>), dim3((unsigned)grid),
                               dim3(256), 0, s, pack, sm, ne, batch, reinterpret_cast<T*>(dst),
                               ld_dst, rounds, stripe_chunks, nchunks);
        else if (tuning().ntidx && D == 128 && __is_same(T, float))
            hipLaunchKernelGGL((k_pooled_vec_striped<T, A, D, U, NT, true>), dim3((unsigned)grid),
                               dim3(256), 0, s, pack, sm, ne, batch, reinterpret_cast<T*>(dst),
                               ld_dst, rounds, stripe_chunks, nchunks);
        else
#endif
            hipLaunchKernelGGL((k_pooled_vec_striped<T, A, D, U, NT>), dim3((unsigned)grid),
                               dim3(256), 0, s, pack, sm, ne, batch, reinterpret_cast<T*>(dst),
                               ld_dst, rounds, stripe_chunks, nchunks);
        ET_LAUNCH_CHECK("k_pooled_vec_striped");
        return ET_OK;
    }
    const int64_t grid = nchunks * n;
    if (grid <= 0) return ET_OK;
    if (grid > 0x7fffffffll) return fail(ET_ERR_ARG, "grid too large");
    if constexpr (kSG) {
        if (sg) {
            hipLaunchKernelGGL((k_pooled_vec<T, A, D, U, NT, false, false, true>),
                               dim3((unsigned)grid), dim3(256), 0, s, pack, n, batch,
                               reinterpret_cast<T*>(dst), ld_dst, rounds);
            ET_LAUNCH_CHECK("k_pooled_vec");
            return ET_OK;
        }
    }
    hipLaunchKernelGGL((k_pooled_vec<T, A, D, U, NT, PG, MK>), dim3((unsigned)grid), dim3(256), 0, s,
                       pack, n, batch, reinterpret_cast<T*>(dst), ld_dst, rounds);
    ET_LAUNCH_CHECK("k_pooled_vec");
    return ET_OK;
}

template <int RB, bool NT>
int launch_gather_rb(const LookupPack& pack, int n, int64_t batch, void* dst, int64_t ld_dst,
                     int es, hipStream_t s) {
    constexpr int VPR = RB / 16;
    constexpr int LPR = VPR < 64 ? VPR : 64;
    constexpr int NV = VPR / LPR;
    constexpr int U = NV >= 8 ? 1 : 8 / NV;
    const int64_t per_round = 4 * (64 / LPR) * U;
    if constexpr (NV == 1 && U == 8) {
        // rows of tables larger than the Infinity Cache load non-temporally, as the pooled
        // kernels' (ntload_bytes): config 2 15.26-15.29 vs 15.99-16.04 us per launch in round 5
        // (profiles/r05/cfg2/ab_gather_pipe.txt)
        bool ntl = tuning().ntload != 0;
        for (int t = 0; t < n && ntl; ++t)
            ntl = pack.d[t].nrows * pack.d[t].ld_table * es > tuning().ntload_bytes;
        bool one = true;
#ifdef ET_EXPERIMENTS
        // ET_GATHER_PIPE=R (R >= 2): round 5's k_gather_pipe over R rounds; 1: k_gather_vec
        const int pr = (int)ET_KNOB("ET_GATHER_PIPE", 0);
        one = pr == 0;
        const int64_t g = pr > 1 ? (batch + per_round * pr - 1) / (per_round * pr) * n : 0;
        if (pr > 1 && g >= 1) {
            if (g > 0x7fffffffll) return fail(ET_ERR_ARG, "grid too large");
            if (ntl)
                hipLaunchKernelGGL((k_gather_pipe<RB, NT, true>), dim3((unsigned)g), dim3(256), 0,
                                   s, pack, n, batch, reinterpret_cast<char*>(dst), ld_dst * es,
                                   es, pr);
            else
                hipLaunchKernelGGL((k_gather_pipe<RB, NT>), dim3((unsigned)g), dim3(256), 0, s,
                                   pack, n, batch, reinterpret_cast<char*>(dst), ld_dst * es, es,
                                   pr);
            ET_LAUNCH_CHECK("k_gather_pipe");
            return ET_OK;
        }
        if constexpr (RB == 512) {
            bool contig = ET_KNOB("ET_GATHER_S", 0) != 0;
            for (int t = 0; t < n && contig; ++t) contig = pack.d[t].ld_idx == 1;
            if (contig) {
                const int64_t gs = (batch + 63) / 64 * n;
                if (ntl)
                    hipLaunchKernelGGL((k_gather_s512<NT, true>), dim3((unsigned)gs), dim3(256), 0,
                                       s, pack, n, batch, reinterpret_cast<char*>(dst),
                                       ld_dst * es, es);
                else
                    hipLaunchKernelGGL((k_gather_s512<NT, false>), dim3((unsigned)gs), dim3(256),
                                       0, s, pack, n, batch, reinterpret_cast<char*>(dst),
                                       ld_dst * es, es);
                ET_LAUNCH_CHECK("k_gather_s512");
                return ET_OK;
            }
        }
        if (const int uo = (int)ET_KNOB("ET_GATHER_ONE", 0)) {  // U / W variants of k_gather_one
            const int w = (int)ET_KNOB("ET_GATHER_W", 4);
            const int64_t pw = w * (64 / LPR) * uo;
            const int64_t g1 = (batch + pw - 1) / pw * n;
            if (g1 > 0x7fffffffll) return fail(ET_ERR_ARG, "grid too large");
#define ET_G1(UU, WW)                                                                            \
    if (uo == UU && w == WW) {                                                                   \
        if (ntl)                                                                                 \
            hipLaunchKernelGGL((k_gather_one<RB, NT, true, UU, WW>), dim3((unsigned)g1),        \
                               dim3(64 * WW), 0, s, pack, n, batch,                              \
                               reinterpret_cast<char*>(dst), ld_dst * es, es);                   \
        else                                                                                     \
            hipLaunchKernelGGL((k_gather_one<RB, NT, false, UU, WW>), dim3((unsigned)g1),       \
                               dim3(64 * WW), 0, s, pack, n, batch,                              \
                               reinterpret_cast<char*>(dst), ld_dst * es, es);                   \
        ET_LAUNCH_CHECK("k_gather_one");                                                         \
        return ET_OK;                                                                            \
    }
            ET_G1(4, 4) ET_G1(16, 4) ET_G1(32, 4) ET_G1(6, 4) ET_G1(12, 4)
            ET_G1(8, 2) ET_G1(8, 8) ET_G1(8, 1) ET_G1(16, 2) ET_G1(4, 8)
#undef ET_G1
        }
#endif
        if (one) {  // the default: one round of 8 rows per lane group, 4 waves per workgroup
            constexpr int kU = 8, kW = 4;
            const int64_t pw = kW * (64 / LPR) * kU;
            const int64_t g1 = (batch + pw - 1) / pw * n;
            if (g1 <= 0) return ET_OK;
            if (g1 > 0x7fffffffll) return fail(ET_ERR_ARG, "grid too large");
            if (ntl)
                hipLaunchKernelGGL((k_gather_one<RB, NT, true, kU, kW>), dim3((unsigned)g1),
                                   dim3(64 * kW), 0, s, pack, n, batch,
                                   reinterpret_cast<char*>(dst), ld_dst * es, es);
            else
                hipLaunchKernelGGL((k_gather_one<RB, NT, false, kU, kW>), dim3((unsigned)g1),
                                   dim3(64 * kW), 0, s, pack, n, batch,
                                   reinterpret_cast<char*>(dst), ld_dst * es, es);
            ET_LAUNCH_CHECK("k_gather_one");
            return ET_OK;
        }
    }
    const int rounds = rounds_for(batch, per_round, n);
    const int64_t nchunks = (batch + per_round * rounds - 1) / (per_round * rounds);
    const int64_t grid = nchunks * n;
    if (grid <= 0) return ET_OK;
    if (grid > 0x7fffffffll) return fail(ET_ERR_ARG, "grid too large");
    hipLaunchKernelGGL((k_gather_vec<RB, NT>), dim3((unsigned)grid), dim3(256), 0, s, pack, n,
                       batch, reinterpret_cast<char*>(dst), ld_dst * es, es, rounds);
    ET_LAUNCH_CHECK("k_gather_vec");
    return ET_OK;
}

template <bool NT>
int launch_gather(const LookupPack& pack, int n, int64_t rb, int64_t batch, void* dst,
                  int64_t ld_dst, int es, hipStream_t s) {
    switch (rb) {
        case 32: return launch_gather_rb<32, NT>(pack, n, batch, dst, ld_dst, es, s);
        case 64: return launch_gather_rb<64, NT>(pack, n, batch, dst, ld_dst, es, s);
        case 128: return launch_gather_rb<128, NT>(pack, n, batch, dst, ld_dst, es, s);
        case 256: return launch_gather_rb<256, NT>(pack, n, batch, dst, ld_dst, es, s);
        case 512: return launch_gather_rb<512, NT>(pack, n, batch, dst, ld_dst, es, s);
        case 1024: return launch_gather_rb<1024, NT>(pack, n, batch, dst, ld_dst, es, s);
        case 2048: return launch_gather_rb<2048, NT>(pack, n, batch, dst, ld_dst, es, s);
        case 4096: return launch_gather_rb<4096, NT>(pack, n, batch, dst, ld_dst, es, s);
    }
    return fail(ET_ERR_UNSUPPORTED, "gather row bytes %lld", (long long)rb);
}

template <typename T, typename A, bool NT, bool PG = false>
int launch_pooled_dim(const LookupPack& pack, int n, int D, int64_t batch, void* dst,
                      int64_t ld_dst, hipStream_t s) {
    switch (D) {
        case 16: return launch_pooled_vec<T, A, 16, NT, PG>(pack, n, batch, dst, ld_dst, s);
        case 32: return launch_pooled_vec<T, A, 32, NT, PG>(pack, n, batch, dst, ld_dst, s);
        case 64: return launch_pooled_vec<T, A, 64, NT, PG>(pack, n, batch, dst, ld_dst, s);
        case 128: return launch_pooled_vec<T, A, 128, NT, PG>(pack, n, batch, dst, ld_dst, s);
        case 256: return launch_pooled_vec<T, A, 256, NT, PG>(pack, n, batch, dst, ld_dst, s);
        case 512: return launch_pooled_vec<T, A, 512, NT, PG>(pack, n, batch, dst, ld_dst, s);
    }
    return fail(ET_ERR_UNSUPPORTED, "vector dim %d", D);
}

template <typename T, typename A, bool NT>
int launch_pooled_masked(const LookupPack& pack, int n, int D, int64_t batch, void* dst,
                         int64_t ld_dst, hipStream_t s) {
#define ET_MK(C)                                                                              \
    case C:                                                                                   \
        if constexpr (C / (16 / (int)sizeof(T)) >= 1)                                         \
            return launch_pooled_vec_u<T, A, C, VecGeom<T, C>::U, NT, false, true>(           \
                pack, n, batch, dst, ld_dst, s);                                              \
        break;
    switch (masked_capacity(D)) {
        ET_MK(16)
        ET_MK(32)
        ET_MK(64)
        ET_MK(128)
        ET_MK(256)
        ET_MK(512)
        ET_MK(1024)
        ET_MK(2048)
    }
#undef ET_MK
    return fail(ET_ERR_UNSUPPORTED, "masked vector dim %d", D);
}

template <typename T, typename A, bool NT>
int launch_generic(const LookupPack& pack, int n, int64_t batch, void* dst, int64_t ld_dst,
                   hipStream_t s) {
    const int64_t grid = (batch + 3) / 4 * n;
    if (grid <= 0) return ET_OK;
    if (grid > 0x7fffffffll) return fail(ET_ERR_ARG, "grid too large");
    hipLaunchKernelGGL((k_pooled_generic<T, A, NT>), dim3((unsigned)grid), dim3(256), 0, s, pack,
                       n, batch, reinterpret_cast<T*>(dst), ld_dst);
    ET_LAUNCH_CHECK("k_pooled_generic");
    return ET_OK;
}

// Kinds of launch group.
enum GroupKind { kGather = 0, kPooledVec = 1, kGeneric = 2, kPagedVec = 3, kMaskedVec = 4 };

template <typename T, typename A, bool NT>
int launch_group_typed(GroupKind kind, const LookupPack& pack, int n, int D, int64_t batch,
                       void* dst, int64_t ld_dst, hipStream_t s) {
    const int es = (int)sizeof(T);
    if (kind == kGather)
        return launch_gather<NT>(pack, n, (int64_t)D * es, batch, dst, ld_dst, es, s);
    if (kind == kPooledVec) return launch_pooled_dim<T, A, NT>(pack, n, D, batch, dst, ld_dst, s);
    if (kind == kPagedVec)
        return launch_pooled_dim<T, A, NT, true>(pack, n, D, batch, dst, ld_dst, s);
    if (kind == kMaskedVec)
        return launch_pooled_masked<T, A, NT>(pack, n, D, batch, dst, ld_dst, s);
    return launch_generic<T, A, NT>(pack, n, batch, dst, ld_dst, s);
}

template <bool NT>
int launch_group(int dtype, bool f32acc, GroupKind kind, const LookupPack& pack, int n, int D,
                 int64_t batch, void* dst, int64_t ld_dst, hipStream_t s) {
    switch (dtype) {
        case ET_F32:
            return launch_group_typed<float, float, NT>(kind, pack, n, D, batch, dst, ld_dst, s);
        case ET_F64:
            return launch_group_typed<double, double, NT>(kind, pack, n, D, batch, dst, ld_dst, s);
        case ET_I32:
            return launch_group_typed<int32_t, uint32_t, NT>(kind, pack, n, D, batch, dst, ld_dst,
                                                            s);
        case ET_I64:
            return launch_group_typed<int64_t, uint64_t, NT>(kind, pack, n, D, batch, dst, ld_dst,
                                                            s);
        case ET_BF16:  // always fp32 accumulation, one RNE rounding per output element
            return launch_group_typed<__bf16, float, NT>(kind, pack, n, D, batch, dst, ld_dst,
                                                         s);
        case ET_F16:
            if (f32acc)
                return launch_group_typed<_Float16, float, NT>(kind, pack, n, D, batch, dst,
                                                               ld_dst, s);
            return launch_group_typed<_Float16, _Float16, NT>(kind, pack, n, D, batch, dst, ld_dst,
                                                              s);
    }
    return fail(ET_ERR_UNSUPPORTED, "dtype %d", dtype);
}

// Validate descriptors, partition them into launch groups and launch.
// force_gather: every table is a vector (pool == 1) lookup => bit-copy path.
// Descriptor checks shared by the dispatchers (1 = nothing to do).
int validate_lookup(const et_lookup_desc* descs, int ntables, int64_t batch, const void* dst,
                    int64_t ld_dst) {
    if (ntables < 0 || batch < 0) return fail(ET_ERR_ARG, "negative ntables/batch");
    if (ntables == 0 || batch == 0) return 1;
    if (!descs) return fail(ET_ERR_ARG, "descs is NULL");
    if (!dst) return fail(ET_ERR_ARG, "dst is NULL");
    for (int t = 0; t < ntables; ++t) {
        const et_lookup_desc& d = descs[t];
        if (d.dim < 0 || d.pool < 0 || d.nrows < 0 || d.cols_per_page < 0)
            return fail(ET_ERR_ARG, "table %d: negative dim/pool/nrows/cols_per_page", t);
        if (d.dim == 0) continue;
        if (d.ld_table < d.dim) return fail(ET_ERR_ARG, "table %d: ld_table < dim", t);
        if (d.dst_row_off < 0 || d.dst_row_off + d.dim > ld_dst)
            return fail(ET_ERR_ARG, "table %d: rows [%lld, %lld) outside ld_dst %lld", t,
                        (long long)d.dst_row_off, (long long)(d.dst_row_off + d.dim),
                        (long long)ld_dst);
        if (d.pool > 0) {
            if (!d.table || !d.idx) return fail(ET_ERR_ARG, "table %d: NULL table/idx", t);
            if (d.nrows == 0)
                return fail(ET_ERR_ARG, "table %d: indices into an empty table", t);
            if (d.ld_idx < d.pool) return fail(ET_ERR_ARG, "table %d: ld_idx < pool", t);
        }
    }
    return ET_OK;
}

int lookup_dispatch(int dtype, const et_lookup_desc* descs, int ntables, int64_t batch,
                    void* dst, int64_t ld_dst, uint32_t flags, hipStream_t s,
                    void* queue = nullptr) {
    const int es = elsize(dtype);
    if (es == 0) return fail(ET_ERR_UNSUPPORTED, "unknown dtype %d", dtype);
    const int v = validate_lookup(descs, ntables, batch, dst, ld_dst);
    if (v != ET_OK) return v == 1 ? ET_OK : v;
    const bool nt = (flags & ET_FLAG_NONTEMPORAL) != 0;
    const bool f32acc = (flags & ET_FLAG_F16_FP32_ACC) != 0;

    // Classify each table; group identical (kind, dim) tables into one launch.
    int kind_of[4096];
    if (ntables > 4096) return fail(ET_ERR_ARG, "too many tables (%d)", ntables);
    for (int t = 0; t < ntables; ++t) {
        const et_lookup_desc& d = descs[t];
        const bool al = aligned16(d.table) && ((d.ld_table * es) % 16 == 0) &&
                        aligned16(static_cast<char*>(dst) + d.dst_row_off * es) &&
                        ((ld_dst * es) % 16 == 0);
        if (d.dim == 0) {
            kind_of[t] = -1;
        } else if (d.cols_per_page != 0) {
            // paged (SplitEmbedding) table: the pooled vector kernel with page addressing
            // (a non-reducing lookup is its pool = 1 case, still a bit copy); pages are
            // 16-byte aligned by contract (include/embtab.h)
            const bool vec = d.pool >= 1 && al && vec_dim_ok(d.dim) && d.nrows < 0xffffffffll &&
                             d.ld_table < 0xffffffffll && d.cols_per_page < 0xffffffffll;
            kind_of[t] = vec ? kPagedVec : kGeneric;
        } else if (d.pool == 1 && al && gather_rb_ok((int64_t)d.dim * es)) {
            kind_of[t] = kGather;
        } else if (d.pool >= 1 && al && vec_dim_ok(d.dim) && d.nrows < 0xffffffffll &&
                   d.ld_table < 0xffffffffll) {
            kind_of[t] = kPooledVec;
        } else if (d.pool >= 1 && al && ((int64_t)d.dim * es) % 16 == 0 && d.dim <= 2048 &&
                   d.nrows < 0xffffffffll && d.ld_table < 0xffffffffll) {
            kind_of[t] = kMaskedVec;  // any other 16-byte-multiple row (96, 200, 1504 ...)
        } else {
            kind_of[t] = kGeneric;
        }
    }
    bool done[4096] = {false};
    for (int t0 = 0; t0 < ntables; ++t0) {
        if (done[t0] || kind_of[t0] < 0) continue;
        // Collect the group of t0 (same kind, and same dim unless generic).
        LookupPack pack;
        pack.queue = static_cast<XcdQueue*>(queue);  // launches of one call are stream-ordered
        int n = 0;
        const GroupKind kind = (GroupKind)kind_of[t0];
        const int D = descs[t0].dim;
        for (int t = t0; t < ntables; ++t) {
            if (done[t] || kind_of[t] != kind_of[t0]) continue;
            if (kind != kGeneric && descs[t].dim != D) continue;
            pack.d[n++] = descs[t];
            done[t] = true;
            if (n == ET_MAX_TABLES_PER_LAUNCH) {
                int rc = nt ? launch_group<true>(dtype, f32acc, kind, pack, n, D, batch, dst,
                                                 ld_dst, s)
                            : launch_group<false>(dtype, f32acc, kind, pack, n, D, batch, dst,
                                                  ld_dst, s);
                if (rc != ET_OK) return rc;
                n = 0;
            }
        }
        if (n > 0) {
            int rc = nt ? launch_group<true>(dtype, f32acc, kind, pack, n, D, batch, dst, ld_dst, s)
                        : launch_group<false>(dtype, f32acc, kind, pack, n, D, batch, dst,
                                              ld_dst, s);
            if (rc != ET_OK) return rc;
        }
    }
    return ET_OK;
}

// Tables of one floating type into a destination of another (generic kernel).
template <typename T, typename A, typename O>
int launch_convert(const et_lookup_desc* descs, int ntables, int64_t batch, void* dst,
                   int64_t ld_dst, bool nt, hipStream_t s) {
    for (int t0 = 0; t0 < ntables; t0 += ET_MAX_TABLES_PER_LAUNCH) {
        LookupPack pack;
        int n = 0;
        for (int t = t0; t < ntables && n < ET_MAX_TABLES_PER_LAUNCH; ++t) pack.d[n++] = descs[t];
        const int64_t grid = (batch + 3) / 4 * n;
        if (grid > 0x7fffffffll) return fail(ET_ERR_ARG, "grid too large");
        if (nt)
            hipLaunchKernelGGL((k_pooled_generic<T, A, true, O>), dim3((unsigned)grid), dim3(256),
                               0, s, pack, n, batch, reinterpret_cast<O*>(dst), ld_dst);
        else
            hipLaunchKernelGGL((k_pooled_generic<T, A, false, O>), dim3((unsigned)grid),
                               dim3(256), 0, s, pack, n, batch, reinterpret_cast<O*>(dst), ld_dst);
        ET_LAUNCH_CHECK("k_pooled_generic");
    }
    return ET_OK;
}

template <typename T, typename A>
int convert_to(int out_dtype, const et_lookup_desc* descs, int ntables, int64_t batch, void* dst,
               int64_t ld_dst, bool nt, hipStream_t s) {
    switch (out_dtype) {
        case ET_F32: return launch_convert<T, A, float>(descs, ntables, batch, dst, ld_dst, nt, s);
        case ET_F64: return launch_convert<T, A, double>(descs, ntables, batch, dst, ld_dst, nt, s);
        case ET_F16:
            return launch_convert<T, A, _Float16>(descs, ntables, batch, dst, ld_dst, nt, s);
        case ET_BF16:
            return launch_convert<T, A, __bf16>(descs, ntables, batch, dst, ld_dst, nt, s);
    }
    return fail(ET_ERR_UNSUPPORTED, "destination dtype %d", out_dtype);
}

int lookup_dispatch_convert(int dtype, int out_dtype, const et_lookup_desc* descs, int ntables,
                            int64_t batch, void* dst, int64_t ld_dst, uint32_t flags,
                            hipStream_t s) {
    const int v = validate_lookup(descs, ntables, batch, dst, ld_dst);
    if (v != ET_OK) return v == 1 ? ET_OK : v;
    const bool nt = (flags & ET_FLAG_NONTEMPORAL) != 0;
    switch (dtype) {
        case ET_F32: return convert_to<float, float>(out_dtype, descs, ntables, batch, dst, ld_dst, nt, s);
        case ET_F64:
            return convert_to<double, double>(out_dtype, descs, ntables, batch, dst, ld_dst, nt, s);
        case ET_BF16:
            return convert_to<__bf16, float>(out_dtype, descs, ntables, batch, dst, ld_dst, nt, s);
        case ET_F16:
            if (flags & ET_FLAG_F16_FP32_ACC)
                return convert_to<_Float16, float>(out_dtype, descs, ntables, batch, dst, ld_dst,
                                                   nt, s);
            return convert_to<_Float16, _Float16>(out_dtype, descs, ntables, batch, dst, ld_dst,
                                                  nt, s);
    }
    return fail(ET_ERR_UNSUPPORTED, "table dtype %d (conversions are between float types)", dtype);
}

}  // namespace et

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------

extern "C" int et_gather(int dtype, const void* table, int64_t ld_table, int64_t nrows,
                         int32_t dim, const int64_t* idx, int64_t n, void* dst, int64_t ld_dst,
                         uint32_t flags, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    if (dim > 0 && ld_dst < dim) return et::fail(ET_ERR_ARG, "ld_dst < dim");
    et_lookup_desc d;
    d.table = table;
    d.ld_table = ld_table;
    d.nrows = nrows;
    d.dim = dim;
    d.pool = 1;
    d.idx = idx;
    d.ld_idx = 1;
    d.dst_row_off = 0;
    d.cols_per_page = 0;
    // A non-reducing lookup is a bit copy whatever the dtype: never the fp32-acc mode.
    return et::lookup_dispatch(dtype, &d, 1, n, dst, ld_dst, flags & ~ET_FLAG_F16_FP32_ACC,
                               static_cast<hipStream_t>(stream));
}

extern "C" int et_pooled_sum(int dtype, const void* table, int64_t ld_table, int64_t nrows,
                             int32_t dim, const int64_t* idx, int32_t pool, int64_t ld_idx,
                             int64_t batch, void* dst, int64_t ld_dst, uint32_t flags,
                             void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    if (dim > 0 && ld_dst < dim) return et::fail(ET_ERR_ARG, "ld_dst < dim");
    // pool == 0: the sum over an empty bag is zero(T); the generic kernel writes zeros.
    et_lookup_desc d;
    d.table = table;
    d.ld_table = ld_table;
    d.nrows = nrows;
    d.dim = dim;
    d.pool = pool;
    d.idx = idx;
    d.ld_idx = ld_idx;
    d.dst_row_off = 0;
    d.cols_per_page = 0;
    // pool == 1 as a *matrix* index is still a sum of one row == that row.
    return et::lookup_dispatch(dtype, &d, 1, batch, dst, ld_dst,
                               pool == 1 ? (flags & ~ET_FLAG_F16_FP32_ACC) : flags,
                               static_cast<hipStream_t>(stream));
}

extern "C" int et_maplookup_prealloc(int dtype, const et_lookup_desc* descs, int32_t ntables,
                                     int64_t batch, void* dst, int64_t ld_dst, uint32_t flags,
                                     void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    hipStream_t s = static_cast<hipStream_t>(stream);
    // Empty bags (pool == 0) are handled by the generic kernel, which writes zeros.
    // f16 pool == 1 tables are bit copies; the flag only matters for pool >= 2, where the
    // group kind is kPooledVec / kGeneric.
    return et::lookup_dispatch(dtype, descs, ntables, batch, dst, ld_dst, flags, s);
}

extern "C" int et_maplookup_prealloc_q(int dtype, const et_lookup_desc* descs, int32_t ntables,
                                       int64_t batch, void* dst, int64_t ld_dst, uint32_t flags,
                                       void* queue, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    if (queue && (reinterpret_cast<uintptr_t>(queue) & 15u))
        return et::fail(ET_ERR_ARG, "queue block is not 16-byte aligned");
    return et::lookup_dispatch(dtype, descs, ntables, batch, dst, ld_dst, flags,
                               static_cast<hipStream_t>(stream), queue);
}

extern "C" int et_maplookup_prealloc_to(int dtype, int dst_dtype, const et_lookup_desc* descs,
                                        int32_t ntables, int64_t batch, void* dst,
                                        int64_t ld_dst, uint32_t flags, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (dst_dtype == dtype)
        return et::lookup_dispatch(dtype, descs, ntables, batch, dst, ld_dst, flags, s);
    return et::lookup_dispatch_convert(dtype, dst_dtype, descs, ntables, batch, dst, ld_dst,
                                       flags, s);
}

ET_OOB_READER(lookup)

#ifdef ET_WG_TIMELINE
// Profiling build only: copies the striped launch's workgroup records (2 x uint4 each)
// to host memory; returns the number copied.
extern "C" int et_debug_timeline(void* host, int64_t cap) {
    const int64_t n = cap < (int64_t)et::kTlCap ? cap : (int64_t)et::kTlCap;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(et::g_tl), (size_t)n * 32, 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return (int)n;
}
#endif
