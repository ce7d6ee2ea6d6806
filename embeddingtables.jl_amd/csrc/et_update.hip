// et_update.hip — fused sparse SGD (Flux.Descent) and the device Indexer for gfx950
//
//
// Replaces (darchr/EmbeddingTables.jl):
//   update!(::Descent, table, ::SparseEmbeddingUpdate, indexer, Val)  src/sparseupdate.jl:160-178
//   index! / histogram! / prefixsum! / remap!                         src/utils.jl:131-314
//   _update_specialized_impl! / _update_generic_impl!                 src/sparseupdate.jl:57-154
//   multi-table update!(opt, tables, grads, indexers; num_splits)     src/sparseupdate.jl:199-238
//
// Pipeline (all stream-ordered, no host synchronisation):
//   1. k_build_keys   occurrence o of table t -> key = row_off[t] + (col - 1), value = o
//                      (o enumerates (table, bag, entry) with the entry fastest — the
//                      reference's `columns(A)` order, src/utils.jl:69-86)
//   2. radix sort      stable, so equal keys keep occurrence order (= remap! order)
//   3. segments        run boundaries of equal keys -> distinct (table, column) pairs
//   4. chunks          each segment is cut into chunks of at most kChunk occurrences
//                      (unless ET_FLAG_EXACT_UPDATE), so a Zipf-hot column cannot
//                      serialise one wave for milliseconds
//   5. k_sgd_chunks    one lane group per chunk: acc = +0; acc += delta[:, bag] in
//                      order; single-chunk segments apply the update directly,
//                      others write a partial row
//   6. k_sgd_combine   multi-chunk segments: acc = +0; acc += partial[p] in chunk order;
//                      apply the update
// The update of one column is  w = fma(-eta, acc, w)  (fused, the specialized path)
// or  w = w - eta*acc  (unfused, the generic path; optionally evaluated in Float64 as
// the reference's multi-table generic path does), chosen by ET_FLAG_SGD_UNFUSED /
// ET_FLAG_SGD_F64_ALPHA.
#include <algorithm>
#include <atomic>
#include <mutex>

#include "et_common.h"
#include "et_chain_asm.h"
#include "et_sort.hip"

namespace et {

constexpr uint32_t kChunk = ET_SGD_CHUNK;  // occurrences per chunk (non-exact mode)

struct UpdatePack {
    et_update_desc d[ET_MAX_TABLES_PER_LAUNCH];
    uint32_t vec_mask;  // bit t: table t is updated by the vector kernels (else generic)
    uint32_t row_off[ET_MAX_TABLES_PER_LAUNCH + 1];  // prefix of nrows
    uint32_t occ_off[ET_MAX_TABLES_PER_LAUNCH + 1];  // prefix of pool * batch
};

// Counters in the workspace.
enum { kCntU = 0, kCntC = 1, kCntM = 2, kCntT = 3,
       kCntNext = 5,     // next chain item (k_sgd_chains)
       kCntSlots = 16 };

__device__ __forceinline__ int table_of_key(const UpdatePack& p, int ntables, uint32_t key) {
    int t = 0;
    // ntables <= 32: a short scan of the (scalar-cached) prefix array
    while (t + 1 < ntables && key >= p.row_off[t + 1]) ++t;
    return t;
}

// 1. keys / values -----------------------------------------------------------
// Workgroup b works on table t with blk_off[t] <= b < blk_off[t+1] (host prefix of
// workgroups per table), so the table is uniform and bags are read with 16-B loads
// of consecutive occurrences.
struct KeyGrid {
    uint32_t blk_off[ET_MAX_TABLES_PER_LAUNCH + 1];
    uint32_t in_b;  // bit t: table t's pairs go to the second sort buffer (see et_sort.hip)
    uint32_t vec;   // bit t: contiguous 16-B aligned indices and 16-B aligned pair slots
    uint32_t snap_mask;  // bit t: copy table t's indices to snap[t] (et_sparse_sgd_snap)
    int64_t* snap[ET_MAX_TABLES_PER_LAUNCH];  // contiguous pool x batch Int64 copies
};

// 4 occurrences per thread: two 16-byte index loads, one 16-byte key and one 16-byte
// value store (config 4: 273 MB of indices in, 273 MB of pairs out).
typedef long long i64x2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_build_keys(UpdatePack pack, KeyGrid kg, int ntables,
                                                    uint32_t* __restrict__ ka,
                                                    uint32_t* __restrict__ va,
                                                    uint32_t* __restrict__ kb,
                                                    uint32_t* __restrict__ vb, uint32_t sent) {
    int t = 0;
    while (t + 1 < ntables && blockIdx.x >= kg.blk_off[t + 1]) ++t;
    const bool second = (kg.in_b >> t) & 1u;
    uint32_t* __restrict__ keys = second ? kb : ka;
    uint32_t* __restrict__ vals = second ? vb : va;
    const et_update_desc& d = pack.d[t];
    const uint32_t pool = (uint32_t)d.pool;
    const uint32_t n_t = pool * (uint32_t)d.batch;
    const uint32_t o0 = pack.occ_off[t], r0 = pack.row_off[t];
    const uint64_t nr = (uint64_t)d.nrows;
    const uint32_t nblk = kg.blk_off[t + 1] - kg.blk_off[t];
    int bad = 0;
    uint32_t ol0 = (blockIdx.x - kg.blk_off[t]) * 256u + threadIdx.x;
    // the snapshot of the indices for indexers[t] (written beside the keys: the index
    // array is read once, 8 more bytes written per occurrence)
    int64_t* __restrict__ snap = (kg.snap_mask >> t) & 1u ? kg.snap[t] : nullptr;
    if ((kg.vec >> t) & 1u) {  // workgroup-uniform
        const uint32_t n4 = n_t / 4u;
        const i64x2* ip = reinterpret_cast<const i64x2*>(d.idx);
        for (uint32_t q = ol0; q < n4; q += nblk * 256u) {
            const i64x2 a = ip[2 * q], b = ip[2 * q + 1];
            if (snap) {  // 16-byte aligned by the host's check
                reinterpret_cast<i64x2*>(snap)[2 * q] = a;
                reinterpret_cast<i64x2*>(snap)[2 * q + 1] = b;
            }
            const uint64_t c[4] = {(uint64_t)(a.x - 1), (uint64_t)(a.y - 1), (uint64_t)(b.x - 1),
                                   (uint64_t)(b.y - 1)};
            u32x4 kv, vv;
            uint32_t kk[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool ok = c[j] < nr;
                bad += ok ? 0 : 1;
                kk[j] = ok ? r0 + (uint32_t)c[j] : sent;
            }
            kv.x = kk[0], kv.y = kk[1], kv.z = kk[2], kv.w = kk[3];
            const uint32_t o = o0 + 4u * q;
            vv.x = o, vv.y = o + 1u, vv.z = o + 2u, vv.w = o + 3u;
            *reinterpret_cast<u32x4*>(keys + o) = kv;
            *reinterpret_cast<u32x4*>(vals + o) = vv;
        }
        ol0 = 4u * n4 + (blockIdx.x - kg.blk_off[t]) * 256u + threadIdx.x;  // the < 4 left
    }
    for (uint32_t ol = ol0; ol < n_t; ol += nblk * 256u) {
        const uint32_t j = ol / pool, i = ol - j * pool;
        const int64_t raw = d.idx[(int64_t)j * d.ld_idx + i];
        if (snap) snap[ol] = raw;
        const uint64_t col = (uint64_t)(raw - 1);
        const bool ok = col < nr;
        bad += ok ? 0 : 1;
        keys[o0 + ol] = ok ? r0 + (uint32_t)col : sent;
        vals[o0 + ol] = o0 + ol;
    }
    if (bad) note_oob(bad);
}

// 3. segments ------------------------------------------------------------------
// Segment starts = stream compaction of the head flags (key differs from the previous
// one), fused into a tile scan: k_seg_reduce counts heads per 4096-key tile,
// k_scan_partials scans the tile counts, k_seg_down recomputes the flags of its tile,
// scans them and writes seg_start[segment] = position (and U, seg_start[U] = n).
// Head flags of keys [i, i + 4) (i a multiple of 4): one 16-byte load of the four keys
// and one load of the key before them (an L1 hit but at a tile's first lane), instead
// of two 4-byte loads per key.
__device__ __forceinline__ void seg_heads4(const uint32_t* __restrict__ keys, int64_t n,
                                           int64_t i, uint32_t (&h)[4]) {
    uint32_t k[4];
    if (i + 3 < n) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(keys + i);
        k[0] = v.x, k[1] = v.y, k[2] = v.z, k[3] = v.w;
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) k[j] = i + j < n ? keys[i + j] : 0u;
    }
    const uint32_t prev = i > 0 ? keys[i - 1] : ~k[0];
    h[0] = (i < n && k[0] != prev) ? 1u : 0u;
#pragma unroll
    for (int j = 1; j < 4; ++j) h[j] = (i + j < n && k[j] != k[j - 1]) ? 1u : 0u;
}

__global__ __launch_bounds__(kScanThreads) void k_seg_reduce(const uint32_t* __restrict__ keys,
                                                             int64_t n,
                                                             uint32_t* __restrict__ part) {
    __shared__ uint32_t lds4[4];
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    uint32_t h = 0;
#pragma unroll
    for (int r = 0; r < kScanItems / 4; ++r) {  // striped 16-byte groups, coalesced
        uint32_t f[4];
        seg_heads4(keys, n, base + 4 * (r * kScanThreads + threadIdx.x), f);
        h += f[0] + f[1] + f[2] + f[3];
    }
    uint32_t total;
    block_inclusive_scan_256(h, lds4, &total);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

__global__ __launch_bounds__(kScanThreads) void k_seg_down(const uint32_t* __restrict__ keys,
                                                           int64_t n,
                                                           const uint32_t* __restrict__ part,
                                                           uint32_t* __restrict__ seg_start,
                                                           uint32_t* __restrict__ counters) {
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t tile[kScanTile + kScanTile / 32];
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
#pragma unroll
    for (int r = 0; r < kScanItems / 4; ++r) {  // striped 16-byte groups, coalesced
        const int e = 4 * (r * kScanThreads + threadIdx.x);
        uint32_t f[4];
        seg_heads4(keys, n, base + e, f);
#pragma unroll
        for (int j = 0; j < 4; ++j) tile[e + j + ((e + j) >> 5)] = f[j];
    }
    __syncthreads();
    uint32_t v[kScanItems];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int e = threadIdx.x * kScanItems + k;
        v[k] = tile[e + (e >> 5)];
        sum += v[k];
    }
    uint32_t total;
    const uint32_t inc = block_inclusive_scan_256(sum, lds4, &total);
    uint32_t run = part[blockIdx.x] + inc - sum;  // exclusive prefix of this thread's run
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t i = base + threadIdx.x * kScanItems + k;
        if (i < n && v[k]) seg_start[run] = (uint32_t)i;
        run += v[k];
        if (i == n - 1) {  // U = heads up to and including the last key
            seg_start[run] = (uint32_t)n;
            counters[kCntU] = run;
        }
    }
}

// nchunks per segment (0 beyond U), multi-chunk partial slots per segment; multi-chunk
// segments are also appended to `mlist` (order irrelevant: each is reduced by exactly
// one workgroup in a fixed order, so results do not depend on it).  The appends are
// aggregated per workgroup round of kSegChunkItems x 256 segments (a block scan of the
// threads' counts, one atomic): the multi-chunk segments are spread over the whole
// segment list (8.5 K of 1.9 M on the config-4 batch), so per-segment atomics on the
// one counter were serialised — 45 us for the pass.
constexpr int kSegChunkItems = 8;

__global__ __launch_bounds__(256) void k_seg_chunks(const uint32_t* __restrict__ seg_start,
                                                    int64_t n, uint32_t* __restrict__ counters,
                                                    uint32_t chunk, uint32_t* __restrict__ nch,
                                                    uint32_t* __restrict__ multi,
                                                    uint32_t* __restrict__ mlist) {
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t base_lds;
    // grid-stride over entries 0..U only (U is known on the device; the scans below
    // stop at U + 1), so a fixed grid covers any n; the loop bound is workgroup-uniform
    const int64_t U = (int64_t)counters[kCntU];
    const int64_t last = U < n ? U : n;
    constexpr int64_t kRound = (int64_t)kSegChunkItems * 256;
    for (int64_t u0 = (int64_t)blockIdx.x * kRound; u0 <= last;
         u0 += (int64_t)gridDim.x * kRound) {
        uint32_t c[kSegChunkItems];
        uint32_t mine = 0;
#pragma unroll
        for (int j = 0; j < kSegChunkItems; ++j) {
            const int64_t u = u0 + j * 256 + threadIdx.x;  // coalesced
            c[j] = 0;
            if (u < U) {
                const uint32_t len = seg_start[u + 1] - seg_start[u];
                c[j] = len <= chunk ? 1u : (len + chunk - 1) / chunk;
            }
            if (u <= last) {
                nch[u] = c[j];
                multi[u] = c[j] > 1 ? c[j] : 0u;
            }
            mine += c[j] > 1 ? 1u : 0u;
        }
        uint32_t total;
        uint32_t at = block_inclusive_scan_256(mine, lds4, &total) - mine;
        if (total == 0) continue;  // workgroup-uniform
        if (threadIdx.x == 0) base_lds = atomicAdd(&counters[kCntM], total);
        __syncthreads();
        at += base_lds;
#pragma unroll
        for (int j = 0; j < kSegChunkItems; ++j)
            if (c[j] > 1) mlist[at++] = (uint32_t)(u0 + j * 256 + threadIdx.x);
        __syncthreads();  // base_lds is rewritten next round
    }
}

// One 16-byte record per chunk — its occurrence range, its column key and where its
// sum goes (kApply: update the column directly; else its partial slot) — so the SGD
// passes fetch a chunk's metadata with one load instead of a chain of dependent ones.
struct ChunkRec {
    uint32_t s0, s1, key, dst;
};
constexpr uint32_t kApply = 0xffffffffu;
constexpr uint32_t kRetired = 0xffffffffu;  // an mlist entry taken by the hot-column pass

__global__ __launch_bounds__(256) void k_chunk_records(
    const uint32_t* __restrict__ chunk_start, const uint32_t* __restrict__ seg_start,
    const uint32_t* __restrict__ partial_start, const uint32_t* __restrict__ keys,
    uint32_t chunk, uint32_t* __restrict__ counters, ChunkRec* __restrict__ recs) {
    // single-chunk segments: one thread each (grid-stride over the device-side U)
    const uint32_t U = counters[kCntU];
    if (blockIdx.x == 0 && threadIdx.x == 0) counters[kCntC] = chunk_start[U];
    for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < (int64_t)U;
         u += (int64_t)gridDim.x * 256) {
        const uint32_t cs = chunk_start[u];
        if (chunk_start[u + 1] - cs != 1) continue;  // k_chunk_records_multi's
        const uint32_t ss = seg_start[u];
        recs[cs] = ChunkRec{ss, seg_start[u + 1], keys[ss], kApply};
    }
}

// multi-chunk segments (from the appended list): one wave each, lanes over chunks
__global__ __launch_bounds__(256) void k_chunk_records_multi(
    const uint32_t* __restrict__ chunk_start, const uint32_t* __restrict__ seg_start,
    const uint32_t* __restrict__ partial_start, const uint32_t* __restrict__ keys,
    const uint32_t* __restrict__ mlist, uint32_t chunk, const uint32_t* __restrict__ counters,
    ChunkRec* __restrict__ recs) {
    const uint32_t M = counters[kCntM];
    const int lane = threadIdx.x & 63;
    for (uint32_t m = blockIdx.x * 4 + (threadIdx.x >> 6); m < M; m += gridDim.x * 4) {
        const uint32_t u = mlist[m];
        const uint32_t ss = seg_start[u], se = seg_start[u + 1], key = keys[ss];
        const uint32_t cs = chunk_start[u], nc = chunk_start[u + 1] - cs, ps = partial_start[u];
        for (uint32_t p = lane; p < nc; p += 64) {
            const uint32_t s0 = ss + p * chunk;
            recs[cs + p] = ChunkRec{s0, s0 + chunk < se ? s0 + chunk : se, key, ps + p};
        }
    }
}

// 5./6. gradient sums and the update ---------------------------------------------

template <int MODE>  // 0 fused fma, 1 unfused f32, 2 unfused f64 alpha
__device__ __forceinline__ float sgd_apply(float w, float acc, float eta32, double eta64) {
    if constexpr (MODE == 0) return __builtin_fmaf(-eta32, acc, w);
    if constexpr (MODE == 1) return __fsub_rn(w, __fmul_rn(eta32, acc));
    return (float)__dsub_rn((double)w, __dmul_rn(eta64, (double)acc));
}

// The update of one element for any table type T with accumulator type C (the
// typed model of include/embtab.h / oracle/embtab_oracle.c): C = T for Float64 and
// Float16 (every Float16 op rounded to half, as Julia's), C = float for Float32,
// BFloat16 and Float16 with ET_FLAG_F16_FP32_ACC.  eta_c = convert(T, eta) held in C.
template <typename T, typename C, int MODE>
__device__ __forceinline__ T sgd_apply_t(T w, C acc, C eta_c, double eta64) {
    if constexpr (MODE == 2) {
        const double v = __dsub_rn((double)w, __dmul_rn(eta64, (double)acc));
        if constexpr (__is_same(T, __bf16))
            return (T)(float)v;
        else
            return (T)v;
    } else if constexpr (__is_same(C, double)) {
        if constexpr (MODE == 0) return __fma_rn(-eta_c, acc, (double)w);
        return __dsub_rn((double)w, __dmul_rn(eta_c, acc));
    } else if constexpr (MODE == 0) {
        // one fp32 fma, THEN one rounding to T.  The barrier keeps the compiler from folding
        // fptrunc(fma) into v_fma_mixlo_f16, which rounds the exact product-sum to half once
        // instead of going through fp32: a different result in rare ties (round 5 found 6 of
        // 64 K Float16 elements off by one ulp against the oracle's fmaf + f32->f16)
        float r = __builtin_fmaf(-(float)eta_c, (float)acc, (float)w);
        asm volatile("" : "+v"(r));
        return (T)r;
    } else if constexpr (__is_same(C, float)) {
        return (T)__fsub_rn((float)w, __fmul_rn(eta_c, acc));
    } else {  // Float16 arithmetic, two roundings (-ffp-contract=off: no fma)
        const C t = eta_c * acc;
        return (T)(C(w) - t);
    }
}

// Value of lane (base + g) for group g (base wave-uniform): readlane + select for <= 4
// groups per wave, ds_bpermute otherwise.
template <int GPW>
__device__ __forceinline__ uint32_t group_pick(uint32_t v, int base, int g) {
    if constexpr (GPW <= 4) {
        uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)v, base);
#pragma unroll
        for (int gg = 1; gg < GPW; ++gg) {
            const uint32_t t = (uint32_t)__builtin_amdgcn_readlane((int)v, base + gg);
            r = g == gg ? t : r;
        }
        return r;
    } else {
        return (uint32_t)__shfl((int)v, base + g, 64);
    }
}

// Sum the delta columns of sorted occurrences [s0, s1) into acc, in order (one lane
// group; a row of D fp32 is LPR lanes x NV 16-B vectors).  The group reads LPR
// occurrence ids at once (coalesced), turns them into bag numbers, broadcasts them
// lane by lane and keeps U column loads in flight.  The groups of a wave walk chunks
// of different lengths, so loop counters are NOT wave-uniform here: the broadcast is a
// ds_bpermute (per-lane source index), never a readlane.
//
// D is the power-of-two capacity of the row; the table's rows have `vpr` <= D/4 16-byte
// vectors (any dim that is a multiple of 4): lanes past the row re-read its last
// vector (vec_index) and never store.
template <int LPR, int NV>
__device__ __forceinline__ void vec_index(int sub, int vpr, int (&vix)[NV]) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const int i = sub + v * LPR;
        vix[v] = i < vpr ? i : vpr - 1;
    }
}

//
// Repeated bags.  A row that occurs k times in one bag has k consecutive sorted
// occurrences with the same bag (the sort is stable and occurrence ids are bag-major),
// so they all add the same delta column.  Each run of equal bags inside a slice of LPR
// occurrences is loaded ONCE and added `run` times in a row — the same sequence of
// fp32 adds as one load per occurrence, bit for bit.  The runs' heads are compacted to
// the front of the group with a forward lane permute (ds_permute), so the load loop
// walks heads only (Zipf(1.05) Criteo batch: 25% fewer delta gathers).
template <int D, int U>
__device__ __forceinline__ void occ_sum(const float* __restrict__ delta, uint32_t ld_delta,
                                        uint32_t occ_off, uint32_t pool,
                                        const uint32_t* __restrict__ vals, uint32_t s0,
                                        uint32_t s1, int g, int sub, int vpr,
                                        float (&acc)[(D / 4 < 64 ? 1 : D / 4 / 64)][4]) {
    constexpr int VPR = D / 4;
    constexpr int LPR = VPR < 64 ? VPR : 64;
    constexpr int NV = VPR / LPR;
    constexpr uint64_t kGroupBits = LPR == 64 ? ~0ull : ((1ull << LPR) - 1);
    const int lane = g * LPR + sub;
    int vix[NV];
    vec_index<LPR, NV>(sub, vpr, vix);
    for (uint32_t c0 = s0; c0 < s1; c0 += LPR) {
        const int cnt = (int)(s1 - c0 < (uint32_t)LPR ? s1 - c0 : (uint32_t)LPR);
        const uint32_t myo = vals[c0 + (uint32_t)(sub < cnt ? sub : cnt - 1)];
        const int mybag = (int)((myo - occ_off) / pool);
        // run heads of this slice: first slot, or a bag different from the previous slot's
        const int prev = __shfl(mybag, sub > 0 ? lane - 1 : lane, 64);
        const bool head = sub < cnt && (sub == 0 || mybag != prev);
        const uint64_t gm = (LPR == 64 ? (uint64_t)__ballot(head)
                                       : ((uint64_t)__ballot(head) >> (g * LPR))) & kGroupBits;
        const int nh = __popcll(gm);
        const int rank = __popcll(gm & ((1ull << sub) - 1));  // heads before this slot
        const uint64_t after = sub + 1 < 64 ? gm >> (sub + 1) : 0ull;
        const int run = (after ? sub + __ffsll((long long)after) : cnt) - sub;
        // heads to slots [0, nh) in order, the other slots behind them (a permutation)
        const int to = g * LPR + (head ? rank : nh + (sub - rank));
        const int hbag = __builtin_amdgcn_ds_permute(to << 2, mybag);
        const int hrun = __builtin_amdgcn_ds_permute(to << 2, run);
        for (int i0 = 0; i0 < nh; i0 += U) {
            const int m = nh - i0 < U ? nh - i0 : U;
            uint64_t off[U];
            int rep[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int slot = g * LPR + i0 + (u < m ? u : m - 1);
                const uint32_t bag = (uint32_t)__shfl(hbag, slot, 64);
                rep[u] = __shfl(hrun, slot, 64);
                off[u] = (uint64_t)bag * ld_delta;
            }
            u32x4 buf[U][NV];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u32x4* src = reinterpret_cast<const u32x4*>(delta + off[u]);
#pragma unroll
                for (int v = 0; v < NV; ++v) buf[u][v] = src[vix[v]];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (u < m) {
                    for (int k = 0; k < rep[u]; ++k) {
#pragma unroll
                        for (int v = 0; v < NV; ++v) {
                            const u32x4 b = buf[u][v];
                            acc[v][0] = acc[v][0] + __uint_as_float(b.x);
                            acc[v][1] = acc[v][1] + __uint_as_float(b.y);
                            acc[v][2] = acc[v][2] + __uint_as_float(b.z);
                            acc[v][3] = acc[v][3] + __uint_as_float(b.w);
                        }
                    }
                }
            }
        }
    }
}

template <int D, int MODE, bool NT>
__device__ __forceinline__ void apply_row(float* __restrict__ w,
                                          const u32x4 (&x)[(D / 4 < 64 ? 1 : D / 4 / 64)],
                                          const float (&acc)[(D / 4 < 64 ? 1 : D / 4 / 64)][4],
                                          int sub, int vpr, float eta32, double eta64) {
    constexpr int VPR = D / 4;
    constexpr int LPR = VPR < 64 ? VPR : 64;
    constexpr int NV = VPR / LPR;
    u32x4* wp = reinterpret_cast<u32x4*>(w) + sub;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        u32x4 y;
        y.x = __float_as_uint(sgd_apply<MODE>(__uint_as_float(x[v].x), acc[v][0], eta32, eta64));
        y.y = __float_as_uint(sgd_apply<MODE>(__uint_as_float(x[v].y), acc[v][1], eta32, eta64));
        y.z = __float_as_uint(sgd_apply<MODE>(__uint_as_float(x[v].z), acc[v][2], eta32, eta64));
        y.w = __float_as_uint(sgd_apply<MODE>(__uint_as_float(x[v].w), acc[v][3], eta32, eta64));
        if (sub + v * LPR < vpr) store16<NT>(wp + v * LPR, y);
    }
}

// Chunk pass.  Each wave takes 64 chunks spaced `nwaves` apart (so the consecutive
// chunks of a hot segment land on different waves), loads their metadata once (one
// chunk per lane), and its lane groups walk them, reading a chunk's fields from the
// metadata lanes with v_readlane.  Single-chunk segments read the table column before
// the gradient sum (so the read overlaps the delta gathers) and apply the update;
// chunks of longer segments store a partial row.
template <int D, int MODE, bool NT>
__device__ __forceinline__ void sgd_chunks_body(
    const UpdatePack& pack, int ntables, const uint32_t* __restrict__ keys,
    const uint32_t* __restrict__ vals, const ChunkRec* __restrict__ recs,
    const uint32_t* __restrict__ counters, float* __restrict__ partials, int pdim,
    uint32_t sent, float eta32, double eta64, uint32_t my_mask, int skip_singles,
    int skip_multi, uint32_t bid, uint32_t nblk) {
    constexpr int VPR = D / 4;
    constexpr int LPR = VPR < 64 ? VPR : 64;
    constexpr int NV = VPR / LPR;
    constexpr int GPW = 64 / LPR;
    constexpr int U = NV >= 8 ? 1 : 8 / NV;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane / LPR, sub = lane % LPR;
    const uint32_t C = counters[kCntC];
    const uint32_t nwaves = nblk * 4u;
    const uint32_t wid = bid * 4u + wave;
    for (uint32_t it = 0; (uint64_t)it * 64u * nwaves + wid < C; ++it) {
        // metadata of chunks (it*64 + l) * nwaves + wid, one per lane l
        const uint64_t cl = ((uint64_t)it * 64u + lane) * nwaves + wid;
        const bool valid = cl < C;
        const ChunkRec r = recs[valid ? (uint32_t)cl : C - 1];
        uint32_t m_s0 = r.s0, m_s1 = r.s1, m_dst = r.dst;
        uint32_t m_key = valid ? r.key : sent;
        const uint64_t left = ((uint64_t)C - wid + nwaves - 1) / nwaves - (uint64_t)it * 64u;
        uint32_t nq = left < 64u ? (uint32_t)left : 64u;
        if (skip_singles) {
            // the records this pass walks (not k_sgd_singles', nor the exact mode's chains:
            // the chunks of multi-chunk columns), compacted to the front
            const bool keep = valid && m_key != sent && !(m_dst == kApply && m_s1 - m_s0 == 1u) &&
                              !(skip_multi && m_dst != kApply);
            const uint64_t bal = (uint64_t)__ballot(keep);
            const int nk = __popcll(bal);
            const int rk = __popcll(bal & ((1ull << lane) - 1ull));
            const int to = (keep ? rk : nk + (lane - rk)) << 2;
            m_s0 = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)m_s0);
            m_s1 = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)m_s1);
            m_dst = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)m_dst);
            m_key = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(keep ? m_key : sent));
            nq = (uint32_t)nk;
        }
        for (uint32_t qq = 0; qq < nq; qq += GPW) {
            const uint32_t kkey = group_pick<GPW>(m_key, (int)qq, g);
            const uint32_t s0 = group_pick<GPW>(m_s0, (int)qq, g);
            const uint32_t s1 = group_pick<GPW>(m_s1, (int)qq, g);
            const uint32_t dsl = group_pick<GPW>(m_dst, (int)qq, g);
            if (qq + g >= nq || kkey == sent) continue;  // past the end / bad indices
            const int t = table_of_key(pack, ntables, kkey);
            const et_update_desc& d = pack.d[t];
            if (!((my_mask >> t) & 1u)) continue;  // another capacity's / the generic table
            float* w = col_ptr<float>(d.table, d.ld_table, d.cols_per_page,
                                      kkey - pack.row_off[t]);
            const int vpr = d.dim / 4;
            int vix[NV];
            vec_index<LPR, NV>(sub, vpr, vix);
            u32x4 x[NV];
            if (dsl == 0xffffffffu) {
                const u32x4* wp = reinterpret_cast<const u32x4*>(w);
#pragma unroll
                for (int v = 0; v < NV; ++v) x[v] = wp[vix[v]];
            }
            float acc[NV][4];
#pragma unroll
            for (int v = 0; v < NV; ++v) acc[v][0] = acc[v][1] = acc[v][2] = acc[v][3] = 0.0f;
            occ_sum<D, U>(reinterpret_cast<const float*>(d.delta), (uint32_t)d.ld_delta,
                          pack.occ_off[t], (uint32_t)d.pool, vals, s0, s1, g, sub, vpr, acc);
            if (dsl == 0xffffffffu) {
                apply_row<D, MODE, NT>(w, x, acc, sub, vpr, eta32, eta64);
            } else {
                u32x4* pp = reinterpret_cast<u32x4*>(partials + (uint64_t)dsl * pdim) + sub;
#pragma unroll
                for (int v = 0; v < NV; ++v)
                    if (sub + v * LPR < vpr)
                        pp[v * LPR] = u32x4{__float_as_uint(acc[v][0]), __float_as_uint(acc[v][1]),
                                            __float_as_uint(acc[v][2]), __float_as_uint(acc[v][3])};
            }
        }
    }
}

#define ET_SGD_CHUNKS_ARGS                                                                     \
    UpdatePack pack, int ntables, const uint32_t* __restrict__ keys,                           \
        const uint32_t* __restrict__ vals, const ChunkRec* __restrict__ recs,                  \
        const uint32_t* __restrict__ counters, float* __restrict__ partials, int pdim,         \
        uint32_t sent, float eta32, double eta64, uint32_t my_mask, int skip_singles
template <int D, int MODE, bool NT>
__global__ __launch_bounds__(256) void k_sgd_chunks(ET_SGD_CHUNKS_ARGS) {
    sgd_chunks_body<D, MODE, NT>(pack, ntables, keys, vals, recs, counters, partials, pdim, sent,
                                 eta32, eta64, my_mask, skip_singles, 0, blockIdx.x, gridDim.x);
}
// The same pass compiled for 5 waves per SIMD (96 VGPRs instead of 97-104: 4 waves).
template <int D, int MODE, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_sgd_chunks5(
    ET_SGD_CHUNKS_ARGS) {
    sgd_chunks_body<D, MODE, NT>(pack, ntables, keys, vals, recs, counters, partials, pdim, sent,
                                 eta32, eta64, my_mask, skip_singles, 0, blockIdx.x, gridDim.x);
}
#undef ET_SGD_CHUNKS_ARGS

// Single-occurrence columns (70% of the chunks on the config-4 batch, 1.34 M of 2.0 M):
// in k_sgd_chunks each is a chain of dependent loads (record -> occurrence id -> Δ
// column and table column -> store) walked one chunk per lane group at a time, so the
// pass waits on memory latency.  Here a wave takes the same 64 records at a time, keeps
// the singles (compacted to the front with a lane permute), and each lane group updates
// K of them together: K occurrence-id loads, then K Δ-column and K table-column loads in
// flight, then K stores.  Same arithmetic as the chunk path (acc = +0 + Δ, then the
// update), bit for bit.
// Per-table fields the singles kernel reads with a per-lane table index, staged in LDS
// (indexing the kernel-argument descriptors per lane would loop over the distinct
// tables of the wave).
struct SingleTab {
    uint64_t table, delta;
    uint32_t ld_table, ld_delta, pool, vpr, row_off, occ_off;
    uint64_t cols_per_page;
};

template <int D, int MODE, bool NT>
__device__ __forceinline__ void sgd_singles_body(
    const UpdatePack& pack, int ntables, const uint32_t* __restrict__ vals,
    const ChunkRec* __restrict__ recs, const uint32_t* __restrict__ counters, uint32_t sent,
    float eta32, double eta64, uint32_t my_mask, uint32_t bid, uint32_t nblk) {
    constexpr int VPR = D / 4;
    constexpr int LPR = VPR < 64 ? VPR : 64;
    constexpr int NV = VPR / LPR;
    constexpr int GPW = 64 / LPR;
    constexpr int K = NV >= 8 ? 1 : 8 / NV;  // singles per lane group at a time
    __shared__ SingleTab tabs[ET_MAX_TABLES_PER_LAUNCH];
    if (threadIdx.x < (unsigned)ntables) {
        const et_update_desc& d = pack.d[threadIdx.x];
        tabs[threadIdx.x] = SingleTab{(uint64_t)d.table, (uint64_t)d.delta, (uint32_t)d.ld_table,
                                      (uint32_t)d.ld_delta, (uint32_t)d.pool, (uint32_t)(d.dim / 4),
                                      pack.row_off[threadIdx.x], pack.occ_off[threadIdx.x],
                                      (uint64_t)d.cols_per_page};
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int g = lane / LPR, sub = lane % LPR;
    const uint32_t C = counters[kCntC];
    const uint32_t nwaves = nblk * 4u;
    const uint32_t wid = bid * 4u + wave;
    for (uint32_t it = 0; (uint64_t)it * 64u * nwaves + wid < C; ++it) {
        // one record per lane: singles get their table-column and Δ-column addresses
        const uint64_t cl = ((uint64_t)it * 64u + lane) * nwaves + wid;
        bool single = false;
        uint64_t wpa = 0, dpa = 0;
        uint32_t vp = 0;
        if (cl < C) {
            const ChunkRec r = recs[(uint32_t)cl];
            if (r.dst == kApply && r.s1 - r.s0 == 1u && r.key != sent) {
                int t = 0;  // wave-uniform loop over the (scalar) prefix, no per-lane branch
                for (int i = 1; i < ntables; ++i) t += r.key >= pack.row_off[i] ? 1 : 0;
                if ((my_mask >> t) & 1u) {
                    const SingleTab tb = tabs[t];
                    const uint32_t bag = (vals[r.s0] - tb.occ_off) / tb.pool;
                    wpa = (uint64_t)col_ptr<float>((const void*)tb.table, tb.ld_table,
                                                   (int64_t)tb.cols_per_page, r.key - tb.row_off);
                    dpa = tb.delta + (uint64_t)bag * tb.ld_delta * 4u;
                    vp = tb.vpr;
                    single = true;
                }
            }
        }
        const uint64_t bal = (uint64_t)__ballot(single);
        const int ns = __popcll(bal);
        if (ns == 0) continue;  // wave-uniform
        const int rank = __popcll(bal & ((1ull << lane) - 1ull));
        const int to = (single ? rank : ns + (lane - rank)) << 2;  // singles first
        const uint32_t wlo = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(uint32_t)wpa);
        const uint32_t whi = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(uint32_t)(wpa >> 32));
        const uint32_t dlo = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(uint32_t)dpa);
        const uint32_t dhi = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)(uint32_t)(dpa >> 32));
        const uint32_t vpp = (uint32_t)__builtin_amdgcn_ds_permute(to, (int)vp);
        // wave-uniform trip count: the lane reads below take other groups' lanes, so every
        // lane stays active through them
        for (int base = 0; base < ns; base += GPW * K) {
            const int q0 = base + g * K;
            const int m = ns - q0 < K ? ns - q0 : K;  // <= 0: this group has none left
            float* wp[K];
            int vpr[K];
            u32x4 x[K][NV], y[K][NV];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                int j = q0 + (k < m ? k : m - 1);
                j = j < ns ? (j < 0 ? 0 : j) : ns - 1;
                const uint64_t w64 = ((uint64_t)(uint32_t)__shfl((int)whi, j, 64) << 32) |
                                     (uint32_t)__shfl((int)wlo, j, 64);
                const uint64_t d64 = ((uint64_t)(uint32_t)__shfl((int)dhi, j, 64) << 32) |
                                     (uint32_t)__shfl((int)dlo, j, 64);
                wp[k] = reinterpret_cast<float*>(w64);
                vpr[k] = __shfl((int)vpp, j, 64);
                int vix[NV];
                vec_index<LPR, NV>(sub, vpr[k], vix);
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    y[k][v] = reinterpret_cast<const u32x4*>(d64)[vix[v]];
                    x[k][v] = reinterpret_cast<const u32x4*>(w64)[vix[v]];
                }
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (k < m) {
                    float acc[NV][4];
#pragma unroll
                    for (int v = 0; v < NV; ++v) {
                        acc[v][0] = 0.0f + __uint_as_float(y[k][v].x);
                        acc[v][1] = 0.0f + __uint_as_float(y[k][v].y);
                        acc[v][2] = 0.0f + __uint_as_float(y[k][v].z);
                        acc[v][3] = 0.0f + __uint_as_float(y[k][v].w);
                    }
                    apply_row<D, MODE, NT>(wp[k], x[k], acc, sub, vpr[k], eta32, eta64);
                }
            }
        }
    }
}

// Combine pass: every multi-chunk segment (from the appended list, one per workgroup
// at a time) is reduced by a whole workgroup.  Its partial rows are split into NR = 8
// contiguous ranges in chunk order, whatever the dim (so a feature slice of a table —
// a shard's piece — combines exactly like the whole table); lane group G sums ranges G,
// G + NG, ... sequentially (U rows in flight), the NR sums are added in range order
// through LDS and group 0 applies the update.  Fixed partition => deterministic.
constexpr uint32_t kLongPartials = 64;

template <int D, int MODE, bool NT>
__device__ __forceinline__ void sgd_combine_body(
    const UpdatePack& pack, int ntables, const uint32_t* __restrict__ keys,
    const uint32_t* __restrict__ seg_start, const uint32_t* __restrict__ partial_start,
    const uint32_t* __restrict__ counters, const uint32_t* __restrict__ mlist,
    const float* __restrict__ partials, int pdim, uint32_t sent, float eta32, double eta64,
    uint32_t my_mask, uint32_t bid, uint32_t nblk) {
    constexpr int VPR = D / 4;
    constexpr int LPR = VPR < 64 ? VPR : 64;
    constexpr int NV = VPR / LPR;
    constexpr int GPW = 64 / LPR;
    constexpr int NG = 4 * GPW;  // lane groups per workgroup (4..64)
    constexpr int NR = 8;        // ranges of partials, independent of the dim
    constexpr int U = NV >= 8 ? 1 : 8 / NV;
    __shared__ u32x4 red[NR][LPR * NV];
    const int lane = threadIdx.x & 63;
    const int G = threadIdx.x / LPR, sub = lane % LPR;
    const uint32_t M = counters[kCntM];
    // two sweeps over the list: segments of more than kLongPartials partials first, so
    // the long sequential range sums (latency chains) start with the kernel, the rest after
    for (int sweep = 0; sweep < 2; ++sweep) {
        for (uint32_t k = bid; k < M; k += nblk) {
            const uint32_t seg = mlist[k];
            if (seg == kRetired) continue;  // a hot column (k_hot_pick), uniform
            {
                const uint32_t npp = partial_start[seg + 1] - partial_start[seg];
                if ((npp > kLongPartials) != (sweep == 0)) continue;  // uniform
            }
            {
                const uint32_t key0 = keys[seg_start[seg]];
                if (key0 == sent || !((my_mask >> table_of_key(pack, ntables, key0)) & 1u))
                    continue;  // uniform across the workgroup
            }
            const uint32_t p0 = partial_start[seg], np = partial_start[seg + 1] - p0;
            const int vpr = pack.d[table_of_key(pack, ntables, keys[seg_start[seg]])].dim / 4;
            int vix[NV];
            vec_index<LPR, NV>(sub, vpr, vix);
            for (int R = G; R < NR; R += NG) {
            const uint32_t a = p0 + (uint32_t)((uint64_t)np * R / NR);
            const uint32_t b = p0 + (uint32_t)((uint64_t)np * (R + 1) / NR);
            float acc[NV][4];
#pragma unroll
            for (int v = 0; v < NV; ++v) acc[v][0] = acc[v][1] = acc[v][2] = acc[v][3] = 0.0f;
            for (uint32_t q0 = a; q0 < b; q0 += U) {
                u32x4 buf[U][NV];
#pragma unroll
                for (int uu = 0; uu < U; ++uu) {
                    const uint32_t q = q0 + uu < b ? q0 + uu : b - 1;
                    const u32x4* pp = reinterpret_cast<const u32x4*>(partials + (uint64_t)q * pdim);
#pragma unroll
                    for (int v = 0; v < NV; ++v) buf[uu][v] = pp[vix[v]];
                }
#pragma unroll
                for (int uu = 0; uu < U; ++uu) {
                    if (q0 + uu < b) {
#pragma unroll
                        for (int v = 0; v < NV; ++v) {
                            acc[v][0] = acc[v][0] + __uint_as_float(buf[uu][v].x);
                            acc[v][1] = acc[v][1] + __uint_as_float(buf[uu][v].y);
                            acc[v][2] = acc[v][2] + __uint_as_float(buf[uu][v].z);
                            acc[v][3] = acc[v][3] + __uint_as_float(buf[uu][v].w);
                        }
                    }
                }
            }
#pragma unroll
            for (int v = 0; v < NV; ++v)
                red[R][v * LPR + sub] = u32x4{__float_as_uint(acc[v][0]), __float_as_uint(acc[v][1]),
                                              __float_as_uint(acc[v][2]), __float_as_uint(acc[v][3])};
            }
            __syncthreads();
            if (G == 0) {
                float tot[NV][4];
#pragma unroll
                for (int v = 0; v < NV; ++v) tot[v][0] = tot[v][1] = tot[v][2] = tot[v][3] = 0.0f;
                for (int gg = 0; gg < NR; ++gg) {
#pragma unroll
                    for (int v = 0; v < NV; ++v) {
                        const u32x4 r = red[gg][v * LPR + sub];
                        tot[v][0] = tot[v][0] + __uint_as_float(r.x);
                        tot[v][1] = tot[v][1] + __uint_as_float(r.y);
                        tot[v][2] = tot[v][2] + __uint_as_float(r.z);
                        tot[v][3] = tot[v][3] + __uint_as_float(r.w);
                    }
                }
                const uint32_t key = keys[seg_start[seg]];
                const int t = table_of_key(pack, ntables, key);
                const et_update_desc& d = pack.d[t];
                float* w = col_ptr<float>(d.table, d.ld_table, d.cols_per_page,
                                          key - pack.row_off[t]);
                u32x4 x[NV];
                const u32x4* wp = reinterpret_cast<const u32x4*>(w);
#pragma unroll
                for (int v = 0; v < NV; ++v) x[v] = wp[vix[v]];
                apply_row<D, MODE, NT>(w, x, tot, sub, vpr, eta32, eta64);
            }
            __syncthreads();
        }
    }
}

template <int D, int MODE, bool NT>
__global__ __launch_bounds__(256) void k_sgd_singles(
    UpdatePack pack, int ntables, const uint32_t* __restrict__ vals,
    const ChunkRec* __restrict__ recs, const uint32_t* __restrict__ counters, uint32_t sent,
    float eta32, double eta64, uint32_t my_mask) {
    sgd_singles_body<D, MODE, NT>(pack, ntables, vals, recs, counters, sent, eta32, eta64,
                                  my_mask, blockIdx.x, gridDim.x);
}

template <int D, int MODE, bool NT>
__global__ __launch_bounds__(256) void k_sgd_combine(
    UpdatePack pack, int ntables, const uint32_t* __restrict__ keys,
    const uint32_t* __restrict__ seg_start, const uint32_t* __restrict__ partial_start,
    const uint32_t* __restrict__ counters, const uint32_t* __restrict__ mlist,
    const float* __restrict__ partials, int pdim, uint32_t sent, float eta32, double eta64,
    uint32_t my_mask) {
    sgd_combine_body<D, MODE, NT>(pack, ntables, keys, seg_start, partial_start, counters, mlist,
                                  partials, pdim, sent, eta32, eta64, my_mask, blockIdx.x,
                                  gridDim.x);
}

// The combine and the singles in one launch: the first `ncomb` workgroups combine, the
// rest update single-occurrence columns.  They touch disjoint columns (multi-chunk vs
// single-occurrence segments) and both only follow the chunk pass, so the combine's
// long sequential range sums (the hottest column's 3.3 K partials: 8 ranges of ~400
// dependent row loads, ~80 us on its own) run under the singles' bandwidth-bound work
// instead of after it.  Every workgroup takes one branch (block-uniform).
template <int D, int MODE, bool NT>
__global__ __launch_bounds__(256) void k_sgd_tail(
    UpdatePack pack, int ntables, const uint32_t* __restrict__ keys,
    const uint32_t* __restrict__ vals, const ChunkRec* __restrict__ recs,
    const uint32_t* __restrict__ seg_start, const uint32_t* __restrict__ partial_start,
    const uint32_t* __restrict__ counters, const uint32_t* __restrict__ mlist,
    const float* __restrict__ partials, int pdim, uint32_t sent, float eta32, double eta64,
    uint32_t my_mask, uint32_t ncomb) {
    if (blockIdx.x < ncomb)
        sgd_combine_body<D, MODE, NT>(pack, ntables, keys, seg_start, partial_start, counters,
                                      mlist, partials, pdim, sent, eta32, eta64, my_mask,
                                      blockIdx.x, ncomb);
    else
        sgd_singles_body<D, MODE, NT>(pack, ntables, vals, recs, counters, sent, eta32, eta64,
                                      my_mask, blockIdx.x - ncomb, gridDim.x - ncomb);
}

// Hot-column pass (non-exact Float32 mode, dim 128, pool <= 32).  The columns with the
// longest occurrence lists of a table — up to kHotSlots of them, chosen by a per-table
// length threshold (a log2 histogram of the multi-chunk segments, so the choice never
// depends on atomic arrival order) — are summed bag-major instead of by gathering one Δ
// column per (column, bag) pair: workgroup (window, table) streams the Δ columns of
// kHotWin consecutive bags once, maps each index to its hot slot through an LDS hash, and
// adds Δ into the slot's LDS accumulator.  Wave w owns the slots s with s % 4 == w and
// walks the bags and pool positions in order, so every (slot, feature) sum runs in
// occurrence order from +0; the per-window partials are added in window order by
// k_hot_combine, which applies the update.  The chunk and combine passes skip the hot
// columns (their records and list entries are retired by k_hot_pick).
constexpr int kHotSlots = 120;   // per table (slot ids fit a byte; 0xff = not hot)
constexpr int kHotWin = 1024;    // bags per workgroup (one partial per window)
constexpr int kHotBatch = 32;    // bags staged in LDS at a time
constexpr int kHotHash = 256;    // open-addressing LDS hash of the hot keys
constexpr int kHotMaxPool = 32;

struct HotList {
    int n;
    int t[ET_MAX_TABLES_PER_LAUNCH];
    uint64_t soff[ET_MAX_TABLES_PER_LAUNCH];  // the table's slot bytes in the workspace
};

__global__ __launch_bounds__(256) void k_hot_hist(UpdatePack pack, int ntables, uint32_t hot_mask,
                                                  const uint32_t* __restrict__ keys,
                                                  const uint32_t* __restrict__ seg_start,
                                                  const uint32_t* __restrict__ mlist,
                                                  const uint32_t* __restrict__ counters,
                                                  uint32_t* __restrict__ hist) {
    const uint32_t M = counters[kCntM];
    for (uint32_t m = blockIdx.x * 256 + threadIdx.x; m < M; m += gridDim.x * 256) {
        const uint32_t u = mlist[m];
        const uint32_t ss = seg_start[u], len = seg_start[u + 1] - ss, key = keys[ss];
        if (key >= pack.row_off[ntables]) continue;  // out-of-range occurrences
        const int t = table_of_key(pack, ntables, key);
        if (!((hot_mask >> t) & 1u)) continue;
        atomicAdd(&hist[t * 32 + (31 - __builtin_clz(len))], 1u);
    }
}

__device__ __forceinline__ int hot_threshold(const uint32_t* __restrict__ hist, int t) {
    // smallest log2 bucket b with (segments of length >= 2^b) <= kHotSlots
    uint32_t acc = 0;
    int b0 = 32;
    for (int b = 31; b >= 0; --b) {
        acc += hist[t * 32 + b];
        if (acc > (uint32_t)kHotSlots) break;
        b0 = b;
    }
    return b0;
}

__global__ __launch_bounds__(256) void k_hot_pick(UpdatePack pack, int ntables, uint32_t hot_mask,
                                                  const uint32_t* __restrict__ keys,
                                                  const uint32_t* __restrict__ seg_start,
                                                  const uint32_t* __restrict__ chunk_start,
                                                  uint32_t* __restrict__ mlist,
                                                  const uint32_t* __restrict__ counters,
                                                  const uint32_t* __restrict__ hist,
                                                  uint32_t* __restrict__ hcnt,
                                                  uint32_t* __restrict__ hkey,
                                                  ChunkRec* __restrict__ recs, uint32_t sent) {
    const uint32_t M = counters[kCntM];
    for (uint32_t m = blockIdx.x * 256 + threadIdx.x; m < M; m += gridDim.x * 256) {
        const uint32_t u = mlist[m];
        const uint32_t ss = seg_start[u], len = seg_start[u + 1] - ss, key = keys[ss];
        if (key >= pack.row_off[ntables]) continue;
        const int t = table_of_key(pack, ntables, key);
        if (!((hot_mask >> t) & 1u)) continue;
        if (31 - __builtin_clz(len) < hot_threshold(hist, t)) continue;
        const uint32_t s = atomicAdd(&hcnt[t], 1u);  // slot ids only place the sums
        hkey[t * kHotSlots + s] = key;
        mlist[m] = kRetired;
        for (uint32_t c = chunk_start[u], ce = chunk_start[u + 1]; c < ce; ++c) recs[c].key = sent;
    }
}

__device__ __forceinline__ uint32_t hot_hash(uint32_t key) {
    return (key * 2654435761u) >> 24;  // kHotHash = 256 buckets
}

// Index phase: the hot slot of every occurrence of a hot table (0xff: not hot or out of
// range), one byte each, bag rows padded to P4 = roundup(pool, 4) bytes so the update
// phase reads a batch of bags as whole words and never touches the indices.
constexpr int kHotSlotBags = 256;  // bags per workgroup of k_hot_slots

__global__ __launch_bounds__(256) void k_hot_slots(UpdatePack pack, HotList hl,
                                                   const uint32_t* __restrict__ hcnt,
                                                   const uint32_t* __restrict__ hkey,
                                                   uint8_t* __restrict__ slots) {
    __shared__ uint32_t hk[kHotHash];
    __shared__ uint8_t hs[kHotHash];
    const int hi = blockIdx.y, t = hl.t[hi];
    const et_update_desc& d = pack.d[t];
    const int64_t bb = (int64_t)blockIdx.x * kHotSlotBags;
    if (bb >= d.batch) return;  // uniform
    const int nbag = d.batch - bb < kHotSlotBags ? (int)(d.batch - bb) : kHotSlotBags;
    const uint32_t H = hcnt[t];
    const int tid = threadIdx.x;
    for (int i = tid; i < kHotHash; i += 256) hk[i] = 0u;
    __syncthreads();
    if (tid < (int)H) {
        const uint32_t key = hkey[t * kHotSlots + tid];
        uint32_t h = hot_hash(key);
        while (atomicCAS(&hk[h], 0u, key + 1u) != 0u) h = (h + 1) & (kHotHash - 1);
        hs[h] = (uint8_t)tid;
    }
    __syncthreads();
    const int P = d.pool, P4 = (P + 3) & ~3, W = P4 / 4;
    const uint32_t r0 = pack.row_off[t];
    const uint64_t nrows = (uint64_t)d.nrows;
    uint32_t* out = reinterpret_cast<uint32_t*>(slots + hl.soff[hi] + (uint64_t)bb * P4);
    for (int e = tid; e < nbag * W; e += 256) {
        const int j = e / W, i0 = (e % W) * 4;
        const int64_t* ip = d.idx + (bb + j) * d.ld_idx;
        uint32_t word = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            uint32_t sv = 0xffu;
            const int i = i0 + b;
            if (i < P && H > 0) {
                const int64_t x = ip[i];
                if (x >= 1 && (uint64_t)x <= nrows) {
                    const uint32_t key = r0 + (uint32_t)(x - 1);
                    uint32_t h = hot_hash(key);
                    for (;;) {
                        const uint32_t v = hk[h];
                        if (v == key + 1u) {
                            sv = hs[h];
                            break;
                        }
                        if (v == 0u) break;
                        h = (h + 1) & (kHotHash - 1);
                    }
                }
            }
            word |= sv << (8 * b);
        }
        out[e] = word;
    }
}

__global__ __launch_bounds__(256, 2) void k_sgd_hot(UpdatePack pack, HotList hl,
                                                    const uint32_t* __restrict__ hcnt,
                                                    const uint8_t* __restrict__ slots,
                                                    float2* __restrict__ part, int nw) {
    __shared__ float2 acc[kHotSlots][64];
    __shared__ float2 dl[kHotBatch][64];
    __shared__ uint32_t sl[kHotBatch * kHotMaxPool / 4];
    const int hi = blockIdx.y, t = hl.t[hi];
    const et_update_desc& d = pack.d[t];
    const int64_t B = d.batch;
    const int64_t b0 = (int64_t)blockIdx.x * kHotWin;
    const uint32_t H = hcnt[t];
    if (b0 >= B || H == 0) return;  // uniform
    const int64_t b1 = b0 + kHotWin < B ? b0 + kHotWin : B;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int P = d.pool, P4 = (P + 3) & ~3, W = P4 / 4;
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(slots + hl.soff[hi]);
    for (int i = tid; i < kHotSlots * 64; i += 256) acc[i >> 6][i & 63] = make_float2(0.0f, 0.0f);

    const float* delta = reinterpret_cast<const float*>(d.delta);
    const int64_t ldd = d.ld_delta;
    float2 rd[8];
    uint32_t rs;
    auto load = [&](int64_t bb) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int64_t b = bb + wv + 4 * k;
            rd[k] = b < b1 ? *reinterpret_cast<const float2*>(delta + b * ldd + 2 * lane)
                           : make_float2(0.0f, 0.0f);
        }
        // the batch's slot words: kHotBatch * W <= 256, one per thread
        rs = (tid < kHotBatch * W && bb + tid / W < b1) ? sw[bb * W + tid] : 0xffffffffu;
    };
    load(b0);
    for (int64_t bb = b0; bb < b1; bb += kHotBatch) {
        const int nbag = b1 - bb < kHotBatch ? (int)(b1 - bb) : kHotBatch;
        __syncthreads();  // the previous batch is processed
#pragma unroll
        for (int k = 0; k < 8; ++k) dl[wv + 4 * k][lane] = rd[k];
        if (tid < kHotBatch * W) sl[tid] = rs;
        __syncthreads();
        if (bb + kHotBatch < b1) load(bb + kHotBatch);
        for (int j = 0; j < nbag; ++j) {
            const float2 dv = dl[j][lane];
            for (int q = 0; q < W; ++q) {
                const uint32_t v = __builtin_amdgcn_readfirstlane(sl[j * W + q]);
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint32_t s = (v >> (8 * b)) & 0xffu;
                    if (s != 0xffu && (s & 3u) == (uint32_t)wv) {
                        float2 a = acc[s][lane];
                        a.x = a.x + dv.x;
                        a.y = a.y + dv.y;
                        acc[s][lane] = a;
                    }
                }
            }
        }
    }
    // window partials, slot-major: part[(hi*kHotSlots + s)*nw + window][64]
    for (uint32_t s = wv; s < H; s += 4)
        part[((uint64_t)(hi * kHotSlots + s) * nw + blockIdx.x) * 64 + lane] = acc[s][lane];
}

template <int MODE, bool NT>
__global__ __launch_bounds__(256) void k_hot_combine(UpdatePack pack, HotList hl,
                                                     const uint32_t* __restrict__ hcnt,
                                                     const uint32_t* __restrict__ hkey,
                                                     const float2* __restrict__ part, int nw,
                                                     float eta32, double eta64) {
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int hi = gw / kHotSlots, s = gw % kHotSlots;
    if (hi >= hl.n) return;
    const int t = hl.t[hi];
    if ((uint32_t)s >= hcnt[t]) return;
    const et_update_desc& d = pack.d[t];
    const int nwt = (int)((d.batch + kHotWin - 1) / kHotWin);
    const float2* p = part + (uint64_t)(hi * kHotSlots + s) * nw * 64 + lane;
    float ax = 0.0f, ay = 0.0f;
    for (int w0 = 0; w0 < nwt; w0 += 8) {
        float2 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = p[(uint64_t)(w0 + k < nwt ? w0 + k : nwt - 1) * 64];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (w0 + k < nwt) {
                ax = ax + v[k].x;
                ay = ay + v[k].y;
            }
    }
    const uint32_t key = hkey[t * kHotSlots + s];
    float* w = col_ptr<float>(d.table, d.ld_table, d.cols_per_page, key - pack.row_off[t]) + 2 * lane;
    store_scalar<NT>(w, sgd_apply<MODE>(w[0], ax, eta32, eta64));
    store_scalar<NT>(w + 1, sgd_apply<MODE>(w[1], ay, eta32, eta64));
}

// ---------------------------------------------------------------------------
// Exact Float32 update: serial chains (ET_FLAG_EXACT_UPDATE)
// ---------------------------------------------------------------------------
// The reference sums every distinct column's gradient serially in occurrence order
// (src/sparseupdate.jl:110-127: acc += delta[:, map[t]] for t in the column's range).
// Columns with at most kChunk occurrences are one chunk of the chunk pass, which is that
// serial sum already; the longer ("chain") columns — the multi-chunk list of the split
// mode — are summed by one wave per 64-feature slice walking the column's run-length
// list: a run of r occurrences in one bag adds the same delta column r times, so the
// index phase cuts every run into entries of at most S adds (S per column, the cheapest
// of 1/2/4/8/16 for its run lengths) and the wave spends exactly S masked fmas per entry
// in the hand-scheduled loop of et_chain_asm.h (no branch and no memory access per add
// beyond the delta load; tools/gen_chain_asm.py).  Same additions in the same order as
// the reference: bit-identical, and no partial sums to combine.
//
// Index phase, over tiles of kChainTile occurrences so a 834,828-occurrence column is
// cut by ~200 workgroups rather than walked by one wave: k_chain_tile_count/_fill (tiles per
// column), k_chain_tcount (per tile, the entries its runs make at each S), k_chain_choose
// (per column, S and the entry count), k_chain_plan (entry offsets; columns in key order, the
// early lists costliest first), k_chain_emit (the entries).  Update phase: the chain role of
// k_sgd_exact, beside the chunk pass (single-chunk columns) and the singles in ONE
// launch, so the hottest chains (834,828 adds on the config-4 batch) overlap the rest.

constexpr int kChainGroup = kChainAsmTrip;  // entries per trip of the asm loop
constexpr int kChainPad = kChainAsmPad;     // readable entries past the last trip
// Issue slots of one entry of a chain at S adds per entry, doubled (et_chain_asm.h: S = 1:
// readlane, address, load, half a wait and the add; S = 2, 4 (the 64-deep loop): two
// readlanes, address, load, half a wait, the mask's compare and select and S masked fmas;
// S = 8, 16 (the streamed loop): the mask's select, load, half a wait, 3/8 for the scalar
// loads and S masked fmas).
__host__ __device__ constexpr uint32_t chain_entry_cost2(uint32_t S) {
#ifdef ET_COST_OLD
    return S <= 1u ? 9u : S <= 4u ? 2u * S + 13u : 2u * S + 11u;
#else
    return S <= 1u ? 9u : S <= 4u ? 2u * S + 13u : 2u * S + 6u;
#endif
}

// A chain entry: r adds (r <= 16) of gradient column `bag`; padding is r = 0 at bag = batch
// (past the gradient: the chain loop's range-checked load returns +0).  The bag takes the low
// 24 bits (`r << 24 | bag`, the layout the Float32 asm and quad loops decode) when the table's
// batch is below 2^24, else the low 27 (`r << 27 | bag`, r <= 16 still fits the top 5 bits;
// read only by chain_walk_wide), so chains cover batches up to 2^27 - 1 bags.
constexpr int64_t kChainNarrowBatch = 1ll << 24;
constexpr int64_t kChainMaxBatch = (1ll << 27) - 1;
__host__ __device__ __forceinline__ uint32_t chain_shift(int64_t batch) {
    return batch < kChainNarrowBatch ? 24u : 27u;
}
__device__ __forceinline__ uint32_t chain_entry(uint32_t r, uint32_t bag, uint32_t sh) {
    return r << sh | bag;
}

// Whether a chain of a table with this gradient can take the hand-scheduled Float32 loops
// (et_chain_asm.h, chain_walk_quad): their gradient addresses are 32-bit byte offsets in one
// range-checked buffer — bag * ld * 4 + 4 * feature from 24-bit factors, and a padding entry
// (bag = batch) must land past the range to load +0 — so (batch + 1) * ld * 4 stays below
// 2^32 and ld below 2^22.  Any other chain takes chain_walk_wide (64-bit addresses).
__host__ __device__ inline bool chain_asm_ok(int64_t batch, int64_t ld) {
    return batch < kChainNarrowBatch && ld < (1ll << 22) &&
           (uint64_t)(batch + 1) * (uint64_t)ld * 4u < (1ull << 32);
}

// The streamed loop's gradient stride in bytes for a chain at S of a table with this gradient,
// 0 when the chain does not take it (the index phase then writes no offsets / masks).
__host__ __device__ inline uint32_t chain_stream_ld4(int64_t batch, int64_t ld, uint32_t S) {
    return S >= (uint32_t)kChainStreamMinS && chain_asm_ok(batch, ld) ? (uint32_t)ld * 4u : 0u;
}

struct ChainCol {
    uint32_t key, e0, ngr, S;  // S == 0: no chain (out-of-range occurrences)
};

// A chain list's entries and, for the streamed Float32 loop (S >= kChainStreamMinS on a
// table chain_asm_ok admits, et_chain_asm.h chain_walk_stream), per entry its gradient byte
// offset bag * ld * 4 and its lane mask (2^r - 1 in each 16-lane row), at the same index.
struct ChainEnt {
    uint32_t* ent;
    uint32_t* off;
    uint64_t* msk;
};

__device__ __forceinline__ uint32_t cdiv_u32(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}

__device__ __forceinline__ uint32_t wave_excl_scan_u32(uint32_t v, int lane) {
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)x, o, 64);
        if (lane >= o) x += t;
    }
    return x - v;
}

constexpr uint32_t kChainTile = 4096;  // occurrences per index-phase tile
constexpr uint32_t kChainTileItems = 16;  // consecutive occurrences per thread in the
                                           // entry scan (x 256)

// A tile's bags in LDS: slot 0 the bag of the occurrence before the tile (~0 at the
// column's start), slots 1..kChainTile the tile's, then kChainHalo past its end (~0 past
// the column's end), so a run that starts in the tile is followed from LDS unless it is
// longer than the halo.  Occurrences are sorted by position inside the column (stable
// sort), and bag = (position - occ_off) / pool.
constexpr uint32_t kChainHalo = 64;
constexpr uint32_t kChainLds = kChainTile + 1 + kChainHalo;

__device__ __forceinline__ void stage_bags(uint32_t* __restrict__ bags,
                                           const uint32_t* __restrict__ vals, uint32_t ss,
                                           uint32_t se, uint32_t a, uint32_t occ_off,
                                           uint32_t pool) {
    for (uint32_t i = threadIdx.x; i < kChainLds; i += blockDim.x) {
        const uint32_t p = a - 1u + i;  // wraps to ~0 only when a == 0 (then p < ss fails)
        bags[i] = (i > 0 || a > ss) && p < se ? (vals[p] - occ_off) / pool : 0xffffffffu;
    }
}

// Length of the run of equal bags starting at LDS slot i (a head, 1 <= i <= kChainTile),
// followed into global memory past the halo.
__device__ __forceinline__ uint32_t run_length(const uint32_t* __restrict__ bags, uint32_t i,
                                               const uint32_t* __restrict__ vals, uint32_t se,
                                               uint32_t a, uint32_t occ_off, uint32_t pool) {
    const uint32_t b = bags[i];
    uint32_t q = i + 1;
    while (q < kChainLds && bags[q] == b) ++q;
    if (q == kChainLds)
        while (a - 1u + q < se && (vals[a - 1u + q] - occ_off) / pool == b) ++q;
    return q - i;
}

// A tile's place: its column m, the column's occurrence range, the tile's first
// occurrence, its index among the column's tiles and their count, and the table — one
// 32-byte record per tile, written by k_chain_tile_fill (so k_chain_tcount / k_chain_emit
// read one record instead of following tile -> column -> segment -> key -> table, five
// dependent loads per tile beside the chunk pass).
struct ChainTile {
    uint32_t m, ss, se, a, ti, nt;
    int t;  // table
    uint32_t pad;
};
static_assert(sizeof(ChainTile) == 32, "tile record");

__device__ __forceinline__ ChainTile chain_tile(const ChainTile* __restrict__ recs, uint32_t tile) {
    const uint4* p = reinterpret_cast<const uint4*>(recs + tile);
    const uint4 x = p[0], y = p[1];
    ChainTile c;
    c.m = x.x;
    c.ss = x.y;
    c.se = x.z;
    c.a = x.w;
    c.ti = y.x;
    c.nt = y.y;
    c.t = (int)y.z;
    c.pad = 0u;
    return c;
}

// Inclusive scan of one value per thread over a workgroup of NW waves.
template <int NW = 16>
__device__ __forceinline__ uint32_t block_inclusive_scan(uint32_t v, uint32_t* lds16,
                                                         uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = (uint32_t)__shfl_up((int)v, o, 64);
        if (lane >= o) v += t;
    }
    if (lane == 63) lds16[wave] = v;
    __syncthreads();
    uint32_t off = 0, all = 0;
    for (int w = 0; w < NW; ++w) {
        off += w < wave ? lds16[w] : 0u;
        all += lds16[w];
    }
    *total = all;
    __syncthreads();
    return v + off;
}

// The one-workgroup step of the regular chains' plan (k_chain_plan) runs at 256 threads: it
// is launched beside the chunk pass, whose persistent workgroups leave each CU a few wave
// slots but never the 16 a 1024-thread workgroup needs (round 4's 1024-thread tile pass waited
// 0.73 ms for a CU, profiles/r05/capture/timeline_none.txt).
constexpr int kPlanThreads = 256;

// The early hot-column candidates of the big tables (ET_EH, see EcList below): kEhK
// ascending columns per table, ~0 past the last; EhMap says which tables have a list and
// where it is.
constexpr int kEhK = 16;  // candidate columns per table
struct EhMap {
    uint32_t mask;                      // bit t: table t has a candidate list
    int8_t e[ET_MAX_TABLES_PER_LAUNCH];  // its entry: the list at cand + e * kEhK
};

// Slot of column c in a table's ascending candidate list (kEhK entries, ~0 = empty), or -1.
__device__ __forceinline__ int eh_slot(const uint32_t* cand, uint32_t c) {
    int lo = 0, hi = kEhK;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cand[mid] < c) lo = mid + 1;
        else hi = mid;
    }
    return lo < kEhK && cand[lo] == c ? lo : -1;
}

// Index phase 1a (grid): tiles per chain column into tile0[m] (none for the out-of-range
// sentinel column, nor for the columns of early-chain tables, ec_mask, nor for the early
// hot-column candidates, eh: those chains are planned from the index arrays, k_ec_*), and
// tile0[M] = 0, ready for the exclusive scan that makes tile0 each column's first tile.
__global__ __launch_bounds__(256) void k_chain_tile_count(UpdatePack pack, int ntables,
                                                          uint32_t ec_mask, EhMap eh,
                                                          const uint32_t* __restrict__ cand,
                                                          const uint32_t* __restrict__ keys,
                                                          const uint32_t* __restrict__ seg_start,
                                                          const uint32_t* __restrict__ mlist,
                                                          const uint32_t* __restrict__ counters,
                                                          uint32_t sent,
                                                          uint32_t* __restrict__ tile0) {
    __shared__ uint32_t sc[ET_MAX_TABLES_PER_LAUNCH * kEhK];  // the candidate lists
    const uint32_t M = counters[kCntM];
    if (eh.mask) {
        const int ne = __popc(eh.mask);
        for (int i = threadIdx.x; i < ne * kEhK; i += 256) sc[i] = cand[i];
        __syncthreads();
    }
    for (uint32_t m = blockIdx.x * 256 + threadIdx.x; m <= M; m += gridDim.x * 256) {
        uint32_t v = 0;
        if (m < M) {
            const uint32_t u = mlist[m], ss = seg_start[u], se = seg_start[u + 1];
            const uint32_t k0 = keys[ss];
            const int t = k0 == sent ? 0 : table_of_key(pack, ntables, k0);
            const bool early = k0 == sent || ((ec_mask >> t) & 1u) ||
                               (((eh.mask >> t) & 1u) &&
                                eh_slot(sc + eh.e[t] * kEhK, k0 - pack.row_off[t]) >= 0);
            v = early ? 0u : cdiv_u32(se - ss, kChainTile);
        }
        tile0[m] = v;
    }
}

// Index phase 1b (grid, after the exclusive scan of tile0): the tile records (ChainTile)
// and the tile total (counters[kCntT] = tile0[M]).
__global__ __launch_bounds__(256) void k_chain_tile_fill(UpdatePack pack, int ntables,
                                                         const uint32_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ seg_start,
                                                         const uint32_t* __restrict__ mlist,
                                                         const uint32_t* __restrict__ tile0,
                                                         uint32_t* __restrict__ counters,
                                                         ChainTile* __restrict__ recs) {
    const uint32_t M = counters[kCntM];
    if (blockIdx.x == 0 && threadIdx.x == 0) counters[kCntT] = tile0[M];
    for (uint32_t m = blockIdx.x * 256 + threadIdx.x; m < M; m += gridDim.x * 256) {
        const uint32_t t0 = tile0[m], t1 = tile0[m + 1];
        if (t0 == t1) continue;
        const uint32_t u = mlist[m], ss = seg_start[u], se = seg_start[u + 1];
        const uint32_t t = (uint32_t)table_of_key(pack, ntables, keys[ss]);
        for (uint32_t k = t0; k < t1; ++k) {
            uint4* p = reinterpret_cast<uint4*>(recs + k);
            p[0] = make_uint4(m, ss, se, ss + (k - t0) * kChainTile);
            p[1] = make_uint4(k - t0, t1 - t0, t, 0u);
        }
    }
}

// Index phase 2: per tile, the entries its runs make at S = 1, 2, 4, 8, 16.
__global__ __launch_bounds__(256) void k_chain_tcount(UpdatePack pack, int ntables,
                                                      const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ vals,
                                                      const uint32_t* __restrict__ seg_start,
                                                      const uint32_t* __restrict__ mlist,
                                                      const uint32_t* __restrict__ counters,
                                                      const uint32_t* __restrict__ tile0,
                                                      const ChainTile* __restrict__ trec,
                                                      uint32_t* __restrict__ tcnt) {
    __shared__ uint32_t bags[kChainLds];
    __shared__ uint32_t red[4][5];
    const uint32_t M = counters[kCntM], T = counters[kCntT];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t tile = blockIdx.x; tile < T; tile += gridDim.x) {
        const ChainTile c = chain_tile(trec, tile);
        const uint32_t occ_off = pack.occ_off[c.t], pool = (uint32_t)pack.d[c.t].pool;
        const uint32_t n = c.a + kChainTile < c.se ? kChainTile : c.se - c.a;
        stage_bags(bags, vals, c.ss, c.se, c.a, occ_off, pool);
        __syncthreads();
        uint32_t E[5] = {0u, 0u, 0u, 0u, 0u};
        for (uint32_t i = 1 + threadIdx.x; i <= n; i += 256) {
            if (bags[i] == bags[i - 1]) continue;
            const uint32_t r = run_length(bags, i, vals, c.se, c.a, occ_off, pool);
#pragma unroll
            for (int k = 0; k < 5; ++k) E[k] += cdiv_u32(r, 1u << k);
        }
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint32_t v = wave_sum_u32(E[k]);
            if (lane == 0) red[wave][k] = v;
        }
        __syncthreads();
        if (threadIdx.x < 5)
            tcnt[5 * tile + threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x] +
                                           red[2][threadIdx.x] + red[3][threadIdx.x];
        __syncthreads();  // bags and red are reused by the next tile
    }
}

// Index phase 3: per chain column (one wave), S minimising entries x (S + per-entry
// overhead), and the padded entry count; (S, entries) in info.  A column without tiles
// (the sentinel) gets S = 0: no chain.
__global__ __launch_bounds__(256) void k_chain_choose(const uint32_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ seg_start,
                                                      const uint32_t* __restrict__ mlist,
                                                      const uint32_t* __restrict__ counters,
                                                      const uint32_t* __restrict__ tile0,
                                                      const uint32_t* __restrict__ tcnt,
                                                      uint32_t* __restrict__ cnt,
                                                      uint2* __restrict__ info,
                                                      ChainCol* __restrict__ chains,
                                                      int kmax) {
    const uint32_t M = counters[kCntM], T = counters[kCntT];
    const int lane = threadIdx.x & 63;
    for (uint32_t m = blockIdx.x * 4 + (threadIdx.x >> 6); m < M; m += gridDim.x * 4) {
        const uint32_t t0 = tile0[m], nt = (m + 1 < M ? tile0[m + 1] : T) - t0;
        if (nt == 0) {
            if (lane == 0) {
                cnt[m] = 0u;
                info[m] = make_uint2(0u, 0u);
                chains[m] = ChainCol{keys[seg_start[mlist[m]]], 0u, 0u, 0u};
            }
            continue;
        }
        uint32_t E[5] = {0u, 0u, 0u, 0u, 0u};
        for (uint32_t i = (uint32_t)lane; i < nt; i += 64)
#pragma unroll
            for (int k = 0; k < 5; ++k) E[k] += tcnt[5 * (t0 + i) + k];
        int best = 0;
        uint64_t bc = ~0ull;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            E[k] = wave_sum_u32(E[k]);
            const uint64_t c = (uint64_t)E[k] * chain_entry_cost2(1u << k);
            if (k <= kmax && c < bc) bc = c, best = k;  // kmax: the largest log2 S
        }
        if (lane == 0) {
            cnt[m] = cdiv_u32(E[best], kChainGroup) * kChainGroup + kChainPad;
            info[m] = make_uint2(1u << best, E[best]);
        }
    }
}

// Index phase 4 (one workgroup): entry offsets (exclusive scan of the padded counts) and the
// dispatch order — key order (table-major, ascending column), so the chains running at any
// moment read the gradient rows of few tables and those stay in the Infinity Cache: config 4
// 3.76-3.81 ms against 3.85-3.87 for round 4's costliest-first order (one box, A/B,
// profiles/r05/exact_grid/ab_r05o.txt; the early lists keep costliest-first — in key order
// their hottest chains start late: 4.01 / 4.70 ms).  The counts come kPlanU x 256 at a time
// (coalesced, all loads issued before the first scan).
constexpr int kPlanU = 8;

__global__ __launch_bounds__(kPlanThreads) void k_chain_plan(const uint32_t* __restrict__ counters,
                                                     const uint32_t* __restrict__ cnt,
                                                     uint32_t* __restrict__ e0,
                                                     uint32_t* __restrict__ order) {
    __shared__ uint32_t lds16[16];
    const uint32_t M = counters[kCntM];
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < M; b0 += kPlanThreads * kPlanU) {
        uint32_t v[kPlanU];
#pragma unroll
        for (int u = 0; u < kPlanU; ++u) {
            const uint32_t m = b0 + (uint32_t)u * kPlanThreads + threadIdx.x;
            v[u] = m < M ? cnt[m] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kPlanU; ++u) {
            const uint32_t m = b0 + (uint32_t)u * kPlanThreads + threadIdx.x;
            uint32_t total;
            const uint32_t inc = block_inclusive_scan<kPlanThreads / 64>(v[u], lds16, &total);
            if (m < M) {
                e0[m] = carry + inc - v[u];
                order[m] = m;
            }
            carry += total;
        }
    }
}

// One run of r adds of delta column `bag` as ceil(r/S) entries (S adds each, the last
// one the remainder); with `ld4` (nonzero: the chain takes the streamed loop) also the
// entry's gradient offset and lane mask.
__device__ __forceinline__ uint64_t chain_lane_mask(uint32_t adds) {
    return (uint64_t)((1u << adds) - 1u) * 0x0001000100010001ull;
}
__device__ __forceinline__ void chain_put(const ChainEnt& ce, uint32_t at, uint32_t i,
                                          uint32_t k, uint32_t r, uint32_t S, uint32_t bag,
                                          uint32_t sh, uint32_t ld4) {
    const uint32_t adds = i + 1 < k ? S : r - S * (k - 1);
    ce.ent[at] = chain_entry(adds, bag, sh);
    if (ld4) {
        ce.off[at] = bag * ld4;
        ce.msk[at] = chain_lane_mask(adds);
    }
}
// A padding entry (no adds, bag = batch: its loads return +0).
__device__ __forceinline__ void chain_pad(const ChainEnt& ce, uint32_t at, uint32_t batch,
                                          uint32_t sh, uint32_t ld4) {
    ce.ent[at] = chain_entry(0u, batch, sh);
    if (ld4) {
        ce.off[at] = batch * ld4;
        ce.msk[at] = 0ull;
    }
}

// Index phase 5, per tile: the entries of the runs that start in it (after the entries
// of the column's earlier tiles at the column's S, in occurrence order); the column's
// last tile pads the entries with zeros (no adds) to the planned count and writes the
// column's descriptor.  Runs are found on the LDS-staged bags (coalesced), their entry
// offsets by a block scan over 16 consecutive occurrences per thread.
__global__ __launch_bounds__(256) void k_chain_emit(UpdatePack pack, int ntables,
                                                    const uint32_t* __restrict__ keys,
                                                    const uint32_t* __restrict__ vals,
                                                    const uint32_t* __restrict__ seg_start,
                                                    const uint32_t* __restrict__ mlist,
                                                    const uint32_t* __restrict__ counters,
                                                    const uint32_t* __restrict__ tile0,
                                                    const ChainTile* __restrict__ trec,
                                                    const uint32_t* __restrict__ tcnt,
                                                    const uint32_t* __restrict__ cnt,
                                                    const uint2* __restrict__ info,
                                                    const uint32_t* __restrict__ e0s,
                                                    ChainEnt ce,
                                                    ChainCol* __restrict__ chains) {
    __shared__ uint32_t bags[kChainLds];
    __shared__ uint32_t rl[kChainTile];  // run length at a head, 0 elsewhere
    __shared__ uint32_t red[2][4];
    const uint32_t M = counters[kCntM], T = counters[kCntT];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t tile = blockIdx.x; tile < T; tile += gridDim.x) {
        const ChainTile c = chain_tile(trec, tile);
        const uint2 in = info[c.m];
        const uint32_t S = in.x, kS = (uint32_t)(__ffs((int)S) - 1);
        const uint32_t occ_off = pack.occ_off[c.t], pool = (uint32_t)pack.d[c.t].pool;
        const uint32_t sh = chain_shift(pack.d[c.t].batch);
        const uint32_t ld4 = chain_stream_ld4(pack.d[c.t].batch, pack.d[c.t].ld_delta, S);
        const uint32_t n = c.a + kChainTile < c.se ? kChainTile : c.se - c.a;
        stage_bags(bags, vals, c.ss, c.se, c.a, occ_off, pool);
        __syncthreads();
        for (uint32_t i = 1 + threadIdx.x; i <= kChainTile; i += 256)
            rl[i - 1] = i <= n && bags[i] != bags[i - 1]
                            ? run_length(bags, i, vals, c.se, c.a, occ_off, pool) : 0u;
        // entries of the column's earlier tiles, and of this thread's 16 occurrences
        uint32_t before = 0, mine = 0;
        const uint32_t t0 = tile - c.ti;
        for (uint32_t i = threadIdx.x; i < c.ti; i += 256) before += tcnt[5 * (t0 + i) + kS];
        __syncthreads();
        const uint32_t j0 = threadIdx.x * kChainTileItems;
#pragma unroll
        for (uint32_t j = 0; j < kChainTileItems; ++j) mine += cdiv_u32(rl[j0 + j], S);
        before = wave_sum_u32(before);
        const uint32_t pre = wave_excl_scan_u32(mine, lane);
        if (lane == 63) red[0][wave] = pre + mine;
        if (lane == 0) red[1][wave] = before;
        __syncthreads();
        uint32_t at = e0s[c.m] + red[1][0] + red[1][1] + red[1][2] + red[1][3] + pre;
        for (int w = 0; w < wave; ++w) at += red[0][w];
        for (uint32_t j = 0; j < kChainTileItems; ++j) {
            const uint32_t r = rl[j0 + j];
            if (r == 0u) continue;
            const uint32_t k = cdiv_u32(r, S), bag = bags[j0 + j + 1];
            for (uint32_t i = 0; i < k; ++i) chain_put(ce, at + i, i, k, r, S, bag, sh, ld4);
            at += k;
        }
        if (c.ti + 1 == c.nt) {
            const uint32_t e0 = e0s[c.m], P = cnt[c.m];
            for (uint32_t i = e0 + in.y + threadIdx.x; i < e0 + P; i += 256)
                chain_pad(ce, i, (uint32_t)pack.d[c.t].batch, sh, ld4);
            if (threadIdx.x == 0)
                chains[c.m] = ChainCol{keys[c.ss], e0, (P - kChainPad) / kChainGroup, S};
        }
        __syncthreads();  // bags, rl and red are reused by the next tile
    }
}

// Debug check of the chain plan (ET_CHAIN_CHECK=1): every entry of every chain addresses
// a gradient column of its table's batch with at most S adds, the entries carrying
// adds number exactly E and precede the padding; a violation is counted in the device
// error word (et_check_errors) as 1 << 20 and the entry neutralised to 0.
__global__ __launch_bounds__(256) void k_chain_check(UpdatePack pack, int ntables,
                                                     const uint32_t* __restrict__ counters,
                                                     const uint32_t* __restrict__ cnt,
                                                     const uint2* __restrict__ info,
                                                     ChainEnt ce,
                                                     const ChainCol* __restrict__ chains,
                                                     const uint32_t* __restrict__ order) {
    const uint32_t M = counters[kCntM];
    const int lane = threadIdx.x & 63;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < M; i += gridDim.x * 256)
        if (order[i] >= M) note_oob(1 << 22);
    for (uint32_t m = blockIdx.x * 4 + (threadIdx.x >> 6); m < M; m += gridDim.x * 4) {
        const ChainCol c = chains[m];
        const uint32_t P = cnt[m];
        if (c.S == 0u) continue;
        const int t = table_of_key(pack, ntables, c.key);
        const uint64_t lim = (uint64_t)pack.d[t].batch;
        const uint32_t sh = chain_shift(pack.d[t].batch), bm = (1u << sh) - 1u;
        const uint32_t ld4 = chain_stream_ld4(pack.d[t].batch, pack.d[t].ld_delta, c.S);
        uint32_t bad = 0, real = 0, pad_then_real = 0;
        if (P != c.ngr * kChainGroup + kChainPad || c.S != info[m].x) bad = 1;
        for (uint32_t i = lane; i < P; i += 64) {
            const uint32_t e = ce.ent[c.e0 + i], r = e >> sh;
            bool ok = ((uint64_t)(e & bm) < lim || (r == 0u && (e & bm) == lim)) && r <= c.S;
            if (ld4)  // the streamed loop's offset and mask say the same as the entry
                ok = ok && ce.off[c.e0 + i] == (e & bm) * ld4 &&
                     ce.msk[c.e0 + i] == (r ? chain_lane_mask(r) : 0ull);
            // a bad entry becomes a padding entry (bag = batch: its range-checked load
            // returns +0), so the debug pass reports the violation without adding
            // gradient column 0 in its place (maskless S = 1 and quad walks add every entry)
            if (!ok) chain_pad(ce, c.e0 + i, (uint32_t)lim, sh, ld4);
            bad += ok ? 0u : 1u;
            real += (ok && r > 0u) ? 1u : 0u;
            pad_then_real += (ok && r > 0u && i >= info[m].y) ? 1u : 0u;
        }
        bad = wave_sum_u32(bad) + wave_sum_u32(pad_then_real);
        real = wave_sum_u32(real);
        if (lane == 0 && (bad || real != info[m].y)) note_oob(1 << 20);
    }
}

// Early chains.  The longest chains of a Zipf batch belong to the smallest tables (the
// 3-row Criteo table's hottest column has 835 K occurrences: a ~3 ms chain), and a chain
// planned from the sorted pairs cannot start before the whole index phase (~1 ms).  For a
// table of at most kEcMaxRows rows the chains are planned straight from its index array,
// on a side stream from the start of the call: the occurrences of column c in bag b are
// a run of r(c, b) equal bags in the column's sorted list (the sort is stable and bags
// are contiguous), so the column's entries are, in bag order, ceil(r / S) entries per
// bag with r > 0 — the same entries k_chain_emit would cut from the sorted list.  Which
// columns are chains (more than `chunk` occurrences) is decided from the same counts
// (occurrences in [1, nrows]), so the main index phase skips exactly these columns
// (k_chain_tile_count) and the chunk pass never sees them (they are multi-chunk).
constexpr int kEcMaxRows = 128;  // tables with at most this many rows
constexpr int kEcBags = 256;     // bags per workgroup of k_ec_count / k_ec_emit
constexpr int kEcMaxPool = 255;  // per-bag counts fit a byte
constexpr int kEcMaxBatch = 1 << 20;
constexpr int kEcStats = 8;      // per (column, block): occurrences, entries at S = 1..16

// Early HOT columns of the larger tables (round 4, ET_EH): every table of more than
// kEcMaxRows rows gets kEhK "slots" — the columns a sample of its first kEhSampleBags bags
// finds hottest (k_eh_pick: at least kEhMinOcc occurrences expected over the batch, at most
// kEhK per table, ascending column order) — planned as early chains of their own (a second
// EcList, hot = 1, on a third side stream), so the big tables' longest chains start with
// the call instead of after the sort.  The slots are counted, planned and emitted by the
// same k_ec_* kernels (a bag's indices are matched against the table's candidate list); a
// candidate with more than `chunk` occurrences is a chain there, and the regular plan skips
// it (k_chain_tile_count), so every column is summed exactly once.
constexpr int kEhSampleBags = 1024;     // bags sampled by k_eh_pick
constexpr uint32_t kEhMinOcc = 32768;   // expected occurrences of a candidate (ET_EH_MIN)
constexpr int kEhHash = 4096;           // LDS hash slots of the sample count
constexpr int kEhProbes = 16;           // linear probes per occurrence

struct EcList {
    int n;                                        // early-chain tables
    uint32_t mask;                                // bit t: table t is one of them
    int hot;                                      // 1: kEhK candidate slots per table (EH)
    int t[ET_MAX_TABLES_PER_LAUNCH];              // their table indices
    uint32_t blk0[ET_MAX_TABLES_PER_LAUNCH + 1];  // prefix of bag blocks
    uint32_t col0[ET_MAX_TABLES_PER_LAUNCH + 1];  // prefix of nrows / kEhK (EC columns)
    uint32_t cb0[ET_MAX_TABLES_PER_LAUNCH + 1];   // prefix of blocks x columns (stat records)
};

inline bool ec_table(const et_update_desc& d) {
    return d.nrows > 0 && d.nrows <= kEcMaxRows && d.pool > 0 && d.pool <= kEcMaxPool &&
           d.batch > 0 && d.batch <= kEcMaxBatch && d.dim > 0;
}

inline bool eh_table(const et_update_desc& d) {
    return d.nrows > kEcMaxRows && d.nrows < (1ll << 31) && d.pool > 0 &&
           d.pool <= kEcMaxPool && d.batch > 0 && d.batch <= kEcMaxBatch && d.dim > 0;
}

// On by default: config-4 exact update 4.05-4.06 ms with, 4.24-4.25 without (the exact
// grid cap on, A/B twice on one box, profiles/r04/ab_exact_grid.txt).
inline bool eh_enabled() { return ET_KNOB("ET_EH", 1) != 0; }

// One workgroup per EH entry: count the sampled bags' columns in an LDS hash table, keep the
// columns expected to reach kEhMinOcc occurrences, at most kEhK of them (the most frequent;
// ties to the smaller column), and write them in ascending order, ~0 past the last.
__global__ __launch_bounds__(1024) void k_eh_pick(UpdatePack pack, EcList ec, uint32_t min_occ,
                                                  int64_t sample_bags,
                                                  uint32_t* __restrict__ cand) {
    __shared__ uint32_t hk[kEhHash], hc[kEhHash];
    __shared__ uint32_t qk[512], qc[512], nq;
    __shared__ uint32_t sel[kEhK], nsel;
    const int e = blockIdx.x;
    const et_update_desc& d = pack.d[ec.t[e]];
    for (int i = threadIdx.x; i < kEhHash; i += 1024) hk[i] = ~0u, hc[i] = 0u;
    if (threadIdx.x == 0) nq = 0u, nsel = 0u;
    __syncthreads();
    const int64_t nb = d.batch < sample_bags ? d.batch : sample_bags;
    const int64_t nocc = nb * d.pool;
    // kEhPickU index loads in flight per thread before the hash updates (round 4 loaded one
    // index per hash update: 20 dependent rounds of memory latency, 214 us beside the index phase)
    constexpr int kEhPickU = 5;
    for (int64_t o0 = threadIdx.x; o0 < nocc; o0 += 1024 * kEhPickU) {
        uint64_t cs[kEhPickU];
#pragma unroll
        for (int u = 0; u < kEhPickU; ++u) {
            const int64_t o = o0 + 1024 * u;
            const int64_t b = o / d.pool, j = o - b * d.pool;
            cs[u] = o < nocc ? (uint64_t)(d.idx[b * d.ld_idx + j] - 1) : ~0ull;
        }
#pragma unroll
        for (int u = 0; u < kEhPickU; ++u) {
            const uint64_t c = cs[u];
            if (c >= (uint64_t)d.nrows) continue;
            uint32_t h = ((uint32_t)c * 2654435761u) >> 20;  // 12 bits
            for (int probe = 0; probe < kEhProbes; ++probe, h = (h + 1) & (kEhHash - 1)) {
                // the hot columns' slots are taken early: a plain read finds them without a CAS
                const uint32_t seen = hk[h];
                const uint32_t prev =
                    seen == (uint32_t)c ? seen : atomicCAS(&hk[h], ~0u, (uint32_t)c);
                if (prev == ~0u || prev == (uint32_t)c) {
                    atomicAdd(&hc[h], 1u);
                    break;
                }
            }  // a crowded neighbourhood drops the occurrence: the sample only ranks columns
        }
    }
    __syncthreads();
    // expected total >= min_occ  <=>  sample count * batch >= min_occ * nb
    for (int i = threadIdx.x; i < kEhHash; i += 1024)
        if (hk[i] != ~0u && (uint64_t)hc[i] * (uint64_t)d.batch >= (uint64_t)min_occ * (uint64_t)nb) {
            const uint32_t q = atomicAdd(&nq, 1u);
            if (q < 512) qk[q] = hk[i], qc[q] = hc[i];
        }
    __syncthreads();
    const uint32_t Q = nq < 512 ? nq : 512u;
    if (threadIdx.x < Q) {  // rank by (count desc, column asc)
        const uint32_t k = qk[threadIdx.x], n = qc[threadIdx.x];
        uint32_t r = 0;
        for (uint32_t i = 0; i < Q; ++i) r += qc[i] > n || (qc[i] == n && qk[i] < k);
        if (r < (uint32_t)kEhK) sel[atomicAdd(&nsel, 1u)] = k;
    }
    __syncthreads();
    const uint32_t S = nsel;
    if (threadIdx.x < kEhK) {  // ascending column order
        uint32_t v = ~0u;
        if (threadIdx.x < S) {
            const uint32_t k = sel[threadIdx.x];
            uint32_t r = 0;
            for (uint32_t i = 0; i < S; ++i) r += sel[i] < k;
            v = k;
            cand[e * kEhK + r] = v;
        }
        if (threadIdx.x >= S) cand[e * kEhK + threadIdx.x] = ~0u;
    }
}

// Per-bag column counts in LDS: row `b` (bag blk * kEcBags + b) holds r(c, bag) for the
// table's R <= kEcMaxRows columns, one byte each (out-of-range indices are not counted; the
// main index phase reports them).  The block's indices are read flat — occurrence o of the
// block is bag o / pool, position o % pool: coalesced, kEcHistU loads in flight per thread —
// and counted with packed LDS atomics (a byte never carries: r <= pool <= 255).  (Round 4
// walked one bag per thread, its pool loads one after another: k_ec_count 162 us on the EC
// list and 202 us on the EH list beside the index phase.)
constexpr int kEcHistU = 8;

__device__ __forceinline__ void ec_hist(const et_update_desc& d, uint32_t blk, uint8_t* hist,
                                        uint32_t RS, const uint32_t* cand = nullptr) {
    const uint32_t R = (uint32_t)d.nrows, pool = (uint32_t)d.pool;
    uint32_t* h32 = reinterpret_cast<uint32_t*>(hist);
    for (uint32_t i = threadIdx.x; i < (uint32_t)kEcBags * RS / 4u; i += kEcBags) h32[i] = 0u;
    __syncthreads();
    const int64_t b0 = (int64_t)blk * kEcBags;
    const int64_t left = d.batch - b0;
    const uint32_t nb = (uint32_t)(left < kEcBags ? left : kEcBags);
    const uint32_t nocc = nb * pool;
    const int64_t* base = d.idx + b0 * d.ld_idx;
    const int64_t ldi = d.ld_idx;
    for (uint32_t o0 = threadIdx.x; o0 < nocc; o0 += kEcHistU * kEcBags) {
        int64_t v[kEcHistU];
#pragma unroll
        for (int u = 0; u < kEcHistU; ++u) {
            const uint32_t o = o0 + (uint32_t)u * kEcBags;
            const uint32_t b = o / pool;
            v[u] = o < nocc ? base[(int64_t)b * ldi + (o - b * pool)] : 0;  // 0: not counted
        }
#pragma unroll
        for (int u = 0; u < kEcHistU; ++u) {
            const uint32_t o = o0 + (uint32_t)u * kEcBags;
            const uint64_t c = (uint64_t)(v[u] - 1);
            if (c < R) {
                const int slot = cand ? eh_slot(cand, (uint32_t)c) : (int)c;  // EH: candidates
                if (slot >= 0) {
                    const uint32_t at = (o / pool) * RS + (uint32_t)slot;
                    atomicAdd(&h32[at >> 2], 1u << (8u * (at & 3u)));
                }
            }
        }
    }
    __syncthreads();
}

// An EH entry's candidate list in LDS (the k_ec_* kernels' slot map), or nullptr.
__device__ __forceinline__ const uint32_t* eh_stage(const EcList& ec, int e,
                                                    const uint32_t* __restrict__ cand,
                                                    uint32_t* lds) {
    if (!ec.hot) return nullptr;
    if (threadIdx.x < kEhK) lds[threadIdx.x] = cand[e * kEhK + threadIdx.x];
    __syncthreads();
    return lds;
}

__device__ __forceinline__ int ec_find(const EcList& ec, uint32_t blk) {
    int e = 0;
    while (e + 1 < ec.n && blk >= ec.blk0[e + 1]) ++e;
    return e;
}

// The columns of a block are summed by "parts": thread (c, p) = (tid % R, tid / R) walks
// bags [p * len, (p + 1) * len) of the block for column c (nparts = kEcBags / R >= 2).
struct EcParts {
    uint32_t R, RS, nparts, len, c, p, b0, b1;
    bool on;
};

__device__ __forceinline__ EcParts ec_parts(uint32_t R) {
    EcParts q;
    q.R = R;
    q.RS = (R + 3u) & ~3u;
    q.nparts = (uint32_t)kEcBags / R;
    q.len = cdiv_u32((uint32_t)kEcBags, q.nparts);
    q.on = threadIdx.x < q.nparts * R;
    q.c = threadIdx.x % R;
    q.p = threadIdx.x / R;
    q.b0 = q.on ? q.p * q.len : 0u;
    const uint32_t e = q.b0 + q.len;
    q.b1 = q.on ? (e < (uint32_t)kEcBags ? e : (uint32_t)kEcBags) : 0u;
    return q;
}

// EC step 1, one workgroup per (table, block of kEcBags bags): per column, its occurrences
// in the block and the entries they make at S = 1, 2, 4, 8, 16.
__global__ __launch_bounds__(256) void k_ec_count(UpdatePack pack, EcList ec,
                                                  uint32_t* __restrict__ stats,
                                                  const uint32_t* __restrict__ cand) {
    extern __shared__ __attribute__((aligned(16))) uint8_t hist[];  // kEcBags x ec_rs(ec)
    __shared__ uint32_t red[kEcBags][6];
    __shared__ uint32_t sc[kEhK];
    const int e = ec_find(ec, blockIdx.x);
    const et_update_desc& d = pack.d[ec.t[e]];
    const uint32_t blk = blockIdx.x - ec.blk0[e];
    const uint32_t nblk = ec.blk0[e + 1] - ec.blk0[e];
    const EcParts q = ec_parts(ec.col0[e + 1] - ec.col0[e]);
    ec_hist(d, blk, hist, q.RS, eh_stage(ec, e, cand, sc));
    uint32_t v[6] = {0u, 0u, 0u, 0u, 0u, 0u};
    for (uint32_t i = q.b0; i < q.b1; ++i) {
        const uint32_t r = hist[i * q.RS + q.c];
        v[0] += r;
#pragma unroll
        for (int k = 0; k < 5; ++k) v[1 + k] += (r + (1u << k) - 1u) >> k;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) red[threadIdx.x][k] = v[k];
    __syncthreads();
    if (threadIdx.x < q.R) {
        uint32_t s6[6] = {0u, 0u, 0u, 0u, 0u, 0u};
        for (uint32_t p = 0; p < q.nparts; ++p)
#pragma unroll
            for (int k = 0; k < 6; ++k) s6[k] += red[p * q.R + threadIdx.x][k];
        uint32_t* o = stats + (uint64_t)(ec.cb0[e] + threadIdx.x * nblk + blk) * kEcStats;
#pragma unroll
        for (int k = 0; k < 6; ++k) o[k] = s6[k];
    }
}

// EC step 2, one wave per column: the totals, whether it is a chain (more than `chunk`
// occurrences), its S (as k_chain_choose), padded entry count, entry offset (allocated
// from counters[kCntT]: the layout depends on arrival order, the entries do not), the
// per-block entry offsets at that S, the padding zeros and its descriptor.
__global__ __launch_bounds__(256) void k_ec_plan(UpdatePack pack, EcList ec, uint32_t chunk,
                                                 const uint32_t* __restrict__ stats,
                                                 uint32_t* __restrict__ boff,
                                                 uint32_t* __restrict__ cnt,
                                                 uint32_t* __restrict__ nocc,
                                                 uint2* __restrict__ info,
                                                 ChainCol* __restrict__ chains,
                                                 ChainEnt ce,
                                                 uint32_t* __restrict__ counters, int kmax,
                                                 const uint32_t* __restrict__ cand) {
    const int lane = threadIdx.x & 63;
    const uint32_t M = ec.col0[ec.n];
    const uint32_t g = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (g >= M) return;  // wave-uniform
    int e = 0;
    while (e + 1 < ec.n && g >= ec.col0[e + 1]) ++e;
    const int t = ec.t[e];
    const uint32_t c = g - ec.col0[e];
    const uint32_t nblk = ec.blk0[e + 1] - ec.blk0[e];
    const uint32_t* st = stats + (uint64_t)(ec.cb0[e] + c * nblk) * kEcStats;
    uint32_t v[6] = {0u, 0u, 0u, 0u, 0u, 0u};
    for (uint32_t b = (uint32_t)lane; b < nblk; b += 64)
#pragma unroll
        for (int k = 0; k < 6; ++k) v[k] += st[(uint64_t)b * kEcStats + k];
#pragma unroll
    for (int k = 0; k < 6; ++k) v[k] = wave_sum_u32(v[k]);
    int best = 0;
    uint64_t bc = ~0ull;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint64_t cc = (uint64_t)v[1 + k] * chain_entry_cost2(1u << k);
        if (k <= kmax && cc < bc) bc = cc, best = k;  // as k_chain_choose
    }
    const bool is_chain = v[0] > chunk;  // wave-uniform
    const uint32_t S = is_chain ? (1u << best) : 0u, E = is_chain ? v[1 + best] : 0u;
    const uint32_t P = is_chain ? cdiv_u32(E, kChainGroup) * kChainGroup + kChainPad : 0u;
    uint32_t e0 = 0;
    if (lane == 0 && is_chain) e0 = atomicAdd(&counters[kCntT], P);
    e0 = (uint32_t)__shfl((int)e0, 0, 64);
    if (lane == 0) {
        cnt[g] = P;
        nocc[g] = v[0];
        info[g] = make_uint2(S, E);
        const uint32_t col = ec.hot ? cand[e * kEhK + c] : c;  // EH: the candidate
        chains[g] = ChainCol{is_chain ? pack.row_off[t] + col : 0u, e0,
                             is_chain ? (P - kChainPad) / kChainGroup : 0u, S};
    }
    if (!is_chain) return;
    uint32_t carry = e0;  // per-block entry offsets at S, in block order
    for (uint32_t b0 = 0; b0 < nblk; b0 += 64) {
        const uint32_t b = b0 + (uint32_t)lane;
        const uint32_t x = b < nblk ? st[(uint64_t)b * kEcStats + 1 + best] : 0u;
        const uint32_t ex = wave_excl_scan_u32(x, lane);
        if (b < nblk) boff[ec.cb0[e] + c * nblk + b] = carry + ex;
        carry += wave_sum_u32(x);
    }
    const uint32_t ld4 = chain_stream_ld4(pack.d[t].batch, pack.d[t].ld_delta, S);
    for (uint32_t i = e0 + E + (uint32_t)lane; i < e0 + P; i += 64)  // ec_table: batch <= 2^20
        chain_pad(ce, i, (uint32_t)pack.d[t].batch, 24u, ld4);
}

// EC step 3 (one workgroup): the cost order of the EC columns — costliest first, so the
// hottest chains start with the list — and their count (counters[kCntM], read by the chain
// role).
__global__ __launch_bounds__(1024) void k_ec_order(EcList ec, const uint2* __restrict__ info,
                                                   int ns,
                                                   uint32_t* __restrict__ order,
                                                   uint32_t* __restrict__ counters) {
    __shared__ uint32_t hist[65];
    const uint32_t M = ec.col0[ec.n];
    if (threadIdx.x < 65) hist[threadIdx.x] = 0u;
    __syncthreads();
    auto bucket = [&](uint32_t g) {  // leading zeros of the cost: 0 = costliest, 64 = none
        const uint2 in = info[g];
        const uint64_t cc = (uint64_t)in.y * chain_entry_cost2(in.x);
        return cc ? (uint32_t)__clzll((long long)cc) : 64u;
    };
    for (uint32_t g = threadIdx.x; g < M; g += 1024) atomicAdd(&hist[bucket(g)], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        for (int k = 0; k < 65; ++k) {
            const uint32_t h = hist[k];
            hist[k] = run;
            run += h;
        }
        counters[kCntM] = M;
    }
    __syncthreads();
    for (uint32_t g = threadIdx.x; g < M; g += 1024) order[atomicAdd(&hist[bucket(g)], 1u)] = g;
}

// EC step 4, per (table, block): the entries of the block's bags for every chain column
// at the column's block offset, in bag order: part (c, p) counts its bags' entries, the
// parts of a column are scanned in LDS, then each part writes its bags' entries.
__global__ __launch_bounds__(256) void k_ec_emit(UpdatePack pack, EcList ec,
                                                 const uint32_t* __restrict__ boff,
                                                 const uint2* __restrict__ info,
                                                 ChainEnt ce,
                                                 const uint32_t* __restrict__ cand) {
    extern __shared__ __attribute__((aligned(16))) uint8_t hist[];  // kEcBags x ec_rs(ec)
    __shared__ uint32_t psum[kEcBags];
    __shared__ uint32_t sc[kEhK];
    const int e = ec_find(ec, blockIdx.x);
    const et_update_desc& d = pack.d[ec.t[e]];
    const uint32_t blk = blockIdx.x - ec.blk0[e];
    const uint32_t nblk = ec.blk0[e + 1] - ec.blk0[e];
    const EcParts q = ec_parts(ec.col0[e + 1] - ec.col0[e]);
    ec_hist(d, blk, hist, q.RS, eh_stage(ec, e, cand, sc));
    const uint32_t S = q.on ? info[ec.col0[e] + q.c].x : 0u;
    uint32_t mine = 0;
    if (S)
        for (uint32_t i = q.b0; i < q.b1; ++i) mine += cdiv_u32(hist[i * q.RS + q.c], S);
    psum[threadIdx.x] = mine;
    __syncthreads();
    if (!S) return;  // no barrier below
    uint32_t at = boff[ec.cb0[e] + q.c * nblk + blk];
    const uint32_t ld4 = chain_stream_ld4(d.batch, d.ld_delta, S);
    for (uint32_t p = 0; p < q.p; ++p) at += psum[p * q.R + q.c];
    for (uint32_t i = q.b0; i < q.b1; ++i) {
        const uint32_t r = hist[i * q.RS + q.c];
        const uint32_t k = cdiv_u32(r, S);
        const uint32_t bag = blk * kEcBags + i;
        for (uint32_t j = 0; j < k; ++j) chain_put(ce, at + j, j, k, r, S, bag, 24u, ld4);
        at += k;
    }
}

// S = 1 chains (every entry one add: the big tables' hot columns, whose runs are single
// occurrences) are bound by memory latency, not issue: a wave keeps at most 63 vector
// loads in flight (vmcnt), i.e. 63 entries of one 64-feature slice, and a random 256-byte
// gradient row takes ~1-2 us to arrive under the update's load.  The quad walk carries
// FOUR entries per load: the wave covers 16 features, its four 16-lane rows load the
// 16-feature slices of four consecutive entries, and the serial sum takes them into row 0
// in order (permlane16 / permlane32 swaps move rows 1-3 down), so 32 loads in flight are
// 128 entries.  The 64-entry chunk is loaded permuted (lane 16r + k holds entry 4k + r),
// so DPP row_newbcast:k hands row r entry 4k + r.  Same adds in the same order as the
// 64-feature loop (bit-identical); rows 1-3 add garbage that is never stored.
// The ring holds R quads (R / 16 chunks, R = kQuadRing = 32: 128 entries in flight).  A
// 64-quad ring on the exclusive SIMDs measured slower (config 4, one box: 3.874-3.877 ms at
// 32 against 3.88-3.91 at 64, profiles/r05/exact_grid/ab_r05o.txt).
constexpr int kQuadRing = 32;   // quads (4 entries each) of gradient loads in flight
constexpr int kQuadItems = 4;   // work items per (column, 64-feature slice): 16-feature quarters
constexpr int kQuadMinGroups = 1024;  // quad walk for S = 1 chains of >= 64 K entries

template <int K>
__device__ __forceinline__ uint32_t row_bcast(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x150 + K, 0xf, 0xf, false);
}

// Quads x[J], J in [J, N) (one half-trip, 32 quads, 128 entries), then their reloads: quad
// q + R into x[J], its bag from the chunk pair (cn0, cn1) R / 16 chunks on.
template <int R, int J, int N>
__device__ __forceinline__ void quad_trip(float (&x)[R], float& acc, uint32_t cn0, uint32_t cn1,
                                          __amdgpu_buffer_rsrc_t rx, uint32_t ld4,
                                          uint32_t lane4) {
    if constexpr (J < N) {
        const uint32_t v = __float_as_uint(x[J]);
        acc = acc + x[J];                                            // entry 4q
        const auto s32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        const auto s16 = __builtin_amdgcn_permlane16_swap(s32[0], s32[0], false, false);
        acc = acc + __uint_as_float(s16[1]);                         // entry 4q + 1
        const uint32_t z = s32[1];                                   // rows: 4q+2, 4q+3, ..
        acc = acc + __uint_as_float(z);                              // entry 4q + 2
        const auto t16 = __builtin_amdgcn_permlane16_swap(z, z, false, false);
        acc = acc + __uint_as_float(t16[1]);                         // entry 4q + 3
        const uint32_t bag = row_bcast<J & 15>((J & 31) < 16 ? cn0 : cn1);
        x[J] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            rx, (int)(__umul24(bag, ld4) + lane4), 0, 0));
        quad_trip<R, J + 1, N>(x, acc, cn0, cn1, rx, ld4, lane4);
    }
}

// Quads 0..R-1: x[J] from chunk J / 16 (c[0..R/16)).
template <int R, int J>
__device__ __forceinline__ void quad_prologue(float (&x)[R], const uint32_t (&c)[R / 16],
                                              __amdgpu_buffer_rsrc_t rx, uint32_t ld4,
                                              uint32_t lane4) {
    if constexpr (J < R) {
        const uint32_t bag = row_bcast<J & 15>(c[J / 16]);
        x[J] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            rx, (int)(__umul24(bag, ld4) + lane4), 0, 0));
        quad_prologue<R, J + 1>(x, c, rx, ld4, lane4);
    }
}

// The serial sum of one S = 1 chain over 16 features (row 0 of the result), R quads of
// gradient loads in flight.  ent: the chain's entries (ngr x 64, then >= kChainPad padding
// entries that address bag `batch`, past the gradient's range: they load +0); P: entries
// readable (range of the entry loads, past it they read 0, i.e. bag 0: loaded into the ring
// but never added).  Half-trips of 2 chunks (32 quads, 128 entries), alternating over the
// ring's halves when R = 64; the last half-trip's adds reach at most 64 entries past
// ngr x 64, inside the padding.
template <int R>
__device__ __forceinline__ float chain_walk_quad(const uint32_t* ent, uint32_t ngr, uint32_t P,
                                                 const float* delta, uint32_t range,
                                                 uint32_t lane4, uint32_t ld4) {
    static_assert(kChainPad >= 64 && (R == 32 || R == 64), "quad walk layout");
    constexpr uint32_t RC = R / 16;  // chunks in the ring
    const int lane = threadIdx.x & 63;
    const uint32_t poff = 4u * (4u * (uint32_t)(lane & 15) + (uint32_t)(lane >> 4));
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(delta), 0, (int)range, 0x00020000);
    const __amdgpu_buffer_rsrc_t re =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(ent), 0, (int)(4u * P), 0x00020000);
    auto chunk = [&](uint32_t c) { return __builtin_amdgcn_raw_buffer_load_b32(re, (int)(c * 256u + poff), 0, 0); };
    uint32_t c[RC];
#pragma unroll
    for (uint32_t k = 0; k < RC; ++k) c[k] = chunk(k);
    uint32_t n0 = chunk(RC), n1 = chunk(RC + 1);  // the reloads of half-trip 0
    float x[R];
    quad_prologue<R, 0>(x, c, rx, ld4, lane4);  // quads 0..R-1
    float acc = 0.0f;
    const uint32_t nh = (ngr + 1u) / 2u;  // half-trips
    for (uint32_t h = 0; h < nh; h += R / 32) {
        {
            const uint32_t m0 = chunk(2u * h + RC + 2u), m1 = chunk(2u * h + RC + 3u);
            quad_trip<R, 0, 32>(x, acc, n0, n1, rx, ld4, lane4);
            n0 = m0;
            n1 = m1;
        }
        if constexpr (R == 64) {
            if (h + 1u == nh) break;
            const uint32_t m0 = chunk(2u * h + RC + 4u), m1 = chunk(2u * h + RC + 5u);
            quad_trip<R, 32, 64>(x, acc, n0, n1, rx, ld4, lane4);
            n0 = m0;
            n1 = m1;
        }
    }
    return acc;
}


// The serial sum of one chain over one 64-feature slice (lane = feature), with 64-bit
// gradient addresses and any element type: the reference's loop (src/sparseupdate.jl:110-127,
// acc += delta[:, bag] once per occurrence, in the accumulator type) taken entry by entry —
// r adds of the entry's gradient column.  The Float32 chains whose gradient the asm loop's
// 32-bit offsets cannot reach (chain_asm_ok) and the Float64 / Float16 / BFloat16 chains
// take it.  Entries are wave-uniform (scalar loads); the gradient loads run kWideAhead
// entries ahead, each from a wave-uniform row address (a padding entry, r = 0, loads row 0
// of the gradient and adds nothing).  ent: ngr x 64 entries, then >= kChainPad padding.
constexpr int kWideAhead = 16;

template <typename T>
__device__ __forceinline__ T wide_load(const T* delta, uint64_t ld, uint32_t fc, uint32_t e,
                                       uint32_t sh) {
    const uint64_t bag = (e >> sh) ? (uint64_t)(e & ((1u << sh) - 1u)) : 0u;
    return delta[bag * ld + fc];
}

// sh: the entries' bag width (chain_shift of the table's batch).
template <typename T, typename C>
__device__ __forceinline__ C chain_walk_wide(const uint32_t* ent, uint32_t ngr, const T* delta,
                                             uint64_t ld, uint32_t fc, C acc, uint32_t sh) {
    static_assert(kChainGroup % kWideAhead == 0 && kChainPad >= kWideAhead, "wide walk layout");
    uint32_t en[kWideAhead];
    T x[kWideAhead];
#pragma unroll
    for (int k = 0; k < kWideAhead; ++k) {
        en[k] = ent[k];
        x[k] = wide_load(delta, ld, fc, en[k], sh);
    }
    const uint32_t ne = ngr * (uint32_t)kChainGroup;
    for (uint32_t h = 0; h < ne; h += kWideAhead) {
#pragma unroll
        for (int k = 0; k < kWideAhead; ++k) {
            const uint32_t r = en[k] >> sh;
            const C v = C(x[k]);
            en[k] = ent[h + kWideAhead + k];  // inside the padding past the last trip
            x[k] = wide_load(delta, ld, fc, en[k], sh);
            for (uint32_t j = 0; j < r; ++j) acc = acc + v;
        }
    }
    return acc;
}

// Update phase, chain role: one (column, 64-feature slice, quarter) item of the cost-
// ordered list: the serial sum of the slice's gradient columns and the update.  A Float32
// S = 1 chain of at least quad_min 64-entry groups takes its four quarters as four items
// (the quad walk, 16 features each); any other chain takes the whole slice in quarter 0
// (the other quarters return at once).  T is the table and gradient type, C the
// accumulator (sgd_apply_t).
// A wave-uniform pointer as an SGPR pair (for the asm loops' "s" operands).
template <typename P>
__device__ __forceinline__ P* uniform_ptr(P* p) {
    const uint64_t b = reinterpret_cast<uint64_t>(p);
    return reinterpret_cast<P*>(
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b) |
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32)) << 32);
}

template <typename T, typename C, int MODE, bool NT>
__device__ __forceinline__ void sgd_chain_item(const UpdatePack& pack, int ntables,
                                               const ChainCol* __restrict__ chains,
                                               const uint32_t* __restrict__ order,
                                               const ChainEnt& ce, int ns,
                                               C eta_c, double eta64, uint32_t it4,
                                               uint32_t quad_min, bool stream) {
    constexpr bool kF32 = __is_same(T, float);
    const int lane = threadIdx.x & 63;
    const uint32_t quarter = it4 % (uint32_t)kQuadItems, it = it4 / (uint32_t)kQuadItems;
    const ChainCol c = chains[order[it / (uint32_t)ns]];
    if (c.S == 0u) return;
    const int t = table_of_key(pack, ntables, c.key);
    const et_update_desc& d = pack.d[t];
    const bool fast = kF32 && chain_asm_ok(d.batch, d.ld_delta);
    // the quad walk spends 4 waves where the 64-feature loop spends one, so short chains,
    // which are throughput- rather than latency-bound, keep the loop
    const bool quad = fast && c.S == 1u && c.ngr >= quad_min;
    if (!quad && quarter != 0u) return;
    const int slice = (int)(it % (uint32_t)ns);
    // the gradient base and the entries as wave-uniform (SGPR) pointers
    const uint64_t db = reinterpret_cast<uint64_t>(d.delta);
    const T* delta = reinterpret_cast<const T*>(
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)db) |
        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(db >> 32)) << 32);
    const uint32_t* e = uniform_ptr(ce.ent + c.e0);
    if constexpr (kF32) {
        if (quad) {
            const int f0 = slice * 64 + (int)quarter * 16;
            if (f0 >= d.dim) return;  // uniform
            const int f = f0 + (lane & 15);
            const uint32_t fc = (uint32_t)(f < d.dim ? f : d.dim - 1);
            const uint32_t ld = (uint32_t)d.ld_delta;
            const float acc = chain_walk_quad<kQuadRing>(e, c.ngr, c.ngr * kChainGroup + kChainPad, delta,
                                              (uint32_t)d.batch * ld * 4u, 4u * fc, 4u * ld);
            if (lane < 16 && f < d.dim) {
                float* w = col_ptr<float>(d.table, d.ld_table, d.cols_per_page,
                                          c.key - pack.row_off[t]) + f;
                store_scalar<NT>(w, sgd_apply<MODE>(*w, acc, eta_c, eta64));
            }
            return;
        }
    }
    const int f = slice * 64 + lane;
    if (slice * 64 >= d.dim) return;  // uniform
    const uint32_t fc = (uint32_t)(f < d.dim ? f : d.dim - 1);
    C acc = C(0);
    bool done = false;
    if constexpr (kF32) {
        if (fast) {
            // range batch * ld * 4 bytes: a padding entry (bag = batch) loads +0
            const uint32_t ld = (uint32_t)d.ld_delta;
            const i32x4 rs = chain_rsrc(delta, (uint32_t)d.batch * ld * 4u);
            if (stream && c.S >= (uint32_t)kChainStreamMinS) {
                // the index phase wrote this chain's offsets and masks (chain_stream_ld4)
                const uint32_t* off = uniform_ptr(ce.off + c.e0);
                const uint64_t* msk = uniform_ptr(ce.msk + c.e0);
                // (64 x loads in flight instead of 32 measured no faster: the hottest early
                // chain 3.16 against 3.05 ms, gpurun_out/r06zf)
                acc = c.S == 8u ? chain_walk_stream<8, 32>(off, msk, c.ngr, rs, 4u * fc, 0.0f)
                                : chain_walk_stream<16, 32>(off, msk, c.ngr, rs, 4u * fc, 0.0f);
            } else switch (c.S) {
                case 1: acc = chain_walk_asm<1>(e, c.ngr, rs, 4u * fc, 4u * ld, 0.0f); break;
                case 2: acc = chain_walk_asm<2>(e, c.ngr, rs, 4u * fc, 4u * ld, 0.0f); break;
                case 4: acc = chain_walk_asm<4>(e, c.ngr, rs, 4u * fc, 4u * ld, 0.0f); break;
                case 8: acc = chain_walk_asm<8>(e, c.ngr, rs, 4u * fc, 4u * ld, 0.0f); break;
                default: acc = chain_walk_asm<16>(e, c.ngr, rs, 4u * fc, 4u * ld, 0.0f); break;
            }
            done = true;
        }
    }
    if (!done)
        acc = chain_walk_wide<T, C>(e, c.ngr, delta, (uint64_t)d.ld_delta, fc, acc,
                                    chain_shift(d.batch));
    if (f < d.dim) {
        T* w = col_ptr<T>(d.table, d.ld_table, d.cols_per_page, c.key - pack.row_off[t]) + f;
        store_scalar<NT>(w, sgd_apply_t<T, C, MODE>(*w, acc, eta_c, eta64));
    }
}

// The chains of an update phase (early, early hot or regular), in their own launch on a side
// stream: each wave takes the next item of the cost-ordered list from counters[kCntNext] (so
// the longest chains start first and a late workgroup takes whatever is left), until the
// list is exhausted.  A chain issues a dependent VALU op about every 4.4 cycles, i.e. it alone
// nearly fills its SIMD's VALU, so two chains must not share a SIMD: the launch reserves more
// than half of a CU's LDS (dynamic, untouched), so no other chain workgroup — of this launch
// or another chain launch — lands on the same CU, and the workgroup's 4 waves take its 4
// SIMDs.  Top priority: the co-resident chunk-pass / singles / index-phase waves (memory
// bound) take the leftover issue slots.
constexpr uint32_t kChainReserveLds = 84 * 1024;  // > 80 KiB: one chain workgroup per CU

#ifdef ET_EXPERIMENTS
// Experiment builds: every chain item's start and end (s_memrealtime, 100 MHz), list, S,
// 64-entry groups, item number and hardware id, read back by et_debug_chain_timeline
// (tools/chain_timeline.py).
constexpr uint32_t kCtlCap = 1u << 17;
__device__ uint4 g_ctl[kCtlCap][2];
__device__ uint32_t g_ctl_n;
#endif

template <typename T, typename C, int MODE, bool NT>
__device__ __forceinline__ void chain_items(const UpdatePack& pack, int ntables,
                                            uint32_t* __restrict__ counters,
                                            const ChainCol* __restrict__ chains,
                                            const uint32_t* __restrict__ order,
                                            const ChainEnt& ce, int ns, C eta_c,
                                            double eta64, uint32_t quad_min, uint32_t list) {
    // list: bits 0-7 the list (0 early, 1 regular, 2 early hot; timelines), bit 8 the streamed
    // loop for S >= kChainStreamMinS (experiment builds can turn it off: ET_CHAIN_STREAM=0)
    const bool stream = (list & 0x100u) != 0u;
    list &= 0xffu;
    const int lane = threadIdx.x & 63;
    __builtin_amdgcn_s_setprio(3);
    const uint32_t items = counters[kCntM] * (uint32_t)ns * (uint32_t)kQuadItems;
    for (;;) {
        uint32_t it = 0;
        if (lane == 0) it = atomicAdd(&counters[kCntNext], 1u);
        it = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)it, 0, 64));
        if (it >= items) break;
#ifdef ET_EXPERIMENTS
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#endif
        sgd_chain_item<T, C, MODE, NT>(pack, ntables, chains, order, ce, ns, eta_c, eta64, it,
                                       quad_min, stream);
#ifdef ET_EXPERIMENTS
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        const ChainCol c = chains[order[(it / (uint32_t)kQuadItems) / (uint32_t)ns]];
        const bool ran = c.S != 0u && ((it % (uint32_t)kQuadItems) == 0u ||
                                        (c.S == 1u && c.ngr >= quad_min));
        if (lane == 0 && ran) {
            const uint32_t k = atomicAdd(&g_ctl_n, 1u);
            uint32_t hw;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            if (k < kCtlCap) {
                g_ctl[k][0] = make_uint4((uint32_t)t0, (uint32_t)(t0 >> 32), (uint32_t)t1,
                                         (uint32_t)(t1 >> 32));
                g_ctl[k][1] = make_uint4(list << 24 | c.S, c.ngr, it, hw);
            }
        }
#endif
    }
    __builtin_amdgcn_s_setprio(0);
}

template <typename T, typename C, int MODE, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_sgd_chains(
    UpdatePack pack, int ntables, uint32_t* __restrict__ counters,
    const ChainCol* __restrict__ chains, const uint32_t* __restrict__ order,
    ChainEnt ce, int ns, C eta_c, double eta64, uint32_t quad_min,
    uint32_t list) {
    chain_items<T, C, MODE, NT>(pack, ntables, counters, chains, order, ce, ns, eta_c, eta64,
                                quad_min, list);
}

// Eight chain waves per workgroup (two per SIMD; one workgroup per CU by the LDS
// reservation): for latency-bound lists (the early hot columns' S = 1 quad walks spend about a
// third of their cycles issuing), so one CU keeps twice the gradient loads in flight.
template <typename T, typename C, int MODE, bool NT>
__global__ __launch_bounds__(512) void k_sgd_chains_w(
    UpdatePack pack, int ntables, uint32_t* __restrict__ counters,
    const ChainCol* __restrict__ chains, const uint32_t* __restrict__ order,
    ChainEnt ce, int ns, C eta_c, double eta64, uint32_t quad_min,
    uint32_t list) {
    chain_items<T, C, MODE, NT>(pack, ntables, counters, chains, order, ce, ns, eta_c, eta64,
                                quad_min, list);
}

// The same chain loop on SIMDs of its own: the kernel writes a255, so it is allocated the
// whole accumulation-register file besides its VGPRs and no other wave — of the chunk pass,
// the singles, the index phase — can be resident on its SIMDs while it runs; the chain waves
// then issue at the SIMD's own rate instead of sharing it (the early chains and the early hot
// columns by default, kChainExcl).
template <typename T, typename C, int MODE, bool NT>
__global__ __launch_bounds__(256) void k_sgd_chains_x(
    UpdatePack pack, int ntables, uint32_t* __restrict__ counters,
    const ChainCol* __restrict__ chains, const uint32_t* __restrict__ order,
    ChainEnt ce, int ns, C eta_c, double eta64, uint32_t quad_min,
    uint32_t list) {
    asm volatile("v_accvgpr_write_b32 a255, 0" ::: "a255");
    chain_items<T, C, MODE, NT>(pack, ntables, counters, chains, order, ce, ns, eta_c, eta64,
                                quad_min, list);
}

// The rest of the update phase of an exact Float32 call in one launch: blocks [0, nch)
// the chunk pass over single-chunk columns of this capacity group, the rest the
// single-occurrence columns (the chains run in k_sgd_chains on the side streams).
template <int D, int MODE, bool NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_sgd_exact(
    UpdatePack pack, int ntables, const uint32_t* __restrict__ keys,
    const uint32_t* __restrict__ vals, const ChunkRec* __restrict__ recs,
    const uint32_t* __restrict__ counters, uint32_t sent, float eta32, double eta64,
    uint32_t my_mask, uint32_t nch) {
    if (blockIdx.x < nch)
        sgd_chunks_body<D, MODE, NT>(pack, ntables, keys, vals, recs, counters, nullptr, 0,
                                     sent, eta32, eta64, my_mask, 1, 1, blockIdx.x, nch);
    else
        sgd_singles_body<D, MODE, NT>(pack, ntables, vals, recs, counters, sent, eta32, eta64,
                                      my_mask, blockIdx.x - nch, gridDim.x - nch);
}

// Generic kernels (any dim / alignment / element type): one wave per chunk or
// combined segment, lanes over features, scalar loads.  T is the table and gradient
// type, C the accumulator (sgd_apply_t).
template <typename T, typename C, int MODE, bool NT>
__global__ __launch_bounds__(256) void k_sgd_chunks_generic(
    UpdatePack pack, int ntables, const uint32_t* __restrict__ keys,
    const uint32_t* __restrict__ vals, const ChunkRec* __restrict__ recs,
    const uint32_t* __restrict__ counters, C* __restrict__ partials, int pdim, uint32_t sent,
    C eta_c, double eta64, int skip_multi) {
    const int lane = threadIdx.x & 63;
    const uint32_t Cn = counters[kCntC];
    const uint32_t waves = gridDim.x * 4;
    for (uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6); c < Cn; c += waves) {
        const ChunkRec r = recs[c];
        const uint32_t key = r.key;
        if (key == sent || (skip_multi && r.dst != kApply)) continue;  // (chains: exact F32)
        const int t = table_of_key(pack, ntables, key);
        const et_update_desc& d = pack.d[t];
        if ((pack.vec_mask >> t) & 1u) continue;  // handled by the vector kernel
        const uint32_t s0 = r.s0, s1 = r.s1;
        const T* delta = reinterpret_cast<const T*>(d.delta);
        for (int f = lane; f < d.dim; f += 64) {
            C acc = C(0);
            for (uint32_t o = s0; o < s1; ++o) {
                const uint32_t bag = (vals[o] - pack.occ_off[t]) / (uint32_t)d.pool;
                acc = acc + C(delta[(uint64_t)bag * (uint64_t)d.ld_delta + f]);
            }
            if (r.dst == kApply) {
                T* w = col_ptr<T>(d.table, d.ld_table, d.cols_per_page, key - pack.row_off[t]) + f;
                store_scalar<NT>(w, sgd_apply_t<T, C, MODE>(*w, acc, eta_c, eta64));
            } else {
                partials[(uint64_t)r.dst * pdim + f] = acc;
            }
        }
    }
}

template <typename T, typename C, int MODE, bool NT>
__global__ __launch_bounds__(256) void k_sgd_combine_generic(
    UpdatePack pack, int ntables, const uint32_t* __restrict__ keys,
    const uint32_t* __restrict__ seg_start, const uint32_t* __restrict__ partial_start,
    const uint32_t* __restrict__ counters, const C* __restrict__ partials, int pdim,
    uint32_t sent, C eta_c, double eta64) {
    const int lane = threadIdx.x & 63;
    const uint32_t Useg = counters[kCntU];
    const uint32_t waves = gridDim.x * 4;
    for (uint32_t u = blockIdx.x * 4 + (threadIdx.x >> 6); u < Useg; u += waves) {
        const uint32_t p0 = partial_start[u], p1 = partial_start[u + 1];
        if (p1 == p0) continue;
        const uint32_t key = keys[seg_start[u]];
        if (key == sent) continue;
        const int t = table_of_key(pack, ntables, key);
        const et_update_desc& d = pack.d[t];
        if ((pack.vec_mask >> t) & 1u) continue;
        // the vector combine's fixed partition (k_sgd_combine: 8 contiguous ranges of
        // partials, each summed from 0, the range sums added in order), so a table taking
        // the generic path combines exactly like a vector-width feature slice of it
        const uint32_t np = p1 - p0;
        for (int f = lane; f < d.dim; f += 64) {
            C tot = C(0);
            for (int R = 0; R < 8; ++R) {
                const uint32_t a = p0 + (uint32_t)((uint64_t)np * R / 8);
                const uint32_t b = p0 + (uint32_t)((uint64_t)np * (R + 1) / 8);
                C acc = C(0);
                for (uint32_t q = a; q < b; ++q) acc = acc + partials[(uint64_t)q * pdim + f];
                tot = tot + acc;
            }
            T* w = col_ptr<T>(d.table, d.ld_table, d.cols_per_page, key - pack.row_off[t]) + f;
            store_scalar<NT>(w, sgd_apply_t<T, C, MODE>(*w, tot, eta_c, eta64));
        }
    }
}

// ---------------------------------------------------------------------------
// Workspace
// ---------------------------------------------------------------------------

struct UpdateWs {
    uint32_t *ka, *va, *kb, *vb, *hist, *part, *seg_start, *nch, *multi, *counters,
        *mlist;
    ChunkRec* recs;
    float* partials;
    // hot-column pass: per-table log2 histograms [32][32] then slot counts [32] (one
    // memset), hot keys [32][kHotSlots], window partials [nhot][kHotSlots][nw][64] float2
    uint32_t *hot_hist, *hot_cnt, *hot_key;
    float2* hot_part;
    uint8_t* hot_slots;  // [sum over hot-shaped tables of batch * roundup(pool, 4)]
    int hot_nw;
    // exact Float32 mode: chain entries (aliasing `partials`: that mode has no partial
    // sums), per chain column (multi-chunk list slot) its descriptor, padded entry count,
    // (S, entries), entry offset, and the cost-ordered slot list
    ChainEnt chain_ent;
    ChainCol* chains;
    uint32_t *chain_cnt, *chain_e0, *chain_order;
    uint2* chain_info;
    // the index phase's tiles: first tile per column, tile -> column, entries per tile at
    // S = 1..16
    uint32_t *chain_tile0, *chain_tcnt;
    ChainTile* chain_trec;
    uint32_t* chain_part;  // the regular plan's scan partials (its own: it runs beside others)
    // early chains (EcList): per (column, block) stats and entry offsets, per EC column the
    // padded entry count, (S, entries), descriptor and cost order, their entries, and a
    // counter block (kCntM = EC columns) for the chain role
    struct EcWs {
        uint32_t *stats, *boff, *cnt, *order, *counters, *nocc;
        ChainEnt ent;
        uint2* info;
        ChainCol* chains;
    };
    EcWs ec, eh;        // the small tables' early chains; the big tables' hot columns (ET_EH)
    uint32_t* eh_cand;  // kEhK candidate columns per EH entry (k_eh_pick)
    int64_t bytes;
};

inline int64_t align256(int64_t x) { return (x + 255) & ~int64_t(255); }

// The entries, offsets and masks of a chain list in one buffer of 16 * n bytes (n even).
inline ChainEnt chain_ent_at(char* p, int64_t n) {
    ChainEnt c;
    c.ent = reinterpret_cast<uint32_t*>(p);
    c.off = p ? c.ent + n : nullptr;
    c.msk = p ? reinterpret_cast<uint64_t*>(p + 8 * n) : nullptr;
    return c;
}

// Index-phase tiles of the chain columns: at most one partial tile per column plus the
// full ones.
inline int64_t chain_tiles_max(int64_t n, uint32_t chunk) {
    return n / kChainTile + n / chunk + 3;
}

// Lay out (or size, when base == nullptr) the update workspace for n occurrences and
// partial rows of pdim floats.
inline UpdateWs carve_update_ws(char* base, int64_t n, int pdim, uint32_t chunk,
                                int nhot = 0, int64_t hot_batch = 0, int64_t hot_bytes = 0,
                                const EcList* ec = nullptr, int64_t ec_occ = 0,
                                const EcList* eh = nullptr, int64_t eh_occ = 0) {
    UpdateWs w;
    // every buffer 256-byte aligned whatever the caller's workspace alignment (the
    // 16-byte key / index / LDS-DMA loads rely on it): the layout starts at the first
    // 256-byte boundary of the workspace, and the size asks for 256 bytes of slack
    int64_t off = base ? (int64_t)((256u - ((uintptr_t)base & 255u)) & 255u) : 256;
    auto take = [&](int64_t bytes) -> char* {
        char* p = base ? base + off : nullptr;
        off += align256(bytes);
        return p;
    };
    const int64_t n1 = n + 1;
    const int64_t hist_m = sort_hist_entries(n, kRsMaxSegs);
    const int64_t scan_m = hist_m > n1 + 1 ? hist_m : n1 + 1;
    w.ka = (uint32_t*)take(4 * n1);
    w.va = (uint32_t*)take(4 * n1);
    w.kb = (uint32_t*)take(4 * n1);
    w.vb = (uint32_t*)take(4 * n1);
    w.hist = (uint32_t*)take(4 * hist_m);
    w.part = (uint32_t*)take(4 * scan_part_entries(scan_m));
    w.seg_start = (uint32_t*)take(4 * (n1 + 1));
    w.nch = (uint32_t*)take(4 * (n1 + 1));
    w.multi = (uint32_t*)take(4 * (n1 + 1));
    const int64_t max_chunks = n + n / chunk + 2;
    w.recs = (ChunkRec*)take((int64_t)sizeof(ChunkRec) * max_chunks);
    w.counters = (uint32_t*)take(4 * kCntSlots);
    w.mlist = (uint32_t*)take(4 * (n / chunk + 2));
    const int64_t max_partials = 2 * (n / chunk) + 2;
    const int64_t mmax = n / chunk + 2;  // multi-chunk (chain) columns
    // 8 bytes per partial element: float (vector path / fp32 accumulators) or double; the
    // exact mode's chain entries (8 bytes, at most one per occurrence + padding) alias it
    const int64_t part_b = 8 * max_partials * (int64_t)(pdim > 0 ? pdim : 1);
    // entries, offsets and masks (4 + 4 + 8 bytes) of up to one entry per occurrence + padding
    const int64_t chain_n = (n + (int64_t)(kChainGroup + kChainPad) * mmax + 64 + 1) & ~int64_t(1);
    const int64_t chain_b = 16 * chain_n;
    w.partials = (float*)take(part_b > chain_b ? part_b : chain_b);
    w.chain_ent = chain_ent_at(reinterpret_cast<char*>(w.partials), chain_n);
    w.chains = (ChainCol*)take((int64_t)sizeof(ChainCol) * mmax);
    w.chain_cnt = (uint32_t*)take(4 * mmax);
    w.chain_e0 = (uint32_t*)take(4 * mmax);
    w.chain_order = (uint32_t*)take(4 * mmax);
    w.chain_info = (uint2*)take(8 * mmax);
    const int64_t tmax = chain_tiles_max(n, chunk);
    w.chain_tile0 = (uint32_t*)take(4 * (mmax + 1));
    w.chain_part = (uint32_t*)take(4 * scan_part_entries(mmax + 1));
    w.chain_trec = (ChainTile*)take((int64_t)sizeof(ChainTile) * tmax);
    w.chain_tcnt = (uint32_t*)take(20 * tmax);
    auto carve_ec = [&](const EcList* l, int64_t occ) {
        const int64_t recs = l && l->n ? l->cb0[l->n] : 0, M = l && l->n ? l->col0[l->n] : 0;
        UpdateWs::EcWs e;
        e.stats = (uint32_t*)take(4 * kEcStats * recs);
        e.boff = (uint32_t*)take(4 * recs);
        e.cnt = (uint32_t*)take(4 * M);
        e.order = (uint32_t*)take(4 * M);
        e.nocc = (uint32_t*)take(4 * M);
        e.info = (uint2*)take(8 * M);
        e.chains = (ChainCol*)take((int64_t)sizeof(ChainCol) * M);
        e.counters = (uint32_t*)take(4 * kCntSlots);
        const int64_t cn = (occ + (int64_t)(kChainGroup + kChainPad) * M + 64 + 1) & ~int64_t(1);
        e.ent = chain_ent_at(take(16 * cn), cn);
        return e;
    };
    w.ec = carve_ec(ec, ec_occ);
    w.eh = carve_ec(eh, eh_occ);
    w.eh_cand = (uint32_t*)take(eh && eh->n ? 4 * (int64_t)kEhK * eh->n : 0);
    w.hot_nw = (int)((hot_batch + kHotWin - 1) / kHotWin);
    w.hot_hist = nullptr;
    w.hot_cnt = nullptr;
    w.hot_key = nullptr;
    w.hot_part = nullptr;
    w.hot_slots = nullptr;
    if (nhot > 0 && w.hot_nw > 0) {
        w.hot_slots = (uint8_t*)take(hot_bytes);
        w.hot_hist = (uint32_t*)take(4 * (32 * 32 + 32));
        w.hot_cnt = w.hot_hist ? w.hot_hist + 32 * 32 : nullptr;
        w.hot_key = (uint32_t*)take(4 * 32 * kHotSlots);
        w.hot_part = (float2*)take((int64_t)nhot * kHotSlots * w.hot_nw * 64 * 8);
    }
    w.bytes = off;
    return w;
}

// Steps 1-4 shared by et_sparse_sgd: sorted keys/values, segments and chunks.
struct Grouped {
    uint32_t* keys;
    uint32_t* vals;
};

// One sort segment per table, sorted on its own column range (et_sort.hip); returns
// the number of radix passes.
inline int sort_segments(const UpdatePack& pack, int ntables, RsSegment* seg) {
    for (int t = 0; t < ntables; ++t) {
        const uint32_t nr = (uint32_t)pack.d[t].nrows;
        seg[t] = RsSegment{pack.occ_off[t], pack.occ_off[t + 1] - pack.occ_off[t],
                           pack.row_off[t], nr, bits_for(nr)};
    }
    return rs_total_passes(seg, ntables);
}

// Where group_occurrences left the sorted pairs (for an APPLY_ONLY call): buffer a
// after an even number of radix passes, b after an odd one (segmented_radix_sort).
inline Grouped grouped_pairs(const UpdatePack& pack, int ntables, const UpdateWs& w) {
    RsSegment seg[ET_MAX_TABLES_PER_LAUNCH];
    const int P = sort_segments(pack, ntables, seg);
    return (P & 1) ? Grouped{w.kb, w.vb} : Grouped{w.ka, w.va};
}

// Exact Float32 mode: the multi-chunk columns become serial chains.  Their plan reads only
// the index phase's segments and multi-chunk list, so it runs on the regular chains' side
// stream (forked after the chunk records) while the caller's stream goes on to the chunk pass
// over the single-chunk columns (k_sgd_exact) — the plan is off the update's critical path.
inline int launch_chain_plan(const UpdatePack& pack, int ntables, int64_t n, uint32_t sent,
                             uint32_t chunk, UpdateWs& w, const Grouped& out, hipStream_t s,
                             uint32_t ec_mask, const EhMap& eh, hipEvent_t cand_ready) {
    if (eh.mask) ET_HIP_CHECK(hipStreamWaitEvent(s, cand_ready, 0));  // k_eh_pick's candidates
    const int64_t mmax = n / chunk + 2;
    const unsigned cg = (unsigned)(cdiv64(mmax, 4) < 2048 ? cdiv64(mmax, 4) : 2048);
    const int64_t tmax = chain_tiles_max(n, chunk);
    // grid-stride over the tiles (about 10 K on config 4): round 4's 8192 workgroups waited
    // beside the chunk pass for slots (k_chain_tcount 127-507 us, k_chain_emit 323-351 us)
    const long long tgmax = ET_KNOB("ET_PLAN_TG", 2048ll);
    const unsigned tg = (unsigned)(tmax < tgmax ? tmax : tgmax);
    // tiles per column, their exclusive scan (device-side length M + 1), the tile map: small
    // grids that fit beside the chunk pass's persistent workgroups (round 4's one-workgroup
    // k_chain_tiles serialised M / 1024 dependent scan rounds and waited up to 0.73 ms for a CU)
    const unsigned mg = (unsigned)(cdiv64(mmax + 1, 256) < 256 ? cdiv64(mmax + 1, 256) : 256);
    hipLaunchKernelGGL(k_chain_tile_count, dim3(mg), dim3(256), 0, s, pack, ntables, ec_mask, eh,
                       w.eh_cand, out.keys, w.seg_start, w.mlist, w.counters, sent,
                       w.chain_tile0);
    int rc = exclusive_scan_u32(w.chain_tile0, w.chain_tile0, mmax + 1, w.chain_part, s,
                                w.counters + kCntM, 1);
    if (rc != ET_OK) return rc;
    hipLaunchKernelGGL(k_chain_tile_fill, dim3(mg), dim3(256), 0, s, pack, ntables, out.keys,
                       w.seg_start, w.mlist, w.chain_tile0, w.counters, w.chain_trec);
    hipLaunchKernelGGL(k_chain_tcount, dim3(tg), dim3(256), 0, s, pack, ntables, out.keys,
                       out.vals, w.seg_start, w.mlist, w.counters, w.chain_tile0,
                       w.chain_trec, w.chain_tcnt);
    hipLaunchKernelGGL(k_chain_choose, dim3(cg), dim3(256), 0, s, out.keys, w.seg_start,
                       w.mlist, w.counters, w.chain_tile0, w.chain_tcnt, w.chain_cnt,
                       w.chain_info, w.chains, 4);
    hipLaunchKernelGGL(k_chain_plan, dim3(1), dim3(kPlanThreads), 0, s, w.counters, w.chain_cnt,
                       w.chain_e0, w.chain_order);
    hipLaunchKernelGGL(k_chain_emit, dim3(tg), dim3(256), 0, s, pack, ntables, out.keys,
                       out.vals, w.seg_start, w.mlist, w.counters, w.chain_tile0,
                       w.chain_trec, w.chain_tcnt, w.chain_cnt, w.chain_info, w.chain_e0,
                       w.chain_ent, w.chains);
    ET_LAUNCH_CHECK("k_chain_emit");
    // ET_CHAIN_CHECK (experiment builds): validate every entry of the plan
    if (ET_KNOB("ET_CHAIN_CHECK", 0))
        hipLaunchKernelGGL(k_chain_check, dim3(cg), dim3(256), 0, s, pack, ntables, w.counters,
                           w.chain_cnt, w.chain_info, w.chain_ent, w.chains, w.chain_order);
    return ET_OK;
}

inline int group_occurrences(const UpdatePack& pack, int ntables, int64_t n, uint32_t sent,
                             uint32_t chunk, UpdateWs& w, Grouped& out, hipStream_t s,
                             uint32_t hot_mask = 0, const HotList* hl = nullptr,
                             bool chain = false, uint32_t ec_mask = 0,
                             int64_t* const* snaps = nullptr) {
    const int64_t blocks = cdiv64(n, 256);
    const unsigned kb_grid = (unsigned)(blocks < 65536 ? blocks : 65536);
    ET_HIP_CHECK(hipMemsetAsync(w.counters, 0, 4 * kCntSlots, s));
    KeyGrid kg;
    kg.blk_off[0] = 0;
    kg.vec = 0;
    kg.snap_mask = 0;
    for (int t = 0; t < ntables; ++t) {
        kg.snap[t] = snaps ? snaps[t] : nullptr;
        if (kg.snap[t]) kg.snap_mask |= 1u << t;
    }
    const bool bufs16 = (((uintptr_t)w.ka | (uintptr_t)w.va | (uintptr_t)w.kb | (uintptr_t)w.vb) &
                         15u) == 0;
    for (int t = 0; t < ntables; ++t) {
        const int64_t nt = pack.occ_off[t + 1] - pack.occ_off[t];
        const et_update_desc& d = pack.d[t];
        const bool vec = bufs16 && (d.ld_idx == d.pool || d.batch == 1) &&
                         ((uintptr_t)d.idx & 15u) == 0 && (pack.occ_off[t] & 3u) == 0 &&
                         ((uintptr_t)kg.snap[t] & 15u) == 0;
        if (vec) kg.vec |= 1u << t;
        int64_t nb = cdiv64(nt, vec ? 1024 : 256);
        nb = nb < 2048 ? nb : 2048;  // grid-stride beyond 2048 workgroups per table
        kg.blk_off[t + 1] = kg.blk_off[t] + (uint32_t)nb;
    }
    (void)kb_grid;
    RsSegment seg[ET_MAX_TABLES_PER_LAUNCH];
    const int P = sort_segments(pack, ntables, seg);
    kg.in_b = 0;
    for (int t = 0; t < ntables; ++t)
        if ((P - rs_passes(seg[t].bits)) & 1) kg.in_b |= 1u << t;
    if (kg.blk_off[ntables] > 0)
        hipLaunchKernelGGL(k_build_keys, dim3(kg.blk_off[ntables]), dim3(256), 0, s, pack, kg,
                           ntables, w.ka, w.va, w.kb, w.vb, sent);
    ET_LAUNCH_CHECK("k_build_keys");
    SortBuffers sb{w.ka, w.va, w.kb, w.vb, w.hist, w.part};
    int rc = segmented_radix_sort(sb, seg, ntables, &out.keys, &out.vals, s);
    if (rc != ET_OK) return rc;
    {
        const int64_t np = cdiv64(n, kScanTile);
        hipLaunchKernelGGL(k_seg_reduce, dim3((unsigned)np), dim3(kScanThreads), 0, s, out.keys,
                           n, w.part);
        launch_scan_partials(w.part, np, nullptr, 0u, s);
        hipLaunchKernelGGL(k_seg_down, dim3((unsigned)np), dim3(kScanThreads), 0, s, out.keys,
                           n, w.part, w.seg_start, w.counters);
        ET_LAUNCH_CHECK("k_seg_down");
    }
    const int64_t blocks1 = cdiv64(n + 1, 256);
    const unsigned fixed_grid = (unsigned)(blocks1 < 8192 ? blocks1 : 8192);
    const int64_t sc_blocks = cdiv64(n + 1, (int64_t)kSegChunkItems * 256);
    hipLaunchKernelGGL(k_seg_chunks, dim3((unsigned)(sc_blocks < 2048 ? sc_blocks : 2048)),
                       dim3(256), 0, s, w.seg_start, n,
                       w.counters, chunk, w.nch, w.multi, w.mlist);
    ET_LAUNCH_CHECK("k_seg_chunks");
    // nch -> chunk_start, multi -> partial_start (in place, n+1 entries)
    rc = exclusive_scan_u32(w.nch, w.nch, n + 1, w.part, s, w.counters + kCntU, 1);
    if (rc != ET_OK) return rc;
    rc = exclusive_scan_u32(w.multi, w.multi, n + 1, w.part, s, w.counters + kCntU, 1);
    if (rc != ET_OK) return rc;
    hipLaunchKernelGGL(k_chunk_records, dim3(fixed_grid), dim3(256), 0, s, w.nch, w.seg_start,
                       w.multi, out.keys, chunk, w.counters, w.recs);
    hipLaunchKernelGGL(k_chunk_records_multi, dim3(512), dim3(256), 0, s, w.nch, w.seg_start,
                       w.multi, out.keys, w.mlist, chunk, w.counters, w.recs);
    ET_LAUNCH_CHECK("k_chunk_records");
    if (hot_mask && w.hot_hist && hl && hl->n > 0) {
        ET_HIP_CHECK(hipMemsetAsync(w.hot_hist, 0, 4 * (32 * 32 + 32), s));
        hipLaunchKernelGGL(k_hot_hist, dim3(256), dim3(256), 0, s, pack, ntables, hot_mask,
                           out.keys, w.seg_start, w.mlist, w.counters, w.hot_hist);
        hipLaunchKernelGGL(k_hot_pick, dim3(256), dim3(256), 0, s, pack, ntables, hot_mask,
                           out.keys, w.seg_start, w.nch, w.mlist, w.counters, w.hot_hist,
                           w.hot_cnt, w.hot_key, w.recs, sent);
        ET_LAUNCH_CHECK("k_hot_pick");
        hipLaunchKernelGGL(k_hot_slots,
                           dim3((unsigned)cdiv64(w.hot_nw * (int64_t)kHotWin, kHotSlotBags),
                                (unsigned)hl->n),
                           dim3(256), 0, s, pack, *hl, w.hot_cnt, w.hot_key, w.hot_slots);
        ET_LAUNCH_CHECK("k_hot_slots");
    }
    return ET_OK;
}

// Float32 tables on the vector kernels, grouped by power-of-two capacity (one pass of
// k_sgd_chunks / k_sgd_combine per capacity; each pass skips the other tables).
struct VecGroups {
    int n = 0;
    int cap[8];
    uint32_t mask[8];
    bool add(int c, int t) {
        for (int i = 0; i < n; ++i)
            if (cap[i] == c) {
                mask[i] |= 1u << t;
                return true;
            }
        if (n == 8) return false;
        cap[n] = c;
        mask[n++] = 1u << t;
        return true;
    }
};

// Single-occurrence columns through k_sgd_singles (ET_SGD_SINGLES=0 in an experiment build
// turns it off) and the chunk pass at 5 waves per SIMD (ET_SGD_OCC5=0: k_sgd_chunks).
inline bool sgd_singles() { return ET_KNOB("ET_SGD_SINGLES", 1) != 0; }
inline bool sgd_chunks_occ5() { return ET_KNOB("ET_SGD_OCC5", 1) != 0; }

// The chains of an exact update phase: the side streams of the early chains and of the early
// hot columns (null: none) and their column counts, the side stream of the regular chains
// (forked from the caller's stream after the index phase).
struct ChainRun {
    hipStream_t ec_side = nullptr;
    uint32_t ec_ncols = 0;
    hipStream_t eh_side = nullptr;  // the early hot columns (EH)
    uint32_t eh_ncols = 0;
    hipStream_t side = nullptr;
};

// Chain workgroups (one CU each): 32 early, 32 early-hot, 128 regular, so the regular chains
// find free CUs when the index phase releases them instead of waiting for early-chain
// workgroups (config 4, one box, twice: 256/256 4.62-4.63 ms, 32/128 4.19-4.27, 16/96
// 4.25-4.29, 64/192 4.42-4.44; profiles/r03/b/ab_exact_knobs.txt; 40/48/64 early-hot
// workgroups 4.14-4.32 against 4.05-4.08, profiles/r04/ab_exact_grid.txt).
constexpr unsigned kEcWg = 32, kEhWg = 32, kRegWg = 128;
// Chain launches on SIMDs of their own (k_sgd_chains_x): bit 0 early, bit 1 regular, bit 2
// early hot.  The early lists only (config 4, A/B twice on one box: none 4.02-4.11 ms, early
// 4.015-4.017, regular 4.33-4.34, both 4.35; profiles/r03/e/ab_chain_excl.txt; non-exclusive
// early hot columns 4.10-4.34 ms, profiles/r04/ab_exact_grid.txt): the regular chains run
// beside the chunk pass, which needs those SIMDs more.
constexpr unsigned kChainExcl = 5;
// The exact mode's chunk pass + singles run at most 512 + 512 grid-stride workgroups: fewer in
// flight than the split mode's 16384 + 16384 leaves the fabric to the latency-bound chains
// beside it (config 4, A/B twice on one box: 4.22-4.24 ms at the split mode's grid, 4.05-4.06
// at 384-768, 4.20 at 256; the split mode itself is faster at its own grid, 3.00 vs 3.61 ms;
// profiles/r04/ab_exact_grid.txt).  384, not 512: 2 x 384 workgroups fit at once beside the 64
// CUs of exclusive early chains (4 per free CU, 1 per chain CU: 832), so none of them is left
// pending in the dispatcher — a pending one held back every dispatch with LDS on the other
// queues (the regular plan's k_scan_down, 17 KB, waited 0.6 ms; 4.01-4.02 ms at 384 against
// 4.16 at 512, profiles/r05/exact_grid/).
constexpr unsigned kExactGrid = 384;

// k_sgd_chains on stream `s`: zero the item counter, at most `nb` workgroups.
template <typename T, typename C, int MODE, bool NT>
int launch_chains(const UpdatePack& pack, int ntables, uint32_t* counters, const ChainCol* chains,
                  const uint32_t* order, const ChainEnt& ce, int ns, C eta_c, double eta64,
                  unsigned nb, hipStream_t s, bool excl, uint32_t list, bool wide = false) {
    if (ET_KNOB("ET_CHAIN_STREAM", 1)) list |= 0x100u;
    // the quad walk for Float32 S = 1 chains of at least this many 64-entry groups (§9 "The
    // quad walk": every S = 1 chain 5.56 ms, >= 4 K / 16 K / 64 K / 128 K entries 5.20 / 4.99 /
    // 4.07-4.16 / 4.36 ms, none 4.48-4.52; profiles/r03/c/ab_quad_min.txt)
    const uint32_t quad_min = (uint32_t)ET_KNOB("ET_QUAD_MIN", (long long)kQuadMinGroups);
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&k_sgd_chains<T, C, MODE, NT>),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)kChainReserveLds);
    ET_HIP_CHECK(attr);
    static const hipError_t attr_x = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&k_sgd_chains_x<T, C, MODE, NT>),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)kChainReserveLds);
    ET_HIP_CHECK(attr_x);
    static const hipError_t attr_w = hipFuncSetAttribute(
        reinterpret_cast<const void*>(&k_sgd_chains_w<T, C, MODE, NT>),
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)kChainReserveLds);
    ET_HIP_CHECK(attr_w);
    ET_HIP_CHECK(hipMemsetAsync(counters + kCntNext, 0, 4, s));
    if (wide) {
        hipLaunchKernelGGL((k_sgd_chains_w<T, C, MODE, NT>), dim3(nb), dim3(512),
                           kChainReserveLds, s, pack, ntables, counters, chains, order, ce, ns,
                           eta_c, eta64, quad_min, list);
        ET_LAUNCH_CHECK("k_sgd_chains_w");
        return ET_OK;
    }
    if (excl) {
        hipLaunchKernelGGL((k_sgd_chains_x<T, C, MODE, NT>), dim3(nb), dim3(256),
                           kChainReserveLds, s, pack, ntables, counters, chains, order, ce, ns,
                           eta_c, eta64, quad_min, list);
        ET_LAUNCH_CHECK("k_sgd_chains_x");
        return ET_OK;
    }
    hipLaunchKernelGGL((k_sgd_chains<T, C, MODE, NT>), dim3(nb), dim3(256), kChainReserveLds, s,
                       pack, ntables, counters, chains, order, ce, ns, eta_c, eta64, quad_min,
                       list);
    ET_LAUNCH_CHECK("k_sgd_chains");
    return ET_OK;
}

// The three chain lists of an exact update phase on their side streams: the early chains and
// the early hot columns (already planned) and the regular chains.
template <typename T, typename C, int MODE, bool NT>
int launch_chain_lists(const UpdatePack& pack, int ntables, UpdateWs& w, int ns, C eta_c,
                       double eta64, const ChainRun& cr) {
    const unsigned excl = (unsigned)ET_KNOB("ET_CHAIN_EXCL", kChainExcl);
    int rc;
    if (cr.ec_side) {
        const int64_t items = (int64_t)cr.ec_ncols * ns;
        const unsigned wg = (unsigned)ET_KNOB("ET_EC_WG", kEcWg);
        const unsigned eb = (unsigned)(cdiv64(items, 4) < wg ? cdiv64(items, 4) : wg);
        rc = launch_chains<T, C, MODE, NT>(pack, ntables, w.ec.counters, w.ec.chains, w.ec.order,
                                           w.ec.ent, ns, eta_c, eta64, eb, cr.ec_side,
                                           (excl & 1u) != 0, 0u);
        if (rc != ET_OK) return rc;
    }
    if (cr.eh_side) {
        const int64_t items = (int64_t)cr.eh_ncols * ns;
        const unsigned wg = (unsigned)ET_KNOB("ET_EH_WG", kEhWg);
        const unsigned eb = (unsigned)(cdiv64(items, 4) < wg ? cdiv64(items, 4) : wg);
        // ET_EH_WIDE (experiments): eight waves per early-hot workgroup (k_sgd_chains_w)
        const bool wide = ET_KNOB("ET_EH_WIDE", 0) != 0;
        rc = launch_chains<T, C, MODE, NT>(pack, ntables, w.eh.counters, w.eh.chains, w.eh.order,
                                           w.eh.ent, ns, eta_c, eta64, eb, cr.eh_side,
                                           (excl & 4u) != 0 && !wide, 2u, wide);
        if (rc != ET_OK) return rc;
    }
    return launch_chains<T, C, MODE, NT>(pack, ntables, w.counters, w.chains, w.chain_order,
                                         w.chain_ent, ns, eta_c, eta64,
                                         (unsigned)ET_KNOB("ET_CHAIN_WG", kRegWg), cr.side,
                                         (excl & 2u) != 0, 1u);
}

// The update phase of an exact Float32 call: the chain lists on the side streams, the chunk
// pass over single-chunk columns + the singles in one launch per capacity group on the
// caller's stream, then the generic tables' single-chunk columns.  No partial sums, no
// combine.
template <int MODE, bool NT>
int launch_sgd_exact(const UpdatePack& pack, int ntables, const Grouped& gr, UpdateWs& w,
                     int pdim, uint32_t sent, float eta32, double eta64, const VecGroups& vg,
                     bool any_generic, hipStream_t s, unsigned grid, const ChainRun& cr) {
    const int ns = (pdim + 63) / 64;
    const unsigned xcap = (unsigned)ET_KNOB("ET_EXACT_GRID", kExactGrid);
    grid = grid < xcap ? grid : xcap;
    int rc = launch_chain_lists<float, float, MODE, NT>(pack, ntables, w, ns, eta32, eta64, cr);
    if (rc != ET_OK) return rc;
#define ET_SGD_EXACT(DD)                                                                       \
    case DD:                                                                                   \
        hipLaunchKernelGGL((k_sgd_exact<DD, MODE, NT>), dim3(2 * grid), dim3(256), 0, s, pack, \
                           ntables, gr.keys, gr.vals, w.recs, w.counters, sent, eta32, eta64,  \
                           vg.mask[i], grid);                                                  \
        break;
    for (int i = 0; i < vg.n; ++i) {
        switch (vg.cap[i]) {
            ET_SGD_EXACT(16)
            ET_SGD_EXACT(32)
            ET_SGD_EXACT(64)
            ET_SGD_EXACT(128)
            ET_SGD_EXACT(256)
            ET_SGD_EXACT(512)
            ET_SGD_EXACT(1024)
            ET_SGD_EXACT(2048)
            default: break;
        }
    }
#undef ET_SGD_EXACT
    ET_LAUNCH_CHECK("k_sgd_exact");
    if (any_generic) {
        hipLaunchKernelGGL((k_sgd_chunks_generic<float, float, MODE, NT>), dim3(grid), dim3(256),
                           0, s, pack, ntables, gr.keys, gr.vals, w.recs, w.counters, w.partials,
                           pdim, sent, eta32, eta64, 1);
        ET_LAUNCH_CHECK("k_sgd_chunks_generic");
    }
    return ET_OK;
}

// The exact update phase of Float64 / Float16 / BFloat16 tables: the same three chain lists
// (walked by chain_walk_wide in the accumulator type) beside the generic chunk pass over the
// single-chunk columns (one wave per chunk, serial in occurrence order).
template <typename T, typename C, int MODE, bool NT>
int launch_sgd_exact_generic(const UpdatePack& pack, int ntables, const Grouped& gr, UpdateWs& w,
                             int pdim, uint32_t sent, C eta_c, double eta64, hipStream_t s,
                             unsigned grid, const ChainRun& cr) {
    int rc = launch_chain_lists<T, C, MODE, NT>(pack, ntables, w, (pdim + 63) / 64, eta_c, eta64,
                                                cr);
    if (rc != ET_OK) return rc;
    hipLaunchKernelGGL((k_sgd_chunks_generic<T, C, MODE, NT>), dim3(grid), dim3(256), 0, s, pack,
                       ntables, gr.keys, gr.vals, w.recs, w.counters,
                       reinterpret_cast<C*>(w.partials), pdim, sent, eta_c, eta64, 1);
    ET_LAUNCH_CHECK("k_sgd_chunks_generic");
    return ET_OK;
}

template <typename T, typename C, int MODE, bool NT>
int launch_sgd_typed(const UpdatePack& pack, int ntables, const Grouped& gr, UpdateWs& w,
                     uint32_t chunk, int pdim, uint32_t sent, C eta_c, double eta64,
                     const VecGroups& vg, bool any_generic, hipStream_t s,
                     const HotList& hl, unsigned grid, bool chain, const ChainRun& cr) {
    if (chain) {
        if constexpr (__is_same(T, float))
            return launch_sgd_exact<MODE, NT>(pack, ntables, gr, w, pdim, sent, eta_c, eta64, vg,
                                              any_generic, s, grid, cr);
        else
            return launch_sgd_exact_generic<T, C, MODE, NT>(pack, ntables, gr, w, pdim, sent,
                                                            eta_c, eta64, s, grid, cr);
    }
    if constexpr (__is_same(T, float)) {
        const bool singles = sgd_singles();
        // combine workgroups of k_sgd_tail: a quarter of one resident wave of workgroups,
        // so the singles start at once beside them
        const unsigned ncomb = grid < 256u ? grid : 256u;
        if (hl.n > 0 && w.hot_part) {
            hipLaunchKernelGGL(k_sgd_hot, dim3((unsigned)w.hot_nw, (unsigned)hl.n), dim3(256), 0, s,
                               pack, hl, w.hot_cnt, w.hot_slots, w.hot_part, w.hot_nw);
            hipLaunchKernelGGL((k_hot_combine<MODE, NT>),
                               dim3((unsigned)cdiv64((int64_t)hl.n * kHotSlots, 4)), dim3(256), 0,
                               s, pack, hl, w.hot_cnt, w.hot_key, w.hot_part, w.hot_nw,
                               (float)eta_c, eta64);
            ET_LAUNCH_CHECK("k_sgd_hot");
        }
#define ET_SGD_VEC(DD)                                                                         \
    case DD:                                                                                   \
        if (sgd_chunks_occ5())                                                                 \
            hipLaunchKernelGGL((k_sgd_chunks5<DD, MODE, NT>), dim3(grid), dim3(256), 0, s,     \
                               pack, ntables, gr.keys, gr.vals, w.recs, w.counters,            \
                               w.partials, pdim, sent, eta_c, eta64, vg.mask[i],               \
                               singles ? 1 : 0);                                               \
        else                                                                                   \
            hipLaunchKernelGGL((k_sgd_chunks<DD, MODE, NT>), dim3(grid), dim3(256), 0, s,      \
                               pack, ntables, gr.keys, gr.vals, w.recs, w.counters,            \
                               w.partials, pdim, sent, eta_c, eta64, vg.mask[i],               \
                               singles ? 1 : 0);                                               \
        if (singles)                                                                           \
            hipLaunchKernelGGL((k_sgd_tail<DD, MODE, NT>), dim3(grid + ncomb), dim3(256), 0, s, \
                               pack, ntables, gr.keys, gr.vals, w.recs, w.seg_start, w.multi,  \
                               w.counters, w.mlist, w.partials, pdim, sent, eta_c, eta64,      \
                               vg.mask[i], ncomb);                                             \
        else                                                                                   \
            hipLaunchKernelGGL((k_sgd_combine<DD, MODE, NT>), dim3(grid), dim3(256), 0, s,     \
                               pack, ntables, gr.keys, w.seg_start, w.multi, w.counters,       \
                               w.mlist, w.partials, pdim, sent, eta_c, eta64, vg.mask[i]);     \
        break;
        for (int i = 0; i < vg.n; ++i) switch (vg.cap[i]) {
            ET_SGD_VEC(16)
            ET_SGD_VEC(32)
            ET_SGD_VEC(64)
            ET_SGD_VEC(128)
            ET_SGD_VEC(256)
            ET_SGD_VEC(512)
            ET_SGD_VEC(1024)
            ET_SGD_VEC(2048)
            default: break;
            }
#undef ET_SGD_VEC
        ET_LAUNCH_CHECK("k_sgd_chunks");
    }
    if (any_generic) {
        C* partials = reinterpret_cast<C*>(w.partials);
        hipLaunchKernelGGL((k_sgd_chunks_generic<T, C, MODE, NT>), dim3(grid), dim3(256), 0, s,
                           pack, ntables, gr.keys, gr.vals, w.recs, w.counters, partials, pdim,
                           sent, eta_c, eta64, 0);
        hipLaunchKernelGGL((k_sgd_combine_generic<T, C, MODE, NT>), dim3(grid), dim3(256), 0, s,
                           pack, ntables, gr.keys, w.seg_start, w.multi, w.counters, partials,
                           pdim, sent, eta_c, eta64);
        ET_LAUNCH_CHECK("k_sgd_chunks_generic");
    }
    return ET_OK;
}

// convert(T, eta) for table type `dtype` (exact in the accumulator type).
inline double convert_eta(int dtype, double eta) {
    switch (dtype) {
        case ET_F32: return (double)(float)eta;
        case ET_F16: return (double)(_Float16)eta;  // correctly rounded from Float64
        case ET_BF16: {
            float f = (float)eta;
            uint32_t x;
            __builtin_memcpy(&x, &f, 4);
            x = (x + 0x7fffu + ((x >> 16) & 1u)) & 0xffff0000u;  // RNE (eta is finite)
            __builtin_memcpy(&f, &x, 4);
            return (double)f;
        }
        default: return eta;
    }
}

// Element type + accumulator dispatch, then MODE / NT.
template <typename T, typename C>
int launch_sgd_dtype(const UpdatePack& pack, int ntables, const Grouped& gr, UpdateWs& w,
                     uint32_t chunk, int pdim, uint32_t sent, double eta_c, double eta64,
                     int mode, bool nt, const VecGroups& vg, bool any_generic, hipStream_t s,
                     const HotList& hl, unsigned grid, bool chain, const ChainRun& cr) {
#define ET_SGD_CALL(M, NTV)                                                                \
    return launch_sgd_typed<T, C, M, NTV>(pack, ntables, gr, w, chunk, pdim, sent, (C)eta_c, \
                                          eta64, vg, any_generic, s, hl, grid, chain, cr)
    if (mode == 0) {
        if (nt) ET_SGD_CALL(0, true);
        ET_SGD_CALL(0, false);
    } else if (mode == 1) {
        if (nt) ET_SGD_CALL(1, true);
        ET_SGD_CALL(1, false);
    }
    if (nt) ET_SGD_CALL(2, true);
    ET_SGD_CALL(2, false);
#undef ET_SGD_CALL
}

// Workgroups of the chunk / combine passes (grid-stride): one per 2048 occurrences,
// 256..16384 — 16384 measured 3% faster than 4096 on the config-4 batch (3.72 vs 3.84
// ms), and small batches launch fewer idle workgroups.
inline unsigned sgd_grid(int64_t n) {
    const int64_t g = cdiv64(n, 2048);
    return (unsigned)(g < 256 ? 256 : g > 16384 ? 16384 : g);
}

// Tables the hot-column pass can take (the workspace is sized for all of them).
inline bool hot_shape(const et_update_desc& d) {
    return d.dim == 128 && d.pool >= 1 && d.pool <= kHotMaxPool && d.batch > 0;
}

// Hot-shaped tables: their count, largest batch, and slot-byte offsets (soff[t]) / total.
inline void hot_sizes(const et_update_desc* descs, int ntables, int* nhot, int64_t* batch,
                      int64_t* bytes, uint64_t* soff = nullptr) {
    *nhot = 0;
    *batch = 0;
    *bytes = 0;
    for (int t = 0; t < ntables; ++t)
        if (hot_shape(descs[t])) {
            ++*nhot;
            if (descs[t].batch > *batch) *batch = descs[t].batch;
            if (soff) soff[t] = (uint64_t)*bytes;
            *bytes += descs[t].batch * ((descs[t].pool + 3) & ~3);
        }
}

inline int validate_update(const et_update_desc* descs, int ntables, int64_t* n_out,
                           uint64_t* rows_out, int* pdim_out, bool need_delta = true) {
    if (ntables < 0) return fail(ET_ERR_ARG, "negative ntables");
    if (ntables > ET_MAX_TABLES_PER_LAUNCH)
        return fail(ET_ERR_ARG, "at most %d tables per update call", ET_MAX_TABLES_PER_LAUNCH);
    if (ntables > 0 && !descs) return fail(ET_ERR_ARG, "descs is NULL");
    int64_t n = 0;
    uint64_t rows = 0;
    int pdim = 0;
    for (int t = 0; t < ntables; ++t) {
        const et_update_desc& d = descs[t];
        if (d.dim < 0 || d.pool < 0 || d.nrows < 0 || d.batch < 0 || d.cols_per_page < 0)
            return fail(ET_ERR_ARG, "table %d: negative size", t);
        if (d.pool > 0 && d.batch > 0) {
            if (!d.idx || (need_delta && (!d.table || !d.delta)))
                return fail(ET_ERR_ARG, "table %d: NULL", t);
            if (d.ld_idx < d.pool) return fail(ET_ERR_ARG, "table %d: ld_idx < pool", t);
            if (d.ld_table < d.dim || d.ld_delta < d.dim)
                return fail(ET_ERR_ARG, "table %d: leading dimension < dim", t);
        }
        n += (int64_t)d.pool * d.batch;
        rows += (uint64_t)d.nrows;
        if (d.dim > pdim) pdim = d.dim;
    }
    if (n >= 0xffffffffll) return fail(ET_ERR_ARG, "too many occurrences (%lld)", (long long)n);
    if (rows >= 0xffffffffull) return fail(ET_ERR_ARG, "too many table columns");
    *n_out = n;
    *rows_out = rows;
    *pdim_out = (pdim + 3) & ~3;
    return ET_OK;
}

// Early-chain tables of these descriptors (ec_table) and their occurrences; the list
// sizes the workspace whatever the flags, and et_sparse_sgd uses it in exact Float32 mode.
// hot = true: the big tables' hot-column list (eh_table, kEhK slots each; empty unless ET_EH).
inline EcList ec_list(const et_update_desc* descs, int ntables, int64_t* occ, bool hot = false) {
    EcList ec;
    ec.n = 0;
    ec.mask = 0;
    ec.hot = hot ? 1 : 0;
    ec.blk0[0] = ec.col0[0] = ec.cb0[0] = 0;
    *occ = 0;
    if (hot && !eh_enabled()) return ec;
    for (int t = 0; t < ntables; ++t) {
        const et_update_desc& d = descs[t];
        if (hot ? !eh_table(d) : !ec_table(d)) continue;
        const uint32_t nb = (uint32_t)cdiv64(d.batch, kEcBags);
        const uint32_t cols = hot ? (uint32_t)kEhK : (uint32_t)d.nrows;
        ec.t[ec.n] = t;
        ec.mask |= 1u << t;
        ec.blk0[ec.n + 1] = ec.blk0[ec.n] + nb;
        ec.col0[ec.n + 1] = ec.col0[ec.n] + cols;
        ec.cb0[ec.n + 1] = ec.cb0[ec.n] + nb * cols;
        *occ += d.pool * d.batch;
        ++ec.n;
    }
    return ec;
}

inline EhMap eh_map(const EcList& eh) {
    EhMap m;
    m.mask = eh.hot ? eh.mask : 0u;
    for (int t = 0; t < ET_MAX_TABLES_PER_LAUNCH; ++t) m.e[t] = 0;
    for (int e = 0; e < eh.n && eh.hot; ++e) m.e[eh.t[e]] = (int8_t)e;
    return m;
}

// Exact mode: columns of more occurrences than this are serial chains (k_sgd_chains), the
// rest single chunks of the chunk pass.
constexpr uint32_t kExactChunk = ET_SGD_CHUNK;

// Three side streams per device (highest priority) for the exact mode's chains: stream 0
// the early chains and stream 2 the early hot columns (both planned from the index arrays,
// forked from the caller's stream at the start of the call), stream 1 the regular chains
// (forked after the index phase); the index phase and the chunk pass run on the caller's
// stream.  All are joined back into the caller's stream inside the same library call, so a
// HIP graph capture of the caller's stream captures every branch.  The fork/join events are
// shared, so a call that uses the side streams holds `mu` from its first fork to its last
// join.
//
// When the side queues are opened matters.  A process's hardware queues
// are spread over the command processor's pipes in the order they are opened (queue i on
// pipe (i - 1) mod 4 fits every measurement below), and a queue that shares a pipe with a
// queue holding a long-running kernel or a blocked barrier (a stream wait) dispatches its
// own kernels 2-4x more slowly.  Round 4 opened the side queues at the first exact update:
// the caller's queue is usually the process's first, so the three side queues took the three
// other pipes — unless the process had opened other queues in between (a torch.cuda.graph
// capture, or ANY stream that ran a kernel: tools/capture_effect.py), which put one side
// queue on the caller's pipe: the index phase's kernels ran 2-4x longer and the config-4
// update took 5.1-5.3 ms instead of 4.03-4.07 (profiles/r05/capture/).  Moving all of the
// call's work to library streams (the caller's queue then holds only the join barriers) was
// tried: 4.15-4.29 ms with other queues open, 4.63-4.69 ms without (the work queue then
// shares the caller's pipe and its blocked join barrier; ET_WORK_STREAM=1 in experiment
// builds, profiles/r05/queue_layout.txt).  So the caller's stream keeps the work, and the
// side queues are opened at the FIRST call into the library on the device, of any entry
// point (et::open_side_streams(), from every stream-taking ABI function), right after the
// caller's own queue, before most programs open other streams; init() touches each with an
// event record, which acquires its hardware queue.
//
// Round 6 (profiles/r06/queue_layout/): a program that opens one or two
// streams (or one stream and a graph capture) BEFORE its first library call still gets a side
// queue on its pipe.  Measured and not kept: reading the pipe from HW_REG_HW_ID (its pipe /
// queue fields name the XCC-local dispatch path and are the same for every stream:
// tools/microbench/hwid_probe.hip), and four candidate side streams with the one to leave out
// learned per caller stream from timed calls (the learned choice was right in a clean process
// but every choice timed slow in the first-streams layouts, though the same choice fixed from
// the start ran at full speed: the cost depends on the queues' history, not only on their
// order).  Kept: the side streams at the least priority (below), which leaves the caller's
// normal-priority queues to the caller and makes a shared pipe cost +16% instead of +30%.
struct SideStreams {
    static constexpr int kN = 4;  // early chains, regular chains, early hot columns, work
    static constexpr int kEc = 0, kReg = 1, kEh = 2, kWork = 3;
    std::mutex mu;
    hipStream_t st[kN] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t fork[kN] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t join[kN] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t cand = nullptr;  // the hot-column candidates are picked (k_eh_pick)
};

// The work stream (kWork) exists only for the ET_WORK_STREAM experiment.
inline int side_stream_count() { return ET_KNOB("ET_WORK_STREAM", 0) ? 4 : 3; }

inline SideStreams* side_streams() {
    static SideStreams streams[64];
    static std::mutex init_mu;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    SideStreams& ss = streams[dev];
    std::lock_guard<std::mutex> lk(init_mu);
    if (!ss.cand) {
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) return nullptr;
        const int n = side_stream_count();
        // The side streams take the LEAST priority (round 6): their queues then come from the
        // low-priority pool, not from the caller's normal-priority queues, and when one does
        // share the caller's pipe the pipe favours the caller's dispatches — config 4 with
        // one or two streams opened before the library's first call: 4.28-4.46 ms instead of
        // 4.72-4.81 at the greatest priority; 3.66-3.71 ms in every other layout measured
        // (profiles/r06/queue_layout/).  ET_SIDE_HIGH=1 (experiment builds): the greatest.
        const int prio = ET_KNOB("ET_SIDE_HIGH", 0) ? greatest : least;
        for (int i = 0; i < n; ++i)
            if ((!ss.fork[i] && hipEventCreateWithFlags(&ss.fork[i], hipEventDisableTiming)) ||
                (!ss.join[i] && hipEventCreateWithFlags(&ss.join[i], hipEventDisableTiming)) ||
                (!ss.st[i] &&
                 hipStreamCreateWithPriority(&ss.st[i], hipStreamNonBlocking, prio)))
                return nullptr;
        // acquire the hardware queues now, back to back (an event record is a packet on the
        // stream's queue)
        for (int i = 0; i < n; ++i)
            if (hipEventRecord(ss.join[i], ss.st[i]) != hipSuccess) return nullptr;
        if (hipEventCreateWithFlags(&ss.cand, hipEventDisableTiming) != hipSuccess) return nullptr;
    }
    return &ss;
}

// fork(i, from): side stream i waits for everything `from` (default: the caller's stream)
// has queued so far; the destructor joins every forked side stream into the caller's stream
// (every return path of et_sparse_sgd).
struct SideFork {
    SideStreams* ss = nullptr;
    hipStream_t main = nullptr;
    std::unique_lock<std::mutex> lk;
    bool forked[SideStreams::kN] = {false, false, false, false};
    SideFork(SideStreams* s, hipStream_t m) : ss(s), main(m) {
        if (ss) lk = std::unique_lock<std::mutex>(ss->mu);
    }
    hipStream_t fork(int i, hipStream_t from = nullptr) {
        if (!ss) return nullptr;
        if (!forked[i]) {
            if (hipEventRecord(ss->fork[i], from ? from : main) != hipSuccess ||
                hipStreamWaitEvent(ss->st[i], ss->fork[i], 0) != hipSuccess)
                return nullptr;
            forked[i] = true;
        }
        return ss->st[i];
    }
    ~SideFork() {
        for (int i = 0; i < SideStreams::kN; ++i)
            if (forked[i]) {
                (void)hipEventRecord(ss->join[i], ss->st[i]);
                (void)hipStreamWaitEvent(main, ss->join[i], 0);
            }
    }
};

// The early-chain plan (k_ec_count -> k_ec_plan -> k_ec_emit) on stream `s`; for the
// hot-column list (ec.hot) after picking the candidates (k_eh_pick), whose completion
// `cand_ready` records for the regular plan (k_chain_tile_count skips the candidates).
inline int launch_ec_plan(const UpdatePack& pack, const EcList& ec, uint32_t chunk,
                          const UpdateWs::EcWs& w, const uint32_t* cand_c, int ns, hipStream_t s,
                          hipEvent_t cand_ready = nullptr) {
    const uint32_t M = ec.col0[ec.n];
    uint32_t* cand = const_cast<uint32_t*>(cand_c);
    if (ec.hot) {
        // ET_EH_MIN (experiment builds): the expected occurrences of a candidate
        const uint32_t min_occ = (uint32_t)ET_KNOB("ET_EH_MIN", (long long)kEhMinOcc);
        // ET_EH_SAMPLE (experiment builds): bags sampled per table
        const int64_t sample = ET_KNOB("ET_EH_SAMPLE", (long long)kEhSampleBags);
        hipLaunchKernelGGL(k_eh_pick, dim3(ec.n), dim3(1024), 0, s, pack, ec, min_occ, sample,
                           cand);
        ET_LAUNCH_CHECK("k_eh_pick");
        if (cand_ready) ET_HIP_CHECK(hipEventRecord(cand_ready, s));
    }
    ET_HIP_CHECK(hipMemsetAsync(w.counters, 0, 4 * kCntSlots, s));
    // the byte histogram in dynamic LDS, sized for the list's widest table (EH: kEhK slots)
    uint32_t rs = 4;
    for (int e = 0; e < ec.n; ++e) {
        const uint32_t r = (ec.col0[e + 1] - ec.col0[e] + 3u) & ~3u;
        rs = r > rs ? r : rs;
    }
    const size_t hist_lds = (size_t)kEcBags * rs;
    hipLaunchKernelGGL(k_ec_count, dim3(ec.blk0[ec.n]), dim3(kEcBags), hist_lds, s, pack, ec,
                       w.stats, cand_c);
    hipLaunchKernelGGL(k_ec_plan, dim3((M + 3u) / 4u), dim3(256), 0, s, pack, ec, chunk,
                       w.stats, w.boff, w.cnt, w.nocc, w.info, w.chains, w.ent, w.counters, 4,
                       cand_c);
    hipLaunchKernelGGL(k_ec_order, dim3(1), dim3(1024), 0, s, ec, w.info, ns, w.order,
                       w.counters);
    hipLaunchKernelGGL(k_ec_emit, dim3(ec.blk0[ec.n]), dim3(kEcBags), hist_lds, s, pack, ec,
                       w.boff, w.info, w.ent, cand_c);
    ET_LAUNCH_CHECK("k_ec_emit");
    return ET_OK;
}

}  // namespace et

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------

extern "C" int et_sgd_workspace_size(const et_update_desc* descs, int32_t ntables,
                                     int64_t* bytes) {
    et::clear_err();
    if (!bytes) return et::fail(ET_ERR_ARG, "bytes is NULL");
    int64_t n;
    uint64_t rows;
    int pdim;
    int rc = et::validate_update(descs, ntables, &n, &rows, &pdim);
    if (rc != ET_OK) return rc;
    int nhot;
    int64_t hb, hbytes;
    et::hot_sizes(descs, ntables, &nhot, &hb, &hbytes);
    int64_t ec_occ, eh_occ;
    const et::EcList ec = et::ec_list(descs, ntables, &ec_occ);
    const et::EcList eh = et::ec_list(descs, ntables, &eh_occ, true);
    *bytes = et::carve_update_ws(nullptr, n, pdim, et::kChunk, nhot, hb, hbytes, &ec, ec_occ, &eh,
                                 eh_occ).bytes;
    return ET_OK;
}

static int sparse_sgd(int dtype, const et_update_desc* descs, int32_t ntables, double eta,
                      uint32_t flags, int64_t* const* snaps, void* workspace, int64_t ws_bytes,
                      void* stream);

extern "C" int et_sparse_sgd(int dtype, const et_update_desc* descs, int32_t ntables, double eta,
                             uint32_t flags, void* workspace, int64_t ws_bytes, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    return sparse_sgd(dtype, descs, ntables, eta, flags, nullptr, workspace, ws_bytes, stream);
}

extern "C" int et_sparse_sgd_snap(int dtype, const et_update_desc* descs, int32_t ntables,
                                  double eta, uint32_t flags, int64_t* const* snaps,
                                  void* workspace, int64_t ws_bytes, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    if (!snaps) return et::fail(ET_ERR_ARG, "snaps is NULL");
    if (ntables > ET_MAX_TABLES_PER_LAUNCH)
        return et::fail(ET_ERR_ARG, "et_sparse_sgd_snap: at most %d tables per call",
                        ET_MAX_TABLES_PER_LAUNCH);
    return sparse_sgd(dtype, descs, ntables, eta, flags, snaps, workspace, ws_bytes, stream);
}

static int sparse_sgd(int dtype, const et_update_desc* descs, int32_t ntables, double eta,
                      uint32_t flags, int64_t* const* snaps, void* workspace, int64_t ws_bytes,
                      void* stream) {
    if (dtype != ET_F32 && dtype != ET_F64 && dtype != ET_F16 && dtype != ET_BF16)
        return et::fail(ET_ERR_UNSUPPORTED, "sparse SGD: dtype %d", dtype);
    const bool index_only = (flags & ET_FLAG_SGD_INDEX_ONLY) != 0;
    const bool apply_only = (flags & ET_FLAG_SGD_APPLY_ONLY) != 0;
    if (index_only && apply_only)
        return et::fail(ET_ERR_ARG, "sparse SGD: INDEX_ONLY and APPLY_ONLY both set");
    int64_t n;
    uint64_t rows;
    int pdim;
    int rc = et::validate_update(descs, ntables, &n, &rows, &pdim, !index_only);
    if (rc != ET_OK) return rc;
    if (n == 0) return ET_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // Exact mode (ET_FLAG_EXACT_UPDATE, and since ABI v9 ET_FLAG_EXACT_IF_FAST too: the chain
    // path covers every element type and gradient size): every column's gradient summed
    // serially in occurrence order, as the reference does.  Columns longer than a chunk are
    // serial chains (k_chain_*, k_sgd_chains) whose entries hold a 24-bit bag below 2^24 bags
    // and a 27-bit one from there (chain_shift), so only a batch of 2^27 bags or more keeps
    // every column in one chunk instead (a chunk then spans a whole segment: exact, one wave
    // per column).
    const bool exact = (flags & (ET_FLAG_EXACT_UPDATE | ET_FLAG_EXACT_IF_FAST)) != 0;
    bool chain = exact;
    for (int t = 0; t < ntables && chain; ++t)
        if (descs[t].batch > et::kChainMaxBatch) chain = false;
    // chain mode: a column of at most kExactChunk occurrences is one chunk of the chunk pass
    // (a lane group's serial sum), a longer one a chain
    const uint32_t chunk = exact && !chain ? (uint32_t)(n < 0x7fffffff ? n + 1 : 0x7fffffff)
                           : chain          ? et::kExactChunk
                                            : et::kChunk;
    int nhot;
    int64_t hb, hbytes;
    uint64_t soff[ET_MAX_TABLES_PER_LAUNCH];
    et::hot_sizes(descs, ntables, &nhot, &hb, &hbytes, soff);
    int64_t ec_occ, eh_occ;
    const et::EcList ec = et::ec_list(descs, ntables, &ec_occ);
    const et::EcList eh = et::ec_list(descs, ntables, &eh_occ, true);
    et::UpdateWs w = et::carve_update_ws(static_cast<char*>(workspace), n, pdim, et::kChunk,
                                         nhot, hb, hbytes, &ec, ec_occ, &eh, eh_occ);
    if (!workspace || ws_bytes < w.bytes)
        return et::fail(ET_ERR_WORKSPACE, "workspace of %lld bytes needed",
                        (long long)w.bytes);

    et::UpdatePack pack;
    uint32_t ro = 0, oo = 0;
    et::VecGroups vg;
    bool any_generic = false;
    uint32_t hot_mask = 0;
    pack.vec_mask = 0;
    for (int t = 0; t < ntables; ++t) {
        const et_update_desc& d = descs[t];
        pack.d[t] = d;
        pack.row_off[t] = ro;
        pack.occ_off[t] = oo;
        ro += (uint32_t)d.nrows;
        oo += (uint32_t)(d.pool * d.batch);
        if (d.pool == 0 || d.batch == 0 || d.dim == 0) continue;
        // paged tables qualify too: their pages are 16-byte aligned by contract
        // vector kernels at the power-of-two capacity of the dim (masked below it)
        const int cap = et::vec_dim_ok(d.dim) ? d.dim : et::masked_capacity(d.dim);
        const bool table_ok = dtype == ET_F32 && (d.cols_per_page > 0 || et::aligned16(d.table)) &&
                              (d.ld_table % 4 == 0) && d.dim % 4 == 0 && d.dim <= 2048;
        const bool delta_ok = et::aligned16(d.delta) && (d.ld_delta % 4 == 0);
        // hot-column pass (Float32 vector tables of dim 128, non-exact mode): chosen from
        // the table alone, so the index phase (which never sees the gradient, delta may be
        // NULL) and the update phase agree; the update phase then needs vector gradients
        const bool hot = table_ok && !exact && (flags & ET_FLAG_SGD_HOT_PASS) && et::hot_shape(d);
        if (hot) {
            if (apply_only && !delta_ok)
                return et::fail(ET_ERR_ARG, "table %d: the hot-column pass chosen by the index "
                                            "phase needs a 16-byte aligned gradient (ld %% 4 == 0)", t);
            if (index_only || delta_ok) hot_mask |= 1u << t;
        }
        if (table_ok && (delta_ok || index_only) && vg.add(cap, t)) {
            pack.vec_mask |= 1u << t;
        } else {
            any_generic = true;
        }
    }
    pack.row_off[ntables] = ro;
    pack.occ_off[ntables] = oo;
    const uint32_t sent = ro;  // key of out-of-range occurrences (sorts last)

    et::HotList hl;
    hl.n = 0;
    for (int t = 0; t < ntables; ++t)
        if ((hot_mask >> t) & 1u) {
            hl.soff[hl.n] = soff[t];
            hl.t[hl.n++] = t;
        }
    // exact mode: the chains run on three side streams — the early chains (small tables) and
    // the early hot columns (the big tables' hottest, sampled), both planned from the index
    // arrays from the start of the call, and the regular ones once the index phase has
    // planned them
    const bool use_ec = chain && ec.n > 0;
    const bool use_eh = chain && eh.n > 0;
    const et::EhMap ehm = et::eh_map(use_eh ? eh : et::EcList{});
    et::SideStreams* sides = chain ? et::side_streams() : nullptr;
    if (chain && !sides) return et::fail(ET_ERR_HIP, "sparse SGD: side streams unavailable");
    et::SideFork fork(sides, s);
    // ET_WORK_STREAM=1 (experiment builds): the main-line work on a library stream
    if (chain && ET_KNOB("ET_WORK_STREAM", 0)) {
        s = fork.fork(et::SideStreams::kWork);
        if (!s) return et::fail(ET_ERR_HIP, "sparse SGD: side stream fork failed");
    }
    hipStream_t ec_side = nullptr;
    if (use_ec) {
        ec_side = fork.fork(et::SideStreams::kEc);
        if (!ec_side) return et::fail(ET_ERR_HIP, "sparse SGD: side stream fork failed");
        if (!apply_only) {
            rc = et::launch_ec_plan(pack, ec, chunk, w.ec, nullptr, (pdim + 63) / 64, ec_side);
            if (rc != ET_OK) return rc;
        }
    }
    hipStream_t eh_side = nullptr;
    if (use_eh) {
        eh_side = fork.fork(et::SideStreams::kEh);
        if (!eh_side) return et::fail(ET_ERR_HIP, "sparse SGD: side stream fork failed");
        if (!apply_only) {
            rc = et::launch_ec_plan(pack, eh, chunk, w.eh, w.eh_cand, (pdim + 63) / 64, eh_side,
                                    sides->cand);
            if (rc != ET_OK) return rc;
        }
    }
    et::Grouped gr;
    if (apply_only) {
        gr = et::grouped_pairs(pack, ntables, w);  // phase 1 ran earlier in stream order
    } else {
        rc = et::group_occurrences(pack, ntables, n, sent, chunk, w, gr, s, hot_mask, &hl, chain,
                                   use_ec ? ec.mask : 0u, snaps);
        if (rc != ET_OK) return rc;
    }
    et::ChainRun cr;
    if (chain) {
        cr.ec_side = ec_side;
        cr.ec_ncols = use_ec ? ec.col0[ec.n] : 0u;
        cr.eh_side = eh_side;
        cr.eh_ncols = use_eh ? eh.col0[eh.n] : 0u;
        // the regular chains' plan: on their side stream beside the chunk pass (default), or
        // on the caller's stream before it (ET_PLAN_SIDE=0 in an experiment build: the chains
        // start earlier, the chunk pass later; 4.13-4.16 vs 4.07 ms, round 4)
        const bool plan_side = ET_KNOB("ET_PLAN_SIDE", 1) != 0;
        if (!apply_only && !plan_side) {
            rc = et::launch_chain_plan(pack, ntables, n, sent, chunk, w, gr, s,
                                       use_ec ? ec.mask : 0u, ehm, sides->cand);
            if (rc != ET_OK) return rc;
        }
        // after the index phase's chunk records (and the plan), on the work stream
        cr.side = fork.fork(et::SideStreams::kReg, s);
        if (!cr.side) return et::fail(ET_ERR_HIP, "sparse SGD: side stream fork failed");
        if (!apply_only && plan_side) {
            rc = et::launch_chain_plan(pack, ntables, n, sent, chunk, w, gr, cr.side,
                                       use_ec ? ec.mask : 0u, ehm, sides->cand);
            if (rc != ET_OK) return rc;
        }
    }
    if (index_only) return ET_OK;

    const bool nt = (flags & ET_FLAG_NONTEMPORAL) != 0;
    const int mode = (flags & ET_FLAG_SGD_UNFUSED) ? ((flags & ET_FLAG_SGD_F64_ALPHA) ? 2 : 1) : 0;
    const double eta_c = et::convert_eta(dtype, eta);
    const unsigned grid = et::sgd_grid(n);
    switch (dtype) {
        case ET_F32:
            return et::launch_sgd_dtype<float, float>(pack, ntables, gr, w, chunk, pdim, sent,
                                                      eta_c, eta, mode, nt, vg, any_generic, s,
                                                      hl, grid, chain, cr);
        case ET_F64:
            return et::launch_sgd_dtype<double, double>(pack, ntables, gr, w, chunk, pdim, sent,
                                                         eta_c, eta, mode, nt, vg, any_generic,
                                                         s, hl, grid, chain, cr);
        case ET_BF16:
            return et::launch_sgd_dtype<__bf16, float>(pack, ntables, gr, w, chunk, pdim, sent,
                                                       eta_c, eta, mode, nt, vg, any_generic, s,
                                                       hl, grid, chain, cr);
        default:  // ET_F16
            if (flags & ET_FLAG_F16_FP32_ACC)
                return et::launch_sgd_dtype<_Float16, float>(pack, ntables, gr, w, chunk, pdim,
                                                             sent, eta_c, eta, mode, nt, vg,
                                                             any_generic, s, hl, grid, chain, cr);
            return et::launch_sgd_dtype<_Float16, _Float16>(pack, ntables, gr, w, chunk, pdim,
                                                            sent, eta_c, eta, mode, nt, vg,
                                                            any_generic, s, hl, grid, chain, cr);
    }
}

// ---------------------------------------------------------------------------
// Device Indexer in the reference's layout (first-seen order)
// ---------------------------------------------------------------------------
namespace et {

__global__ __launch_bounds__(256) void k_first_occ(const uint32_t* __restrict__ keys,
                                                   const uint32_t* __restrict__ vals,
                                                   const uint32_t* __restrict__ seg_start,
                                                   const uint32_t* __restrict__ counters,
                                                   int64_t n, uint32_t sent, uint32_t pad,
                                                   uint32_t* __restrict__ fo,
                                                   uint32_t* __restrict__ seg) {
    const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (u >= n) return;
    const uint32_t U = counters[kCntU];
    uint32_t f = pad;
    if (u < U && keys[seg_start[u]] != sent) f = vals[seg_start[u]];  // stable => minimum
    fo[u] = f;
    seg[u] = (uint32_t)u;
}

// cnt[k] = occurrences of the k-th distinct column in first-seen order (0 beyond).
__global__ __launch_bounds__(256) void k_count_fs(const uint32_t* __restrict__ order_fo,
                                                  const uint32_t* __restrict__ order_seg,
                                                  const uint32_t* __restrict__ seg_start,
                                                  int64_t n, uint32_t pad,
                                                  uint32_t* __restrict__ cnt) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k > n) return;
    uint32_t c = 0;
    if (k < n && order_fo[k] != pad) {
        const uint32_t u = order_seg[k];
        c = seg_start[u + 1] - seg_start[u];
    }
    cnt[k] = c;
}

__global__ __launch_bounds__(256) void k_write_index(
    const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
    const uint32_t* __restrict__ seg_start, const uint32_t* __restrict__ order_fo,
    const uint32_t* __restrict__ order_seg, const uint32_t* __restrict__ off, int64_t n,
    uint32_t pad, uint32_t pool, int64_t* __restrict__ cum_col, int64_t* __restrict__ cum_off,
    int64_t* __restrict__ map, int64_t* __restrict__ nunique) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * 4;
    for (int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); k < n; k += waves) {
        const bool valid = order_fo[k] != pad;
        const bool last_valid = valid && (k + 1 == n || order_fo[k + 1] == pad);
        if (k == 0 && !valid && lane == 0) {  // no valid occurrence at all
            cum_col[0] = 0;
            cum_off[0] = 1;
            *nunique = 0;
        }
        if (!valid) continue;
        const uint32_t u = order_seg[k];
        const uint32_t s0 = seg_start[u], len = seg_start[u + 1] - s0;
        if (lane == 0) {
            cum_col[k] = (int64_t)keys[s0] + 1;
            cum_off[k] = (int64_t)off[k] + 1;
            if (last_valid) {
                cum_col[k + 1] = 0;
                cum_off[k + 1] = (int64_t)off[k] + len + 1;
                *nunique = k + 1;
            }
        }
        for (uint32_t q = lane; q < len; q += 64)
            map[off[k] + q] = (int64_t)(vals[s0 + q] / pool) + 1;
    }
}

struct IndexWs {
    UpdateWs u;
    uint32_t *fk, *fv, *fk2, *fv2, *cnt;
    int64_t bytes;
};

inline IndexWs carve_index_ws(char* base, int64_t n) {
    IndexWs w;
    w.u = carve_update_ws(base, n, 0, kChunk);
    int64_t off = w.u.bytes;
    auto take = [&](int64_t bytes) -> char* {
        char* p = base ? base + off : nullptr;
        off += align256(bytes);
        return p;
    };
    const int64_t n1 = n + 1;
    w.fk = (uint32_t*)take(4 * n1);
    w.fv = (uint32_t*)take(4 * n1);
    w.fk2 = (uint32_t*)take(4 * n1);
    w.fv2 = (uint32_t*)take(4 * n1);
    w.cnt = (uint32_t*)take(4 * (n1 + 1));
    w.bytes = off;
    return w;
}

}  // namespace et

extern "C" int et_index_workspace_size(int64_t n, int64_t* bytes) {
    et::clear_err();
    if (!bytes || n < 0) return et::fail(ET_ERR_ARG, "bad arguments");
    *bytes = et::carve_index_ws(nullptr, n).bytes;
    return ET_OK;
}

extern "C" int et_index_build(const int64_t* idx, int32_t pool, int64_t ld_idx, int64_t batch,
                              int64_t nrows, int64_t* cumulative_col, int64_t* cumulative_off,
                              int64_t* map, int64_t* nunique_dev, void* workspace,
                              int64_t ws_bytes, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    if (pool < 0 || batch < 0 || nrows < 0) return et::fail(ET_ERR_ARG, "negative size");
    const int64_t n = (int64_t)pool * batch;
    if (n >= 0x7fffffffll) return et::fail(ET_ERR_ARG, "too many occurrences");
    if (nrows >= 0xffffffffll) return et::fail(ET_ERR_ARG, "too many columns");
    if (!cumulative_col || !cumulative_off || !nunique_dev || (n > 0 && (!map || !idx)))
        return et::fail(ET_ERR_ARG, "NULL argument");
    if (n > 0 && ld_idx < pool) return et::fail(ET_ERR_ARG, "ld_idx < pool");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (n == 0) {
        const int64_t term[2] = {0, 1};
        const int64_t zero = 0;
        ET_HIP_CHECK(hipMemcpyAsync(cumulative_col, &term[0], 8, hipMemcpyHostToDevice, s));
        ET_HIP_CHECK(hipMemcpyAsync(cumulative_off, &term[1], 8, hipMemcpyHostToDevice, s));
        ET_HIP_CHECK(hipMemcpyAsync(nunique_dev, &zero, 8, hipMemcpyHostToDevice, s));
        ET_HIP_CHECK(hipStreamSynchronize(s));  // the host sources are on this stack frame
        return ET_OK;
    }
    et::IndexWs w = et::carve_index_ws(static_cast<char*>(workspace), n);
    if (!workspace || ws_bytes < w.bytes)
        return et::fail(ET_ERR_WORKSPACE, "workspace of %lld bytes needed", (long long)w.bytes);

    et::UpdatePack pack;
    et_update_desc d{};
    d.nrows = nrows;
    d.dim = 0;
    d.pool = pool;
    d.idx = idx;
    d.ld_idx = ld_idx;
    d.batch = batch;
    pack.d[0] = d;
    pack.vec_mask = 0;
    pack.row_off[0] = 0;
    pack.row_off[1] = (uint32_t)nrows;
    pack.occ_off[0] = 0;
    pack.occ_off[1] = (uint32_t)n;
    const uint32_t sent = (uint32_t)nrows;

    et::Grouped gr;
    int rc = et::group_occurrences(pack, 1, n, sent, et::kChunk, w.u, gr, s);
    if (rc != ET_OK) return rc;

    const uint32_t pad = (uint32_t)n;  // > every occurrence id
    const int64_t blocks = et::cdiv64(n, 256);
    hipLaunchKernelGGL(et::k_first_occ, dim3((unsigned)blocks), dim3(256), 0, s, gr.keys, gr.vals,
                       w.u.seg_start, w.u.counters, n, sent, pad, w.fk, w.fv);
    ET_LAUNCH_CHECK("k_first_occ");
    et::SortBuffers sb{w.fk, w.fv, w.fk2, w.fv2, w.u.hist, w.u.part};
    uint32_t *ofo, *oseg;
    rc = et::radix_sort_pairs(sb, n, et::bits_for(pad), &ofo, &oseg, s);
    if (rc != ET_OK) return rc;
    hipLaunchKernelGGL(et::k_count_fs, dim3((unsigned)et::cdiv64(n + 1, 256)), dim3(256), 0, s,
                       ofo, oseg, w.u.seg_start, n, pad, w.cnt);
    ET_LAUNCH_CHECK("k_count_fs");
    rc = et::exclusive_scan_u32(w.cnt, w.cnt, n + 1, w.u.part, s);
    if (rc != ET_OK) return rc;
    const int64_t wb = et::cdiv64(n, 4);
    hipLaunchKernelGGL(et::k_write_index, dim3((unsigned)(wb < 65536 ? wb : 65536)), dim3(256), 0,
                       s, gr.keys, gr.vals, w.u.seg_start, ofo, oseg, w.cnt, n, pad,
                       (uint32_t)pool, cumulative_col, cumulative_off, map, nunique_dev);
    ET_LAUNCH_CHECK("k_write_index");
    return ET_OK;
}

// ---------------------------------------------------------------------------
// Update from a reference-layout Indexer range (IndexerView)
// ---------------------------------------------------------------------------
namespace et {

template <typename T, typename C, int MODE, bool NT>
__global__ __launch_bounds__(256) void k_update_indexed(
    void* __restrict__ table, int64_t ld_table, int64_t cols_per_page, int64_t nrows, int dim,
    const T* __restrict__ delta, int64_t ld_delta, const int64_t* __restrict__ cum_col,
    const int64_t* __restrict__ cum_off, int64_t ubegin, int64_t uend,
    const int64_t* __restrict__ map, C eta_c, double eta64) {
    const int lane = threadIdx.x & 63;
    const int64_t waves = (int64_t)gridDim.x * 4;
    for (int64_t e = ubegin + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); e < uend; e += waves) {
        const uint64_t col = (uint64_t)(cum_col[e] - 1);
        if (col >= (uint64_t)nrows) {
            if (lane == 0) note_oob();
            continue;
        }
        const int64_t k0 = cum_off[e] - 1, k1 = cum_off[e + 1] - 1;
        T* w = col_ptr<T>(table, ld_table, cols_per_page, col);
        for (int f = lane; f < dim; f += 64) {
            C acc = C(0);  // zero(Tiled) / zero!(scratchspace)
            for (int64_t k = k0; k < k1; ++k)
                acc = acc + C(delta[(uint64_t)(map[k] - 1) * (uint64_t)ld_delta + f]);
            store_scalar<NT>(w + f, sgd_apply_t<T, C, MODE>(w[f], acc, eta_c, eta64));
        }
    }
}

template <typename T, typename C>
int launch_update_indexed(void* table, int64_t ld_table, int64_t cols_per_page, int64_t nrows,
                          int dim, const void* delta, int64_t ld_delta, const int64_t* cum_col,
                          const int64_t* cum_off, int64_t ubegin, int64_t uend,
                          const int64_t* map, double eta_c, double eta, int mode, bool nt,
                          hipStream_t s) {
    const int64_t nb = cdiv64(uend - ubegin, 4);
    const unsigned grid = (unsigned)(nb < 8192 ? nb : 8192);
#define ET_UI(M, NTV)                                                                           \
    hipLaunchKernelGGL((k_update_indexed<T, C, M, NTV>), dim3(grid), dim3(256), 0, s, table,   \
                       ld_table, cols_per_page, nrows, dim, (const T*)delta, ld_delta, cum_col, \
                       cum_off, ubegin, uend, map, (C)eta_c, eta)
    if (mode == 0) {
        if (nt) ET_UI(0, true); else ET_UI(0, false);
    } else if (mode == 1) {
        if (nt) ET_UI(1, true); else ET_UI(1, false);
    } else {
        if (nt) ET_UI(2, true); else ET_UI(2, false);
    }
#undef ET_UI
    ET_LAUNCH_CHECK("k_update_indexed");
    return ET_OK;
}

}  // namespace et

extern "C" int et_update_indexed(int dtype, void* table, int64_t ld_table,
                                 int64_t cols_per_page, int64_t nrows, int32_t dim,
                                 const void* delta, int64_t ld_delta,
                                 const int64_t* cumulative_col, const int64_t* cumulative_off,
                                 int64_t ubegin, int64_t uend, const int64_t* map, double eta,
                                 uint32_t flags, void* stream) {
    et::clear_err();
    et::open_side_streams(static_cast<hipStream_t>(stream));
    if (dtype != ET_F32 && dtype != ET_F64 && dtype != ET_F16 && dtype != ET_BF16)
        return et::fail(ET_ERR_UNSUPPORTED, "update: dtype %d", dtype);
    if (uend <= ubegin || dim == 0) return ET_OK;
    if (ubegin < 0 || dim < 0 || ld_table < dim || ld_delta < dim || cols_per_page < 0)
        return et::fail(ET_ERR_ARG, "bad sizes");
    if (!table || !delta || !cumulative_col || !cumulative_off || !map)
        return et::fail(ET_ERR_ARG, "NULL argument");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool nt = (flags & ET_FLAG_NONTEMPORAL) != 0;
    const int mode = (flags & ET_FLAG_SGD_UNFUSED) ? ((flags & ET_FLAG_SGD_F64_ALPHA) ? 2 : 1) : 0;
    const double eta_c = et::convert_eta(dtype, eta);
#define ET_UI_T(T, C)                                                                     \
    return et::launch_update_indexed<T, C>(table, ld_table, cols_per_page, nrows, dim, delta, \
                                           ld_delta, cumulative_col, cumulative_off, ubegin,  \
                                           uend, map, eta_c, eta, mode, nt, s)
    switch (dtype) {
        case ET_F32: ET_UI_T(float, float);
        case ET_F64: ET_UI_T(double, double);
        case ET_BF16: ET_UI_T(__bf16, float);
        default:
            if (flags & ET_FLAG_F16_FP32_ACC) ET_UI_T(_Float16, float);
            ET_UI_T(_Float16, _Float16);
    }
#undef ET_UI_T
}

ET_OOB_READER(update)

namespace et {
// Open this device's side queues at the first library call (see SideStreams); a no-op after
// that, and while the caller's stream is capturing a graph.
void open_side_streams(hipStream_t caller) {
    static std::atomic<uint64_t> done{0};  // bit d: device d's side streams are open
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return;
    if (done.load(std::memory_order_relaxed) & (1ull << dev)) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(caller, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
    if (side_streams()) done.fetch_or(1ull << dev);
}
}  // namespace et

#ifdef ET_EXPERIMENTS
// Experiment builds only: copy (and reset) the chain-item timeline, 2 x uint4 per item
// (et_update.hip chain_items); *n = items recorded (may exceed cap).
extern "C" int et_debug_chain_timeline(void* host, int64_t cap, int64_t* n) {
    uint32_t k = 0, zero = 0;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(&k, HIP_SYMBOL(et::g_ctl_n), 4, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    const int64_t m = std::min<int64_t>(std::min<int64_t>(k, cap), et::kCtlCap);
    if (m > 0 && hipMemcpyFromSymbol(host, HIP_SYMBOL(et::g_ctl), (size_t)m * 32, 0,
                                     hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(et::g_ctl_n), &zero, 4, 0, hipMemcpyHostToDevice) != hipSuccess)
        return -1;
    *n = k;
    return 0;
}
#endif
