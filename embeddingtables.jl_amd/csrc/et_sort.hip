// et_sort.hip — device-wide exclusive scan and stable LSD radix sort of
// (uint32 key, uint32 value) pairs for gfx950 (included by et_update.hip).
//
// These build the GPU equivalent of the reference's Indexer (src/utils.jl:88-314):
// sorting occurrences by table column with a STABLE sort keeps each column's
// occurrences in occurrence order, which is the order remap! (src/utils.jl:242-272)
// lays them out in `map`, so per-column gradient sums see the same addends in
// the same order as the reference.
//
// Scan: reduce tiles -> scan tile sums (one workgroup) -> scan tiles with offset.
// Sort pass (8- or 9-bit digit): per-tile digit histogram (LDS atomics) -> segment-,
// then digit-major exclusive scan -> stable scatter, where each 8192-key tile is ranked in 32 rounds of
// 256 keys (striped, so rounds follow input order) and each round ranks a key among
// equal digits of lower lanes by one wave ballot per digit bit + per-wave digit counts
// in LDS.
#include "et_common.h"

namespace et {

constexpr int kScanThreads = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanThreads * kScanItems;  // 4096
constexpr int kScanPartialsLds = 16384;               // partials staged in LDS (64 KB)
constexpr int kScanStageMin = 1024;                   // fewer partials: read in place

constexpr int kRsMaxBits = 9;  // digit width: 9 bits -> 3 passes for keys < 2^27
constexpr int kRsMaxBuckets = 1 << kRsMaxBits;
constexpr int kRsThreads = 256;
constexpr int kRsItems = 32;
constexpr int kRsTile = kRsThreads * kRsItems;  // 8192 keys per workgroup

inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Inclusive scan of one value per thread across a 256-thread workgroup.
// Returns the inclusive prefix; *total receives the workgroup sum.
__device__ __forceinline__ uint32_t block_inclusive_scan_256(uint32_t v, uint32_t* lds4,
                                                             uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, 64);
        if (lane >= o) v += t;
    }
    if (lane == 63) lds4[wave] = v;
    __syncthreads();
    uint32_t off = 0;
    for (int w = 0; w < wave; ++w) off += lds4[w];
    *total = lds4[0] + lds4[1] + lds4[2] + lds4[3];
    __syncthreads();
    return v + off;
}

// `mlen` (optional, device): the scan covers min(m, *mlen + madd) elements — a length
// only known on the device (e.g. the number of segments); tiles beyond it do nothing.
__device__ __forceinline__ int64_t scan_len(int64_t m, const uint32_t* mlen, uint32_t madd) {
    if (!mlen) return m;
    const int64_t l = (int64_t)*mlen + madd;
    return l < m ? l : m;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const uint32_t* __restrict__ in,
                                                              int64_t m,
                                                              uint32_t* __restrict__ part,
                                                              const uint32_t* __restrict__ mlen,
                                                              uint32_t madd) {
    __shared__ uint32_t lds4[4];
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    m = scan_len(m, mlen, madd);
    if (base >= m) {
        if (threadIdx.x == 0) part[blockIdx.x] = 0;
        return;
    }
    uint32_t s = 0;
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const int64_t i = base + r * kScanThreads + threadIdx.x;
        if (i < m) s += in[i];
    }
    uint32_t total;
    block_inclusive_scan_256(s, lds4, &total);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

// Exclusive scan of part[0..np) in place by one workgroup; part[np] = total.  STAGED (host
// chosen, np > kScanStageMin) stages the partials in 64 KB of LDS; the unstaged variant
// asks for 16 bytes, so it finds a CU at once beside persistent workgroups that hold most
// of the LDS (the exact update's chain-plan scan, 2-3 partials, waited 585 us for 64 KB
// beside k_sgd_exact).
template <bool STAGED>
__global__ __launch_bounds__(kScanThreads) void k_scan_partials(uint32_t* __restrict__ part,
                                                                int64_t np,
                                                                const uint32_t* __restrict__ mlen,
                                                                uint32_t madd) {
    __shared__ uint32_t lds4[4];
    if (mlen) {  // tiles past the device-side length hold zeros and are never read
        const int64_t used = ((int64_t)*mlen + madd + kScanTile - 1) / kScanTile;
        np = used < np ? used : np;
    }
    // one block scan: thread t owns the contiguous run [t*per, (t+1)*per) (a loop of
    // 256-wide block scans costs two barriers and a dependent load per 256 entries —
    // 26 us for the 8.3 K tiles of a 34 M-key segment scan)
    // Up to 16384 partials (a 64 M-element scan) are staged in LDS with coalesced loads
    // and stores; the per-thread runs then read LDS instead of strided global words.
    __shared__ uint32_t sp[STAGED ? kScanPartialsLds : 1];
    const bool staged = STAGED && np <= kScanPartialsLds;  // workgroup-uniform
    uint32_t* p = staged ? sp : part;
    if (staged) {  // all loads issued before the LDS stores (one memory latency)
        uint32_t buf[kScanPartialsLds / kScanThreads];
#pragma unroll
        for (int r = 0; r < kScanPartialsLds / kScanThreads; ++r) {
            const int64_t i = r * kScanThreads + threadIdx.x;
            buf[r] = i < np ? part[i] : 0u;
        }
#pragma unroll
        for (int r = 0; r < kScanPartialsLds / kScanThreads; ++r)
            sp[r * kScanThreads + threadIdx.x] = buf[r];
        __syncthreads();
    }
    const int64_t per = (np + kScanThreads - 1) / kScanThreads;
    const int64_t i0 = (int64_t)threadIdx.x * per;
    const int64_t i1 = i0 + per < np ? i0 + per : np;
    uint32_t s = 0;
    for (int64_t i = i0; i < i1; ++i) s += p[i];
    uint32_t total;
    uint32_t run = block_inclusive_scan_256(s, lds4, &total) - s;
    for (int64_t i = i0; i < i1; ++i) {
        const uint32_t v = p[i];
        p[i] = run;
        run += v;
    }
    if (staged) {
        __syncthreads();
        for (int64_t i = threadIdx.x; i < np; i += kScanThreads) part[i] = sp[i];
    }
    if (threadIdx.x == 0) part[np] = total;
}

// Blocked per-thread segments: thread t scans elements [t*16, t*16+16) of the tile.
__global__ __launch_bounds__(kScanThreads) void k_scan_down(const uint32_t* __restrict__ in,
                                                            uint32_t* __restrict__ out, int64_t m,
                                                            const uint32_t* __restrict__ part,
                                                            const uint32_t* __restrict__ mlen,
                                                            uint32_t madd) {
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t tile[kScanTile + kScanTile / 32];
    const int64_t base = (int64_t)blockIdx.x * kScanTile;
    m = scan_len(m, mlen, madd);
    if (base >= m) return;
    // striped, coalesced load into LDS (padded every 32 words against bank conflicts)
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const int e = r * kScanThreads + threadIdx.x;
        const int64_t i = base + e;
        tile[e + (e >> 5)] = i < m ? in[i] : 0u;
    }
    __syncthreads();
    uint32_t v[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int e = threadIdx.x * kScanItems + k;
        v[k] = tile[e + (e >> 5)];
        s += v[k];
    }
    uint32_t total;
    const uint32_t inc = block_inclusive_scan_256(s, lds4, &total);
    uint32_t run = part[blockIdx.x] + inc - s;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int e = threadIdx.x * kScanItems + k;
        tile[e + (e >> 5)] = run;
        run += v[k];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kScanItems; ++r) {
        const int e = r * kScanThreads + threadIdx.x;
        const int64_t i = base + e;
        if (i < m) out[i] = tile[e + (e >> 5)];
    }
}

inline void launch_scan_partials(uint32_t* part, int64_t np, const uint32_t* mlen, uint32_t madd,
                                 hipStream_t s) {
    if (np > kScanStageMin)
        hipLaunchKernelGGL(k_scan_partials<true>, dim3(1), dim3(kScanThreads), 0, s, part, np,
                           mlen, madd);
    else
        hipLaunchKernelGGL(k_scan_partials<false>, dim3(1), dim3(kScanThreads), 0, s, part, np,
                           mlen, madd);
}

// Exclusive scan of m (< 2^32 total) uint32 values; out may alias in.  out[m] is NOT
// written; the total is left in part[np].  `part` needs cdiv(m, 4096) + 1 entries.
// With `mlen`, only the first min(m, *mlen + madd) elements (a device-side length) are
// scanned and written.
inline int exclusive_scan_u32(const uint32_t* in, uint32_t* out, int64_t m, uint32_t* part,
                              hipStream_t s, const uint32_t* mlen = nullptr,
                              uint32_t madd = 0) {
    if (m <= 0) return ET_OK;
    const int64_t np = cdiv64(m, kScanTile);
    if (np > 0x7fffffffll) return fail(ET_ERR_ARG, "scan too large");
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)np), dim3(kScanThreads), 0, s, in, m, part,
                       mlen, madd);
    launch_scan_partials(part, np, mlen, madd, s);
    hipLaunchKernelGGL(k_scan_down, dim3((unsigned)np), dim3(kScanThreads), 0, s, in, out, m,
                       part, mlen, madd);
    ET_LAUNCH_CHECK("exclusive_scan_u32");
    return ET_OK;
}

inline int64_t scan_part_entries(int64_t m) { return cdiv64(m, kScanTile) + 1; }

// --- radix sort -----------------------------------------------------------
//
// Segmented: the elements are up to kRsMaxSegs contiguous segments (the tables of an
// update), each sorted on its own key range with its own number of passes — a
// 3-row table needs one 9-bit pass, a 10 M-row table three — so the passes over
// all segments cost sum_t n_t * passes_t instead of n * passes(max key).  Keys of
// segment k are reduced to min(key - key_base[k], key_cap[k]) (table-local column,
// the out-of-range sentinel clamped to the segment's largest value).  A segment with
// passes_t passes takes part in the LAST passes_t of the P passes, so every segment
// ends in the same buffer; its keys start in buffer (P - passes_t) % 2.

constexpr int kRsMaxSegs = 32;

struct RsPass {
    int nseg;                            // segments taking part in this pass
    uint32_t tile_off[kRsMaxSegs + 1];   // prefix of their tiles
    uint32_t elem0[kRsMaxSegs];          // first element of the segment
    uint32_t n[kRsMaxSegs];              // its elements
    uint32_t pos_base[kRsMaxSegs];       // elem0 - elements of earlier taking-part segments
    uint32_t key_base[kRsMaxSegs];
    uint32_t key_cap[kRsMaxSegs];
    uint32_t shift[kRsMaxSegs];
};

__device__ __forceinline__ int rs_segment(const RsPass& p, uint32_t b) {
    int k = 0;
    while (k + 1 < p.nseg && b >= p.tile_off[k + 1]) ++k;
    return k;
}

template <int NB>
__device__ __forceinline__ uint32_t rs_digit(uint32_t key, uint32_t base, uint32_t cap,
                                             uint32_t shift) {
    uint32_t l = key - base;
    l = l < cap ? l : cap;
    return (l >> shift) & (NB - 1);
}

// LDS digit-count increment of one wave instruction whose lanes hold consecutive
// elements (valid lanes a prefix): equal digits in adjacent lanes are added once per run
// by the run's first lane.  A skewed tile — a Zipf-hot column, or a table of a few rows,
// whose keys are nearly all equal — otherwise serialises up to 64 lane atomics on one
// LDS address (the last sort pass's histogram took 87 us for 34 M keys, the first pass's
// 12 us for 7.9 M keys of the large tables).  Not used in the staged scatter's counts:
// there the extra ballots cost more than the conflicts (passes over the large tables
// 51 / 140 us -> 56 / 160 us, the last pass unchanged).
__device__ __forceinline__ void lds_count_runs(uint32_t* row, uint32_t d, bool valid) {
    const int lane = threadIdx.x & 63;
    const uint32_t prev = (uint32_t)__shfl_up((int)d, 1, 64);
    const bool head = valid && (lane == 0 || d != prev);
    const uint64_t heads = (uint64_t)__ballot(head);
    const int nvalid = __popcll((uint64_t)__ballot(valid));
    if (head) {
        const uint64_t after = lane < 63 ? heads >> (lane + 1) : 0ull;
        const int end = after ? lane + __ffsll((long long)after) : nvalid;
        atomicAdd(&row[d], (uint32_t)(end - lane));
    }
}

template <int BITS>
__global__ __launch_bounds__(kRsThreads) void k_rs_hist(const uint32_t* __restrict__ keys,
                                                        RsPass p, uint32_t* __restrict__ hist) {
    constexpr int NB = 1 << BITS;
    __shared__ uint32_t h[4][NB];
    const int wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 4 * NB; i += kRsThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const int k = rs_segment(p, blockIdx.x);
    const uint32_t tl = blockIdx.x - p.tile_off[k], tiles = p.tile_off[k + 1] - p.tile_off[k];
    const uint32_t n = p.n[k], kb = p.key_base[k], cap = p.key_cap[k], sh = p.shift[k];
    const uint32_t* kp = keys + p.elem0[k];
    const uint32_t base = tl * kRsTile;
    // 8 keys in flight per thread, then their LDS increments
    for (int r0 = 0; r0 < kRsItems; r0 += 8) {
        uint32_t kk[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t i = base + (r0 + q) * kRsThreads + threadIdx.x;
            kk[q] = i < n ? kp[i] : 0xffffffffu;
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t i = base + (r0 + q) * kRsThreads + threadIdx.x;
            lds_count_runs(h[wave], rs_digit<NB>(kk[q], kb, cap, sh), i < n);
        }
    }
    __syncthreads();
    uint32_t* hs = hist + (uint64_t)NB * p.tile_off[k];
    for (int d = threadIdx.x; d < NB; d += kRsThreads)
        hs[(uint64_t)d * tiles + tl] = h[0][d] + h[1][d] + h[2][d] + h[3][d];
}

// Stable scatter of one tile (8192 keys).  Full tiles of a 16-byte aligned segment are
// staged in LDS by LDS-DMA (74 KB, 2 workgroups per CU), sorted by digit in LDS and
// written out in bucket runs (below).  The tail tile takes the round path: 32 rounds of
// 256 keys in input order; a key's rank among equal digits is (keys of this digit in
// earlier rounds) + (lower waves of this round) + (lower lanes of its wave, found with
// one ballot per digit bit).  Config-4 update, passes in order (8-bit over the 6 largest
// tables' 7.9 M pairs, 9-bit over 22 M, 9-bit over 34 M; rocprofv3 kernel trace): 49 /
// 143 / 211 us staged against 141 / 359 / 231 us with the round path alone — its
// scattered 4-byte stores (one L2 write request each) were its bound.
template <int BITS>
__global__ __launch_bounds__(kRsThreads) void k_rs_scatter(
    const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
    uint32_t* __restrict__ kout, uint32_t* __restrict__ vout, RsPass p,
    const uint32_t* __restrict__ hist_scanned) {
    constexpr int NB = 1 << BITS;
    __shared__ uint32_t base_of[NB];
    __shared__ uint32_t wcnt[4][NB];
    // the whole tile's keys and values, staged by LDS-DMA (full, 16-byte aligned tiles)
    __shared__ uint32_t skey[kRsTile];
    __shared__ uint32_t sval[kRsTile];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int k = rs_segment(p, blockIdx.x);
    const uint32_t tl = blockIdx.x - p.tile_off[k], tiles = p.tile_off[k + 1] - p.tile_off[k];
    const uint32_t n = p.n[k], kb = p.key_base[k], cap = p.key_cap[k], sh = p.shift[k];
    const uint32_t e0 = p.elem0[k], pb = p.pos_base[k];
    const uint32_t* hs = hist_scanned + (uint64_t)NB * p.tile_off[k];
    const uint32_t base = tl * kRsTile;
    // Full tiles of a 16-byte aligned segment: every key and value of the tile is
    // requested at once (16 global_load_lds_dwordx4 per wave, no VGPRs), so the tile
    // pays one memory latency instead of one per round of 256 keys; the tail tile
    // keeps the register path with a one-round prefetch.
    const bool staged = base + kRsTile <= n && ((e0 & 3u) == 0);  // workgroup-uniform
    if (staged) {
#pragma unroll
        for (int j = 0; j < kRsItems / 4; ++j) {
            const int c = (j * 4 + wave) * 256;  // this wave-instruction's 256 keys (1 KiB)
            __builtin_amdgcn_global_load_lds(kin + e0 + base + c + lane * 4, &skey[c], 16, 0, 0);
            __builtin_amdgcn_global_load_lds(vin + e0 + base + c + lane * 4, &sval[c], 16, 0, 0);
        }
    }
    for (int d = threadIdx.x; d < NB; d += kRsThreads) {
        base_of[d] = hs[(uint64_t)d * tiles + tl] + pb;
        wcnt[0][d] = wcnt[1][d] = wcnt[2][d] = wcnt[3][d] = 0;
    }
    __syncthreads();  // (with LDS-DMA in flight this waits vmcnt(0): the tile has landed)
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    // register path: keys / values of the next round are loaded while this round is ranked
    uint32_t key_n = 0, val_n = 0;
    if (!staged) {
        const uint32_t i = base + threadIdx.x;
        if (i < n) {
            key_n = kin[e0 + i];
            val_n = vin[e0 + i];
        }
    }
    if (staged) {
        // Staged tile, sorted in LDS, written out in bucket runs.  Wave q owns the
        // tile's keys [q * 2048, (q + 1) * 2048) (input order = wave-major):
        //  1. each wave counts its keys' digits in its own LDS row (wcnt[q]);
        //  2. tile-local offsets: dpre[d] = keys of smaller digits in the tile, and row
        //     (q, d) starts at dpre[d] + keys of digit d in waves < q;
        //  3. each wave walks its keys in order: a key's rank among equal digits within a
        //     64-key round comes from the ballots, the running offset from its wave's
        //     row, which only that wave updates (LDS ops of one wave run in program
        //     order) — stable, no barrier per round; keys, values and tile-local sorted
        //     positions stay in registers;
        //  4. after a barrier every key and value is written to its sorted slot of the
        //     LDS tile, and after another the tile is written out slot by slot: digit d's
        //     run (about 16 keys at 512 buckets) lands at consecutive global positions, so
        //     a store instruction touches a few cache lines instead of 64 (one L2 write
        //     request per scattered 4-byte key was this kernel's bound).
        constexpr int kPer = kRsTile / 4;
        constexpr int kRounds = kPer / 64;
        __shared__ uint32_t dpre[NB];
        const uint32_t* wk = skey + wave * kPer;
        const uint32_t* wv = sval + wave * kPer;
        for (int rr = 0; rr < kPer; rr += 64)
            atomicAdd(&wcnt[wave][rs_digit<NB>(wk[rr + lane], kb, cap, sh)], 1u);
        __syncthreads();
        {
            // exclusive scan of the tile's digit totals (NB / 256 digits per thread)
            constexpr int DPT = NB / kRsThreads;
            uint32_t tot[DPT], sum = 0;
#pragma unroll
            for (int q = 0; q < DPT; ++q) {
                const int d = threadIdx.x * DPT + q;
                tot[q] = wcnt[0][d] + wcnt[1][d] + wcnt[2][d] + wcnt[3][d];
                sum += tot[q];
            }
            __shared__ uint32_t lds4[4];
            uint32_t total;
            uint32_t run = block_inclusive_scan_256(sum, lds4, &total) - sum;
#pragma unroll
            for (int q = 0; q < DPT; ++q) {
                const int d = threadIdx.x * DPT + q;
                dpre[d] = run;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const uint32_t c = wcnt[w][d];
                    wcnt[w][d] = run;
                    run += c;
                }
            }
        }
        __syncthreads();
        uint32_t rk[kRounds], rv[kRounds], rl[kRounds];
#pragma unroll
        for (int q = 0; q < kRounds; ++q) {
            const uint32_t key = wk[q * 64 + lane];
            const uint32_t d = rs_digit<NB>(key, kb, cap, sh);
            uint64_t same = ~0ull;
#pragma unroll
            for (int b = 0; b < BITS; ++b) {
                const uint64_t ones = __ballot((d >> b) & 1u);
                same &= ((d >> b) & 1u) ? ones : ~ones;
            }
            const uint32_t rank = __popcll(same & lt_mask);
            rl[q] = wcnt[wave][d] + rank;
            if (rank == 0) wcnt[wave][d] += (uint32_t)__popcll(same);  // after every lane's read
            rk[q] = key;
            rv[q] = wv[q * 64 + lane];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < kRounds; ++q) {
            skey[rl[q]] = rk[q];
            sval[rl[q]] = rv[q];
        }
        __syncthreads();
        for (int j = threadIdx.x; j < kRsTile; j += kRsThreads) {
            const uint32_t key = skey[j];
            const uint32_t d = rs_digit<NB>(key, kb, cap, sh);
            const uint32_t pos = base_of[d] + (uint32_t)j - dpre[d];
            kout[pos] = key;
            vout[pos] = sval[j];
        }
        return;
    }
    for (int r = 0; r < kRsItems; ++r) {
        const uint32_t i = base + r * kRsThreads + threadIdx.x;
        const bool valid = i < n;
        const uint32_t key = key_n, val = val_n;
        if (r + 1 < kRsItems) {
            const uint32_t i2 = i + kRsThreads;
            if (i2 < n) {
                key_n = kin[e0 + i2];
                val_n = vin[e0 + i2];
            }
        }
        const uint32_t d = rs_digit<NB>(key, kb, cap, sh);
        uint64_t same = __ballot(valid);
#pragma unroll
        for (int b = 0; b < BITS; ++b) {
            const uint64_t ones = __ballot((d >> b) & 1u);
            same &= ((d >> b) & 1u) ? ones : ~ones;
        }
        const uint32_t rank = __popcll(same & lt_mask);
        const bool leader = valid && rank == 0;  // lowest lane of its digit in the wave
        const uint32_t cnt = (uint32_t)__popcll(same);
        if (leader) wcnt[wave][d] = cnt;
        __syncthreads();
        uint32_t pos = 0;
        if (valid) {
            pos = base_of[d] + rank;
            for (int w = 0; w < wave; ++w) pos += wcnt[w][d];
        }
        __syncthreads();
        // only the digits present in this round move: each (wave, digit) leader adds
        // its count and clears its slot (instead of a pass over all NB digits)
        if (leader) {
            atomicAdd(&base_of[d], cnt);
            wcnt[wave][d] = 0;
        }
        __syncthreads();
        if (valid) {
            kout[pos] = key;
            vout[pos] = val;
        }
    }
}

struct SortBuffers {
    uint32_t* ka;
    uint32_t* va;
    uint32_t* kb;
    uint32_t* vb;
    uint32_t* hist;  // kRsMaxBuckets * (tiles + segments) + 1
    uint32_t* part;  // scan partials
};

inline int64_t sort_hist_entries(int64_t n, int nseg = 1) {
    return (int64_t)kRsMaxBuckets * (cdiv64(n, kRsTile) + nseg) + 1;
}

// One segment of a sort: elements [elem0, elem0 + n), keys reduced to
// min(key - key_base, key_cap) < 2^bits.
struct RsSegment {
    uint32_t elem0, n, key_base, key_cap;
    int bits;
};

inline int rs_passes(int bits) { return (bits + kRsMaxBits - 1) / kRsMaxBits; }

// Passes over all segments; returns the number P of passes (the result is in buffer a
// if P is even, b if odd; segment s must start in buffer (P - rs_passes(bits_s)) % 2).
inline int rs_total_passes(const RsSegment* seg, int nseg) {
    int P = 0;
    for (int k = 0; k < nseg; ++k)
        if (seg[k].n > 0 && rs_passes(seg[k].bits) > P) P = rs_passes(seg[k].bits);
    return P;
}

inline int segmented_radix_sort(SortBuffers& sb, const RsSegment* seg, int nseg,
                                uint32_t** sorted_k, uint32_t** sorted_v, hipStream_t s) {
    if (nseg > kRsMaxSegs) return fail(ET_ERR_ARG, "too many sort segments");
    const int P = rs_total_passes(seg, nseg);
    uint32_t *k0 = sb.ka, *v0 = sb.va, *k1 = sb.kb, *v1 = sb.vb;
    for (int pass = 0; pass < P; ++pass) {
        RsPass rp;
        rp.nseg = 0;
        rp.tile_off[0] = 0;
        uint32_t before = 0;
        bool wide = false;
        for (int k = 0; k < nseg; ++k) {
            const int pt = rs_passes(seg[k].bits);
            if (seg[k].n == 0 || pass < P - pt) continue;
            const int width = (seg[k].bits + pt - 1) / pt;  // <= 9
            wide |= width > 8;
            const int j = rp.nseg++;
            rp.tile_off[j + 1] = rp.tile_off[j] + (uint32_t)cdiv64(seg[k].n, kRsTile);
            rp.elem0[j] = seg[k].elem0;
            rp.n[j] = seg[k].n;
            rp.pos_base[j] = seg[k].elem0 - before;
            rp.key_base[j] = seg[k].key_base;
            rp.key_cap[j] = seg[k].key_cap;
            rp.shift[j] = (uint32_t)((pass - (P - pt)) * width);
            before += seg[k].n;
        }
        const uint32_t tiles = rp.tile_off[rp.nseg];
        const int nb = wide ? 512 : 256;
        if (wide) {
            hipLaunchKernelGGL(k_rs_hist<9>, dim3(tiles), dim3(kRsThreads), 0, s, k0, rp, sb.hist);
        } else {
            hipLaunchKernelGGL(k_rs_hist<8>, dim3(tiles), dim3(kRsThreads), 0, s, k0, rp, sb.hist);
        }
        ET_LAUNCH_CHECK("k_rs_hist");
        int rc = exclusive_scan_u32(sb.hist, sb.hist, (int64_t)nb * tiles, sb.part, s);
        if (rc != ET_OK) return rc;
        if (wide) {
            hipLaunchKernelGGL(k_rs_scatter<9>, dim3(tiles), dim3(kRsThreads), 0, s, k0, v0, k1,
                               v1, rp, sb.hist);
        } else {
            hipLaunchKernelGGL(k_rs_scatter<8>, dim3(tiles), dim3(kRsThreads), 0, s, k0, v0, k1,
                               v1, rp, sb.hist);
        }
        ET_LAUNCH_CHECK("k_rs_scatter");
        uint32_t* t = k0;
        k0 = k1;
        k1 = t;
        t = v0;
        v0 = v1;
        v1 = t;
    }
    *sorted_k = k0;
    *sorted_v = v0;
    return ET_OK;
}

// Stable sort of n (ka, va) pairs by the low `bits` key bits (one segment).
inline int radix_sort_pairs(SortBuffers& sb, int64_t n, int bits, uint32_t** sorted_k,
                            uint32_t** sorted_v, hipStream_t s) {
    if (n >= 0xffffffffll) return fail(ET_ERR_ARG, "sort too large");
    RsSegment seg{0u, (uint32_t)n, 0u, 0xffffffffu, bits};
    return segmented_radix_sort(sb, &seg, 1, sorted_k, sorted_v, s);
}

inline int bits_for(uint64_t maxval) {
    int b = 0;
    while (b < 32 && (maxval >> b) != 0) ++b;
    return b;
}

}  // namespace et
