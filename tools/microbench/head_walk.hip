// Cost of walking one column's run-length list ("heads": one delta column added `rep`
// times in a row) on one wave, one feature per lane — the critical path of the exact
// sparse SGD (the hottest config-4 column: 65,536 heads, 834,828 dependent adds).
// Variants differ in how `rep` adds are sequenced; the head entries are prefetched with
// scalar loads two batches ahead and the delta values with vector loads one batch ahead.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/microbench/head_walk.hip -o head_walk
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../embeddingtables.jl_amd/csrc/et_chain_asm.h"

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

constexpr int kMaxRep = 20;
constexpr int NB = 16;  // heads per batch

template <int V>
__device__ __forceinline__ float add_rep(float acc, float x, uint32_t r) {
    if constexpr (V == 0) {  // 4 at a time + remainder
        while (r >= 4) {
            acc = acc + x;
            acc = acc + x;
            acc = acc + x;
            acc = acc + x;
            r -= 4;
        }
        if (r & 2) {
            acc = acc + x;
            acc = acc + x;
        }
        if (r & 1) acc = acc + x;
        return acc;
    } else if constexpr (V == 1) {  // computed jump over 20 unrolled adds
        const uint32_t skip = (uint32_t)(kMaxRep - r) * 4u + 12u;  // + the 3 SALU after getpc
        asm volatile(
            "s_getpc_b64 s[90:91]\n\t"
            "s_add_u32 s90, s90, %[sk]\n\t"
            "s_addc_u32 s91, s91, 0\n\t"
            "s_setpc_b64 s[90:91]\n\t"
            ".rept 20\n\t"
            "v_add_f32_e32 %[a], %[a], %[x]\n\t"
            ".endr\n\t"
            : [a] "+v"(acc)
            : [x] "v"(x), [sk] "s"(skip)
            : "scc", "s90", "s91");
        return acc;
    } else {  // fall-through switch
        switch (r) {
#define C(n) case n: acc = acc + x; [[fallthrough]];
            C(20) C(19) C(18) C(17) C(16) C(15) C(14) C(13) C(12) C(11)
            C(10) C(9) C(8) C(7) C(6) C(5) C(4) C(3) C(2)
#undef C
            case 1: acc = acc + x;
            default: break;
        }
        return acc;
    }
}

// heads[h] = bag | rep << 24 ; delta: column b at delta + b * ld, 64 features
template <int V>
__global__ void k_walk(const uint32_t* __restrict__ heads, int nh, const float* __restrict__ delta,
                       int ld, float* out, long long* cyc) {
    const int lane = threadIdx.x;
    float acc = 0.0f;
    uint32_t e0[NB], e1[NB];
    float x0[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) e0[j] = heads[j];
#pragma unroll
    for (int j = 0; j < NB; ++j) e1[j] = heads[NB + j];
#pragma unroll
    for (int j = 0; j < NB; ++j) x0[j] = delta[(size_t)(e0[j] & 0xffffffu) * ld + lane];
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int h0 = 0; h0 < nh; h0 += NB) {
        uint32_t e2[NB];
        float x1[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) e2[j] = heads[h0 + 2 * NB + j];  // padded list
#pragma unroll
        for (int j = 0; j < NB; ++j) x1[j] = delta[(size_t)(e1[j] & 0xffffffu) * ld + lane];
#pragma unroll
        for (int j = 0; j < NB; ++j) acc = add_rep<V>(acc, x0[j], e0[j] >> 24);
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            e0[j] = e1[j];
            e1[j] = e2[j];
            x0[j] = x1[j];
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = acc;
    if (lane == 0) cyc[0] = t1 - t0;
}

// pure dependent chain with k independent scalar ops per add
template <int K>
__global__ void k_salu(const float* x, float* out, long long* cyc, int n) {
    float a = x[threadIdx.x], b = x[64 + threadIdx.x];
    uint32_t s0 = (uint32_t)n, s1 = 7u, s2 = 9u, s3 = 11u;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i += 16) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            if constexpr (K == 0)
                asm volatile("v_add_f32_e32 %[a], %[a], %[b]" : [a] "+v"(a) : [b] "v"(b));
            else if constexpr (K == 1)
                asm volatile("v_add_f32_e32 %[a], %[a], %[b]\n\ts_add_u32 %[s0], %[s0], 3"
                             : [a] "+v"(a), [s0] "+s"(s0) : [b] "v"(b) : "scc");
            else if constexpr (K == 2)
                asm volatile("v_add_f32_e32 %[a], %[a], %[b]\n\ts_add_u32 %[s0], %[s0], 3\n\t"
                             "s_xor_b32 %[s1], %[s1], 5"
                             : [a] "+v"(a), [s0] "+s"(s0), [s1] "+s"(s1) : [b] "v"(b) : "scc");
            else
                asm volatile(
                    "v_add_f32_e32 %[a], %[a], %[b]\n\ts_add_u32 %[s0], %[s0], 3\n\t"
                    "s_xor_b32 %[s1], %[s1], 5\n\ts_add_u32 %[s2], %[s2], 3\n\ts_xor_b32 %[s3], %[s3], 5"
                    : [a] "+v"(a), [s0] "+s"(s0), [s1] "+s"(s1), [s2] "+s"(s2), [s3] "+s"(s3)
                    : [b] "v"(b) : "scc");
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + (float)(s0 + s1 + s2 + s3);
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// per-occurrence stream: x for occurrence t at stream + t*64 (pre-expanded), 1 load + 1 add
__global__ void k_stream(const float* __restrict__ stream, int n, float* out, long long* cyc) {
    const int lane = threadIdx.x;
    float acc = 0.0f;
    float a[32], b[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) a[j] = stream[(size_t)j * 64 + lane];
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int t0i = 0; t0i < n; t0i += 32) {
#pragma unroll
        for (int j = 0; j < 32; ++j) b[j] = stream[(size_t)(t0i + 32 + j) * 64 + lane];
#pragma unroll
        for (int j = 0; j < 32; ++j) acc = acc + a[j];
#pragma unroll
        for (int j = 0; j < 32; ++j) a[j] = b[j];
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = acc;
    if (lane == 0) cyc[0] = t1 - t0;
}


// masks: row r of S floats = [1]*r + [0]*(S-r); fma(x, 1, acc) == acc + x exactly and
// fma(x, 0, acc) == acc (acc is never -0), so a head of r <= S adds is S branch-free fmas
__constant__ float kMaskTab[17][16] = {
#define R(r) {r > 0, r > 1, r > 2, r > 3, r > 4, r > 5, r > 6, r > 7, r > 8, r > 9, r > 10, r > 11, \
              r > 12, r > 13, r > 14, r > 15}
    R(0), R(1), R(2), R(3), R(4), R(5), R(6), R(7), R(8), R(9), R(10), R(11), R(12), R(13), R(14),
    R(15), R(16)
#undef R
};

// entries: (delta element offset = bag * ld, mask-row byte offset = r * 64), r <= S; list
// padded with (0, 0) to a multiple of 8 plus 8
struct Ent8 {
    uint32_t v[16];
};

template <int S>
struct Masks {
    float m[S];
};

__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xc07f); }

// one wave, one feature per lane: acc over entries [0, ne) (ne a multiple of 8; 16 readable
// entries past the end); masks of head j+1 and entries of batch b+2 are issued right after
// the wait for what head j needs, so no scalar load is outstanding behind a needed one
template <int S>
__device__ __forceinline__ float chain_walk(const Ent8* __restrict__ eb, uint32_t nb,
                                            const float* __restrict__ xb, uint32_t ld) {
    constexpr int NB = 8;
    const char* mt = reinterpret_cast<const char*>(&kMaskTab[0][0]);
    Ent8 ec = eb[0], en = eb[1];
    float x[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) x[j] = xb[(uint64_t)ec.v[2 * j] * ld];
    Masks<S> mc = *reinterpret_cast<const Masks<S>*>(mt + ec.v[1]);
    float acc = 0.0f;
    for (uint32_t b = 0; b < nb; ++b) {
        Ent8 enn;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
            wait_lgkm0();
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t mrow = j < NB - 1 ? ec.v[2 * j + 3] : en.v[1];
            const Masks<S> mn = *reinterpret_cast<const Masks<S>*>(mt + mrow);
            if (j == NB - 1) enn = eb[b + 2];
            __builtin_amdgcn_sched_barrier(0);
            const float xv = x[j];
            x[j] = xb[(uint64_t)en.v[2 * j] * ld];
#pragma unroll
            for (int k = 0; k < S; ++k) acc = __builtin_fmaf(xv, mc.m[k], acc);
            __builtin_amdgcn_sched_barrier(0);
            mc = mn;
        }
        ec = en;
        en = enn;
    }
    return acc;
}

// entries: (bag, mask-row byte offset = r * 64), r <= S; padded with (0, 0) to a multiple of
// 8 plus 16
template <int S>
__global__ void k_chain(const uint2* __restrict__ ent, int ne, const float* __restrict__ delta,
                        int ld, float* out, long long* cyc) {
    const long long t0 = __builtin_amdgcn_s_memtime();
    const float acc = chain_walk<S>(reinterpret_cast<const Ent8*>(ent), (uint32_t)ne / 8,
                                    delta + threadIdx.x, (uint32_t)ld);
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// the generated hand-scheduled loop (csrc/et_chain_asm.h): entries r << 24 | bag
template <int S>
__global__ void k_chain_asm(const uint32_t* __restrict__ ent, int trips, const float* __restrict__ delta,
                            int ld, float* out, long long* cyc) {
    const long long t0 = __builtin_amdgcn_s_memtime();
    const float acc = et::chain_walk_asm<S>(ent, (uint32_t)trips, delta, 4u * threadIdx.x,
                                            4u * (uint32_t)ld, 0.0f);
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// reference: the same entries summed with plain sequential adds
__global__ void k_chain_ref(const uint32_t* __restrict__ ent, int ne, int ld,
                            const float* __restrict__ delta, float* out) {
    float acc = 0.0f;
    for (int h = 0; h < ne; ++h) {
        const float x = delta[(size_t)(ent[h] & 0xffffffu) * ld + threadIdx.x];
        const int r = (int)(ent[h] >> 24);
        for (int k = 0; k < r; ++k) acc = acc + x;
    }
    out[threadIdx.x] = acc;
}

int main() {
    const int nh = 65536, ncols = 4096, ld = 64;
    std::vector<uint32_t> hh(nh + 4 * NB, 1u << 24);
    long long adds = 0;
    srand(1);
    for (int h = 0; h < nh; ++h) {
        int r = 0;
        for (int k = 0; k < 20; ++k) r += (rand() % 1000) < 638;
        if (r == 0) r = 1;
        adds += r;
        hh[h] = (uint32_t)(rand() % ncols) | ((uint32_t)r << 24);
    }
    std::vector<float> hd((size_t)ncols * ld);
    for (size_t i = 0; i < hd.size(); ++i) hd[i] = 1e-3f * (float)((i * 7919) % 1000) - 0.5f;
    uint32_t* heads;
    float *delta, *out, *stream;
    long long* cyc;
    CHECK(hipMalloc(&heads, hh.size() * 4));
    CHECK(hipMalloc(&delta, hd.size() * 4));
    CHECK(hipMalloc(&out, 64 * 4));
    CHECK(hipMalloc(&cyc, 8));
    const size_t nstream = (size_t)(adds + 64) * 64;
    CHECK(hipMalloc(&stream, nstream * 4));
    CHECK(hipMemset(stream, 0, nstream * 4));
    CHECK(hipMemcpy(heads, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(delta, hd.data(), hd.size() * 4, hipMemcpyHostToDevice));
    auto run = [&](const char* name, auto launch, double steps) {
        long long best = -1;
        for (int rep = 0; rep < 5; ++rep) {
            launch();
            CHECK(hipDeviceSynchronize());
            long long c;
            CHECK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            if (best < 0 || c < best) best = c;
        }
        printf("%-40s %10lld cycles %7.2f cycles/add\n", name, best, (double)best / steps);
    };
    printf("heads %d, adds %lld (%.2f per head)\n", nh, adds, (double)adds / nh);
    const int n = 1 << 18;
    run("chain, 0 SALU per add", [&] { k_salu<0><<<1, 64>>>(delta, out, cyc, n); }, n);
    run("chain, 1 SALU per add", [&] { k_salu<1><<<1, 64>>>(delta, out, cyc, n); }, n);
    run("chain, 2 SALU per add", [&] { k_salu<2><<<1, 64>>>(delta, out, cyc, n); }, n);
    run("chain, 4 SALU per add", [&] { k_salu<4><<<1, 64>>>(delta, out, cyc, n); }, n);
    run("heads, 4-at-a-time", [&] { k_walk<0><<<1, 64>>>(heads, nh, delta, ld, out, cyc); },
        (double)adds);
    run("heads, computed jump", [&] { k_walk<1><<<1, 64>>>(heads, nh, delta, ld, out, cyc); },
        (double)adds);
    run("heads, switch", [&] { k_walk<2><<<1, 64>>>(heads, nh, delta, ld, out, cyc); },
        (double)adds);
    run("stream, load+add per occurrence",
        [&] { k_stream<<<1, 64>>>(stream, (int)(adds / 32 * 32), out, cyc); }, (double)(adds / 32 * 32));

    {  // chain with S-slot masks: the hottest column (r ~ Binom(20, .638) split at S = 16)
        // and a mid one (r ~ 1 + Geom, mean ~2.9, S = 4)
        for (int which = 0; which < 2; ++which) {
            const int S = which == 0 ? 16 : 4;
            std::vector<uint32_t> ee;
            long long adds2 = 0;
            for (int h = 0; h < nh; ++h) {
                int r = 0;
                if (which == 0) {
                    for (int k = 0; k < 20; ++k) r += (rand() % 1000) < 638;
                } else {
                    r = 1;
                    while ((rand() % 1000) < 655 && r < 20) ++r;
                }
                if (r == 0) r = 1;
                adds2 += r;
                const uint32_t bag = (uint32_t)(rand() % ncols);
                while (r > 0) {
                    const int q = r < S ? r : S;
                    ee.push_back(bag);
                    ee.push_back((uint32_t)q * 64u);
                    r -= q;
                }
            }
            const int ne = (int)ee.size() / 2;
            const int nep = (ne + 7) / 8 * 8;
            ee.resize((size_t)(nep + 24) * 2, 0u);
            uint2* dent;
            CHECK(hipMalloc(&dent, ee.size() * 4));
            CHECK(hipMemcpy(dent, ee.data(), ee.size() * 4, hipMemcpyHostToDevice));
            char name[96];
            snprintf(name, sizeof name, "chain S=%d (%d entries, %.2f adds/entry)", S, ne,
                     (double)adds2 / ne);
            if (S == 16)
                run(name, [&] { k_chain<16><<<1, 64>>>(dent, nep, delta, ld, out, cyc); }, (double)adds2);
            else
                run(name, [&] { k_chain<4><<<1, 64>>>(dent, nep, delta, ld, out, cyc); }, (double)adds2);
            long long best = 0;
            CHECK(hipMemcpy(&best, cyc, 8, hipMemcpyDeviceToHost));
            printf("    %.1f cycles per entry\n", (double)best / ne);
            CHECK(hipFree(dent));

            // the hand-scheduled loop on the same run lengths: gradient in L2 (the
            // columns above) and in HBM (65,536 columns of the config-4 stride, 872 MB)
            for (int big = 0; big < 2; ++big) {
                const int bcols = big ? 65536 : ncols, bld = big ? 3328 : ld;
                float* bdelta = delta;
                if (big) {
                    CHECK(hipMalloc(&bdelta, (size_t)bcols * bld * 4));
                    std::vector<float> hb((size_t)bcols * bld);
                    for (size_t i = 0; i < hb.size(); ++i)
                        hb[i] = 1e-3f * (float)((i * 7919) % 1000) - 0.5f;
                    CHECK(hipMemcpy(bdelta, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
                }
                std::vector<uint32_t> ea;
                for (size_t i = 0; i < (size_t)ne; ++i) {
                    const uint32_t bag = big ? (uint32_t)(rand() % bcols) : ee[2 * i];
                    ea.push_back((ee[2 * i + 1] / 64u) << 24 | bag);
                }
                const int trips = (ne + 63) / 64;
                ea.resize((size_t)(trips * 64 + 64), 0u);
                uint32_t* da;
                float* ref;
                CHECK(hipMalloc(&da, ea.size() * 4));
                CHECK(hipMalloc(&ref, 64 * 4));
                CHECK(hipMemcpy(da, ea.data(), ea.size() * 4, hipMemcpyHostToDevice));
                snprintf(name, sizeof name, "asm chain S=%d (%s)", S, big ? "HBM" : "L2");
                if (S == 16)
                    run(name, [&] { k_chain_asm<16><<<1, 64>>>(da, trips, bdelta, bld, out, cyc); }, (double)adds2);
                else
                    run(name, [&] { k_chain_asm<4><<<1, 64>>>(da, trips, bdelta, bld, out, cyc); }, (double)adds2);
                long long best2 = 0;
                CHECK(hipMemcpy(&best2, cyc, 8, hipMemcpyDeviceToHost));
                printf("    %.1f cycles per entry\n", (double)best2 / ne);
                k_chain_ref<<<1, 64>>>(da, ne, bld, bdelta, ref);
                CHECK(hipDeviceSynchronize());
                float a[64], b[64];
                CHECK(hipMemcpy(a, out, 256, hipMemcpyDeviceToHost));
                CHECK(hipMemcpy(b, ref, 256, hipMemcpyDeviceToHost));
                int bad = 0;
                for (int l = 0; l < 64; ++l) bad += memcmp(&a[l], &b[l], 4) != 0;
                printf("    bit-identical to sequential adds: %s (%d lanes differ)\n", bad ? "NO" : "yes", bad);
                CHECK(hipFree(da));
                CHECK(hipFree(ref));
                if (big) CHECK(hipFree(bdelta));
            }
        }
    }
    return 0;
}
