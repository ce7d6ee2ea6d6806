// Dependent fp32 add-chain cost on gfx950, one wave alone on the chip.
// The exact (serial) update's critical path is the hottest column's chain of
// dependent adds (834,828 on the config-4 Zipf batch); this measures what one step of
// that chain costs in the instruction forms the hot-column kernel can use, and what a
// run-length ("head": one delta column added `rep` times in a row) costs on top.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/microbench/chain_lat.hip -o chain_lat
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                             \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

constexpr int kSteps = 1 << 16;

// (a) one float per lane, one dependent v_add_f32 per step
__global__ void k_add1(const float* x, float* out, long long* cyc) {
    float a = x[threadIdx.x], b = x[64 + threadIdx.x];
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
    for (int i = 0; i < kSteps; ++i) a = a + b;
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// (b) two floats per lane as one packed add (v_pk_add_f32) per step
__global__ void k_pk(const float* x, float* out, long long* cyc) {
    f2 a = {x[threadIdx.x], x[threadIdx.x + 64]}, b = {x[128 + threadIdx.x], x[192 + threadIdx.x]};
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
    for (int i = 0; i < kSteps; ++i) a = a + b;
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a.x + a.y;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// (c) two independent float chains per lane (two v_add_f32 per step)
__global__ void k_add2(const float* x, float* out, long long* cyc) {
    float a = x[threadIdx.x], c = x[threadIdx.x + 64], b = x[128 + threadIdx.x];
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
    for (int i = 0; i < kSteps; ++i) {
        a = a + b;
        c = c + b;
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + c;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// (d) run-length walk: heads[h] = (lds slot << 8) | rep; the head's delta pair is read
// from LDS and added rep times (reps 5-20, binomial like the hottest column's).
// MODE 0: plain counted loop; MODE 1: switch with fall-through (20 unrolled adds);
// MODE 2: 4 at a time then the remainder.
template <int MODE>
__global__ void k_heads(const uint32_t* heads, int nheads, const f2* src, float* out,
                        long long* cyc) {
    __shared__ f2 lds[64][64];
    for (int i = threadIdx.x; i < 64 * 64; i += 64) lds[i >> 6][i & 63] = src[i];
    __syncthreads();
    f2 a = {0.0f, 0.0f};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int h = 0; h < nheads; ++h) {
        const uint32_t e = heads[h];
        const f2 v = lds[(e >> 8) & 63][threadIdx.x];
        int r = (int)(e & 0xffu);
        if constexpr (MODE == 0) {
            for (int k = 0; k < r; ++k) a = a + v;
        } else if constexpr (MODE == 1) {
            switch (r) {
#define C(n) case n: a = a + v; [[fallthrough]];
                C(20) C(19) C(18) C(17) C(16) C(15) C(14) C(13) C(12) C(11)
                C(10) C(9) C(8) C(7) C(6) C(5) C(4) C(3) C(2)
#undef C
                case 1: a = a + v;
                default: break;
            }
        } else {
            while (r >= 4) {
                a = a + v;
                a = a + v;
                a = a + v;
                a = a + v;
                r -= 4;
            }
            if (r >= 2) {
                a = a + v;
                a = a + v;
                r -= 2;
            }
            if (r) a = a + v;
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a.x + a.y;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    float *x, *out;
    long long* cyc;
    CHECK(hipMalloc(&x, 4096 * sizeof(float)));
    CHECK(hipMalloc(&out, 64 * sizeof(float)));
    CHECK(hipMalloc(&cyc, sizeof(long long)));
    std::vector<float> hx(4096);
    for (int i = 0; i < 4096; ++i) hx[i] = 1e-3f * (float)((i * 7919) % 1000);
    CHECK(hipMemcpy(x, hx.data(), 4096 * sizeof(float), hipMemcpyHostToDevice));
    auto run = [&](const char* name, auto launch, double steps) {
        long long best = -1;
        for (int rep = 0; rep < 5; ++rep) {
            launch();
            CHECK(hipDeviceSynchronize());
            long long c;
            CHECK(hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost));
            if (best < 0 || c < best) best = c;
        }
        // s_memtime counts shader-clock cycles
        printf("%-34s %10lld cycles  %6.2f cycles/add-step\n", name, best, (double)best / steps);
    };
    run("v_add_f32 chain (1 feature/lane)", [&] { k_add1<<<1, 64>>>(x, out, cyc); }, kSteps);
    run("packed chain (2 features/lane)", [&] { k_pk<<<1, 64>>>(x, out, cyc); }, kSteps);
    run("2 v_add_f32 chains (2/lane)", [&] { k_add2<<<1, 64>>>(x, out, cyc); }, kSteps);

    const int nh = 65536;
    std::vector<uint32_t> hh(nh);
    long long adds = 0;
    srand(1);
    for (int h = 0; h < nh; ++h) {
        int r = 0;
        for (int k = 0; k < 20; ++k) r += (rand() % 1000) < 638;
        if (r == 0) r = 1;
        adds += r;
        hh[h] = ((uint32_t)(rand() % 64) << 8) | (uint32_t)r;
    }
    uint32_t* heads;
    CHECK(hipMalloc(&heads, nh * 4));
    CHECK(hipMemcpy(heads, hh.data(), nh * 4, hipMemcpyHostToDevice));
    printf("heads %d, adds %lld (%.2f per head)\n", nh, adds, (double)adds / nh);
    const f2* src = reinterpret_cast<const f2*>(x);
    run("heads: counted loop", [&] { k_heads<0><<<1, 64>>>(heads, nh, src, out, cyc); }, (double)adds);
    run("heads: switch fall-through", [&] { k_heads<1><<<1, 64>>>(heads, nh, src, out, cyc); },
        (double)adds);
    run("heads: 4-at-a-time + remainder", [&] { k_heads<2><<<1, 64>>>(heads, nh, src, out, cyc); },
        (double)adds);
    return 0;
}
