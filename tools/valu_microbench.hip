// VALU issue / dependency microbenchmark for the chain loops (build: hipcc --offload-arch=gfx950
// -O3 -o tools/exp/valu_microbench tools/valu_microbench.hip; run on the GPU box).  One workgroup of 4 waves (one per SIMD, nothing else on the GPU); each wave
// runs ITER trips of 16 instructions of one form and records s_memtime (core clock) and
// s_memrealtime (100 MHz) around the loop.  Prints cycles and ns per instruction per form:
//   add      16 dependent v_add_f32
//   fmac     16 dependent v_fmac_f32
//   fmacdpp  16 dependent v_fmac_f32_dpp row_newbcast:k (the masked chain add)
//   fmacdpp2 two chains interleaved (8 + 8 dependent v_fmac_f32_dpp)
//   add2     two chains interleaved (8 + 8 dependent v_add_f32)
//   pkadd    16 dependent v_pk_add_f32 (two features per lane)
//   pkfma    16 dependent v_pk_fma_f32
//   perm     16 v_permlane16_swap on one register pair (dependent)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITER = 4096;

#define REP16(X) X X X X X X X X X X X X X X X X
#define REP8(X) X X X X X X X X

template <int FORM>
__global__ __launch_bounds__(256) void k_bench(float* out, uint64_t* t) {
    float a0 = threadIdx.x * 1e-7f, a1 = a0 + 1.0f, x = 1e-8f, m = 1.0f;
    float p0 = a0, p1 = a1, y0 = x, y1 = x;
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < ITER; ++i) {
        if constexpr (FORM == 0) {
            asm volatile(REP16("v_add_f32_e32 %0, %0, %1\n\t") : "+v"(a0) : "v"(x));
        } else if constexpr (FORM == 1) {
            asm volatile(REP16("v_fmac_f32_e32 %0, %1, %2\n\t") : "+v"(a0) : "v"(m), "v"(x));
        } else if constexpr (FORM == 2) {
            asm volatile(
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %0, %1, %2 row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
                : "+v"(a0) : "v"(m), "v"(x));
        } else if constexpr (FORM == 3) {
            asm volatile(REP8(
                "v_fmac_f32_dpp %0, %2, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
                "v_fmac_f32_dpp %1, %2, %3 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t")
                : "+v"(a0), "+v"(a1) : "v"(m), "v"(x));
        } else if constexpr (FORM == 4) {
            asm volatile(REP8("v_add_f32_e32 %0, %0, %2\n\tv_add_f32_e32 %1, %1, %2\n\t")
                : "+v"(a0), "+v"(a1) : "v"(x));
        } else if constexpr (FORM == 5) {
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 acc = {p0, p1}, xv = {y0, y1};
            asm volatile(REP16("v_pk_add_f32 %0, %0, %1\n\t") : "+v"(acc) : "v"(xv));
            p0 = acc.x;
            p1 = acc.y;
        } else if constexpr (FORM == 6) {
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 acc = {p0, p1}, xv = {y0, y1}, mv = {m, m};
            asm volatile(REP16("v_pk_fma_f32 %0, %1, %2, %0\n\t") : "+v"(acc) : "v"(mv), "v"(xv));
            p0 = acc.x;
            p1 = acc.y;
        } else {
            uint32_t u = __float_as_uint(a0), v = __float_as_uint(a1);
            asm volatile(REP16("v_permlane16_swap_b32 %0, %1\n\t") : "+v"(u), "+v"(v));
            a0 = __uint_as_float(u);
            a1 = __uint_as_float(v);
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + p0 + p1;
    if (threadIdx.x == 0) {
        t[0] = c1 - c0;
        t[1] = r1 - r0;
    }
}

template <int FORM>
static void run(const char* name, float* out, uint64_t* t) {
    uint64_t h[2];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_bench<FORM>, dim3(1), dim3(256), 0, 0, out, t);
        if (hipDeviceSynchronize() != hipSuccess) { printf("%s: failed\n", name); return; }
    }
    if (hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return;
    const double n = 16.0 * ITER;
    printf("%-9s %6.2f clk/instr  %6.3f ns/instr  (clock %.2f GHz)\n", name, h[0] / n,
           h[1] * 10.0 / n, h[0] / (h[1] * 10.0));
}

int main() {
    float* out;
    uint64_t* t;
    if (hipMalloc(&out, 4096) != hipSuccess || hipMalloc(&t, 64) != hipSuccess) return 1;
    run<0>("add", out, t);
    run<1>("fmac", out, t);
    run<2>("fmacdpp", out, t);
    run<3>("fmacdpp2", out, t);
    run<4>("add2", out, t);
    run<5>("pkadd", out, t);
    run<6>("pkfma", out, t);
    run<7>("perm", out, t);
    return 0;
}
