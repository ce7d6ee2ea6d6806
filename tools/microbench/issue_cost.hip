// Issue costs that decide how the exact update's serial chain is sequenced (gfx950, one
// wave alone on the chip, s_memtime cycles).  Each kernel is one dependent v_add_f32 chain
// with something else interleaved:
//   dep<KS,KV>   : KS independent SALU ops and KV independent VALU ops after every add
//   exec0        : adds issued with EXEC = 0 (do masked-off adds cost an issue slot?)
//   dppfmac      : v_fmac_f32_dpp row_newbcast (the round-3 masked slot) as the chain op
//   readlane     : a v_readlane_b32 after every add
//   ladder       : per entry of r adds, one s_setpc_b64 into a 20-add ladder (r = 9..16)
//   straight     : the same entries' bookkeeping without the jump, exactly 12 adds each
//   cbranch      : per entry, r adds as a binary ladder of s_cbranch_scc0 over 16/8/4/2/1 blocks
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/issue_cost.hip -o issue_cost
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

#define STR_(x) #x
#define STR(x) STR_(x)

#define DEP_KERNEL(NAME, KS, KV)                                                         \
    __global__ void NAME(float* out, long long* cyc, int iters) {                        \
        float a = (float)threadIdx.x, b = 1e-3f, c = 0.5f;                               \
        uint32_t s0 = 1;                                                                 \
        const long long t0 = __builtin_amdgcn_s_memtime();                               \
        for (int i = 0; i < iters; ++i) {                                                \
            asm volatile(".rept 16\n\tv_add_f32_e32 %0, %0, %2\n\t"                       \
                         ".rept " STR(KS) "\n\ts_add_u32 %3, %3, 3\n\t.endr\n\t"         \
                         ".rept " STR(KV) "\n\tv_add_f32_e32 %1, %1, %2\n\t.endr\n\t"    \
                         ".endr"                                                         \
                         : "+v"(a), "+v"(c), "+v"(b), "+s"(s0)                           \
                         :                                                               \
                         : "scc");                                                       \
        }                                                                                \
        const long long t1 = __builtin_amdgcn_s_memtime();                               \
        out[threadIdx.x] = a + c + (float)s0;                                            \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                          \
    }

DEP_KERNEL(k_dep00, 0, 0)
DEP_KERNEL(k_dep10, 1, 0)
DEP_KERNEL(k_dep20, 2, 0)
DEP_KERNEL(k_dep40, 4, 0)
DEP_KERNEL(k_dep01, 0, 1)
DEP_KERNEL(k_dep02, 0, 2)
DEP_KERNEL(k_dep11, 1, 1)

__global__ void k_exec0(float* out, long long* cyc, int iters) {
    float a = (float)threadIdx.x, b = 1e-3f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "s_mov_b64 s[20:21], exec\n\t"
            "s_mov_b64 exec, 0\n\t"
            ".rept 16\n\tv_add_f32_e32 %0, %0, %1\n\t.endr\n\t"
            "s_mov_b64 exec, s[20:21]"
            : "+v"(a), "+v"(b)
            :
            : "s20", "s21");
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_dppfmac(float* out, long long* cyc, int iters) {
    float a = (float)threadIdx.x, b = 1e-3f, m = 1.0f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            ".rept 16\n\tv_fmac_f32_dpp %0, %2, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t.endr"
            : "+v"(a), "+v"(b), "+v"(m));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_readlane(float* out, long long* cyc, int iters) {
    float a = (float)threadIdx.x, b = 1e-3f;
    uint32_t v = threadIdx.x;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            ".rept 16\n\tv_add_f32_e32 %0, %0, %1\n\tv_readlane_b32 s22, %2, 5\n\t.endr"
            : "+v"(a), "+v"(b), "+v"(v)
            :
            : "s22");
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// entries: r = 9 + (k & 7) for k = 1, 6, 11, ... (k += 5), i.e. r cycles through 9..16
// (mean 12.5); n entries.  One s_setpc_b64 per entry into a 20-add ladder: the entry's
// bookkeeping sits after the ladder and jumps back into it (or to the exit).
__global__ void k_ladder(float* out, long long* cyc, int n) {
    float a = (float)threadIdx.x, b = 1e-3f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
        "s_mov_b32 s40, %2\n\t"
        "s_mov_b32 s41, 0\n\t"
        "s_getpc_b64 s[30:31]\n"
        "0:\n\t"
        "s_add_u32 s30, s30, 2f-0b\n\t"
        "s_addc_u32 s31, s31, 0\n\t"
        "s_getpc_b64 s[50:51]\n"
        "8:\n\t"
        "s_add_u32 s50, s50, 3f-8b\n\t"
        "s_addc_u32 s51, s51, 0\n\t"
        "s_branch 2f\n"
        "1:\n\t"
        ".rept 20\n\tv_add_f32_e32 %0, %0, %1\n\t.endr\n"
        "2:\n\t"
        "s_add_u32 s41, s41, 5\n\t"
        "s_and_b32 s42, s41, 7\n\t"
        "s_add_u32 s42, s42, 9\n\t"
        "s_lshl_b32 s42, s42, 2\n\t"
        "s_sub_u32 s34, s30, s42\n\t"
        "s_subb_u32 s35, s31, 0\n\t"
        "s_sub_u32 s40, s40, 1\n\t"
        "s_cmp_eq_u32 s40, -1\n\t"
        "s_cselect_b64 s[34:35], s[50:51], s[34:35]\n\t"
        "s_setpc_b64 s[34:35]\n"
        "3:"
        : "+v"(a), "+v"(b)
        : "s"(n)
        : "s30", "s31", "s50", "s51", "s34", "s35", "s40", "s41", "s42", "scc");
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// the ladder's bookkeeping, no jump: 12 adds per entry (a counted loop of 4 entries per
// back edge, so the loop branch is 1/4 per entry)
__global__ void k_straight(float* out, long long* cyc, int n) {
    float a = (float)threadIdx.x, b = 1e-3f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
        "s_mov_b32 s40, %2\n\t"
        "s_mov_b32 s41, 0\n"
        "1:\n\t"
        ".rept 4\n\t"
        ".rept 12\n\tv_add_f32_e32 %0, %0, %1\n\t.endr\n\t"
        "s_add_u32 s41, s41, 5\n\t"
        "s_and_b32 s42, s41, 7\n\t"
        "s_add_u32 s42, s42, 9\n\t"
        "s_lshl_b32 s42, s42, 2\n\t"
        "s_sub_u32 s34, s30, s42\n\t"
        "s_subb_u32 s35, s31, 0\n\t"
        ".endr\n\t"
        "s_sub_u32 s40, s40, 4\n\t"
        "s_cmp_gt_i32 s40, 0\n\t"
        "s_cbranch_scc1 1b"
        : "+v"(a), "+v"(b)
        : "s"(n)
        : "s30", "s31", "s34", "s35", "s40", "s41", "s42", "scc");
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// binary ladder: blocks of 8/4/2/1 adds each behind an s_bitcmp1 + s_cbranch_scc0
// (r = 9..16 -> the 8-block always, r - 8 in 1..8 as 4/2/1 + one more 8? no: r - 8 <= 8,
// so blocks 8 (unconditional) + 8/4/2/1 conditional on r - 8's bits 3..0)
__global__ void k_cbranch(float* out, long long* cyc, int n) {
    float a = (float)threadIdx.x, b = 1e-3f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    asm volatile(
        "s_mov_b32 s40, %2\n\t"
        "s_mov_b32 s41, 0\n"
        "1:\n\t"
        "s_add_u32 s41, s41, 5\n\t"
        "s_and_b32 s42, s41, 7\n\t"
        "s_add_u32 s42, s42, 1\n\t"  // r - 8 in 1..8
        ".rept 8\n\tv_add_f32_e32 %0, %0, %1\n\t.endr\n\t"
        "s_bitcmp1_b32 s42, 3\n\t"
        "s_cbranch_scc0 4f\n\t"
        ".rept 8\n\tv_add_f32_e32 %0, %0, %1\n\t.endr\n"
        "4:\n\t"
        "s_bitcmp1_b32 s42, 2\n\t"
        "s_cbranch_scc0 5f\n\t"
        ".rept 4\n\tv_add_f32_e32 %0, %0, %1\n\t.endr\n"
        "5:\n\t"
        "s_bitcmp1_b32 s42, 1\n\t"
        "s_cbranch_scc0 6f\n\t"
        ".rept 2\n\tv_add_f32_e32 %0, %0, %1\n\t.endr\n"
        "6:\n\t"
        "s_bitcmp1_b32 s42, 0\n\t"
        "s_cbranch_scc0 7f\n\t"
        "v_add_f32_e32 %0, %0, %1\n"
        "7:\n\t"
        "s_sub_u32 s40, s40, 1\n\t"
        "s_cmp_gt_i32 s40, 0\n\t"
        "s_cbranch_scc1 1b"
        : "+v"(a), "+v"(b)
        : "s"(n)
        : "s40", "s41", "s42", "scc");
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}


// dependent chains of one instruction form (16 per loop trip), acc is the chained operand
#define CHAIN_KERNEL(NAME, INSTR)                                                         \
    __global__ void NAME(float* out, long long* cyc, int iters) {                         \
        float a = (float)threadIdx.x, b = 1e-3f, m = 1.0f;                                \
        float a2 = 0.5f, b2 = 2e-3f;                                                      \
        const long long t0 = __builtin_amdgcn_s_memtime();                                \
        for (int i = 0; i < iters; ++i) {                                                 \
            asm volatile(".rept 16\n\t" INSTR "\n\t.endr"                                 \
                         : "+v"(a), "+v"(b), "+v"(m), "+v"(a2), "+v"(b2)                  \
                         :                                                                \
                         : "s24", "s25");                                                 \
        }                                                                                 \
        const long long t1 = __builtin_amdgcn_s_memtime();                                \
        out[threadIdx.x] = a + a2;                                                        \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                           \
    }
CHAIN_KERNEL(k_c_add32, "v_add_f32_e32 %0, %1, %0")
CHAIN_KERNEL(k_c_add64, "v_add_f32_e64 %0, %1, %0")
CHAIN_KERNEL(k_c_fmacv, "v_fmac_f32_e32 %0, %2, %1")
CHAIN_KERNEL(k_c_fmacs, "v_fmac_f32_e32 %0, s24, %1")
CHAIN_KERNEL(k_c_dpp_bc, "v_add_f32_dpp %0, %1, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf")
CHAIN_KERNEL(k_c_dpp_shr, "v_add_f32_dpp %0, %1, %0 row_shr:1 row_mask:0xf bank_mask:0xf")
CHAIN_KERNEL(k_c_dpp_qp, "v_add_f32_dpp %0, %1, %0 quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf")
CHAIN_KERNEL(k_c_dpp_bc15, "v_add_f32_dpp %0, %1, %0 row_bcast:15 row_mask:0xf bank_mask:0xf")

typedef float f2v __attribute__((ext_vector_type(2)));
#define PK_KERNEL(NAME, INSTR)                                                           \
    __global__ void NAME(float* out, long long* cyc, int iters) {                        \
        f2v a = {(float)threadIdx.x, 1.0f}, b = {1e-3f, 2e-3f};                          \
        const long long t0 = __builtin_amdgcn_s_memtime();                               \
        for (int i = 0; i < iters; ++i) {                                                \
            asm volatile("s_mov_b32 s24, 1.0\n\ts_mov_b32 s25, 1.0\n\t"                   \
                         ".rept 16\n\t" INSTR "\n\t.endr"                                \
                         : "+v"(a), "+v"(b)                                              \
                         :                                                               \
                         : "s24", "s25");                                                \
        }                                                                                \
        const long long t1 = __builtin_amdgcn_s_memtime();                               \
        out[threadIdx.x] = a.x + a.y;                                                    \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                          \
    }
PK_KERNEL(k_p_pkadd, "v_pk_add_f32 %0, %0, %1")
PK_KERNEL(k_p_pkfma_s, "v_pk_fma_f32 %0, s[24:25], %1, %0 op_sel_hi:[0,1,1]")
PK_KERNEL(k_p_pkfma_s2, "v_pk_fma_f32 %0, s[24:25], %1, %0")


// 16 dependent fmacs, each with its own SGPR mask (the wave-uniform-r form)
__global__ void k_c_fmacs16(float* out, long long* cyc, int iters) {
    float a = (float)threadIdx.x, b = 1e-3f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        asm volatile(
            "s_mov_b32 s24, 1.0\n\ts_mov_b32 s25, 1.0\n\ts_mov_b32 s26, 0\n\ts_mov_b32 s27, 1.0\n\t"
            "v_fmac_f32_e32 %0, s24, %1\n\tv_fmac_f32_e32 %0, s25, %1\n\t"
            "v_fmac_f32_e32 %0, s26, %1\n\tv_fmac_f32_e32 %0, s27, %1\n\t"
            "v_fmac_f32_e32 %0, s24, %1\n\tv_fmac_f32_e32 %0, s25, %1\n\t"
            "v_fmac_f32_e32 %0, s26, %1\n\tv_fmac_f32_e32 %0, s27, %1\n\t"
            "v_fmac_f32_e32 %0, s24, %1\n\tv_fmac_f32_e32 %0, s25, %1\n\t"
            "v_fmac_f32_e32 %0, s26, %1\n\tv_fmac_f32_e32 %0, s27, %1\n\t"
            "v_fmac_f32_e32 %0, s24, %1\n\tv_fmac_f32_e32 %0, s25, %1\n\t"
            "v_fmac_f32_e32 %0, s26, %1\n\tv_fmac_f32_e32 %0, s27, %1"
            : "+v"(a), "+v"(b)
            :
            : "s24", "s25", "s26", "s27");
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// 16 independent adds (4 accumulators in rotation): the VALU issue rate of one wave
__global__ void k_indep(float* out, long long* cyc, int iters) {
    float a = (float)threadIdx.x, b = 1e-3f, c = 1.0f, d = 2.0f, e = 3.0f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        asm volatile(".rept 4\n\tv_add_f32_e32 %0, %0, %1\n\tv_add_f32_e32 %2, %2, %1\n\t"
                     "v_add_f32_e32 %3, %3, %1\n\tv_add_f32_e32 %4, %4, %1\n\t.endr"
                     : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e));
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + c + d + e;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// 16 dependent adds then N independent SALU ops (not a chain): do SALU ops hide in the
// VALU dependency stall when they come in a block?
#define BLK_KERNEL(NAME, NS)                                                             \
    __global__ void NAME(float* out, long long* cyc, int iters) {                        \
        float a = (float)threadIdx.x, b = 1e-3f;                                         \
        const long long t0 = __builtin_amdgcn_s_memtime();                               \
        for (int i = 0; i < iters; ++i) {                                                \
            asm volatile(".rept 16\n\tv_add_f32_e32 %0, %0, %1\n\t.endr\n\t"            \
                         ".rept " STR(NS) "\n\ts_mov_b32 s30, 7\n\t.endr"                \
                         : "+v"(a), "+v"(b) : : "s30");                                  \
        }                                                                                \
        const long long t1 = __builtin_amdgcn_s_memtime();                               \
        out[threadIdx.x] = a;                                                            \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                          \
    }
BLK_KERNEL(k_blk0, 0)
BLK_KERNEL(k_blk2, 2)
BLK_KERNEL(k_blk4, 4)
BLK_KERNEL(k_blk8, 8)

// 16 dependent adds then one buffer_load with an SGPR offset (no wait)
__global__ void k_blkload(const float* src, float* out, long long* cyc, int iters) {
    float a = (float)threadIdx.x, b = 1e-3f, x;
    const uint64_t p = reinterpret_cast<uint64_t>(src);
    int r0 = __builtin_amdgcn_readfirstlane((int)(uint32_t)p);
    int r1 = __builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32) & 0xffff);
    uint32_t off = threadIdx.x * 4;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        asm volatile("s_mov_b32 s40, %4\n\ts_mov_b32 s41, %5\n\ts_mov_b32 s42, 256\n\ts_mov_b32 s43, 0x00020000\n\t"
                     ".rept 16\n\tv_add_f32_e32 %0, %0, %1\n\t.endr\n\t"
                     "s_mov_b32 s44, 0\n\t"
                     "buffer_load_dword %2, %3, s[40:43], s44 offen\n\t"
                     "s_waitcnt vmcnt(8)"
                     : "+v"(a), "+v"(b), "=v"(x) : "v"(off), "s"(r0), "s"(r1) : "s40", "s41", "s42", "s43", "s44", "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = a + x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    float* out;
    long long* cyc;
    CHECK(hipMalloc(&out, 64 * sizeof(float)));
    CHECK(hipMalloc(&cyc, sizeof(long long)));
    auto run = [&](const char* name, auto launch, double units, const char* unit) {
        long long best = -1;
        for (int rep = 0; rep < 5; ++rep) {
            launch();
            CHECK(hipDeviceSynchronize());
            long long c;
            CHECK(hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost));
            if (best < 0 || c < best) best = c;
        }
        printf("%-44s %10lld cycles  %7.2f cycles/%s\n", name, best, (double)best / units, unit);
    };
    const int it = 4096;
    const double adds = 16.0 * it;
    run("dep add", [&] { k_dep00<<<1, 64>>>(out, cyc, it); }, adds, "add");
    run("dep add + 1 SALU", [&] { k_dep10<<<1, 64>>>(out, cyc, it); }, adds, "add");
    run("dep add + 2 SALU", [&] { k_dep20<<<1, 64>>>(out, cyc, it); }, adds, "add");
    run("dep add + 4 SALU", [&] { k_dep40<<<1, 64>>>(out, cyc, it); }, adds, "add");
    run("dep add + 1 indep VALU", [&] { k_dep01<<<1, 64>>>(out, cyc, it); }, adds, "add");
    run("dep add + 2 indep VALU", [&] { k_dep02<<<1, 64>>>(out, cyc, it); }, adds, "add");
    run("dep add + 1 SALU + 1 indep VALU", [&] { k_dep11<<<1, 64>>>(out, cyc, it); }, adds, "add");
    run("add with EXEC=0", [&] { k_exec0<<<1, 64>>>(out, cyc, it); }, adds, "add");
    run("dep v_fmac_f32_dpp row_newbcast", [&] { k_dppfmac<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("dep add + v_readlane", [&] { k_readlane<<<1, 64>>>(out, cyc, it); }, adds, "add");

    run("chain v_add_f32_e32", [&] { k_c_add32<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("chain v_add_f32_e64", [&] { k_c_add64<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("chain v_fmac_f32 vgpr mask", [&] { k_c_fmacv<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("chain v_fmac_f32 sgpr mask", [&] { k_c_fmacs<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("chain v_add dpp row_newbcast", [&] { k_c_dpp_bc<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("chain v_add dpp row_shr:1", [&] { k_c_dpp_shr<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("chain v_add dpp quad_perm", [&] { k_c_dpp_qp<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("chain v_add dpp row_bcast:15", [&] { k_c_dpp_bc15<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("chain v_pk_add_f32", [&] { k_p_pkadd<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("chain v_pk_fma_f32 sgpr mask (op_sel_hi)", [&] { k_p_pkfma_s<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("chain v_pk_fma_f32 sgpr pair", [&] { k_p_pkfma_s2<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("chain v_fmac_f32 16 sgpr masks", [&] { k_c_fmacs16<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("16 indep adds (4 accs)", [&] { k_indep<<<1, 64>>>(out, cyc, it); }, adds, "op");
    run("16 dep adds + 0 SALU block", [&] { k_blk0<<<1, 64>>>(out, cyc, it); }, it, "16adds");
    run("16 dep adds + 2 SALU block", [&] { k_blk2<<<1, 64>>>(out, cyc, it); }, it, "16adds");
    run("16 dep adds + 4 SALU block", [&] { k_blk4<<<1, 64>>>(out, cyc, it); }, it, "16adds");
    run("16 dep adds + 8 SALU block", [&] { k_blk8<<<1, 64>>>(out, cyc, it); }, it, "16adds");
    run("16 dep adds + buffer_load soffset", [&] { k_blkload<<<1, 64>>>(out, out, cyc, it); }, it, "16adds");
    const int n = 65536;
    // r cycles through 9 + ((5k) & 7) for k = 1..n: mean 12.5
    double sum_r = 0;
    for (int k = 1; k <= n; ++k) sum_r += 9 + ((5 * k) & 7);
    run("ladder: setpc per entry (r 9..16)", [&] { k_ladder<<<1, 64>>>(out, cyc, n); }, n, "entry");
    printf("    = %.2f cycles/add over %.0f adds\n", 0.0, sum_r);
    run("straight: same SALU, 12 adds, no jump", [&] { k_straight<<<1, 64>>>(out, cyc, n); }, n,
        "entry");
    run("cbranch: 8 + 8/4/2/1 blocks (r 9..16)", [&] { k_cbranch<<<1, 64>>>(out, cyc, n); }, n,
        "entry");
    printf("mean r = %.3f\n", sum_r / n);
    return 0;
}
