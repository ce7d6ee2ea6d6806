// Which hardware queue (ME, pipe, queue slot from HW_REG_HW_ID) does each HIP stream land on?
// Creates normal-priority streams and then high-priority ones, runs a one-wave probe kernel on
// each (the first use acquires the stream's queue) and prints the HW_ID fields its wave reads.
// Build: hipcc --offload-arch=gfx950 -O2 tools/microbench/hwid_probe.hip -o tools/microbench/hwid_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_probe(unsigned* out) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x == 0) {
        out[0] = hw;
        out[1] = xcc;
    }
}

static void probe(const char* what, hipStream_t s, unsigned* d, unsigned* h) {
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, s, d);
    (void)hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    const unsigned hw = h[0];
    printf("%-10s hw=0x%08x me=%u pipe=%u queue=%u vmid=%u se=%u cu=%u xcc=%u\n", what, hw,
           (hw >> 30) & 3, (hw >> 6) & 3, (hw >> 24) & 7, (hw >> 20) & 15, (hw >> 13) & 7,
           (hw >> 8) & 15, h[1] & 15);
}

int main(int argc, char** argv) {
    const int nnorm = argc > 1 ? atoi(argv[1]) : 6, nhigh = argc > 2 ? atoi(argv[2]) : 5;
    unsigned *d, *h;
    (void)hipMalloc(&d, 64);
    (void)hipHostMalloc(&h, 64);
    int least = 0, greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
    printf("priority range least=%d greatest=%d\n", least, greatest);
    probe("null", nullptr, d, h);
    char name[32];
    for (int i = 0; i < nnorm; ++i) {
        hipStream_t s;
        (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        snprintf(name, sizeof name, "norm%d", i);
        probe(name, s, d, h);
    }
    for (int i = 0; i < nhigh; ++i) {
        hipStream_t s;
        (void)hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest);
        snprintf(name, sizeof name, "high%d", i);
        probe(name, s, d, h);
    }
    for (int i = 0; i < nhigh; ++i) {
        hipStream_t s;
        (void)hipStreamCreateWithPriority(&s, hipStreamNonBlocking, least);
        snprintf(name, sizeof name, "low%d", i);
        probe(name, s, d, h);
    }
    probe("null", nullptr, d, h);
    return 0;
}
