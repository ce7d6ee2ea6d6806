#include <cstring>
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <vector>
#include <random>
int main() {
  const size_t n = 34078720;
  std::vector<unsigned> hk(n), hv(n);
  std::mt19937 g(1); for (size_t i = 0; i < n; ++i) { hk[i] = g() & ((1u<<26)-1); hv[i] = i; }
  unsigned *k0,*k1,*v0,*v1; hipMalloc(&k0,n*4); hipMalloc(&k1,n*4); hipMalloc(&v0,n*4); hipMalloc(&v1,n*4);
  hipMemcpy(k0,hk.data(),n*4,hipMemcpyHostToDevice); hipMemcpy(v0,hv.data(),n*4,hipMemcpyHostToDevice);
  size_t tb=0; rocprim::radix_sort_pairs(nullptr,tb,k0,k1,v0,v1,n,0,26); void* t; hipMalloc(&t,tb);
  printf("temp bytes %zu\n", tb);
  hipEvent_t a,b; hipEventCreate(&a); hipEventCreate(&b);
  for (int bits : {26, 32}) {
    for (int w=0; w<3; ++w) rocprim::radix_sort_pairs(t,tb,k0,k1,v0,v1,n,0,bits);
    hipEventRecord(a);
    for (int r=0;r<10;++r) rocprim::radix_sort_pairs(t,tb,k0,k1,v0,v1,n,0,bits);
    hipEventRecord(b); hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms,a,b);
    printf("rocprim radix_sort_pairs n=%zu bits=%d: %.3f ms\n", n, bits, ms/10);
  }
  // stability check
  std::vector<unsigned> ok(n), ov(n); hipMemcpy(ok.data(),k1,n*4,hipMemcpyDeviceToHost); hipMemcpy(ov.data(),v1,n*4,hipMemcpyDeviceToHost);
  size_t bad=0; for (size_t i=1;i<n;++i) if (ok[i]<ok[i-1] || (ok[i]==ok[i-1] && ov[i]<ov[i-1])) ++bad;
  printf("order violations %zu\n", bad);
  return 0;
}
