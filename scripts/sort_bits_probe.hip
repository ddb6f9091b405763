// Radix bits per onesweep pass for K2's index sort (u32 keys carrying u64
// values, pairs_index.hip): rocPRIM's gfx950 default is 8 bits (4 passes
// over a 32-bit key); 10 or 11 bits sort the same keys in 3 passes.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/sort_bits_probe.hip -o scripts/sort_bits_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void fill(uint32_t* k, uint64_t* v, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint64_t x = (i / 8) * 0x9E3779B97F4A7C15ull;  // runs of ~8 equal keys, as clustered sketches give
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 32;
    k[i] = (uint32_t)x;
    v[i] = x ^ i;
  }
}

template <unsigned Bits>
using Cfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::radix_sort_onesweep_config<
    rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>, Bits, rocprim::block_radix_rank_algorithm::match>>;

template <class C>
int time_sort(const char* name, size_t n, uint32_t* k0, uint32_t* k1, uint64_t* v0, uint64_t* v1) {
  size_t bytes = 0;
  CHK(rocprim::radix_sort_pairs<C>(nullptr, bytes, k0, k1, v0, v1, n, 0, 32));
  void* tmp;
  CHK(hipMalloc(&tmp, bytes));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  float best = 1e9f;
  for (int r = 0; r < 6; ++r) {
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, k0, v0, n);
    CHK(hipEventRecord(a));
    CHK(rocprim::radix_sort_pairs<C>(tmp, bytes, k0, k1, v0, v1, n, 0, 32));
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    if (r) best = ms < best ? ms : best;
  }
  std::printf("{\"n\": %zu, \"config\": \"%s\", \"best_ms\": %.4f}\n", n, name, best);
  CHK(hipFree(tmp));
  return 0;
}

int main() {
  for (size_t n : {10000000ull, 100000000ull}) {
    uint32_t *k0, *k1;
    uint64_t *v0, *v1;
    CHK(hipMalloc(&k0, n * 4));
    CHK(hipMalloc(&k1, n * 4));
    CHK(hipMalloc(&v0, n * 8));
    CHK(hipMalloc(&v1, n * 8));
    int rc = time_sort<rocprim::default_config>("default", n, k0, k1, v0, v1);
    rc |= time_sort<Cfg<8>>("onesweep 8 bits", n, k0, k1, v0, v1);
    rc |= time_sort<Cfg<10>>("onesweep 10 bits", n, k0, k1, v0, v1);
    rc |= time_sort<Cfg<11>>("onesweep 11 bits", n, k0, k1, v0, v1);
    CHK(hipFree(k0));
    CHK(hipFree(k1));
    CHK(hipFree(v0));
    CHK(hipFree(v1));
    if (rc) return rc;
  }
  return 0;
}
