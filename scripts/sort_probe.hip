// How fast does hipCUB/rocPRIM radix-sort (u64 hash, u32 value) pairs on one
// MI355X?  Sizing probe for an inverted-index pair kernel: N x s sketch
// entries are 1e7 at C3, 1e8 at C4 and C5.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/sort_probe.hip -o scripts/sort_probe
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdio>
#include <vector>

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void fill(uint64_t* k, uint32_t* v, size_t n, uint64_t mask) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint64_t x = i * 0x9E3779B97F4A7C15ull;
    x ^= x >> 29;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 32;
    k[i] = x & mask;
    v[i] = (uint32_t)i;
  }
}

int main() {
  for (size_t n : {10000000ull, 100000000ull}) {
    for (int bits : {58, 32}) {
      uint64_t *k0, *k1;
      uint32_t *v0, *v1;
      CHK(hipMalloc(&k0, n * 8));
      CHK(hipMalloc(&k1, n * 8));
      CHK(hipMalloc(&v0, n * 4));
      CHK(hipMalloc(&v1, n * 4));
      const uint64_t mask = bits == 64 ? ~0ull : ((1ull << bits) - 1);
      hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, k0, v0, n, mask);
      size_t tmp_bytes = 0;
      CHK(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, k0, k1, v0, v1, (int)n, 0, bits));
      void* tmp;
      CHK(hipMalloc(&tmp, tmp_bytes));
      hipEvent_t a, b;
      CHK(hipEventCreate(&a));
      CHK(hipEventCreate(&b));
      CHK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k0, k1, v0, v1, (int)n, 0, bits));
      CHK(hipDeviceSynchronize());
      float best = 1e9;
      for (int r = 0; r < 3; ++r) {
        CHK(hipEventRecord(a));
        CHK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, k0, k1, v0, v1, (int)n, 0, bits));
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        best = ms < best ? ms : best;
      }
      std::printf("{\"n\": %zu, \"key_bits\": %d, \"ms\": %.3f, \"Mpairs_per_s\": %.0f}\n", n, bits, best,
                  n / (best * 1e-3) / 1e6);
      CHK(hipFree(tmp));
      CHK(hipFree(k0));
      CHK(hipFree(k1));
      CHK(hipFree(v0));
      CHK(hipFree(v1));
    }
  }
  return 0;
}
