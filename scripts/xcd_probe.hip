// Dispatch probe: which XCD (HW_REG_XCC_ID) and CU each workgroup of a
// pair-kernel-shaped launch (1024 threads, 76 KiB dynamic LDS) runs on, and
// when it starts / ends.  Used to check the blockIdx -> XCD assumption of
// the gate kernel's work-item ordering.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(1024, 8) void probe(unsigned* out, unsigned spin) {
  extern __shared__ unsigned sm[];
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  unsigned long long t0 = wall_clock64();
  sm[threadIdx.x] = threadIdx.x;
  __syncthreads();
  unsigned acc = sm[(threadIdx.x * 7) & 1023];
  for (unsigned i = 0; i < spin; ++i) acc = acc * 1664525u + 1013904223u;
  __syncthreads();
  unsigned long long t1 = wall_clock64();
  if (threadIdx.x == 0) {
    out[blockIdx.x * 6 + 0] = xcc & 0xF;
    out[blockIdx.x * 6 + 1] = hw;
    out[blockIdx.x * 6 + 2] = (unsigned)t0;
    out[blockIdx.x * 6 + 3] = (unsigned)(t0 >> 32);
    out[blockIdx.x * 6 + 4] = (unsigned)t1;
    out[blockIdx.x * 6 + 5] = (unsigned)(t1 >> 32) + (acc == 12345u);
  }
}

int main() {
  const int n = 4096;
  unsigned* d;
  hipMalloc(&d, n * 6 * 4);
  const size_t lds = 76 * 1024;
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(probe, dim3(n), dim3(1024), lds, 0, d, 20000u);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(probe, dim3(n), dim3(1024), lds, 0, d, 20000u);
  hipDeviceSynchronize();
  std::vector<unsigned> h(n * 6);
  hipMemcpy(h.data(), d, n * 6 * 4, hipMemcpyDeviceToHost);
  for (int b = 0; b < n; ++b)
    printf("%d %u %u %llu %llu\n", b, h[b * 6], h[b * 6 + 1],
           ((unsigned long long)h[b * 6 + 3] << 32) | h[b * 6 + 2],
           ((unsigned long long)h[b * 6 + 5] << 32) | h[b * 6 + 4]);
  return 0;
}
