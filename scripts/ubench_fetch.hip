// FETCH_SIZE calibration per load width (round-2 roofline traffic figures).
//
// MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports half the bytes of a
// 16-B-per-lane streaming read; other widths are uncalibrated.  K1 reads its
// 2-bit words with 4-B loads (each lane a 5-word window), K2's gate streams
// 4-B low words.  Each kernel here reads a 2 GiB buffer (8x the Infinity
// Cache) exactly once with one access shape; run under
//   rocprofv3 --pmc FETCH_SIZE ...
// and divide FETCH_SIZE (KiB) by the bytes read to get the factor.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/ubench_fetch.hip -o scripts/ubench_fetch
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

constexpr size_t kBytes = 2ull << 30;

// W = 4, 8, 16: coalesced loads of W bytes per lane, grid-stride
template <int W>
__global__ __launch_bounds__(256) void stream_kernel(const uint8_t* __restrict__ p, uint32_t* out) {
  uint32_t acc = 0;
  const size_t n = kBytes / W;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    if (W == 4) acc ^= ((const uint32_t*)p)[i];
    if (W == 8) {
      const uint2 v = ((const uint2*)p)[i];
      acc ^= v.x ^ v.y;
    }
    if (W == 16) {
      const uint4 v = ((const uint4*)p)[i];
      acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// K1's shape: lane l of segment s reads the 5 words starting at word
// floor(44 s / 16) (44 k-mer positions per lane, 16 bases per word)
__global__ __launch_bounds__(256) void window_kernel(const uint32_t* __restrict__ w, uint32_t* out) {
  uint32_t acc = 0;
  const size_t nw = kBytes / 4;
  const size_t nseg = (nw - 8) * 16 / 44;
  for (size_t seg = (size_t)blockIdx.x * 256 + threadIdx.x; seg < nseg; seg += (size_t)gridDim.x * 256) {
    const size_t wi = seg * 44 / 16;
#pragma unroll
    for (int j = 0; j < 5; ++j) acc ^= w[wi + j];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  int n_cu = 0;
  CHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t* buf;
  uint32_t* out;
  CHK(hipMalloc(&buf, kBytes));
  CHK(hipMemset(buf, 0x5A, kBytes));
  const int grid = n_cu * 8;
  CHK(hipMalloc(&out, (size_t)grid * 256 * 4));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  auto time = [&](const char* name, auto launch) -> int {
    launch();
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(a));
    launch();
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, a, b));
    std::printf("{\"shape\": \"%s\", \"bytes\": %zu, \"ms\": %.4f, \"GBps\": %.1f}\n", name, kBytes, ms,
                kBytes / (ms * 1e-3) / 1e9);
    return 0;
  };
  int rc = 0;
  rc |= time("dword coalesced", [&] { hipLaunchKernelGGL(stream_kernel<4>, dim3(grid), dim3(256), 0, 0, buf, out); });
  rc |= time("dwordx2 coalesced", [&] { hipLaunchKernelGGL(stream_kernel<8>, dim3(grid), dim3(256), 0, 0, buf, out); });
  rc |= time("dwordx4 coalesced", [&] { hipLaunchKernelGGL(stream_kernel<16>, dim3(grid), dim3(256), 0, 0, buf, out); });
  rc |= time("K1 5-word windows", [&] {
    hipLaunchKernelGGL(window_kernel, dim3(grid), dim3(256), 0, 0, (const uint32_t*)buf, out);
  });
  CHK(hipFree(buf));
  CHK(hipFree(out));
  return rc;
}
