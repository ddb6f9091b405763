// Benchmark input generator: synthetic clustered genomes written straight
// into HBM in the 2-bit layout kernel K1 reads (SURVEY.md 8(d), configs
// C2-C4).  Counter-based (splitmix64 of (seed, stream, index)), so the
// output depends only on the arguments, not on the launch geometry.
#include "gg_internal.hpp"

namespace gg {
namespace {

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ uint64_t rng(uint64_t seed, uint64_t stream, uint64_t i) {
  return splitmix(splitmix(seed ^ (stream * 0xD6E8FEB86659FD93ull)) + i);
}

__global__ __launch_bounds__(256) void synth_kernel(uint32_t first_genome, uint32_t n_genomes, uint32_t wpg,
                                                    uint32_t cluster_size, float max_rate,
                                                    uint64_t seed, uint32_t* __restrict__ words) {
  const uint64_t total = (uint64_t)n_genomes * wpg;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total;
       w += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t g = first_genome + (uint32_t)(w / wpg);
    const uint32_t wg = (uint32_t)(w % wpg);
    const uint32_t cl = g / cluster_size;
    const uint32_t m = g % cluster_size;
    uint32_t word = (uint32_t)rng(seed, 1 + (uint64_t)cl, wg);
    if (m != 0) {
      // member rate r ~ U(0, max_rate), fixed per genome
      const float u = (float)(rng(seed, 0x5EEDull, g) >> 40) * (1.0f / 16777216.0f);
      const uint32_t thr = (uint32_t)(u * max_rate * 65536.0f);
      const uint64_t r0 = rng(seed ^ 0xA5A5A5A5ull, g, 4ull * wg);
      const uint64_t r1 = rng(seed ^ 0xA5A5A5A5ull, g, 4ull * wg + 1);
      const uint64_t r2 = rng(seed ^ 0xA5A5A5A5ull, g, 4ull * wg + 2);
      const uint64_t r3 = rng(seed ^ 0xA5A5A5A5ull, g, 4ull * wg + 3);
      const uint64_t rs = rng(seed ^ 0x3C3C3C3Cull, g, wg);
      const uint64_t rr[4] = {r0, r1, r2, r3};
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        const uint32_t u16 = (uint32_t)(rr[b >> 2] >> (16 * (b & 3))) & 0xFFFFu;
        if (u16 < thr) {
          const uint32_t sh = 30 - 2 * b;
          const uint32_t base = (word >> sh) & 3u;
          const uint32_t v = (uint32_t)(rs >> (4 * b)) & 0xFu;  // 0..15 -> 1..3
          const uint32_t nb = (base + 1u + (v % 3u)) & 3u;
          word = (word & ~(3u << sh)) | (nb << sh);
        }
      }
    }
    words[w] = word;
  }
}

}  // namespace

hipError_t launch_synth(uint32_t first_genome, uint32_t n_genomes, uint32_t genome_len, uint32_t cluster_size,
                        float max_sub_rate, uint64_t seed, uint32_t* words, hipStream_t st) {
  const uint32_t wpg = genome_len / 16;
  hipLaunchKernelGGL(synth_kernel, dim3(4096), dim3(256), 0, st, first_genome, n_genomes, wpg,
                     cluster_size, max_sub_rate, seed, words);
  return hipGetLastError();
}

}  // namespace gg
