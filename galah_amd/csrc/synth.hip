// Benchmark input generator: synthetic clustered genomes written straight
// into HBM in the 2-bit layout kernel K1 reads (SURVEY.md 8(d), configs
// C2-C4).  Counter-based (splitmix64 of (seed, stream, index)), so the
// output depends only on the arguments, not on the launch geometry.
#include <algorithm>

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

// Mixed lengths (config C5): genome g occupies words [woff[g], woff[g+1]);
// the members of a cluster share the root's length.  blockIdx.y = genome.
__global__ __launch_bounds__(256) void synth_mixed_kernel(uint32_t first_genome, const uint64_t* __restrict__ woff,
                                                          uint32_t cluster_size, float max_rate, uint64_t seed,
                                                          uint32_t* __restrict__ words) {
  const uint32_t gl = blockIdx.y;
  const uint32_t g = first_genome + gl;
  const uint64_t w0 = woff[gl], nw = woff[gl + 1] - w0;
  const uint32_t cl = g / cluster_size;
  const uint32_t m = g % cluster_size;
  const float u = (float)(rng(seed, 0x5EEDull, g) >> 40) * (1.0f / 16777216.0f);
  const uint32_t thr = m ? (uint32_t)(u * max_rate * 65536.0f) : 0u;
  for (uint64_t wg = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; wg < nw; wg += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t word = (uint32_t)rng(seed, 1 + (uint64_t)cl, wg);
    if (thr) {
      const uint64_t rr[4] = {rng(seed ^ 0xA5A5A5A5ull, g, 4ull * wg), rng(seed ^ 0xA5A5A5A5ull, g, 4ull * wg + 1),
                              rng(seed ^ 0xA5A5A5A5ull, g, 4ull * wg + 2), rng(seed ^ 0xA5A5A5A5ull, g, 4ull * wg + 3)};
      const uint64_t rs = rng(seed ^ 0x3C3C3C3Cull, g, wg);
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        const uint32_t u16 = (uint32_t)(rr[b >> 2] >> (16 * (b & 3))) & 0xFFFFu;
        if (u16 < thr) {
          const uint32_t sh = 30 - 2 * b;
          const uint32_t base = (word >> sh) & 3u;
          const uint32_t v = (uint32_t)(rs >> (4 * b)) & 0xFu;
          word = (word & ~(3u << sh)) | (((base + 1u + (v % 3u)) & 3u) << sh);
        }
      }
    }
    words[w0 + wg] = word;
  }
}

}  // namespace

hipError_t launch_synth_mixed(uint32_t first_genome, uint32_t n_genomes, const uint64_t* d_woff,
                              uint64_t max_words, uint32_t cluster_size, float max_sub_rate, uint64_t seed,
                              uint32_t* words, hipStream_t st) {
  if (n_genomes == 0) return hipSuccess;
  const uint32_t bx = (uint32_t)std::min<uint64_t>(64, (max_words + 255) / 256);
  hipLaunchKernelGGL(synth_mixed_kernel, dim3(std::max(1u, bx), n_genomes), dim3(256), 0, st, first_genome, d_woff,
                     cluster_size, max_sub_rate, seed, words);
  return hipGetLastError();
}

hipError_t launch_synth(uint32_t first_genome, uint32_t n_genomes, uint32_t genome_len, uint32_t cluster_size,
                        float max_sub_rate, uint64_t seed, uint32_t* words, hipStream_t st) {
  const uint32_t wpg = genome_len / 16;
  hipLaunchKernelGGL(synth_kernel, dim3(4096), dim3(256), 0, st, first_genome, n_genomes, wpg,
                     cluster_size, max_sub_rate, seed, words);
  return hipGetLastError();
}

}  // namespace gg
