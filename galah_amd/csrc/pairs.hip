// Kernel K2: all-pairs sorted-sketch intersection + threshold + compaction.
//
// Restates src/finch.rs:53-73 (serial upper-triangle loop over
// finch::distance::distance(s_i, s_j, false)):
//   merge the two ascending sketches until EITHER is exhausted;
//   common = #equal, total = i + j - common;
//   ani = 1 - clamp(-ln(2J/(1+J))/k, 0, 1), J = common/total (f64);
//   keep (i, j) iff ani >= (min_ani as f64).
// ani(common, total) is monotone in common for fixed total, so the host
// inverts the f64 test once into cmin[total] (same libm, same expression)
// and the device decides with an integer compare: common >= cmin[total].
// No device log ever decides membership (ties near the cut are ~1e-8 apart).
//
// Pair space: upper-triangle tiles of GG_PAIR_TILE x GG_PAIR_TILE, row-major.
// Passing pairs are appended with one atomic per wave (ballot + mbcnt).
#include "gg_internal.hpp"

namespace gg {
namespace {

constexpr uint32_t kTile = GG_PAIR_TILE;
constexpr int kBlock = 256;

__device__ __forceinline__ uint64_t row_start(uint64_t I, uint64_t nb) {
  // tiles before row I: sum_{r<I} (nb - r)
  return I * nb - I * (I - 1) / 2;
}

__device__ __forceinline__ void decode_tile(uint64_t t, uint32_t nb, uint32_t& I, uint32_t& J) {
  uint32_t lo = 0, hi = nb;  // row_start(lo) <= t < row_start(hi)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (row_start(mid, nb) <= t) lo = mid;
    else hi = mid;
  }
  I = lo;
  J = lo + (uint32_t)(t - row_start(lo, nb));
}

__global__ __launch_bounds__(kBlock) void pairs_merge_kernel(PairsLaunch a) {
  const uint64_t t = a.tile_begin + blockIdx.x;
  if (t >= a.tile_end) return;
  uint32_t I, J;
  decode_tile(t, a.n_row_tiles, I, J);
  const uint32_t lane = threadIdx.x & 63;

  for (uint32_t e = threadIdx.x; e < kTile * kTile; e += kBlock) {
    const uint32_t i = I * kTile + e / kTile;
    const uint32_t j = J * kTile + e % kTile;
    const bool valid = (i < j) && (j < a.n);
    uint32_t common = 0, total = 0;
    bool pass = false;
    if (valid) {
      const uint64_t* A = a.sketches + (uint64_t)i * a.stride;
      const uint64_t* B = a.sketches + (uint64_t)j * a.stride;
      const uint32_t la = a.lens[i], lb = a.lens[j];
      uint32_t x = 0, y = 0, c = 0;
      while (x < la && y < lb) {
        const uint64_t va = A[x], vb = B[y];
        x += (va <= vb);
        y += (vb <= va);
        c += (va == vb);
      }
      common = c;
      total = x + y - c;
      pass = (total <= a.tmax) && (common >= a.cmin[total]);
    }
    const unsigned long long m = __ballot(pass);
    if (m) {
      const uint32_t npass = __popcll(m);
      unsigned long long base = 0;
      if (lane == __builtin_ctzll(m)) base = atomicAdd(a.count, (unsigned long long)npass);
      base = __shfl(base, __builtin_ctzll(m));
      if (pass) {
        const uint32_t rank = __popcll(m & ((1ull << lane) - 1ull));
        const unsigned long long slot = base + rank;
        if (slot < a.out_cap) a.out[slot] = gg_pair{i, j, common, total};
      }
    }
  }
}

}  // namespace

hipError_t launch_pairs(const PairsLaunch& a, hipStream_t st) {
  if (a.tile_end <= a.tile_begin) return hipSuccess;
  const uint64_t n = a.tile_end - a.tile_begin;
  if (n > 0x7fffffffull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pairs_merge_kernel, dim3((uint32_t)n), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

}  // namespace gg
