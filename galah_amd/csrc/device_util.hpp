// Small device helpers shared by the pair kernels (pairs.hip, pairs_gate.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace gg {

__device__ __forceinline__ uint32_t top32(uint64_t b, uint32_t sr, uint32_t sl) {
  return (uint32_t)((b >> sr) << sl);
}

// Value bucket of b in [0, nb): the top 32 significant bits of the row
// block's largest key scaled into nb buckets.  Monotone in b, so bucket
// order is key order.
__device__ __forceinline__ uint32_t bucket_of(uint64_t b, uint32_t sr, uint32_t sl, uint32_t scale) {
  return (uint32_t)(((uint64_t)top32(b, sr, sl) * scale) >> 32);
}

// bytes 0..3 of the result = bits 0..3 of x
__device__ __forceinline__ uint32_t spread4(uint32_t x) {
  return ((x & 15u) * 0x204081u) & 0x01010101u;
}

// Sum over the 64 lanes with DPP (VALU-native; __shfl_xor would go through
// ds_bpermute): row_shr 1/2/4/8 gives each 16-lane row's inclusive prefix,
// row_bcast 15/31 carries the row totals, lane 63 holds the wave total.
// The result is wave-uniform.
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ uint32_t uni32(uint32_t v) { return __builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)uni32((uint32_t)(v >> 32)) << 32) | uni32((uint32_t)v);
}

// Number of lanes below this one whose bit is set in m.
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

}  // namespace gg
