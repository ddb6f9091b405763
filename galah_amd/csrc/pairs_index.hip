// Kernel K2, inverted-index form: all-pairs shared-hash counts from one sort.
//
// Same contract as pairs_gate.hip / pairs.hip (src/finch.rs:53-73: finch's
// merge-to-first-exhaustion, common = |A n B|, total = i + j - common, pass
// iff common >= cmin[total]).  common(i, j) is the number of hash values
// that occur in both sketches, and a hash occurs at most once per sketch, so
//
//   1. every sketch entry (hash, row, position) is radix-sorted by hash
//      (hipCUB / rocPRIM onesweep, 64-bit keys): equal hashes form runs;
//   2. each run of g >= 2 entries writes (run start, g) to every member's
//      row-major slot (runinfo), g = 1 writes 0;
//   3. one workgroup per row i walks its own runinfo (coalesced), reads the
//      members of its runs and counts every partner j > i in an LDS hash map
//      -> common(i, j) exactly, for every pair that shares a hash;
//   4. pairs whose count reaches sufmin[min(|A|, |B|)] get finch's total from
//      two rank searches and are emitted if common >= cmin[total].
//
// Pairs sharing no hash have common = 0 and can pass only when some
// cmin[t] = 0 (min_ani <= 0): the host uses the gate kernel then.  Work is
// N s log-free sorting + the shared-hash events sum_runs g (g - 1), against
// the gate kernel's N^2 s / R column tests: for clustered genome sets (every
// BASELINE config) the events are a few per entry.  A run longer than
// kMaxRun (the same hash in thousands of genomes: a highly redundant set)
// sends the call back to the gate kernel before anything is emitted.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "device_util.hpp"
#include "gg_internal.hpp"

namespace gg {
namespace {

constexpr int kRowThreads = 256;
constexpr uint32_t kMapLog2 = 11;
constexpr uint32_t kMap = 1u << kMapLog2;  // LDS partner map slots per row
constexpr uint32_t kMapFull = kMap * 3 / 4;

// #{ e < n : a[e] <= x }, a ascending
__device__ __forceinline__ uint32_t count_le(const uint64_t* __restrict__ a, uint32_t n, uint64_t x) {
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// keys[e] = hash of entry e = (row i, position k) of the [n x stride] array
// (2^64 - 1 for padding k >= len_i), vals[e] = i << kbits | k.
__global__ __launch_bounds__(256) void index_fill_kernel(const uint64_t* __restrict__ sk,
                                                         const uint32_t* __restrict__ lens, uint32_t n,
                                                         uint32_t stride, uint32_t kbits, uint64_t* __restrict__ keys,
                                                         uint32_t* __restrict__ vals) {
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t len = lens[i];
    const uint64_t* row = sk + (uint64_t)i * stride;
    for (uint32_t k = threadIdx.x; k < stride; k += 256) {
      const uint64_t e = (uint64_t)i * stride + k;
      keys[e] = k < len ? row[k] : ~0ull;
      vals[e] = (i << kbits) | k;
    }
  }
}

// Largest hash of any sketch (its last entry) -> *out (for the sort's bit
// range: the radix sort skips the high bits that are zero in every key).
__global__ __launch_bounds__(256) void index_max_kernel(const uint64_t* __restrict__ sk,
                                                        const uint32_t* __restrict__ lens, uint32_t n, uint32_t stride,
                                                        unsigned long long* __restrict__ out) {
  unsigned long long m = 0;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const uint32_t l = lens[i];
    if (l) m = max(m, (unsigned long long)sk[(uint64_t)i * stride + l - 1]);
  }
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned long long)__shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0 && m) atomicMax(out, m);
}

// Run starts write their run to every member's runinfo slot:
// (start | g << 32) for g >= 2 (bit 63 set for the 2^64 - 1 run, whose
// members may include padding), 0 for g = 1.  Runs longer than max_run set
// *overflow (the host then uses the gate kernel).
__global__ __launch_bounds__(256) void index_runs_kernel(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ vals, uint64_t total,
                                                         uint32_t stride, uint32_t kbits, uint32_t max_run,
                                                         uint64_t* __restrict__ runinfo, uint32_t* __restrict__ overflow) {
  // (no device-wide event counter: one atomic per wave on one address
  // serialises at ~12 ns each, 1.9 ms at C3)
  const uint32_t kmask = (1u << kbits) - 1u;
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < total; p += (uint64_t)gridDim.x * 256) {
    const uint64_t key = keys[p];
    if (p > 0 && keys[p - 1] == key) continue;  // not a run start
    uint64_t e = p + 1;
    while (e < total && keys[e] == key && e - p <= max_run) ++e;
    const uint64_t g = e - p;
    if (g > max_run) {
      atomicOr(overflow, 1u);
      continue;
    }
    const uint64_t info = g >= 2 ? (p | (g << 32) | (key == ~0ull ? (1ull << 63) : 0ull)) : 0ull;
    for (uint64_t q = p; q < e; ++q) {
      const uint32_t v = vals[q];
      runinfo[(uint64_t)(v >> kbits) * stride + (v & kmask)] = info;
    }
  }
}

// Allowed column interval [jlo, jhi) of row i inside tiles [tb, te) (tile
// row I holds tiles rs(I) .. rs(I) + nb - I - 1, tile (I, J) = rs(I) + J - I).
__device__ __forceinline__ void row_columns(uint32_t i, uint32_t n, uint64_t nb, uint64_t tb, uint64_t te,
                                            uint32_t& jlo, uint32_t& jhi) {
  const uint64_t I = i / GG_PAIR_TILE;
  const uint64_t rs = I * nb - I * (I - 1) / 2;
  const uint64_t t0 = rs, t1 = rs + (nb - I);
  const uint64_t a = max(t0, tb), b = min(t1, te);
  if (a >= b) {
    jlo = jhi = 0;
    return;
  }
  const uint64_t J0 = I + (a - rs), J1 = I + (b - rs);
  jlo = (uint32_t)max<uint64_t>(J0 * GG_PAIR_TILE, (uint64_t)i + 1);
  jhi = (uint32_t)min<uint64_t>(J1 * GG_PAIR_TILE, (uint64_t)n);
}

__device__ __forceinline__ uint32_t part_of(uint32_t j, uint32_t plog2) {
  return plog2 ? (j * 0x9E3779B1u) >> (32 - plog2) : 0u;
}

// One workgroup per row i: common(i, j) for every partner j > i in the
// row's column interval, from the runs of its hashes, then the finch test.
// Rows whose partners overflow the LDS map are redone in 2, 4, ... passes,
// each counting one hash class of partners.
__global__ __launch_bounds__(kRowThreads) void index_pairs_kernel(IndexLaunch a) {
  __shared__ uint32_t mkey[kMap];  // partner + 1 (0 = empty)
  __shared__ uint32_t mcnt[kMap];
  __shared__ uint32_t fill;
  __shared__ volatile uint32_t over;
  const uint32_t tid = threadIdx.x;
  const uint32_t i = a.row0 + blockIdx.x;
  if (i >= a.n) return;
  uint32_t jlo, jhi;
  row_columns(i, a.n, a.nb, a.tile_begin, a.tile_end, jlo, jhi);
  const uint32_t la = a.lens[i];
  if (jlo >= jhi || la == 0) return;
  const uint32_t kmask = (1u << a.kbits) - 1u;
  const uint64_t* ri = a.runinfo + (uint64_t)i * a.stride;
  const uint64_t* A = a.sketches + (uint64_t)i * a.stride;
  const uint64_t xa = A[la - 1];
  uint32_t plog2 = 0;
  for (uint32_t p = 0; p < (1u << plog2);) {
    for (uint32_t x = tid; x < kMap; x += kRowThreads) mkey[x] = 0u, mcnt[x] = 0u;
    if (tid == 0) fill = 0u, over = 0u;
    __syncthreads();
    for (uint32_t k = tid; k < la; k += kRowThreads) {
      if (over) break;
      const uint64_t info = ri[k];
      const uint32_t g = (uint32_t)(info >> 32) & 0x7FFFFFFFu;
      if (g < 2) continue;
      const uint32_t st = (uint32_t)info;
      const bool maxrun = (info >> 63) != 0;
      for (uint32_t q = st; q < st + g; ++q) {
        const uint32_t v = a.vals[q];
        const uint32_t j = v >> a.kbits;
        if (j < jlo || j >= jhi) continue;
        if (plog2 && part_of(j, plog2) != p) continue;
        if (maxrun && (v & kmask) >= a.lens[j]) continue;  // padding, not the hash 2^64 - 1
        uint32_t h = (j * 0x85EBCA6Bu) >> (32 - kMapLog2);
        for (uint32_t probe = 0;; ++probe) {
          const uint32_t old = atomicCAS(&mkey[h], 0u, j + 1u);
          if (old == 0u) {
            if (atomicAdd(&fill, 1u) >= kMapFull) over = 1u;
          }
          if (old == 0u || old == j + 1u) {
            atomicAdd(&mcnt[h], 1u);
            break;
          }
          if (probe >= kMap) {
            over = 1u;
            break;
          }
          h = (h + 1) & (kMap - 1);
        }
        if (over) break;
      }
    }
    __syncthreads();
    if (over && plog2 < 16) {  // too many partners for one map: split them in twice as many classes
      ++plog2;
      p = 0;
      __syncthreads();
      continue;
    }
    for (uint32_t x = tid; x < kMap; x += kRowThreads) {
      const uint32_t key = mkey[x];
      if (!key) continue;
      const uint32_t j = key - 1u, common = mcnt[x];
      const uint32_t lb = a.lens[j];
      if (common < a.sufmin[min(la, lb)]) continue;
      const uint64_t* B = a.sketches + (uint64_t)j * a.stride;
      const uint64_t xb = B[lb - 1];
      const uint32_t total = xa <= xb ? la + count_le(B, lb, xa) - common : count_le(A, la, xb) + lb - common;
      if (total <= a.tmax && common >= a.cmin[total]) {
        const unsigned long long slot = atomicAdd(a.count, 1ull);
        if (slot < a.out_cap) a.out[slot] = gg_pair{i, j, common, total};
      }
    }
    __syncthreads();
    ++p;
  }
}

}  // namespace

hipError_t index_fill(const IndexBuild& b, hipStream_t st) {
  hipError_t e = hipMemsetAsync(b.flags, 0, 16, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(index_fill_kernel, dim3(std::min<uint32_t>(b.n, 16384)), dim3(256), 0, st, b.sketches, b.lens,
                     b.n, b.stride, b.kbits, b.keys_in, b.vals_in);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(index_max_kernel, dim3(std::min<uint32_t>((b.n + 255) / 256, 1024)), dim3(256), 0, st,
                     b.sketches, b.lens, b.n, b.stride, (unsigned long long*)(b.flags + 2));
  return hipGetLastError();
}

hipError_t index_build(const IndexBuild& b, uint32_t end_bit, hipStream_t st) {
  const uint64_t total = (uint64_t)b.n * b.stride;
  size_t bytes = b.sort_tmp_bytes;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(b.sort_tmp, bytes, b.keys_in, b.keys_out, b.vals_in, b.vals_out,
                                                    (int)total, 0, (int)end_bit, st);
  if (e != hipSuccess) return e;
  const uint64_t blocks = std::min<uint64_t>(65536, (total + 255) / 256);
  hipLaunchKernelGGL(index_runs_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, b.keys_out, b.vals_out, total,
                     b.stride, b.kbits, b.max_run, b.runinfo, b.flags);
  return hipGetLastError();
}

size_t index_sort_tmp_bytes(uint64_t total) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)total, 0, 64);
  return bytes;
}

hipError_t launch_index_pairs(const IndexLaunch& a, uint32_t n_rows, hipStream_t st) {
  if (n_rows == 0) return hipSuccess;
  hipLaunchKernelGGL(index_pairs_kernel, dim3(n_rows), dim3(kRowThreads), 0, st, a);
  return hipGetLastError();
}

}  // namespace gg
