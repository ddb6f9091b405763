// Kernel K2, inverted-index form: all-pairs shared-hash counts from one sort.
//
// Same contract as pairs_gate.hip / pairs.hip (src/finch.rs:53-73: finch's
// merge-to-first-exhaustion, common = |A n B|, total = i + j - common, pass
// iff common >= cmin[total]).  common(i, j) is the number of hash values
// that occur in both sketches, and a hash occurs at most once per sketch, so
//
//   1. every sketch entry (row i, position k < len_i) is grouped with the
//      entries of equal hash: the bucketed build (default) sorts the entries
//      by a monotone, population-balanced bucket of their hash (16-bit ids,
//      two radix passes) and groups equal hashes per bucket in an LDS hash
//      table; the full build (fallback) radix-sorts the top 32 significant
//      bits of each hash, carrying its low 32 bits, in four passes;
//   2. each group of g >= 2 equal hashes ("run") lies contiguous in ents,
//      and (run start, g) goes to every member's row-major slot (runinfo;
//      g = 1 writes 0);
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
// (the pairs kernel's LDS partner map per row: 2^11 slots, 2^13 for heavy
// indexes; index_pairs_kernel)
constexpr int kScanThreads = 1024;
constexpr uint32_t kXcds = 8;  // MI355X: 8 XCDs, each with its own L2

// Key shape of the index (index_scan_kernel leaves the largest hash in
// info[1]): the sort key of the full build is the top 32 significant bits
// of a hash (h >> sh, end_bit significant bits); the bucketed build
// top-aligns that key (norm = 32 - end_bit) and splits it into a coarse bin
// (top 12 bits) and the 20 bits below.
struct KeyShape {
  uint32_t sh, norm;
};
__device__ __forceinline__ KeyShape key_shape(unsigned long long maxh) {
  const uint32_t bits = maxh ? 64u - (uint32_t)__builtin_clzll(maxh) : 0u;
  const uint32_t sh = bits > 32 ? bits - 32 : 0u;
  const uint32_t eb = bits - sh > 1u ? bits - sh : 1u;
  return KeyShape{sh, 32u - eb};
}

// Bucketed build: 4096 coarse bins of the top-aligned key, each split into
// nsub = ceil(count / per) equal sub-ranges (bbase[c] = first bucket of bin c,
// bbase[4096] = buckets).  bucket_of is monotone in the hash and equal
// hashes share a bucket; the buckets hold ~per entries whatever the shape of
// the hash distribution (C5's sketches of 0.5-12 Mbp genomes put 25x more
// entries near 0 than near the largest hash).
constexpr uint32_t kCoarseBits = 12;
constexpr uint32_t kBucketPad = 0xFFFFu;
constexpr uint32_t kBucketKeyBits = 16;  // sort key of an unused slot (every bucket id is below: <= 64096 buckets)
constexpr uint32_t kCoarse = 1u << kCoarseBits;
__device__ __forceinline__ uint32_t bucket_of(uint64_t h, KeyShape ks, const uint32_t* __restrict__ bbase) {
  const uint32_t key = (uint32_t)(h >> ks.sh) << ks.norm;
  const uint32_t c = key >> (32 - kCoarseBits);
  const uint32_t rel = key & ((1u << (32 - kCoarseBits)) - 1u);
  const uint32_t b0 = bbase[c], ns = bbase[c + 1] - b0;
  return b0 + (uint32_t)(((uint64_t)rel * ns) >> (32 - kCoarseBits));
}

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

// One workgroup: offs[i] = sum of lens[0..i) (entries before row i), the
// total -> info[0], the largest hash of any sketch (its last entry) ->
// info[1].  n is at most a few 10^5 rows.
__global__ __launch_bounds__(kScanThreads) void index_scan_kernel(const uint64_t* __restrict__ sk,
                                                                  const uint32_t* __restrict__ lens, uint32_t n,
                                                                  uint32_t stride, uint64_t* __restrict__ offs,
                                                                  unsigned long long* __restrict__ info) {
  __shared__ unsigned long long wsum[kScanThreads / 64], wmax[kScanThreads / 64];
  const uint32_t tid = threadIdx.x;
  const uint32_t per = (n + kScanThreads - 1) / kScanThreads;
  const uint32_t b0 = min(tid * per, n), b1 = min(b0 + per, n);
  unsigned long long sum = 0, mx = 0;
  for (uint32_t i = b0; i < b1; ++i) {
    const uint32_t l = lens[i];
    sum += l;
    if (l) mx = max(mx, (unsigned long long)sk[(uint64_t)i * stride + l - 1]);
  }
  unsigned long long inc = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(inc, o);
    if ((tid & 63) >= (uint32_t)o) inc += y;
  }
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, (unsigned long long)__shfl_xor(mx, o));
  if ((tid & 63) == 63) wsum[tid >> 6] = inc;
  if ((tid & 63) == 0) wmax[tid >> 6] = mx;
  __syncthreads();
  unsigned long long run = inc - sum;
  for (uint32_t w = 0; w < (tid >> 6); ++w) run += wsum[w];
  for (uint32_t i = b0; i < b1; ++i) {
    offs[i] = run;
    run += lens[i];
  }
  if (tid == kScanThreads - 1) {
    info[0] = run;  // the last thread's running sum ends at the total
    unsigned long long m = 0;
    for (int w = 0; w < kScanThreads / 64; ++w) m = max(m, wmax[w]);
    info[1] = m;
  }
}

// Entry of row i, k < len_i, value i << kbits | k:
//   full build:     at offs[i] + k, keys = h >> sh (32 bits), vals = lo32(h) << 32 | value
//   bucketed build: at i * stride + k (every slot k < stride: the sort's item
//                   count is known before the row lengths are), 16-bit keys =
//                   bucket_of(h) or kBucketPad past len_i, vals32 = value
template <bool BUCKET>
__global__ __launch_bounds__(256) void index_fill_kernel(const uint64_t* __restrict__ sk,
                                                         const uint32_t* __restrict__ lens,
                                                         const uint64_t* __restrict__ offs, uint32_t n,
                                                         uint32_t stride, uint32_t kbits, uint32_t sh,
                                                         const unsigned long long* __restrict__ info,
                                                         const uint32_t* __restrict__ bbase,
                                                         uint32_t* __restrict__ keys, uint64_t* __restrict__ vals) {
  const KeyShape ks = BUCKET ? key_shape(info[1]) : KeyShape{sh, 0u};
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
    const uint32_t len = lens[i];
    const uint64_t* row = sk + (uint64_t)i * stride;
    if (BUCKET) {  // row-major slots i * stride + k, unused slots keyed past every bucket
      const uint64_t o = (uint64_t)i * stride;
      for (uint32_t k = threadIdx.x; k < stride; k += 256) {
        ((uint16_t*)keys)[o + k] = (uint16_t)(k < len ? bucket_of(row[k], ks, bbase) : kBucketPad);
        ((uint32_t*)vals)[o + k] = (i << kbits) | k;
      }
      continue;
    }
    const uint64_t o = offs[i];
    for (uint32_t k = threadIdx.x; k < len; k += 256) {
      const uint64_t h = row[k];
      const uint32_t v = (i << kbits) | k;
      {
        keys[o + k] = (uint32_t)(h >> sh);
        vals[o + k] = (h << 32) | v;
      }
    }
  }
}

// Adds the lanes' values to the LDS counts h for a wave whose active lanes
// (`in`, a prefix of the wave) hold non-decreasing values: the first lane of
// each run of equal values adds the run's length x weight (one atomic per
// run).
__device__ __forceinline__ void wave_runs_add(uint32_t* h, uint32_t v, bool in, uint32_t weight = 1) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t prev = __shfl_up(v, 1);
  const bool head = in && (lane == 0 || prev != v);
  const uint64_t heads = __ballot(head);
  const uint32_t n_in = (uint32_t)__popcll(__ballot(in));
  if (head) {
    const uint64_t after = (heads >> lane) >> 1;
    const uint32_t next = after ? lane + 1u + (uint32_t)__builtin_ctzll(after) : 64u;
    atomicAdd(&h[v], (min(next, n_in) - lane) * weight);
  }
}

// Coarse-bin histogram of every sketch entry (one LDS histogram per
// workgroup over a contiguous slice of rows, merged with one atomic per
// non-empty bin).
__global__ __launch_bounds__(256) void bucket_hist_kernel(const uint64_t* __restrict__ sk,
                                                          const uint32_t* __restrict__ lens, uint32_t n,
                                                          uint32_t stride,
                                                          const unsigned long long* __restrict__ info,
                                                          uint32_t* __restrict__ hist, uint32_t may_sample) {
  __shared__ uint32_t lh[kCoarse];
  for (uint32_t x = threadIdx.x; x < kCoarse; x += 256) lh[x] = 0u;
  __syncthreads();
  const KeyShape ks = key_shape(info[1]);
  const uint32_t i0 = (uint32_t)((uint64_t)n * blockIdx.x / gridDim.x);
  const uint32_t i1 = (uint32_t)((uint64_t)n * (blockIdx.x + 1) / gridDim.x);
  auto bin = [&](uint64_t h) { return ((uint32_t)(h >> ks.sh) << ks.norm) >> (32 - kCoarseBits); };
  // A row is sorted, so its bins never decrease: the lanes of a wave read 64
  // consecutive entries (coalesced) and only the first lane of each run of
  // equal bins adds the run's length (C5's s = 10000 rows hold ~2.4 entries
  // per bin: one atomic per entry put the lanes of a wave on a few
  // neighbouring bins, 21.5 conflict cycles per LDS instruction; a contiguous
  // piece per thread instead spread every load over 64 lines and read the
  // sketches ~6x over, 0.25 -> 0.76 ms)
  // Past 2^26 entries the histogram is sampled: one 16-entry line (128 B) of
  // every 8 of a row, its offset varying with the row, each entry counted 8
  // times.  The counts only shape the buckets (any bucket_of is exact), and
  // a coarse bin then holds >= ~2k sampled entries at C5's skew, so a bucket
  // comes out within a few % of `per` (the capacity is 1.8x).
  const bool sample = may_sample && info[0] >= (1ull << 26);
  for (uint32_t i = i0; i < i1; ++i) {
    const uint32_t len = lens[i];
    const uint64_t* row = sk + (uint64_t)i * stride;
    if (sample) {
      const uint32_t lines = (len + 15) / 16, first = i & 7;
      const uint32_t q_end = lines > first ? (lines - first + 7) / 8 * 16 : 0;
      for (uint32_t q0 = 0; q0 < q_end; q0 += 256) {
        const uint32_t q = q0 + threadIdx.x;
        const uint32_t k = (first + (q >> 4) * 8) * 16 + (q & 15);
        const bool in = q < q_end && k < len;
        const uint32_t b = in ? bin(row[k]) : ~0u;
        wave_runs_add(lh, b, in, 8);
      }
      continue;
    }
    for (uint32_t k0 = 0; k0 < len; k0 += 256) {
      const uint32_t k = k0 + threadIdx.x;
      const bool in = k < len;
      const uint32_t b = in ? bin(row[k]) : ~0u;
      wave_runs_add(lh, b, in);
    }
  }
  __syncthreads();
  for (uint32_t x = threadIdx.x; x < kCoarse; x += 256)
    if (lh[x]) atomicAdd(&hist[x], lh[x]);
}

// bbase from the histogram: per = max(1024, ceil(entries / 60000)) entries
// per bucket at most on average, so that there are at most 60000 + 4096
// buckets (16-bit bucket ids: two digit passes of the sort).
constexpr uint32_t kBaseThreads = 1024;
__global__ __launch_bounds__(kBaseThreads) void bucket_base_kernel(const uint32_t* __restrict__ hist,
                                                                   const unsigned long long* __restrict__ info,
                                                                   uint32_t* __restrict__ bbase) {
  __shared__ uint32_t wsum[kBaseThreads / 64];
  __shared__ unsigned long long wtot[kBaseThreads / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  constexpr uint32_t q = kCoarse / kBaseThreads;
  // per from the histogram's own total (a sampled histogram's differs from
  // the entries a little): sum ceil(c / per) <= 60000 + 4096 buckets either way
  uint32_t hc[q];
  unsigned long long t = 0;
#pragma unroll
  for (uint32_t x = 0; x < q; ++x) {
    hc[x] = hist[tid * q + x];
    t += hc[x];
  }
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o);
  if (lane == 0) wtot[tid >> 6] = t;
  __syncthreads();
  unsigned long long total = 0;
  for (uint32_t w = 0; w < kBaseThreads / 64; ++w) total += wtot[w];
  (void)info;
  const uint32_t per = (uint32_t)max(1024ull, (total + 59999ull) / 60000ull);
  uint32_t ns[q], sum = 0;
#pragma unroll
  for (uint32_t x = 0; x < q; ++x) {
    ns[x] = max(1u, (hc[x] + per - 1u) / per);  // (a bin the sample missed still gets its own bucket)
    sum += ns[x];
  }
  uint32_t inc = sum;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) wsum[tid >> 6] = inc;
  __syncthreads();
  uint32_t run = inc - sum;
  for (uint32_t w = 0; w < (tid >> 6); ++w) run += wsum[w];
#pragma unroll
  for (uint32_t x = 0; x < q; ++x) {
    bbase[tid * q + x] = run;
    run += ns[x];
  }
  if (tid == kBaseThreads - 1) bbase[kCoarse] = run;
}

// Split build (bucketed, every row): the sort of the bucket ids is replaced
// by two placements that use what the sort did not know -- a row is sorted,
// so bucket ids never decrease along it and its entries of one super-bin
// (bucket >> 8, at most 256 of them) are one contiguous piece:
//   split_keys     one workgroup per row: bucket ids (16 bits, row-major
//                  slots as index_fill writes them) and the row's count per
//                  super-bin -> cnt[D * n + i];
//   (scan)         off = exclusive sum of cnt (super-bin major, row minor):
//                  super-bin D's entries from off[D * n], row i's at
//                  off[D * n + i];
//   split_scatter  one workgroup per row: each entry to off[D * n + i] plus
//                  its place in the row's piece of D, as its 8 low bucket
//                  bits (keys8) and its entry value (vals);
//   superbin_count, superbin_place  an LDS counting sort of each super-bin's
//                  entries by the low bits (the bucket), giving the buckets'
//                  bounds (bstart) and the entries in bucket order.
// The entries move 3 times at 5 B instead of a fill and two radix passes at
// 6 B each (no digit look-back, no bounds pass).
constexpr uint32_t kSuper = 256;  // super-bins: bucket >> 8 (buckets < 2^16)

__device__ __forceinline__ uint32_t row_of_block(uint32_t n) {
  // XCD-aware: the workgroups of XCD x (blockIdx % kXcds) take the x-th
  // contiguous range of rows, so the counts and pieces of neighbouring rows
  // (adjacent in every super-bin) are written through the same L2
  const uint32_t per_xcd = (n + kXcds - 1) / kXcds;
  return (blockIdx.x % kXcds) * per_xcd + blockIdx.x / kXcds;
}

__global__ __launch_bounds__(256) void split_keys_kernel(const uint64_t* __restrict__ sk,
                                                         const uint32_t* __restrict__ lens, uint32_t n,
                                                         uint32_t stride,
                                                         const unsigned long long* __restrict__ info,
                                                         const uint32_t* __restrict__ bbase,
                                                         uint16_t* __restrict__ keys, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t lc[kSuper];
  const uint32_t i = row_of_block(n);
  if (i >= n) return;
  const uint32_t tid = threadIdx.x;
  lc[tid] = 0u;
  if (i == 0 && tid == 0) cnt[(uint64_t)kSuper * n] = 0u;  // (the scan's last item: off[256 n] = entries)
  __syncthreads();
  const KeyShape ks = key_shape(info[1]);
  const uint32_t len = lens[i];
  const uint64_t* row = sk + (uint64_t)i * stride;
  uint16_t* krow = keys + (uint64_t)i * stride;
  for (uint32_t k0 = 0; k0 < stride; k0 += 256) {
    const uint32_t k = k0 + tid;
    const bool in = k < len;
    const uint32_t b = in ? bucket_of(row[k], ks, bbase) : kBucketPad;
    if (k < stride) krow[k] = (uint16_t)b;
    if (k0 < len) wave_runs_add(lc, b >> 8, in);  // (uniform: k0 < len)
  }
  __syncthreads();
  cnt[(uint64_t)tid * n + i] = lc[tid];
}

__global__ __launch_bounds__(256) void split_scatter_kernel(const uint16_t* __restrict__ keys,
                                                            const uint32_t* __restrict__ lens, uint32_t n,
                                                            uint32_t stride, uint32_t kbits,
                                                            const uint32_t* __restrict__ cnt,
                                                            const uint32_t* __restrict__ off,
                                                            uint8_t* __restrict__ keys8,
                                                            uint32_t* __restrict__ vals) {
  __shared__ uint32_t base[kSuper];
  __shared__ uint32_t wsum[256 / 64];
  const uint32_t i = row_of_block(n);
  if (i >= n) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  // base[D] = off[D n + i] - (the row's entries before its piece of D)
  const uint32_t c = cnt[(uint64_t)tid * n + i];
  uint32_t inc = c;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) wsum[tid >> 6] = inc;
  __syncthreads();
  uint32_t before = inc - c;
  for (uint32_t w = 0; w < (tid >> 6); ++w) before += wsum[w];
  base[tid] = off[(uint64_t)tid * n + i] - before;
  __syncthreads();
  const uint32_t len = lens[i];
  const uint16_t* krow = keys + (uint64_t)i * stride;
  for (uint32_t k = tid; k < len; k += 256) {
    const uint32_t b = krow[k];
    const uint32_t p = base[b >> 8] + k;
    keys8[p] = (uint8_t)b;
    vals[p] = (i << kbits) | k;
  }
}

// The super-bin sort: super-bin D's entries [off[D n], off[(D + 1) n]) are
// cut into up to kSuperParts equal slices, one workgroup each (a
// workgroup per super-bin left the chip at one workgroup per CU: 0.57 ms at
// C5).  A slice is read in groups of 16 entries (one 16-byte load of keys8,
// four of vals; groups aligned to 16 entries, the slice ends masked).
//   superbin_count  the slice's counts per low key byte -> shist[D][part][256]
//   superbin_place  bucket x of super-bin D starts at off[D n] + the counts of
//                   buckets < x over all slices (bstart; part 0 writes it,
//                   the last workgroup also bstart[65536] = entries); the
//                   slice's entries of bucket x follow those of earlier
//                   slices (order inside a bucket is free: index_bucket
//                   groups by hash)
constexpr uint32_t kSuperParts = 16;  // slices per super-bin at most (fewer for small inputs)

__device__ __forceinline__ void super_slice(const uint32_t* __restrict__ off, uint32_t n, uint32_t D, uint32_t part,
                                            uint32_t parts, uint32_t& a, uint32_t& e) {
  const uint32_t s0 = off[(uint64_t)D * n], s1 = off[(uint64_t)(D + 1) * n];
  a = s0 + (uint32_t)((uint64_t)(s1 - s0) * part / parts);
  e = s0 + (uint32_t)((uint64_t)(s1 - s0) * (part + 1) / parts);
}

// XCD-aware: the slices of a super-bin run on one XCD (blockIdx
// % kXcds), so the bucket-ordered lines of its output are written through
// one L2 (slices dealt round-robin over the XCDs wrote each line from up to
// 8 L2s)
__device__ __forceinline__ void super_block(uint32_t parts, uint32_t& D, uint32_t& part) {
  constexpr uint32_t per_xcd = kSuper / kXcds;
  const uint32_t j = blockIdx.x / kXcds;
  D = (blockIdx.x % kXcds) * per_xcd + j / parts;
  part = j % parts;
}

__device__ __forceinline__ uint32_t key_byte(const uint32_t (&w)[4], uint32_t e) {
  return (w[e >> 2] >> (8 * (e & 3))) & 0xFFu;
}

__global__ __launch_bounds__(256) void superbin_count_kernel(const uint8_t* __restrict__ keys8,
                                                             const uint32_t* __restrict__ off, uint32_t n,
                                                             uint32_t parts, uint32_t* __restrict__ shist) {
  __shared__ uint32_t h[kSuper];
  const uint32_t tid = threadIdx.x;
  uint32_t D, part, a, e;
  super_block(parts, D, part);
  super_slice(off, n, D, part, parts, a, e);
  h[tid] = 0u;
  __syncthreads();
  for (uint64_t g = a / 16 + tid; g < (e + 15ull) / 16; g += 256) {
    const uint4 kw = *(const uint4*)(keys8 + g * 16);
    const uint32_t w[4] = {kw.x, kw.y, kw.z, kw.w};
#pragma unroll
    for (uint32_t x = 0; x < 16; ++x) {
      const uint64_t p = g * 16 + x;
      if (p >= a && p < e) atomicAdd(&h[key_byte(w, x)], 1u);
    }
  }
  __syncthreads();
  shist[((uint64_t)D * parts + part) * kSuper + tid] = h[tid];
}

// superbin_place stages a chunk of up to kPlaceChunk entries in LDS in bucket
// order (an LDS counting sort of the chunk), then writes each bucket's piece
// as one contiguous run: ~48 entries per bucket per chunk at C5.  (Placing
// each entry straight at its bucket's cursor was one 4-byte store per entry
// to a scattered line: 0.63-0.67 ms at C5.)
constexpr uint32_t kPlaceThreads = 512;
constexpr uint32_t kPlaceChunk = 12288;  // (65 KB of LDS: two workgroups per CU)

// exclusive scan of v over threads 0..255 (waves 0-3, uniform), into the
// running total of waves before; wsum holds the 4 wave totals after a barrier
__device__ __forceinline__ uint32_t scan256_wave(uint32_t v, uint32_t* wsum) {
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  uint32_t inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o);
    if (lane >= (uint32_t)o) inc += y;
  }
  if (lane == 63) wsum[tid >> 6] = inc;
  return inc - v;
}

__global__ __launch_bounds__(kPlaceThreads) void superbin_place_kernel(const uint8_t* __restrict__ keys8,
                                                                       const uint32_t* __restrict__ vals,
                                                                       const uint32_t* __restrict__ off, uint32_t n,
                                                                       uint32_t parts,
                                                                       const uint32_t* __restrict__ shist,
                                                                       uint32_t* __restrict__ bstart,
                                                                       uint32_t* __restrict__ sorted) {
  __shared__ uint32_t cur[kSuper], lcnt[kSuper], lpos[kSuper], lstart[kSuper], wsum[kSuper / 64];
  __shared__ uint32_t stage[kPlaceChunk];
  __shared__ uint8_t sbk[kPlaceChunk];
  const uint32_t tid = threadIdx.x;
  const bool bt = tid < kSuper;  // (threads 0-255: one bucket each)
  uint32_t D, part, a, e;
  super_block(parts, D, part);
  super_slice(off, n, D, part, parts, a, e);
  // bucket tid: its count over all slices and over the slices before this one
  uint32_t tot = 0, before = 0, ex = 0;
  if (bt) {
    const uint32_t* hd = shist + (uint64_t)D * parts * kSuper + tid;
    for (uint32_t q = 0; q < parts; ++q) {
      const uint32_t c = hd[q * kSuper];
      tot += c;
      before += q < part ? c : 0u;
    }
    ex = scan256_wave(tot, wsum);
  }
  __syncthreads();
  if (bt) {
    uint32_t start = off[(uint64_t)D * n] + ex;
    for (uint32_t w = 0; w < (tid >> 6); ++w) start += wsum[w];
    if (part == 0) bstart[D * kSuper + tid] = start;
    if (D == kSuper - 1 && part == parts - 1 && tid == 0) bstart[(uint64_t)kSuper * kSuper] = e;
    cur[tid] = start + before;
  }
  for (uint32_t c0 = a; c0 < e; c0 += kPlaceChunk) {
    const uint32_t c1 = min(e, c0 + kPlaceChunk);
    if (bt) lcnt[tid] = 0u;
    __syncthreads();
    for (uint64_t g = c0 / 16 + tid; g < (c1 + 15ull) / 16; g += kPlaceThreads) {
      const uint4 kw = *(const uint4*)(keys8 + g * 16);
      const uint32_t w[4] = {kw.x, kw.y, kw.z, kw.w};
#pragma unroll
      for (uint32_t x = 0; x < 16; ++x) {
        const uint64_t p = g * 16 + x;
        if (p >= c0 && p < c1) atomicAdd(&lcnt[key_byte(w, x)], 1u);
      }
    }
    __syncthreads();
    uint32_t lex = 0;
    if (bt) lex = scan256_wave(lcnt[tid], wsum);
    __syncthreads();
    if (bt) {
      for (uint32_t w = 0; w < (tid >> 6); ++w) lex += wsum[w];
      lstart[tid] = lex;
      lpos[tid] = lex;
    }
    __syncthreads();
    for (uint64_t g = c0 / 16 + tid; g < (c1 + 15ull) / 16; g += kPlaceThreads) {
      const uint4 kw = *(const uint4*)(keys8 + g * 16);
      const uint4* vp = (const uint4*)(vals + g * 16);
      const uint4 v0 = vp[0], v1 = vp[1], v2 = vp[2], v3 = vp[3];
      const uint32_t w[4] = {kw.x, kw.y, kw.z, kw.w};
      const uint32_t v[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                              v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
#pragma unroll
      for (uint32_t x = 0; x < 16; ++x) {
        const uint64_t p = g * 16 + x;
        if (p >= c0 && p < c1) {
          const uint32_t bk = key_byte(w, x);
          const uint32_t l = atomicAdd(&lpos[bk], 1u);
          stage[l] = v[x];
          sbk[l] = (uint8_t)bk;
        }
      }
    }
    __syncthreads();
    for (uint32_t l = tid; l < c1 - c0; l += kPlaceThreads) {
      const uint32_t bk = sbk[l];
      sorted[cur[bk] + (l - lstart[bk])] = stage[l];
    }
    __syncthreads();
    if (bt) cur[tid] += lcnt[tid];
  }
}

// Row-range index.  A blocked Bloom filter of the hashes of rows [r0, r1):
// one 32-bit word per hash, two bits in it, so a test is one load (the
// filter holds ~16 bits per row entry: ~2% false positives, which only add
// entries to the sort).
__device__ __forceinline__ void bloom_probe(uint64_t h, uint32_t log2b, uint32_t& word, uint32_t& mask) {
  const uint64_t x = (h + 0x632BE59BD9B4E019ull) * 0x9E3779B97F4A7C15ull;
  word = (uint32_t)(x >> (64 - (log2b - 5)));
  mask = (1u << ((uint32_t)(x >> 20) & 31u)) | (1u << ((uint32_t)(x >> 26) & 31u));
}

__global__ __launch_bounds__(256) void bloom_build_kernel(const uint64_t* __restrict__ sk,
                                                          const uint32_t* __restrict__ lens, uint32_t r0,
                                                          uint32_t r1, uint32_t stride, uint32_t* __restrict__ bloom,
                                                          uint32_t log2b) {
  for (uint32_t i = r0 + blockIdx.x; i < r1; i += gridDim.x) {
    const uint32_t len = lens[i];
    const uint64_t* row = sk + (uint64_t)i * stride;
    for (uint32_t k = threadIdx.x; k < len; k += 256) {
      uint32_t w, m;
      bloom_probe(row[k], log2b, w, m);
      atomicOr(&bloom[w], m);
    }
  }
}

__device__ __forceinline__ bool bloom_test(const uint32_t* __restrict__ bloom, uint32_t log2b, uint64_t h) {
  uint32_t w, m;
  bloom_probe(h, log2b, w, m);
  return (bloom[w] & m) == m;
}

// The kept entries, compacted: rows [r0, r1) keep all of theirs, other rows
// the entries that pass the filter.  Workgroup w owns a contiguous slice of
// rows: it counts its kept entries, reserves their space with one atomic on
// *kept, and writes them in row order (a wave-ballot prefix per 256-entry
// chunk).  The key shift comes from the largest hash (info[1], written by
// index_scan_kernel before this launch), as the host computes it.
template <bool BUCKET>
__global__ __launch_bounds__(256) void index_fill_range_kernel(
    const uint64_t* __restrict__ sk, const uint32_t* __restrict__ lens, uint32_t n, uint32_t stride, uint32_t kbits,
    const uint32_t* __restrict__ bloom, uint32_t log2b, uint32_t r0, uint32_t r1,
    const unsigned long long* __restrict__ info, const uint32_t* __restrict__ bbase, uint32_t* __restrict__ kept,
    uint32_t* __restrict__ keys, uint64_t* __restrict__ vals) {
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t base_s;
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t i0 = (uint32_t)((uint64_t)n * blockIdx.x / gridDim.x);
  const uint32_t i1 = (uint32_t)((uint64_t)n * (blockIdx.x + 1) / gridDim.x);
  const KeyShape ks = key_shape(info[1]);
  const uint32_t sh = ks.sh;
  uint32_t c = 0;
  for (uint32_t i = i0; i < i1; ++i) {
    const uint32_t len = lens[i];
    if (i >= r0 && i < r1) {
      if (threadIdx.x == 0) c += len;
      continue;
    }
    const uint64_t* row = sk + (uint64_t)i * stride;
    for (uint32_t k = threadIdx.x; k < len; k += 256) c += bloom_test(bloom, log2b, row[k]) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if (lane == 0) wsum[wave] = c;
  __syncthreads();
  if (threadIdx.x == 0) base_s = atomicAdd(kept, wsum[0] + wsum[1] + wsum[2] + wsum[3]);
  __syncthreads();
  uint64_t o = base_s;
  for (uint32_t i = i0; i < i1; ++i) {
    const uint32_t len = lens[i];
    const uint64_t* row = sk + (uint64_t)i * stride;
    const bool all = i >= r0 && i < r1;
    for (uint32_t k0 = 0; k0 < len; k0 += 256) {
      const uint32_t k = k0 + threadIdx.x;
      const uint64_t h = k < len ? row[k] : 0ull;
      const bool keep = k < len && (all || bloom_test(bloom, log2b, h));
      const uint64_t m = __ballot(keep);
      const uint32_t before = __popcll(m & ((1ull << lane) - 1ull));
      __syncthreads();  // (the previous chunk's readers of wsum are done)
      if (lane == 0) wsum[wave] = __popcll(m);
      __syncthreads();
      uint32_t base = 0;
      for (uint32_t w = 0; w < wave; ++w) base += wsum[w];
      if (keep) {
        const uint64_t at = o + base + before;
        const uint32_t v = (i << kbits) | k;
        if (BUCKET) {
          ((uint16_t*)keys)[at] = (uint16_t)bucket_of(h, ks, bbase);
          ((uint32_t*)vals)[at] = v;
        } else {
          keys[at] = (uint32_t)(h >> sh);
          vals[at] = (h << 32) | v;
        }
      }
      o += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    }
  }
}

// The member-read count of a build (IndexBuild::cost) is summed in
// kCostSlots partial counters 128 B apart (one per workgroup modulo the
// slots; a single counter, added to by every wave of the run passes, cost
// C3's K2 1.8 ms of atomics on one address), then into cost[0] by
// index_cost_sum_kernel before the pairs kernel reads it.
// The longest run goes the same way (word 1 of each slot, cost[1]): a run
// longer than the partner map's fill limit means rows with that many
// partners, which the large map serves in one pass.
constexpr uint32_t kCostSlots = 64, kCostStride = 16;  // (u64 words: 128 B apart)
__device__ __forceinline__ void cost_add(unsigned long long* cost, unsigned long long reads, uint32_t g) {
  for (int o = 32; o > 0; o >>= 1) {
    reads += __shfl_xor(reads, o);
    g = max(g, (uint32_t)__shfl_xor(g, o));
  }
  if ((threadIdx.x & 63) == 0 && reads) {
    unsigned long long* slot = &cost[kCostStride * (1 + (blockIdx.x + (threadIdx.x >> 6)) % kCostSlots)];
    atomicAdd(slot, reads);
    atomicMax(slot + 1, (unsigned long long)g);
  }
}
__global__ void index_cost_sum_kernel(unsigned long long* cost) {
  unsigned long long v = cost[kCostStride * (1 + threadIdx.x)], g = cost[kCostStride * (1 + threadIdx.x) + 1];
  for (int o = 32; o > 0; o >>= 1) {
    v += __shfl_xor(v, o);
    g = max(g, (unsigned long long)__shfl_xor(g, o));
  }
  if (threadIdx.x == 0) {
    cost[0] = v;
    cost[1] = g;
  }
}

// runinfo of an entry of a hash other sketches hold too: the members of its
// run the pairs kernel reads for it, ents[first, first + count) -- when the
// run is in row order, the members after the entry (count = g - 1 - rank,
// 0 for the last: nothing to read), otherwise the whole run (count = g; the
// kernel skips the entry's own row).  0: a hash no other sketch holds.
__device__ __forceinline__ uint64_t run_reads(uint64_t first, uint32_t count) {
  return count ? first | ((uint64_t)count << 32) : 0ull;
}

// Runs of equal keys, one thread per sorted entry p (every lane busy: the
// run pass was thread-per-run before, with ~4 of 5 lanes idle at the
// non-starts and its 8-byte runinfo stores issued by one lane per run).
// A wave covers 64 consecutive entries; the ballot of "p starts a run" and
// of "p + 1 starts a run" give every lane its run [start, end) from bit
// scans; a run that begins before the wave or ends after it is extended by
// one lane walking the sorted keys (runs are a few entries; longer than
// max_run sets *overflow and the host uses the gate kernel).  Each entry then
//   ents[p] = its (row << kbits | k), and
//   runinfo[row, k] = start | g << 32 (g >= 2) or 0 (a hash no other
//   sketch holds; every evaluated row's entries are written, so runinfo needs
//   no clearing).
// When the fill wrote the entries in row-major order (rows_ordered: every
// build but the row-range one, whose workgroups append), the stable sort
// keeps each run in row order: the entry's rank p - start goes into runinfo
// as run_reads' count, and the pairs kernel reads only the members after it.
// Every entry adds the member reads the pairs kernel will make for it (the
// members after it in a sorted run, else all g) to *cost.
// A run of equal keys whose members do not all carry the start's low hash
// word (two hashes with the same top bits: rare) marks its start in the
// `mixed` bitset; index_mixed_kernel then sorts it and writes its sub-runs.
__device__ __forceinline__ uint32_t run_start_back(const uint32_t* __restrict__ keys, uint64_t p, uint32_t key,
                                                   uint32_t max_run) {
  // first position of the run holding p (bounded: a longer run overflows anyway)
  uint64_t q = p;
  while (q > 0 && keys[q - 1] == key && p - q <= max_run) --q;
  return (uint32_t)q;
}

__global__ __launch_bounds__(256) void index_runs_kernel(const uint32_t* __restrict__ keys,
                                                         const uint64_t* __restrict__ vals, uint64_t total,
                                                         uint32_t stride, uint32_t kbits, uint32_t max_run,
                                                         uint64_t* __restrict__ runinfo, uint32_t* __restrict__ ents,
                                                         uint32_t* __restrict__ mixed, uint32_t* __restrict__ overflow,
                                                         uint32_t rows_ordered, unsigned long long* __restrict__ cost) {
  const uint32_t kmask = (1u << kbits) - 1u;
  const uint32_t lane = threadIdx.x & 63;
  unsigned long long reads = 0;
  uint32_t gmax = 0;
  // XCD-aware: the sorted entries are cut into kXcds contiguous chunks and
  // the workgroups of XCD x (blockIdx % kXcds, the dispatcher's round robin)
  // sweep chunk x.  The runinfo stores land on every row wherever the sweep
  // is, but at a given moment an XCD's sweep covers 1/kXcds of the hash range
  // and so a few cache lines per row, which its own L2 can gather into whole
  // lines (the grid-strided sweep spread every XCD over the whole range).
  const uint64_t W = (total + 63) / 64;
  const uint32_t x = blockIdx.x % kXcds;
  const uint64_t wend = W * (x + 1) / kXcds;
  const uint64_t step = (uint64_t)(gridDim.x / kXcds) * 4;
  for (uint64_t wi = W * x / kXcds + (uint64_t)(blockIdx.x / kXcds) * 4 + (threadIdx.x >> 6); wi < wend; wi += step) {
    const uint64_t w0 = wi * 64;
    const uint64_t p = w0 + lane;
    const bool in = p < total;
    const uint32_t key = in ? keys[p] : 0u;
    const uint32_t prev = (in && p > 0) ? keys[p - 1] : ~key;
    const uint32_t next = (p + 1 < total) ? keys[p + 1] : ~key;
    const uint64_t v = in ? vals[p] : 0ull;
    // S: bit t = entry w0 + t starts a run; E: bit t = entry w0 + t ends one
    const uint64_t S = __ballot(in && (p == 0 || prev != key));
    const uint64_t E = __ballot(in && (p + 1 == total || next != key));
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
    const uint64_t sb = S & upto, eb = E & ~(upto >> 1);  // starts at or below / ends at or above the lane
    // the wave's first run may begin before w0, its last may end after w0 + 63
    uint32_t head = (uint32_t)w0, tail_end = 0;
    if (!(S & 1ull)) {  // (uniform) walk back from w0
      uint32_t h = 0;
      if (lane == 0) h = run_start_back(keys, w0, key, max_run);
      head = __builtin_amdgcn_readlane(h, 0);
    }
    const uint32_t last = (uint32_t)(63 - __builtin_clzll(__ballot(in)));  // last lane in range
    if (!((E >> last) & 1ull)) {  // (uniform) walk forward from the wave's end
      uint32_t t = 0;
      if (lane == last) {
        uint64_t q = p + 1;
        while (q < total && keys[q] == key && q - p <= max_run) ++q;
        t = (uint32_t)q;
      }
      tail_end = __builtin_amdgcn_readlane(t, last);
    }
    if (!in) continue;
    const uint32_t start = sb ? (uint32_t)(w0 + 63 - __builtin_clzll(sb)) : head;
    const uint32_t end = eb ? (uint32_t)(w0 + __builtin_ctzll(eb) + 1) : tail_end;
    const uint32_t g = end - start;
    // the start's low hash word: from its lane, or (a run begun before the
    // wave) from memory
    const uint32_t lo = (uint32_t)(v >> 32);
    const uint32_t src = start >= w0 ? (uint32_t)(start - w0) : 0u;
    uint32_t lo0 = __shfl(lo, (int)src);
    if (start < w0) lo0 = (uint32_t)(vals[start] >> 32);
    const uint32_t e = (uint32_t)v;
    ents[p] = e;
    if (g > max_run) {
      atomicOr(overflow, 1u);
      continue;
    }
    const uint32_t after = end - (uint32_t)p - 1u;  // the run's members after this entry
    const uint32_t cnt = g < 2 ? 0u : rows_ordered ? after : g;
    runinfo[(uint64_t)(e >> kbits) * stride + (e & kmask)] = run_reads(rows_ordered ? p + 1 : start, cnt);
    reads += cnt;
    gmax = max(gmax, g);
    if (lo != lo0) atomicOr(&mixed[start >> 5], 1u << (start & 31));
  }
  // (every lane of the wave is here: the sweep's bounds are the wave's)
  cost_add(cost, reads, gmax);
}

// The runs index_runs_kernel marked mixed (equal top bits, more than one
// hash): sorted in place by (low word, entry) by one thread each, split by
// low word, ents and runinfo rewritten for their members.  One thread per
// bitset word.
constexpr uint32_t kMixedRegs = 16;
__global__ __launch_bounds__(256) void index_mixed_kernel(const uint32_t* __restrict__ keys,
                                                          uint64_t* __restrict__ vals, uint64_t total,
                                                          uint32_t stride, uint32_t kbits,
                                                          const uint32_t* __restrict__ mixed,
                                                          uint64_t* __restrict__ runinfo,
                                                          uint32_t* __restrict__ ents) {
  const uint32_t kmask = (1u << kbits) - 1u;
  const uint64_t nw = (total + 31) / 32;
  for (uint64_t wi = (uint64_t)blockIdx.x * 256 + threadIdx.x; wi < nw; wi += (uint64_t)gridDim.x * 256) {
    uint32_t m = mixed[wi];
    while (m) {
      const uint64_t p = wi * 32 + (uint64_t)__builtin_ctz(m);
      m &= m - 1;
      const uint32_t key = keys[p];
      uint64_t e = p + 1;
      while (e < total && keys[e] == key) ++e;
      if (e - p <= kMixedRegs) {  // sort by (low word, entry) in registers
        uint64_t r[kMixedRegs];
#pragma unroll
        for (uint32_t q = 0; q < kMixedRegs; ++q) r[q] = p + q < e ? vals[p + q] : ~0ull;
#pragma unroll
        for (uint32_t q = 1; q < kMixedRegs; ++q) {
#pragma unroll
          for (uint32_t w = q; w > 0; --w) {
            const uint64_t a = r[w - 1], b = r[w];
            r[w - 1] = a < b ? a : b;
            r[w] = a < b ? b : a;
          }
        }
#pragma unroll
        for (uint32_t q = 0; q < kMixedRegs; ++q)
          if (p + q < e) vals[p + q] = r[q];
      } else {
        for (uint64_t q = p + 1; q < e; ++q) {  // insertion sort in place
          const uint64_t x = vals[q];
          uint64_t w = q;
          while (w > p && vals[w - 1] > x) {
            vals[w] = vals[w - 1];
            --w;
          }
          vals[w] = x;
        }
      }
      for (uint64_t a = p; a < e;) {
        const uint32_t lo = (uint32_t)(vals[a] >> 32);
        uint64_t b = a + 1;
        while (b < e && (uint32_t)(vals[b] >> 32) == lo) ++b;
        // (sorted by (low word, entry): each sub-run is in row order)
        for (uint64_t q = a; q < b; ++q) {
          const uint32_t v = (uint32_t)vals[q];
          ents[q] = v;
          runinfo[(uint64_t)(v >> kbits) * stride + (v & kmask)] = run_reads(q + 1, (uint32_t)(b - q - 1));
        }
        a = b;
      }
    }
  }
}

// Bucketed build, after the sort by bucket (16-bit keys, entry values):
// bstart[b] = first sorted entry of bucket b (bstart[nb] = total), written
// where the bucket changes (one coalesced pass over the keys).
constexpr uint32_t kRowSortedRun = 32;  // longer runs of the bucketed build keep their arrival order
constexpr uint32_t kBucketCap = 3072;    // entries of one bucket grouped in LDS
constexpr uint32_t kBucketSlots = 4096;  // its LDS hash table (load <= 0.75)
static_assert(kSuper % kXcds == 0, "super-bins per XCD");
static_assert(kBucketSlots * sizeof(uint64_t) >= kBucketCap * sizeof(uint32_t), "row-order pass: entries in tkey's space");
static_assert(kBucketCap < 4096,
              "bucket table: group start and size packed as 12 + 12 bits");

__global__ __launch_bounds__(256) void bucket_bounds_kernel(const uint16_t* __restrict__ keys, uint64_t total,
                                                            const uint32_t* __restrict__ nbuckets_p,
                                                            uint32_t* __restrict__ bstart) {
  const uint32_t nbuckets = *nbuckets_p;
  // 8 consecutive positions per thread (one 16-byte load of keys)
  for (uint64_t p0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 8; p0 <= total; p0 += (uint64_t)gridDim.x * 256 * 8) {
    uint16_t k[8];
    if (p0 + 8 <= total) {
      const uint4 v = *(const uint4*)(keys + p0);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        k[2 * j] = (uint16_t)w[j];
        k[2 * j + 1] = (uint16_t)(w[j] >> 16);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) k[j] = p0 + j < total ? keys[p0 + j] : 0;
    }
    uint32_t prev = p0 > 0 ? min((uint32_t)keys[p0 - 1], nbuckets) : 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t p = p0 + j;
      if (p > total) break;
      const uint32_t cur = p < total ? min((uint32_t)k[j], nbuckets) : nbuckets;
      const uint32_t first = p > 0 ? prev + 1u : 0u;
      for (uint32_t bk = first; bk <= cur; ++bk) bstart[bk] = (uint32_t)p;
      prev = cur;
    }
  }
}

// One workgroup per bucket.  Each entry reads its hash from its sketch row
// (buckets are ranges of hash values, swept in order by the workgroups of
// one XCD, so every row is read forward and its runinfo written forward, a
// few lines at a time, which the XCD's L2 gathers), and equal hashes meet in
// an LDS hash table: one atomicCAS per entry (2^64 - 1 has a slot of its own,
// the empty marker being that value), a second atomic gives the entry its
// rank among equal hashes, a scan over the table gives every hash its
// group's start, and every entry writes its ents word at start + rank and
// its runinfo slot (group start and size g >= 2, or 0) as index_runs_kernel
// does.  A bucket over kBucketCap entries sets flags[3] (the host rebuilds
// with the full sort).
template <int kBucketThreads>
__global__ __launch_bounds__(kBucketThreads) void index_bucket_kernel(
    const uint32_t* __restrict__ sorted, const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ nbuckets_p,
    uint64_t total, const uint64_t* __restrict__ sk, uint32_t stride, uint32_t kbits,
    uint32_t max_run, uint64_t* __restrict__ runinfo, uint32_t* __restrict__ ents, uint32_t ents16,
    uint32_t* __restrict__ flags, unsigned long long* __restrict__ cost) {
  __shared__ uint64_t tkey[kBucketSlots];
  __shared__ uint32_t tcnt[kBucketSlots + 1];  // group size; after the scan start << 12 | size
  constexpr uint32_t kBucketPer = kBucketCap / kBucketThreads;
  static_assert(kBucketCap % kBucketThreads == 0 && kBucketSlots % kBucketThreads == 0, "bucket table");
  __shared__ uint32_t wsum[kBucketThreads / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t kmask = (1u << kbits) - 1u;
  constexpr uint64_t none = ~0ull;
  constexpr uint32_t smask = kBucketSlots - 1u;
  // XCD-aware: the workgroups of XCD x (blockIdx % kXcds) take the x-th
  // contiguous range of buckets, in order (the grid is a bound on the
  // buckets, whose count the device computed)
  const uint32_t nbuckets = *nbuckets_p;
  const uint32_t per_xcd = (nbuckets + kXcds - 1) / kXcds;
  if (blockIdx.x / kXcds >= per_xcd) return;
  const uint32_t bk = (blockIdx.x % kXcds) * per_xcd + blockIdx.x / kXcds;
  if (bk >= nbuckets) return;
  const uint32_t lo = bstart[bk], hi = bstart[bk + 1], n = hi - lo;
  if (lo > hi || hi > total) {  // unsorted keys: never read through
    if (tid == 0) atomicOr(&flags[3], 2u);
    return;
  }
  if (n == 0) return;
  if (n == 1) {  // a hash no other entry shares
    if (tid == 0) {
      const uint32_t e = sorted[lo];
      if (ents16) ((uint16_t*)ents)[lo] = (uint16_t)(e >> kbits);
      else ents[lo] = e;
      runinfo[(uint64_t)(e >> kbits) * stride + (e & kmask)] = 0ull;
    }
    return;
  }
  if (n > kBucketCap) {
    if (tid == 0) atomicOr(&flags[3], 1u);
    return;
  }
  for (uint32_t x = tid; x <= kBucketSlots; x += kBucketThreads) {
    if (x < kBucketSlots) tkey[x] = none;
    tcnt[x] = 0u;
  }
  __syncthreads();
  // the entries, then their hashes, all loads in flight before the first
  // atomic (one dependent pair of loads per entry at a time left the
  // workgroup waiting on memory latency)
  uint32_t slot[kBucketPer], rank[kBucketPer], ent[kBucketPer];
  uint64_t hv[kBucketPer];
#pragma unroll
  for (uint32_t r = 0; r < kBucketPer; ++r) {
    const uint32_t q = tid + r * kBucketThreads;
    ent[r] = q < n ? sorted[lo + q] : 0u;
  }
#pragma unroll
  for (uint32_t r = 0; r < kBucketPer; ++r) {
    const uint32_t q = tid + r * kBucketThreads;
    const uint32_t e = ent[r];
    hv[r] = q < n ? sk[(uint64_t)(e >> kbits) * stride + (e & kmask)] : 0ull;
  }
#pragma unroll
  for (uint32_t r = 0; r < kBucketPer; ++r) {
    const uint32_t q = tid + r * kBucketThreads;
    slot[r] = 0u;
    rank[r] = 0u;
    if (q < n) {
      const uint64_t h = hv[r];
      uint32_t s = kBucketSlots;
      if (h != none) {
        s = (uint32_t)(h ^ (h >> 29)) & smask;
        for (;;) {
          const unsigned long long old =
              atomicCAS((unsigned long long*)&tkey[s], (unsigned long long)none, (unsigned long long)h);
          if (old == none || old == h) break;
          s = (s + 1u) & smask;
        }
      }
      slot[r] = s;
      rank[r] = atomicAdd(&tcnt[s], 1u);
    }
  }
  __syncthreads();
  // exclusive scan of the group sizes in slot order (slot kBucketSlots, the
  // hash 2^64 - 1, last): each thread 16 consecutive slots, then the wave
  // and workgroup totals
  {
    constexpr uint32_t per = kBucketSlots / kBucketThreads;
    const uint32_t s0 = tid * per;
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t x = 0; x < per; ++x) sum += tcnt[s0 + x];
    uint32_t inc = sum;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t run = inc - sum;
    for (uint32_t w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll
    for (uint32_t x = 0; x < per; ++x) {
      const uint32_t g = tcnt[s0 + x];
      tcnt[s0 + x] = (run << 12) | g;
      run += g;
    }
    if (tid == kBucketThreads - 1) tcnt[kBucketSlots] |= run << 12;
  }
  __syncthreads();
  // A group of g <= kRowSortedRun is stored in row order: the entries are
  // laid out in LDS by their arrival rank (in tkey's space, free now), each
  // counts the members of lower row (a hash is in a row at most once), and
  // its runinfo carries that rank, so the pairs kernel reads only the
  // members after it -- the partners j > i (sum g (g - 1) / 2 member reads
  // instead of sum g^2).  Longer groups keep the arrival order (rank flag 0:
  // every member is read and filtered, as the full build's runs are).
  uint32_t* grp = reinterpret_cast<uint32_t*>(tkey);
#pragma unroll
  for (uint32_t r = 0; r < kBucketPer; ++r) {
    const uint32_t q = tid + r * kBucketThreads;
    if (q < n) grp[(tcnt[slot[r]] >> 12) + rank[r]] = ent[r];
  }
  __syncthreads();
  uint32_t reads = 0, gmax = 0;  // the pairs kernel's member reads for this thread's entries (index_runs_kernel's *cost)
#pragma unroll
  for (uint32_t r = 0; r < kBucketPer; ++r) {
    const uint32_t q = tid + r * kBucketThreads;
    if (q < n) {
      const uint32_t t = tcnt[slot[r]];
      const uint32_t start = t >> 12, g = t & 0xFFFu;
      const uint32_t e = ent[r];
      uint32_t rk = rank[r];
      bool sorted_run = false;
      if (g >= 2 && g <= kRowSortedRun) {
        const uint32_t row = e >> kbits;
        rk = 0;
        for (uint32_t x = 0; x < g; ++x) rk += (grp[start + x] >> kbits) < row ? 1u : 0u;
        sorted_run = true;
      }
      if (ents16) ((uint16_t*)ents)[lo + start + rk] = (uint16_t)(e >> kbits);
      else ents[lo + start + rk] = e;
      if (g > max_run) {
        atomicOr(&flags[0], 1u);
        continue;
      }
      const uint32_t cnt = g < 2 ? 0u : sorted_run ? g - 1u - rk : g;
      runinfo[(uint64_t)(e >> kbits) * stride + (e & kmask)] =
          run_reads((uint64_t)lo + start + (sorted_run ? rk + 1u : 0u), cnt);
      reads += cnt;
      gmax = max(gmax, g);
    }
  }
  cost_add(cost, reads, gmax);
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
constexpr uint32_t kMemberLoads = 8;  // run members loaded together per step
template <bool E16, uint32_t MAPLOG2>
__global__ __launch_bounds__(kRowThreads) void index_pairs_kernel(IndexLaunch a) {
  // (MAPLOG2: 11, or 13 for an index whose rows read thousands of run
  // members each -- clusters of thousands of near-identical genomes: their
  // partners overflow the 2,048-slot map and every extra pass reads the
  // row's runs again; 64 KB of LDS, 2 workgroups per CU)
  constexpr uint32_t kMapLog2 = MAPLOG2, kMap = 1u << kMapLog2, kMapFull = kMap * 3 / 4;
  __shared__ uint32_t mkey[kMap];  // partner + 1 (0 = empty)
  __shared__ uint32_t mcnt[kMap];
  __shared__ uint32_t fill;
  __shared__ volatile uint32_t over;
  const uint32_t tid = threadIdx.x;
  // XCD-aware rows: the workgroups of XCD x (blockIdx % kXcds) take the x-th
  // contiguous range of rows, in order, so rows near each other share that
  // XCD's L2 (the run members one row reads, a row next to it in the input
  // order often reads too: related genomes sit together in many inputs)
  const uint32_t per_xcd = (a.n_rows + kXcds - 1) / kXcds;
  const uint32_t ri_ = (blockIdx.x % kXcds) * per_xcd + blockIdx.x / kXcds;
  if (ri_ >= a.n_rows) return;
  const uint32_t i = a.row0 + ri_;
  if (i >= a.n) return;
  // (launched right after the build, before the host has seen its flags: a
  // run over the limit or a bucket too large left runinfo incomplete)
  if (a.build_flags && ((a.build_flags[0] | a.build_flags[3]) || (a.cost && *a.cost > a.cost_limit))) return;
  uint32_t jlo, jhi;
  row_columns(i, a.n, a.nb, a.tile_begin, a.tile_end, jlo, jhi);
  const uint32_t la = a.lens[i];
  if (jlo >= jhi || la == 0) return;
  const uint64_t* ri = a.runinfo + (uint64_t)i * a.stride;
  const uint64_t* A = a.sketches + (uint64_t)i * a.stride;
  const uint64_t xa = A[la - 1];
  uint32_t plog2 = 0;
  for (uint32_t p = 0; p < (1u << plog2);) {
    for (uint32_t x = tid; x < kMap; x += kRowThreads) mkey[x] = 0u, mcnt[x] = 0u;
    if (tid == 0) fill = 0u, over = 0u;
    __syncthreads();
    // the next entry's runinfo and up to kMemberLoads members of a run are
    // loaded before the map's atomics (one member load at a time left each
    // thread waiting on L2 latency per member)
    uint64_t info_next = tid < la ? ri[tid] : 0ull;
    for (uint32_t k = tid; k < la; k += kRowThreads) {
      if (over) break;
      const uint64_t info = info_next;
      info_next = k + kRowThreads < la ? ri[k + kRowThreads] : 0ull;
      // the members to read (run_reads): in a run in row order only those
      // after row i's own (j > i)
      const uint32_t cnt = (uint32_t)(info >> 32);
      if (cnt == 0) continue;
      const uint32_t q_first = (uint32_t)info, end = q_first + cnt;
      bool stop = false;
      for (uint32_t q0 = q_first; q0 < end && !stop; q0 += kMemberLoads) {
        uint32_t jv[kMemberLoads];
#pragma unroll
        for (uint32_t u = 0; u < kMemberLoads; ++u) {
          const uint32_t q = q0 + u;
          jv[u] = q < end ? (E16 ? (uint32_t)((const uint16_t*)a.vals)[q] : a.vals[q] >> a.kbits) : jhi;
        }
#pragma unroll
        for (uint32_t u = 0; u < kMemberLoads; ++u) {
          const uint32_t j = jv[u];
          if (stop || j < jlo || j >= jhi) continue;
          if (plog2 && part_of(j, plog2) != p) continue;
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
          if (over) stop = true;
        }
      }
      if (stop) break;
    }
    __syncthreads();
    if (over) {
      if (plog2 < a.max_split_log2) {  // too many partners for one map: split them in twice as many classes
        // part_of takes the top plog2 bits of one hash, so class p at plog2 is
        // classes 2p and 2p + 1 at plog2 + 1: the classes below p were already
        // emitted as classes below 2p, which must not be counted again
        ++plog2;
        p *= 2;
        __syncthreads();
        continue;
      }
      // still too many in one class: the counts would be incomplete, so emit
      // nothing; the host discards this launch's output and runs the gate kernel
      if (tid == 0) atomicOr(a.overflow, 1u);
      return;
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

// GALAHGPU_INDEX_HIST_SAMPLE=0: the coarse histogram over every entry at any size
static bool hist_sampling() {
  const char* e = getenv("GALAHGPU_INDEX_HIST_SAMPLE");
  return !(e && *e == '0');
}

hipError_t index_fill(const IndexBuild& b, hipStream_t st) {
  // (flags [4] u32 and the cost counters after them: one clear)
  hipError_t e = hipMemsetAsync(b.flags, 0, 4 * sizeof(uint32_t) + index_cost_bytes(), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(index_scan_kernel, dim3(1), dim3(kScanThreads), 0, st, b.sketches, b.lens, b.n, b.stride,
                     b.offs, (unsigned long long*)b.info);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const unsigned long long* info = (const unsigned long long*)b.info;
  if (b.bucket) {  // coarse-bin histogram of every entry -> bucket bases (bbase[kCoarse] = buckets)
    e = hipMemsetAsync(b.hist, 0, kCoarse * sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(bucket_hist_kernel, dim3(std::max(1u, std::min<uint32_t>(b.n, 1024))), dim3(256), 0, st,
                       b.sketches, b.lens, b.n, b.stride, info, b.hist, hist_sampling() ? 1u : 0u);
    hipLaunchKernelGGL(bucket_base_kernel, dim3(1), dim3(kBaseThreads), 0, st, b.hist, info, b.bbase);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (!b.bloom) return hipSuccess;
  // row-range index: filter, then the kept entries (their count -> flags[1])
  e = hipMemsetAsync(b.bloom, 0, ((size_t)1 << b.bloom_log2) / 8, st);
  if (e != hipSuccess) return e;
  if (b.r1 > b.r0)
    hipLaunchKernelGGL(bloom_build_kernel, dim3(std::min<uint32_t>(b.r1 - b.r0, 16384)), dim3(256), 0, st,
                       b.sketches, b.lens, b.r0, b.r1, b.stride, b.bloom, b.bloom_log2);
  const dim3 grid(std::max(1u, std::min<uint32_t>(b.n, 4096)));
  if (b.bucket)
    hipLaunchKernelGGL(index_fill_range_kernel<true>, grid, dim3(256), 0, st, b.sketches, b.lens, b.n, b.stride,
                       b.kbits, b.bloom, b.bloom_log2, b.r0, b.r1, info, b.bbase, b.flags + 1, b.keys_in, b.vals_in);
  else
    hipLaunchKernelGGL(index_fill_range_kernel<false>, grid, dim3(256), 0, st, b.sketches, b.lens, b.n, b.stride,
                       b.kbits, b.bloom, b.bloom_log2, b.r0, b.r1, info, nullptr, b.flags + 1, b.keys_in,
                       b.vals_in);
  return hipGetLastError();
}

hipError_t index_build(const IndexBuild& b, uint64_t total, uint32_t sh, uint32_t end_bit, hipStream_t st) {
  if (total == 0) return hipSuccess;
  if (!b.bloom)  // (the row-range index filled its kept entries in index_fill)
    hipLaunchKernelGGL(index_fill_kernel<false>, dim3(std::min<uint32_t>(b.n, 16384)), dim3(256), 0, st,
                       b.sketches, b.lens, b.offs, b.n, b.stride, b.kbits, sh, nullptr, nullptr, b.keys_in,
                       b.vals_in);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t bytes = b.sort_tmp_bytes;
  e = hipcub::DeviceRadixSort::SortPairs(b.sort_tmp, bytes, b.keys_in, b.keys_out, b.vals_in, b.vals_out,
                                         (int)total, 0, (int)end_bit, st);
  if (e != hipSuccess) return e;
  // runinfo needs no clearing: the run pass writes the slot of every entry it
  // sees, which includes every entry of every evaluated row (writing only the
  // g >= 2 slots after a clear of the evaluated rows measured slower: C5 pairs
  // phase 10.35 vs 9.98 ms, profiles/r03_d/runinfo_g2_memset_c5.json)
  e = hipMemsetAsync(b.mixed, 0, ((total + 31) / 32) * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  const uint64_t waves = (total + 63) / 64;
  // a multiple of kXcds workgroups, ~8 per CU-slot of the chip at most
  const uint32_t blocks = (uint32_t)(std::min<uint64_t>(8192, std::max<uint64_t>(1, (waves + 4 * kXcds - 1) /
                                                                                  (4 * kXcds))) * kXcds);
  // the entries of shared hashes land in keys_in (free after the sort)
  hipLaunchKernelGGL(index_runs_kernel, dim3(blocks), dim3(256), 0, st, b.keys_out, b.vals_out, total, b.stride,
                     b.kbits, b.max_run, b.runinfo, b.keys_in, b.mixed, b.flags, b.bloom ? 0u : 1u, b.cost);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint64_t words = (total + 31) / 32;
  hipLaunchKernelGGL(index_mixed_kernel, dim3((uint32_t)std::min<uint64_t>(4096, (words + 255) / 256)), dim3(256), 0,
                     st, b.keys_out, b.vals_out, total, b.stride, b.kbits, b.mixed, b.runinfo, b.keys_in);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(index_cost_sum_kernel, dim3(1), dim3(kCostSlots), 0, st, b.cost);
  return hipGetLastError();
}

size_t index_cost_bytes() { return (size_t)(1 + kCostSlots) * kCostStride * sizeof(unsigned long long); }

static hipError_t index_sort_buckets(const IndexBuild& b, uint64_t total, uint32_t nb_bound, hipStream_t st);

hipError_t index_build_buckets(const IndexBuild& b, uint64_t total, uint32_t nb_bound, hipStream_t st) {
  if (total == 0 || nb_bound == 0) return hipSuccess;
  const uint32_t* nbuckets_d = b.bbase + kCoarse;
  uint32_t* vout = (uint32_t*)b.vals_out;
  if (b.split_cnt && !b.bloom) {  // split build: two placements instead of the fill and the sort
    const dim3 rows((b.n + kXcds - 1) / kXcds * kXcds);
    hipLaunchKernelGGL(split_keys_kernel, rows, dim3(256), 0, st, b.sketches, b.lens, b.n, b.stride,
                       (const unsigned long long*)b.info, b.bbase, (uint16_t*)b.keys_in, b.split_cnt);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t bytes = b.sort_tmp_bytes;
    e = hipcub::DeviceScan::ExclusiveSum(b.sort_tmp, bytes, b.split_cnt, b.split_off, (int)(kSuper * b.n + 1), st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(split_scatter_kernel, rows, dim3(256), 0, st, (const uint16_t*)b.keys_in, b.lens, b.n,
                       b.stride, b.kbits, b.split_cnt, b.split_off, (uint8_t*)b.keys_out, (uint32_t*)b.vals_in);
    // slices per super-bin: ~1.5 LDS chunks each (C5: 16; C3's 39k-entry
    // super-bins: 2 -- 16 slices of 2.4k entries took 0.12 ms there, mostly
    // per-workgroup latency)
    const uint32_t parts = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>(kSuperParts, total / ((uint64_t)kSuper * 3 * kPlaceChunk / 2)));
    hipLaunchKernelGGL(superbin_count_kernel, dim3(kSuper * parts), dim3(256), 0, st, (const uint8_t*)b.keys_out,
                       b.split_off, b.n, parts, b.split_hist);
    hipLaunchKernelGGL(superbin_place_kernel, dim3(kSuper * parts), dim3(kPlaceThreads), 0, st,
                       (const uint8_t*)b.keys_out, (const uint32_t*)b.vals_in, b.split_off, b.n, parts, b.split_hist,
                       b.bstart, vout);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  } else {
    hipError_t e = index_sort_buckets(b, total, nb_bound, st);
    if (e != hipSuccess) return e;
  }
  // the entries land in keys_in (free after the sort), as with the run pass
  const uint32_t per_xcd = (nb_bound + kXcds - 1) / kXcds;
  // 1024 threads per bucket (GALAHGPU_BUCKET_THREADS=256|512: A/B; C5 index_bucket
  // 1.76 ms at 256, 1.74 at 512, 1.63 at 1024)
  const char* bt = getenv("GALAHGPU_BUCKET_THREADS");
  const int threads = bt && *bt ? atoi(bt) : 1024;
  auto go = [&](auto kern, int t) {
    hipLaunchKernelGGL(kern, dim3(per_xcd * kXcds), dim3(t), 0, st, vout, b.bstart, nbuckets_d, total, b.sketches,
                       b.stride, b.kbits, b.max_run, b.runinfo, b.keys_in, index_ents16(b.n) ? 1u : 0u, b.flags,
                       b.cost);
  };
  if (threads == 256) go(index_bucket_kernel<256>, 256);
  else if (threads == 512) go(index_bucket_kernel<512>, 512);
  else go(index_bucket_kernel<1024>, 1024);
  hipError_t e2 = hipGetLastError();
  if (e2 != hipSuccess) return e2;
  hipLaunchKernelGGL(index_cost_sum_kernel, dim3(1), dim3(kCostSlots), 0, st, b.cost);
  return hipGetLastError();
}

// The bucketed build's fill and 16-bit sort (the row-range index, whose
// kept entries are compacted, or GALAHGPU_INDEX_SPLIT=0), then the bucket
// bounds.
static hipError_t index_sort_buckets(const IndexBuild& b, uint64_t total, uint32_t nb_bound, hipStream_t st) {
  const uint32_t* nbuckets_d = b.bbase + kCoarse;
  if (!b.bloom)
    hipLaunchKernelGGL(index_fill_kernel<true>, dim3(std::min<uint32_t>(b.n, 16384)), dim3(256), 0, st, b.sketches,
                       b.lens, nullptr, b.n, b.stride, b.kbits, 0u, (const unsigned long long*)b.info, b.bbase,
                       b.keys_in, b.vals_in);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // bucket ids as keys, entries as values, every key bit sorted (bit 0 up:
  // rocPRIM's merge-sort path, used up to 2^20 items, mis-sorts ranges that
  // begin above bit 0; scripts/sortchk_probe.hip,
  // profiles/r03_g/rocprim_partial_bits_sortchk.txt)
  uint32_t* vin = (uint32_t*)b.vals_in;
  uint32_t* vout = (uint32_t*)b.vals_out;
  size_t bytes = b.sort_tmp_bytes;
  e = hipcub::DeviceRadixSort::SortPairs(b.sort_tmp, bytes, (const uint16_t*)b.keys_in, (uint16_t*)b.keys_out, vin,
                                         vout, (int)total, 0, (int)kBucketKeyBits, st);
  if (e != hipSuccess) return e;
  // (every bucket start is written when the keys are sorted; a bucket whose
  // bounds come out inconsistent is reported, never read through)
  e = hipMemsetAsync(b.bstart, 0xFF, ((size_t)nb_bound + 1) * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(bucket_bounds_kernel, dim3((uint32_t)std::min<uint64_t>(16384, total / 2048 + 1)), dim3(256), 0,
                     st, (const uint16_t*)b.keys_out, total, nbuckets_d, b.bstart);
  return hipGetLastError();
}

size_t index_split_tmp_bytes(uint32_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (int)(kSuper * n + 1));
  return bytes;
}

uint32_t index_bucket_bound(uint64_t entries) {
  return (uint32_t)std::min<uint64_t>(kBucketPad - 1, entries / 1024 + kCoarse);
}

size_t index_sort_tmp_bytes(uint64_t total, uint32_t end_bit) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (const uint64_t*)nullptr, (uint64_t*)nullptr, (int)total, 0, (int)end_bit);
  return bytes;
}

size_t index_bucket_sort_tmp_bytes(uint64_t total) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint16_t*)nullptr, (uint16_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)total, 0,
                                           (int)kBucketKeyBits);
  return bytes;
}

hipError_t launch_index_pairs(const IndexLaunch& a, uint32_t n_rows, hipStream_t st) {
  if (n_rows == 0) return hipSuccess;
  IndexLaunch b = a;
  b.n_rows = n_rows;
  const dim3 grid((n_rows + kXcds - 1) / kXcds * kXcds);
  if (a.ents16) {
    if (a.big_map) hipLaunchKernelGGL((index_pairs_kernel<true, 13>), grid, dim3(kRowThreads), 0, st, b);
    else hipLaunchKernelGGL((index_pairs_kernel<true, 11>), grid, dim3(kRowThreads), 0, st, b);
  } else {
    if (a.big_map) hipLaunchKernelGGL((index_pairs_kernel<false, 13>), grid, dim3(kRowThreads), 0, st, b);
    else hipLaunchKernelGGL((index_pairs_kernel<false, 11>), grid, dim3(kRowThreads), 0, st, b);
  }
  return hipGetLastError();
}

// Passing pairs in (i, j) order on the device (the output of every K2 form
// is an atomic append): key i * n + j, value the pair's position, radix
// sorted over the key's significant bits, then the pairs gathered in that
// order, so the host copies them out as they are (C4's 153k pairs: the host
// radix sort took ~1 ms of a 2.3 ms merge; unpacking sorted keys and values
// on the host, one 64-bit division per pair, ~0.1 ms of C3's 15k).
namespace {
__global__ __launch_bounds__(256) void pair_keys_kernel(const gg_pair* __restrict__ p, uint32_t cnt, uint32_t n,
                                                        uint64_t* __restrict__ keys, uint32_t* __restrict__ idx) {
  for (uint32_t x = blockIdx.x * 256 + threadIdx.x; x < cnt; x += gridDim.x * 256) {
    const gg_pair q = p[x];
    keys[x] = (uint64_t)q.i * n + q.j;
    idx[x] = x;
  }
}

__global__ __launch_bounds__(256) void pair_gather_kernel(const gg_pair* __restrict__ p, uint32_t cnt,
                                                          const uint32_t* __restrict__ idx,
                                                          gg_pair* __restrict__ sorted) {
  for (uint32_t y = blockIdx.x * 256 + threadIdx.x; y < cnt; y += gridDim.x * 256) sorted[y] = p[idx[y]];
}
}  // namespace

uint32_t pair_key_bits(uint32_t n) {
  const uint64_t mx = (uint64_t)n * n;
  uint32_t bits = 1;
  while (bits < 64 && (mx >> bits) != 0) ++bits;
  return bits;
}

size_t pair_sort_tmp_bytes(uint64_t cnt, uint32_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)cnt, 0,
                                           (int)pair_key_bits(n));
  return bytes;
}

hipError_t sort_pairs_device(const gg_pair* d_pairs, uint64_t cnt, uint32_t n, uint64_t* keys, uint64_t* keys_out,
                             uint32_t* idx, uint32_t* idx_out, gg_pair* sorted, void* tmp, size_t tmp_bytes,
                             hipStream_t st) {
  if (cnt == 0) return hipSuccess;
  if (cnt >= (1ull << 31)) return hipErrorInvalidValue;  // (the sort's count is an int)
  const dim3 grid((uint32_t)std::min<uint64_t>(4096, (cnt + 255) / 256));
  hipLaunchKernelGGL(pair_keys_kernel, grid, dim3(256), 0, st, d_pairs, (uint32_t)cnt, n, keys, idx);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  // (bit 0 up: see index_build_buckets on rocPRIM's merge-sort path)
  e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys, keys_out, idx, idx_out, (int)cnt, 0,
                                         (int)pair_key_bits(n), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(pair_gather_kernel, grid, dim3(256), 0, st, d_pairs, (uint32_t)cnt, idx_out, sorted);
  return hipGetLastError();
}

// The bucketed build stores each run member as its 16-bit row when rows fit
// (C3/C5's 10k rows: C5's 10^8 members in 200 MB instead of 400 MB, inside
// the 256 MB MALL that the pairs kernel's member reads then hit).
bool index_ents16(uint32_t n) { return n <= 65536u; }

}  // namespace gg
