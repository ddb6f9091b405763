// Kernel K2, gated-table form (the default pair kernel).
//
// Same contract as pairs.hip (src/finch.rs:53-73: finch's merge-to-first-
// exhaustion, common = |A n B|, total = i + j - common, pass iff
// common >= cmin[total]), organised so that the work per pair is a few
// VALU instructions instead of a merge:
//
//  * Row blocks.  The R (<= 32) rows of a row block share one table, built
//    once per launch by gate_build_kernel into HBM: the block's keys in
//    buckets chosen by a hash of the key's low word (dir = start | count <<
//    16, ~8 entries per bucket; a key shared by several rows appears once
//    per row, buckets unsorted), the row of each entry as a one-bit mask,
//    and a gate: a Bloom filter over the low words.  R * s <= 32768 keys,
//    so at s = 1000 a row block holds 32 rows.
//  * Gate.  pairs_gate_kernel copies the row block's gate into LDS and
//    streams the low words of column sketches (a compact copy made per
//    launch) through it.  For s < 2048: one gate bit in 2^19 bits (64 KiB;
//    one LDS read per column hash; ~6% of an unrelated column's hashes pass
//    at 32k keys) and ~2-key buckets whose directory stays in HBM.  For
//    s >= 2048 ("wide": few rows per block, thousands of hashes per column
//    visit): two gate bits in 2^18 bits (2-5% pass) and ~8-key buckets whose
//    directory (16 KiB) is copied to LDS too.  Passing hashes are queued
//    per wave (LDS ring of low words and positions) and resolved 64 at a
//    time: directory, then the bucket's keys read 8 at a time; only a
//    low-word match reads the column's high word.  The masks of the equal
//    keys are ORed into per-lane byte counters.  One column hash serves all
//    R rows.
//  * Work order.  Work items (row block x column segment) are dealt to
//    blockIdx column-segment-major in runs of 64 per XCD (the host does
//    it: pairs_gate in api.cpp), so the workgroups resident on an XCD
//    stream the same columns through its L2.
//  * Totals.  A pair can pass only if common >= min(cmin[t], t >= min(|A|,
//    |B|)) (the first exhaustion leaves total >= |A| or >= |B|), so the
//    ranks that finch's total needs are computed (binary searches) only for
//    those rows -- in practice for related pairs only.
//
// Bound: VALU issue of the gate loop (~10 instructions per 64 column
// hashes, shared by R rows) and L2 bandwidth for the streamed columns.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "device_util.hpp"
#include "gg_internal.hpp"

namespace gg {
namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kRing = 128;      // per-wave queue (<= 63 + 64 pending)
constexpr int kRounds = 8;           // 64-hash rounds per register chunk
constexpr uint32_t kMetaBytes = 512;

struct GateMeta {
  uint64_t last[kGateRowsMax];  // largest hash of each row
  uint32_t len[kGateRowsMax];
  uint32_t nrows;
};
static_assert(sizeof(GateMeta) <= kMetaBytes, "meta");

// One row block's table in HBM: meta | gate[bm_words] | dir[nb] | keys[cap] | masks[cap]
struct BlockView {
  const GateMeta* meta;
  uint32_t* dir;
  uint32_t* bm;
  uint64_t* keys;
  uint32_t* masks;
};

__device__ __forceinline__ BlockView block_view(const uint8_t* base, const GateParams& p) {
  uint8_t* b = const_cast<uint8_t*>(base);
  BlockView v;
  v.meta = reinterpret_cast<const GateMeta*>(b);
  v.bm = reinterpret_cast<uint32_t*>(b + kMetaBytes);
  v.dir = v.bm + p.bm_words;
  v.keys = reinterpret_cast<uint64_t*>(v.dir + p.nb);
  v.masks = reinterpret_cast<uint32_t*>(v.keys + p.cap);
  return v;
}

// Bucket of a key from its low word (multiplicative hash, independent of
// the gate bits).
__device__ __forceinline__ uint32_t bucket_lo(uint32_t lo, uint32_t nb_log2) {
  return (lo * 0x9E3779B1u) >> (32 - nb_log2);
}
// The two gate bits of a key: a two-hash Bloom filter over the low word.
__device__ __forceinline__ uint32_t gate_bit1(uint32_t lo, uint32_t bm_log2) { return lo & ((1u << bm_log2) - 1); }
__device__ __forceinline__ uint32_t gate_bit2(uint32_t lo, uint32_t bm_log2) {
  return (lo * 0x85EBCA6Bu) >> (32 - bm_log2);
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

// ---------------------------------------------------------------------------
// Table build: one workgroup per row block.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void gate_build_kernel(GateBuildLaunch a) {
  extern __shared__ __align__(16) uint32_t sm[];
  const GateParams p = a.p;
  uint32_t* cnt = sm;          // [nb]: counts, then bucket starts, then bucket ends
  uint32_t* bm = sm + p.nb;    // [bm_words]
  __shared__ GateMeta meta;
  __shared__ uint32_t pre[kGateRowsMax + 1];
  __shared__ uint32_t wsum[kWaves];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t blk = blockIdx.x;
  const uint32_t I = a.tile_row0 + blk / p.G, rb = blk % p.G;
  const uint32_t row0 = I * GG_PAIR_TILE + rb * p.R;
  const uint32_t row_end = min(min(row0 + p.R, (I + 1) * GG_PAIR_TILE), a.n);
  BlockView v = block_view(a.tables + (size_t)blk * p.block_bytes, p);

  const uint32_t nrows = row0 < row_end ? row_end - row0 : 0;
  if (tid < kGateRowsMax) {  // one thread per row: the loads overlap
    uint32_t l = 0;
    uint64_t last = 0;
    if (tid < nrows) {
      l = a.lens[row0 + tid];
      if (l) last = a.sketches[(uint64_t)(row0 + tid) * a.stride + l - 1];
    }
    meta.len[tid] = l;
    meta.last[tid] = last;
  }
  for (uint32_t i = tid; i < p.nb + p.bm_words; i += kThreads) sm[i] = 0;
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (uint32_t r = 0; r < kGateRowsMax; ++r) {
      pre[r] = acc;
      acc += meta.len[r];
    }
    pre[kGateRowsMax] = acc;
    meta.nrows = nrows;
  }
  __syncthreads();
  const uint32_t E = pre[kGateRowsMax];
  auto entry = [&](uint32_t e, uint32_t& r) {
    r = 0;
    for (uint32_t x = 1; x < p.R; ++x) r += (e >= pre[x]) ? 1u : 0u;
    return a.sketches[(uint64_t)(row0 + r) * a.stride + (e - pre[r])];
  };

  // pass 1: bucket counts and the gate bitmap
  for (uint32_t e = tid; e < E; e += kThreads) {
    uint32_t r;
    const uint64_t key = entry(e, r);
    const uint32_t lo = (uint32_t)key;
    atomicAdd(&cnt[bucket_lo(lo, p.nb_log2)], 1u);
    const uint32_t b1 = gate_bit1(lo, p.bm_log2), b2 = gate_bit2(lo, p.bm_log2);
    atomicOr(&bm[b1 >> 5], 1u << (b1 & 31));
    if (p.wide) atomicOr(&bm[b2 >> 5], 1u << (b2 & 31));
  }
  __syncthreads();
  // exclusive scan of the counts -> bucket starts
  {
    const uint32_t per = (p.nb + kThreads - 1) / kThreads;
    const uint32_t b0 = min(tid * per, p.nb), b1 = min(b0 + per, p.nb);
    uint32_t s = 0;
    for (uint32_t b = b0; b < b1; ++b) s += cnt[b];
    uint32_t inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t run = inc - s;
    for (uint32_t w = 0; w < wave; ++w) run += wsum[w];
    for (uint32_t b = b0; b < b1; ++b) {
      const uint32_t c = cnt[b];
      cnt[b] = run;
      run += c;
    }
  }
  __syncthreads();
  // pass 2: scatter (afterwards cnt[b] = end of bucket b = start of b + 1)
  for (uint32_t e = tid; e < E; e += kThreads) {
    uint32_t r;
    const uint64_t key = entry(e, r);
    const uint32_t slot = atomicAdd(&cnt[bucket_lo((uint32_t)key, p.nb_log2)], 1u);
    v.keys[slot] = key;
    v.masks[slot] = 1u << r;
  }
  __syncthreads();
  // buckets stay unsorted: a lookup compares every entry of its bucket
  // (~8 at R * s = 32k keys in 4k buckets) and ORs the masks of equal keys
  for (uint32_t b = tid; b < p.nb; b += kThreads) {
    const uint32_t s0 = b ? cnt[b - 1] : 0u, s1 = cnt[b];
    v.dir[b] = s0 | ((s1 - s0) << 16);
  }
  for (uint32_t i = tid; i < p.bm_words; i += kThreads) v.bm[i] = bm[i];
  if (tid == 0) *const_cast<GateMeta*>(v.meta) = meta;
}

// Low 32 bits of every hash of rows [row0, n): the gate reads 4 B per
// column hash instead of 8.
__global__ __launch_bounds__(256) void gate_lo32_kernel(const uint64_t* __restrict__ sk, uint32_t* __restrict__ lo,
                                                        uint64_t begin, uint64_t end) {
  for (uint64_t i = begin + (uint64_t)blockIdx.x * 256 + threadIdx.x; i < end; i += (uint64_t)gridDim.x * 256)
    lo[i] = (uint32_t)sk[i];
}

// ---------------------------------------------------------------------------
// Column streaming: one workgroup per (row block, column segment).
// ---------------------------------------------------------------------------
template <bool WIDE>
__global__ __launch_bounds__(kThreads, 8) void pairs_gate_kernel(GateLaunch a) {
  extern __shared__ __align__(16) uint32_t sm[];
  const GateParams p = a.p;
  uint32_t* bm = sm;                                 // [bm_words] gate
  uint32_t* dir = bm + p.bm_words;                   // WIDE: [nb] bucket directory
  uint32_t* rings_lo = dir + (WIDE ? p.nb : 0u);     // [kWaves][kRing] queued low words
  uint16_t* rings_e = reinterpret_cast<uint16_t*>(rings_lo + kWaves * kRing);  // their column positions
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // work item of this workgroup (the host orders items so that the
  // workgroups resident on one XCD share a column segment)
  const PairSeg sg = a.items[blockIdx.x];
  if (sg.I == UINT32_MAX) return;
  const uint32_t rb = sg.pad;
  const uint32_t row0 = sg.I * GG_PAIR_TILE + rb * p.R;
  if (row0 >= a.n || rb * p.R >= GG_PAIR_TILE) return;
  const uint32_t c0 = max(sg.J0 * GG_PAIR_TILE, row0 + 1);
  const uint32_t c1 = min(sg.J1 * GG_PAIR_TILE, a.n);
  if (c0 >= c1) return;
  const uint32_t blk = (sg.I - a.tile_row0) * p.G + rb;
  const BlockView v = block_view(a.tables + (size_t)blk * p.block_bytes, p);

  {
    // gate and directory are adjacent in both places
    const uint4* src = reinterpret_cast<const uint4*>(v.bm);
    uint4* dst = reinterpret_cast<uint4*>(bm);
    for (uint32_t i = tid; i < (p.bm_words + (WIDE ? p.nb : 0u)) / 4; i += kThreads) dst[i] = src[i];
  }
  const GateMeta& gm = *v.meta;
  const uint32_t nrows = gm.nrows;
  // lane r < R holds row r
  const uint32_t la = lane < kGateRowsMax ? gm.len[lane] : 0u;
  const uint64_t xa = lane < kGateRowsMax ? gm.last[lane] : 0ull;
  const uint32_t nacc = (p.R + 3) / 4;
  uint32_t* ring_lo = rings_lo + wave * kRing;
  uint16_t* ring_e = rings_e + wave * kRing;
  __syncthreads();

  for (uint32_t j = c0 + wave; j < c1; j += kWaves) {
    const uint32_t lb = uni32(a.lens[j]);
    const uint64_t* B = a.sketches + (uint64_t)j * a.stride;
    uint32_t head = 0, tail = 0;  // wave-uniform
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // byte counters, rows 4q..4q+3
    bool hits = false;
    const uint32_t* Bw = reinterpret_cast<const uint32_t*>(B);  // [2e] low, [2e+1] high word
    // table walk for up to 64 queued hashes: directory in LDS, one read of
    // the bucket's keys; the column's high word only for low-word matches
    auto drain = [&](uint32_t count) {
      uint32_t m = 0;
      if (lane < count) {
        const uint32_t q = (head + lane) & (kRing - 1);
        const uint32_t lo = ring_lo[q];
        const uint32_t d = (WIDE ? dir : v.dir)[bucket_lo(lo, p.nb_log2)];
        const uint32_t st = d & 0xFFFFu, n = d >> 16;
        // the bucket's keys, 8 loads in flight at a time; low-word matches
        // collected as a bit set
        const uint32_t* kw = reinterpret_cast<const uint32_t*>(v.keys + st);
        uint32_t hi = 0;
        bool have_hi = false;
        for (uint32_t k0 = 0; k0 < n; k0 += 8) {
          uint32_t kl[8];
#pragma unroll
          for (uint32_t t = 0; t < 8; ++t) kl[t] = kw[2 * min(k0 + t, n - 1)];
          uint32_t match = 0;
#pragma unroll
          for (uint32_t t = 0; t < 8; ++t) match |= (kl[t] == lo && k0 + t < n) ? (1u << t) : 0u;
          while (match) {
            const uint32_t k = k0 + __builtin_ctz(match);
            match &= match - 1;
            if (!have_hi) {
              hi = Bw[2 * (uint32_t)ring_e[q] + 1];
              have_hi = true;
            }
            if (kw[2 * k + 1] == hi) m |= v.masks[st + k];
          }
        }
      }
      if (__ballot(m != 0)) {
        hits = true;
#pragma unroll
        for (uint32_t c = 0; c < 8; ++c)
          if (c < nacc) acc[c] += spread4(m >> (4 * c));
      }
      head += count;
    };

    // the gate needs the low 32 bits of each hash only
    const uint32_t* B32 = a.lo32 + (uint64_t)j * a.stride;
    // One chunk of kRounds x 64 column hashes: all loads, then all bitmap
    // reads, then the tests, so the latencies overlap.  TAIL: the chunk
    // reaches past the column end; those lanes re-read its last hash and
    // are masked out of the hit test (branch-free).
    auto chunk = [&](uint32_t cb, auto tail_tag) {
      constexpr bool TAIL = decltype(tail_tag)::value;
      uint32_t lo[kRounds], w1[kRounds], w2[kRounds];
      const uint32_t* src = B32 + cb + lane;
#pragma unroll
      for (int t = 0; t < kRounds; ++t)
        lo[t] = TAIL ? B32[min(cb + t * 64 + lane, lb - 1)] : src[64 * t];
#pragma unroll
      for (int t = 0; t < kRounds; ++t) {
        w1[t] = bm[gate_bit1(lo[t], p.bm_log2) >> 5];
        if (WIDE) w2[t] = bm[gate_bit2(lo[t], p.bm_log2) >> 5];
      }
#pragma unroll
      for (int t = 0; t < kRounds; ++t) {
        if (TAIL && cb + t * 64 >= lb) break;  // wave-uniform
        const uint32_t e = cb + t * 64 + lane;
        uint32_t hit = (w1[t] >> (lo[t] & 31)) & 1u;
        if (WIDE) hit &= w2[t] >> (gate_bit2(lo[t], p.bm_log2) & 31);
        if (TAIL) hit &= (e < lb) ? 1u : 0u;
        const uint64_t mm = __ballot(hit);
        if (mm) {
          if (hit) {
            const uint32_t q = (tail + lanes_below(mm)) & (kRing - 1);
            ring_lo[q] = lo[t];
            ring_e[q] = (uint16_t)e;
          }
          tail += __popcll(mm);
          if (tail - head >= 64) drain(64);
        }
      }
    };
    uint32_t cb = 0;
    for (; cb + 64 * kRounds <= lb; cb += 64 * kRounds) chunk(cb, std::false_type{});
    if (cb < lb) chunk(cb, std::true_type{});
    while (tail != head) drain(min(64u, tail - head));

    if (!hits && !a.zero_passes) continue;  // no row shares a hash with column j
    // lane r < R: common of pair (row0 + r, j)
    uint32_t common = 0;
    if (hits) {
#pragma unroll
      for (uint32_t c = 0; c < 8; ++c) {
        if (c >= nacc) break;
        const uint32_t s02 = wave_sum(acc[c] & 0x00FF00FFu);         // rows 4c, 4c+2
        const uint32_t s13 = wave_sum((acc[c] >> 8) & 0x00FF00FFu);  // rows 4c+1, 4c+3
        if ((lane >> 2) == c) {
          const uint32_t w = lane & 3;
          common = (((w & 1) ? s13 : s02) >> (16 * (w >> 1))) & 0xFFFFu;
        }
      }
    }
    const uint32_t i = row0 + lane;
    bool cand = false;
    if (lane < nrows && j > i) {
      if (la == 0 || lb == 0) cand = a.cmin[0] == 0;  // finch: common 0, total 0
      else cand = common >= a.sufmin[min(la, lb)];
    }
    if (!__ballot(cand)) continue;
    bool pass = false;
    uint32_t total = 0;
    if (cand) {
      if (la == 0 || lb == 0) {
        common = 0;
        pass = true;
      } else {
        const uint64_t lastB = B[lb - 1];
        if (xa <= lastB) total = la + count_le(B, lb, xa) - common;
        else total = count_le(a.sketches + (uint64_t)i * a.stride, la, lastB) + lb - common;
        pass = total <= a.tmax && common >= a.cmin[total];
      }
    }
    const uint64_t mk = __ballot(pass);
    if (mk) {
      const uint32_t first = __builtin_ctzll(mk);
      unsigned long long obase = 0;
      if (lane == first) obase = atomicAdd(a.count, (unsigned long long)__popcll(mk));
      obase = __shfl(obase, first);
      if (pass) {
        const unsigned long long slot = obase + lanes_below(mk);
        if (slot < a.out_cap) a.out[slot] = gg_pair{i, j, common, total};
      }
    }
  }
}

uint32_t pow2_at_least(uint64_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace

GateParams gate_params(uint32_t s) {
  GateParams g;
  g.R = std::min<uint32_t>(kGateRowsMax, std::max<uint32_t>(1, kGateCap / std::max<uint32_t>(s, 1)));
  g.G = (GG_PAIR_TILE + g.R - 1) / g.R;
  g.cap = g.R * s;
  // Wide sketches (few rows per block, s hashes per column visit): a
  // two-hash gate in 2^18 bits and the directory (~8 keys per bucket) in
  // LDS, so gate misses are rarer and a table walk is one L2 round trip.
  // Small sketches: a one-bit gate in 2^19 bits (cheaper per hash) and a
  // directory of ~2-key buckets in HBM.
  // GALAHGPU_GATE_WIDE_MIN_S: sketch size from which the wide regime is
  // used (default 2048; for A/B runs only, results do not depend on it)
  static const uint32_t wide_min = [] {
    const char* e = getenv("GALAHGPU_GATE_WIDE_MIN_S");
    return e && *e ? (uint32_t)strtoul(e, nullptr, 10) : 2048u;
  }();
  g.wide = s >= wide_min;
  if (g.wide) {
    // Keys per wide row block: up to 65535 (the 16-bit bucket starts), twice
    // kGateCap.  More keys = more rows per block = fewer passes over each
    // column's hashes, with a gate (2^19 bits) and directory twice as large
    // (C5, s = 10000: R = 6 instead of 3, pairs 193.8 -> 95.5 ms).
    // GALAHGPU_GATE_WIDE_CAP overrides it for A/B runs (results do not
    // depend on it).
    static const uint32_t wide_cap = [] {
      const char* e = getenv("GALAHGPU_GATE_WIDE_CAP");
      const uint32_t v = e && *e ? (uint32_t)strtoul(e, nullptr, 10) : 65535u;
      return std::min<uint32_t>(65535u, std::max<uint32_t>(kGateCap, v));
    }();
    g.R = std::min<uint32_t>(kGateRowsMax, std::max<uint32_t>(1, wide_cap / std::max<uint32_t>(s, 1)));
    g.G = (GG_PAIR_TILE + g.R - 1) / g.R;
    g.cap = g.R * s;
    const uint32_t big = g.cap > kGateCap ? 1u : 0u;
    g.nb = std::min<uint32_t>(4096u << big, std::max<uint32_t>(64, pow2_at_least((g.cap + 7) / 8)));
    g.bm_words = std::min<uint32_t>(1u << (13 + big), std::max<uint32_t>(128, pow2_at_least((uint64_t)g.cap * 8) / 32));
  } else {
    g.nb = std::min<uint32_t>(16384, std::max<uint32_t>(64, pow2_at_least((g.cap + 1) / 2)));
    g.bm_words = std::min<uint32_t>(1u << 14, std::max<uint32_t>(128, pow2_at_least((uint64_t)g.cap * 16) / 32));
  }
  g.nb_log2 = __builtin_ctz(g.nb);
  g.bm_log2 = __builtin_ctz(g.bm_words * 32);
  const uint64_t bytes = kMetaBytes + 4ull * g.nb + 4ull * g.bm_words + 12ull * g.cap;
  g.block_bytes = (bytes + 255) & ~255ull;
  return g;
}

hipError_t launch_gate_build(const GateBuildLaunch& a, hipStream_t st) {
  if (a.n_blocks == 0) return hipSuccess;
  {
    const uint64_t begin = (uint64_t)a.tile_row0 * GG_PAIR_TILE * a.stride, end = (uint64_t)a.n * a.stride;
    if (begin < end) {
      const uint64_t blocks = std::min<uint64_t>(8192, (end - begin + 255) / 256);
      hipLaunchKernelGGL(gate_lo32_kernel, dim3((uint32_t)blocks), dim3(256), 0, st, a.sketches, a.lo32, begin, end);
    }
  }
  const size_t lds = 4ull * (a.p.nb + a.p.bm_words);
  hipError_t e = hipFuncSetAttribute((const void*)gate_build_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(gate_build_kernel, dim3(a.n_blocks), dim3(kThreads), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_pairs_gate(const GateLaunch& a, hipStream_t st) {
  if (a.n_items == 0) return hipSuccess;
  const size_t lds = 4ull * (a.p.bm_words + (a.p.wide ? a.p.nb : 0u)) + 6ull * kWaves * kRing;
  const void* fn = a.p.wide ? (const void*)pairs_gate_kernel<true> : (const void*)pairs_gate_kernel<false>;
  hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  if (a.p.wide) hipLaunchKernelGGL(pairs_gate_kernel<true>, dim3(a.n_items), dim3(kThreads), lds, st, a);
  else hipLaunchKernelGGL(pairs_gate_kernel<false>, dim3(a.n_items), dim3(kThreads), lds, st, a);
  return hipGetLastError();
}

}  // namespace gg
