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
#include "device_util.hpp"
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

// ---------------------------------------------------------------------------
// K2 table kernel.
//
// A workgroup owns R consecutive row sketches (a "row block") and a run of
// up to kSegTiles column tiles of the same tile row.  It builds, in LDS, a
// value-bucketed table of the row block's hashes: keys sorted inside each
// bucket, an R-bit row mask per entry (a hash shared by several rows is
// several entries).  Its 16 waves then stream column sketches: each lane
// looks one column hash up (bucket directory read + short sorted scan), and
// the hit masks are accumulated per row in byte counters.  For a column
// this replaces R sorted merges of ~2s steps by s table lookups.
//
// total = i + j - common at first exhaustion of finch's merge equals
//   |A| + rank_B(last A) - common        if last A <= last B
//   rank_A(last B) + |B| - common        otherwise
// rank_B comes from a ballot per streamed round; rank_A from a 64-way
// search of the row sketch.  Pass test: common >= cmin[total].
//
// Blocks of one segment are placed 8 apart in blockIdx so they share an XCD
// (round-robin dispatch) and stream the same columns through one L2.
// ---------------------------------------------------------------------------
constexpr int kTableThreads = 1024;
constexpr int kTableWaves = kTableThreads / 64;
constexpr uint32_t kNB = 8192;  // buckets
constexpr uint32_t kNG = kNB / 64;  // bucket groups (rank_A prefix samples)
constexpr uint32_t kKeyCap = 8192;
constexpr uint32_t kEPT = kKeyCap / kTableThreads;  // entries per thread in the build
constexpr int kChunk = 16;                          // column rounds held in registers
constexpr int kGroup = 8;                           // rounds whose LDS probes are issued together

// LDS layout (dynamic, base 16-B aligned):
//   meta 256 B | ent u64[cap+2] (build: kNB u32 counters) | masks u8[cap+8]
//   | dir u32[kNB] (start | count << 16) | samp u16[(kNG+1)*8]
// Packed mode (row block max key < 2^56): ent = key << 8 | row mask.
// Otherwise ent = key and masks[] holds the row mask.
__host__ __device__ constexpr size_t tk_ent(uint32_t cap) {
  return ((size_t)cap + 2) * 8 > (size_t)kNB * 4 ? ((size_t)cap + 2) * 8 : (size_t)kNB * 4;
}
__host__ __device__ constexpr size_t tk_masks(uint32_t cap) { return ((size_t)cap + 8 + 15) & ~(size_t)15; }
__host__ __device__ constexpr size_t tk_dir() { return (size_t)kNB * 4; }
__host__ __device__ constexpr size_t tk_samp() { return (((size_t)kNG + 1) * 8 * 2 + 15) & ~(size_t)15; }
constexpr uint32_t kRing = 128;  // per-wave ring of column hashes needing a full bucket walk
__host__ __device__ constexpr size_t tk_ring() { return (size_t)kTableWaves * kRing * 8; }
__host__ __device__ constexpr size_t table_lds_bytes(uint32_t cap) {
  return 256 + tk_ent(cap) + tk_masks(cap) + tk_dir() + tk_samp() + tk_ring();
}

struct TableMeta {
  uint64_t last[8];     // last (largest) hash of each row
  uint32_t len[8];
  uint32_t pre[9];      // prefix of len
  uint64_t maxkey;
  uint32_t shift_r;     // top32(b) = (b >> shift_r) << shift_l
  uint32_t shift_l;
  uint32_t scale;
  uint32_t nrows;
  uint32_t packed;
};

// Lane r < R receives #{ e < lb : B[e] <= x_r } (B ascending, lb > 0).
// Level 1: 64 samples shared by all rows; level 2: 64/R lanes per row scan
// the remaining window.  x[] and B are wave-uniform.
template <int R>
__device__ __forceinline__ uint32_t rank_rows_B(const uint64_t* __restrict__ B, uint32_t lb,
                                               const uint64_t* __restrict__ meta_last,
                                               const uint64_t (&x)[R], uint32_t lane) {
  const uint32_t step = (lb + 63) / 64;
  const uint32_t e = (lane + 1) * step - 1;  // sample index; past the end for some lanes
  const bool ok = e < lb;
  const uint64_t sv = ok ? B[e] : 0;
  uint32_t cvec = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t c = __popcll(__ballot(ok && sv <= x[r]));
    if (lane == (uint32_t)r) cvec = c;
  }
  constexpr uint32_t LPR = 64 / R;  // lanes per row
  const uint32_t my_row = lane / LPR, sub = lane % LPR;
  const uint32_t c_my = __shfl(cvec, my_row);
  const uint64_t x_my = meta_last[my_row];
  const uint32_t w0 = c_my * step;
  const uint32_t w1 = min(lb, w0 + step - 1);
  uint32_t cnt = 0;
  for (uint32_t i = w0 + sub; i < w1; i += LPR) cnt += (B[i] <= x_my) ? 1u : 0u;
#pragma unroll
  for (uint32_t o = LPR / 2; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
  // lane r (r < R) reads the group total of row r (group leader lane r*LPR)
  const uint32_t tot = w0 + cnt;
  return __shfl(tot, (lane % R) * LPR);
}


// Per-row byte counters (acc_lo: rows 0-3, acc_hi: rows 4-7) summed over
// the wave; lane r < 8 receives row r's total.
__device__ __forceinline__ uint32_t row_totals(uint32_t acc_lo, uint32_t acc_hi, uint32_t lane) {
  const uint32_t s0 = wave_sum(acc_lo & 0x00FF00FFu);         // rows 0, 2
  const uint32_t s1 = wave_sum((acc_lo >> 8) & 0x00FF00FFu);  // rows 1, 3
  const uint32_t s2 = wave_sum(acc_hi & 0x00FF00FFu);         // rows 4, 6
  const uint32_t s3 = wave_sum((acc_hi >> 8) & 0x00FF00FFu);  // rows 5, 7
  const uint32_t which = (lane & 1) + 2 * ((lane >> 2) & 1);
  const uint32_t sv = which == 0 ? s0 : which == 1 ? s1 : which == 2 ? s2 : s3;
  return (sv >> (16 * ((lane >> 1) & 1))) & 0xFFFFu;
}

// Per-row 16-bit counters for walks over whole buckets (a bucket can hold
// more than 255 entries): c[0] rows 0|2, c[1] rows 1|3, c[2] rows 4|6,
// c[3] rows 5|7, row in the low / high half.
struct RowCount16 {
  uint32_t c[4] = {0, 0, 0, 0};
  __device__ __forceinline__ void add(uint32_t m) {
    c[0] += (m & 1u) | ((m & 4u) << 14);
    c[1] += ((m >> 1) & 1u) | ((m & 8u) << 13);
    c[2] += ((m >> 4) & 1u) | ((m & 64u) << 10);
    c[3] += ((m >> 5) & 1u) | ((m & 128u) << 9);
  }
  // lane r < 8 receives row r's wave total
  __device__ __forceinline__ uint32_t totals(uint32_t lane) const {
    const uint32_t s0 = wave_sum(c[0]), s1 = wave_sum(c[1]), s2 = wave_sum(c[2]), s3 = wave_sum(c[3]);
    const uint32_t which = (lane & 1) + 2 * ((lane >> 2) & 1);
    const uint32_t sv = which == 0 ? s0 : which == 1 ? s1 : which == 2 ? s2 : s3;
    return (sv >> (16 * ((lane >> 1) & 1))) & 0xFFFFu;
  }
};

template <bool PACKED>
__device__ __forceinline__ uint64_t ent_key(const uint64_t* ent, uint32_t i) {
  return PACKED ? (ent[i] >> 8) : ent[i];
}
template <bool PACKED>
__device__ __forceinline__ uint32_t ent_mask(const uint64_t* ent, const uint8_t* masks, uint32_t i) {
  return PACKED ? (uint32_t)(ent[i] & 0xFFu) : (uint32_t)masks[i];
}

// First-probe lookup: examines the first two entries of the bucket only.
// Returns the row mask when the key is among them; sets `more` when the
// key may sit further in the bucket (count > 2 and both entries smaller).
template <bool PACKED>
__device__ __forceinline__ uint32_t lookup2(const uint64_t* __restrict__ ent,
                                            const uint8_t* __restrict__ masks, uint32_t st,
                                            uint32_t n, uint64_t bv, bool& more) {
  const uint64_t e0 = ent[st], e1 = ent[st + 1];
  uint32_t m = 0;
  if (PACKED) {
    const uint64_t bvs = bv << 8;
    const uint64_t x0 = e0 ^ bvs, x1 = e1 ^ bvs;
    if (n > 1 && x1 < 256) m = (uint32_t)x1;
    if (n > 0 && x0 < 256) m = (uint32_t)x0;
    more = (n > 2) && (e1 < bvs);
  } else {
    if (n > 1 && e1 == bv) m = masks[st + 1];
    if (n > 0 && e0 == bv) m = masks[st];
    more = (n > 2) && (e1 < bv);
  }
  return m;
}

// Row mask of column hash bv (0 when absent).  Buckets hold distinct keys
// in ascending order; entries past a bucket's count are ignored.
template <bool PACKED>
__device__ __forceinline__ uint32_t lookup(const uint64_t* __restrict__ ent,
                                           const uint8_t* __restrict__ masks, uint32_t st,
                                           uint32_t n, uint64_t bv) {
  uint32_t m = 0;
  if (PACKED) {
    const uint64_t bvs = bv << 8, top = bvs | 0xFFull;
    for (uint32_t k = 0; k < n; k += 2) {
      const uint64_t e0 = ent[st + k], e1 = ent[st + k + 1];
      const uint64_t x0 = e0 ^ bvs, x1 = e1 ^ bvs;
      if (x0 < 256) m = (uint32_t)x0;
      if (x1 < 256 && k + 1 < n) m = (uint32_t)x1;
      if (e1 > top) break;
    }
  } else {
    for (uint32_t k = 0; k < n; k += 2) {
      const uint64_t k0 = ent[st + k], k1 = ent[st + k + 1];
      if (k0 == bv) m = masks[st + k];
      if (k1 == bv && k + 1 < n) m = masks[st + k + 1];
      if (k1 >= bv) break;
    }
  }
  return m;
}

template <int R, bool PACKED>
__device__ __forceinline__ void table_build_and_stream(const PairsTableLaunch& a, uint8_t* smem,
                                                       uint32_t row0, uint32_t c0, uint32_t c1) {
  TableMeta& meta = *reinterpret_cast<TableMeta*>(smem);
  const uint32_t cap = (uint32_t)R * a.stride;
  uint64_t* ent = reinterpret_cast<uint64_t*>(smem + 256);
  uint8_t* masks = smem + 256 + tk_ent(cap);
  uint32_t* dir = reinterpret_cast<uint32_t*>(smem + 256 + tk_ent(cap) + tk_masks(cap));
  uint16_t* samp = reinterpret_cast<uint16_t*>(smem + 256 + tk_ent(cap) + tk_masks(cap) + tk_dir());
  uint32_t* cnt = reinterpret_cast<uint32_t*>(ent);  // build-time bucket counters
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t E = meta.pre[8];
  const uint32_t sr = meta.shift_r, sl = meta.shift_l, scale = meta.scale;

  // ---- build pass 1: bucket counts, each entry's rank inside its bucket
  // (all kEPT loads issued before the first use)
  uint64_t bkey[kEPT];
  uint32_t brow[kEPT];
#pragma unroll
  for (uint32_t t = 0; t < kEPT; ++t) {
    const uint32_t e = min(tid + t * kTableThreads, E ? E - 1 : 0u);
    uint32_t r = 0;
#pragma unroll
    for (int x = 1; x < R; ++x) r += (e >= meta.pre[x]) ? 1u : 0u;
    brow[t] = r;
    bkey[t] = E ? a.sketches[(uint64_t)(row0 + r) * a.stride + (e - meta.pre[r])] : 0ull;
  }
  uint32_t pos[kEPT];
#pragma unroll
  for (uint32_t t = 0; t < kEPT; ++t) {
    pos[t] = 0;
    if (tid + t * kTableThreads < E) pos[t] = atomicAdd(&cnt[bucket_of(bkey[t], sr, sl, scale)], 1u);
  }
  __syncthreads();
  // exclusive scan of the kNB counters -> dir = start | count << 16
  {
    __shared__ uint32_t wsum[kTableWaves];
    constexpr uint32_t PT = kNB / kTableThreads;
    const uint32_t base = tid * PT;
    uint32_t v[PT];
    uint32_t s = 0;
#pragma unroll
    for (uint32_t i = 0; i < PT; ++i) {
      v[i] = cnt[base + i];
      s += v[i];
    }
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
#pragma unroll
    for (uint32_t i = 0; i < PT; ++i) {
      dir[base + i] = run | (v[i] << 16);
      run += v[i];
    }
  }
  __syncthreads();
  // ---- build pass 2: scatter
#pragma unroll
  for (uint32_t t = 0; t < kEPT; ++t) {
    if (tid + t * kTableThreads < E) {
      const uint64_t key = bkey[t];
      const uint32_t slot = (dir[bucket_of(key, sr, sl, scale)] & 0xFFFFu) + pos[t];
      if (PACKED) {
        ent[slot] = (key << 8) | (1ull << brow[t]);
      } else {
        ent[slot] = key;
        masks[slot] = (uint8_t)(1u << brow[t]);
      }
    }
  }
  if (tid < 2) {
    ent[E + tid] = ~0ull;  // pads for paired reads past the last bucket
    masks[E + tid] = 0;
  }
  __syncthreads();
  // ---- per bucket: insertion sort, merge equal keys (OR the row masks)
  for (uint32_t bk = tid; bk < kNB; bk += kTableThreads) {
    const uint32_t d = dir[bk];
    const uint32_t s0 = d & 0xFFFFu, s1 = s0 + (d >> 16);
    for (uint32_t i = s0 + 1; i < s1; ++i) {
      const uint64_t k = ent[i];
      const uint8_t m = PACKED ? 0 : masks[i];
      uint32_t j = i;
      while (j > s0 && ent[j - 1] > k) {
        ent[j] = ent[j - 1];
        if (!PACKED) masks[j] = masks[j - 1];
        --j;
      }
      ent[j] = k;
      if (!PACKED) masks[j] = m;
    }
    uint32_t w = s0;
    for (uint32_t i = s0; i < s1; ++i) {
      if (i > s0 && ent_key<PACKED>(ent, i) == ent_key<PACKED>(ent, w - 1)) {
        if (PACKED) ent[w - 1] |= ent[i] & 0xFFull;
        else masks[w - 1] |= masks[i];
      } else {
        ent[w] = ent[i];
        if (!PACKED) masks[w] = masks[i];
        ++w;
      }
    }
    dir[bk] = s0 | ((w - s0) << 16);
  }
  __syncthreads();
  // ---- rank_A support: per-row entry counts before each 64-bucket group
  for (uint32_t g = wave; g < kNG; g += kTableWaves) {
    const uint32_t d = dir[g * 64 + lane];
    RowCount16 rc;
    for (uint32_t k = 0; k < (d >> 16); ++k) rc.add(ent_mask<PACKED>(ent, masks, (d & 0xFFFFu) + k));
    const uint32_t c = rc.totals(lane);
    if (lane < 8) samp[(g + 1) * 8 + lane] = (uint16_t)c;
  }
  __syncthreads();
  if (tid < 8) {
    uint32_t run = 0;
    samp[tid] = 0;
    for (uint32_t g = 1; g <= kNG; ++g) {
      run += samp[g * 8 + tid];
      samp[g * 8 + tid] = (uint16_t)run;
    }
  }
  __syncthreads();

  // ---- stream columns
  const uint64_t maxkey = uni64(meta.maxkey);
  const uint32_t nrows = uni32(meta.nrows);
  uint64_t xr[R];
  uint32_t lr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    xr[r] = uni64(meta.last[r]);
    lr[r] = uni32(meta.len[r]);
  }
  uint64_t* ring = reinterpret_cast<uint64_t*>(smem + 256 + tk_ent(cap) + tk_masks(cap) + tk_dir() + tk_samp()) +
                   wave * kRing;
  for (uint32_t j = c0 + wave; j < c1; j += kTableWaves) {
    const uint32_t lb = uni32(a.lens[j]);
    const uint64_t* B = a.sketches + (uint64_t)j * a.stride;
    const uint64_t lastB = lb ? uni64(B[lb - 1]) : 0;
    uint32_t acc_lo = 0, acc_hi = 0;
    uint32_t head = 0, tail = 0;  // ring indices (wave-uniform)
    // full bucket walks for up to 64 queued hashes
    auto drain = [&](uint32_t count) {
      uint32_t m = 0;
      if (lane < count) {
        const uint64_t bv = ring[(head + lane) & (kRing - 1)];
        const uint32_t d = dir[bucket_of(bv, sr, sl, scale)];
        m = lookup<PACKED>(ent, masks, (d & 0xFFFFu) + 2, (d >> 16) - 2, bv);
      }
      acc_lo += spread4(m);
      if (R > 4) acc_hi += spread4(m >> 4);
      head += count;
    };
    for (uint32_t cb = 0; cb < lb; cb += kChunk * 64) {
      uint64_t v[kChunk];
#pragma unroll
      for (int t = 0; t < kChunk; ++t) {
        const uint32_t e = cb + t * 64 + lane;
        v[t] = e < lb ? B[e] : ~0ull;
      }
      // groups of kGroup rounds: all directory reads, then all entry
      // reads, then the compares -- branch-free so the LDS latencies of
      // the group overlap; lanes past the column end or above maxkey probe
      // bucket 0 and are masked out.
#pragma unroll
      for (int g0 = 0; g0 < kChunk; g0 += kGroup) {
        if (cb + g0 * 64 >= lb) continue;  // wave-uniform
        uint32_t d[kGroup];
        bool ok[kGroup];
#pragma unroll
        for (int t = 0; t < kGroup; ++t) {
          const uint64_t bv = v[g0 + t];
          ok[t] = (cb + (g0 + t) * 64 + lane < lb) && (bv <= maxkey);
          const uint32_t bk = ok[t] ? bucket_of(bv, sr, sl, scale) : 0u;
          d[t] = dir[bk];
        }
        uint64_t e0[kGroup], e1[kGroup];
#pragma unroll
        for (int t = 0; t < kGroup; ++t) {
          const uint32_t st = d[t] & 0xFFFFu;
          e0[t] = ent[st];
          e1[t] = ent[st + 1];
        }
        uint32_t more_bits = 0;
#pragma unroll
        for (int t = 0; t < kGroup; ++t) {
          const uint64_t bv = v[g0 + t];
          const uint32_t n = d[t] >> 16;
          uint32_t m = 0;
          bool more;
          if (PACKED) {
            const uint64_t bvs = bv << 8;
            const uint64_t x0 = e0[t] ^ bvs, x1 = e1[t] ^ bvs;
            m = (n > 1 && x1 < 256) ? (uint32_t)x1 : 0u;
            m = (n > 0 && x0 < 256) ? (uint32_t)x0 : m;
            more = (n > 2) && (e1[t] < bvs);
          } else {
            const uint32_t st = d[t] & 0xFFFFu;
            const uint32_t m0 = masks[st], m1 = masks[st + 1];
            m = (n > 1 && e1[t] == bv) ? m1 : 0u;
            m = (n > 0 && e0[t] == bv) ? m0 : m;
            more = (n > 2) && (e1[t] < bv);
          }
          m = ok[t] ? m : 0u;
          more_bits |= (ok[t] && more) ? (1u << t) : 0u;
          acc_lo += spread4(m);
          if (R > 4) acc_hi += spread4(m >> 4);
        }
        // queue the lanes whose key may sit past the first two entries
#pragma unroll
        for (int t = 0; t < kGroup; ++t) {
          const bool more = (more_bits >> t) & 1u;
          const unsigned long long mm = __ballot(more);
          if (mm) {
            if (more) ring[(tail + __popcll(mm & ((1ull << lane) - 1ull))) & (kRing - 1)] = v[g0 + t];
            tail += __popcll(mm);
            if (tail - head >= 64) drain(64);
          }
        }
      }
    }
    while (tail != head) drain(min(64u, tail - head));
    const uint32_t common_lane = row_totals(acc_lo, acc_hi, lane);
    // rank_A(last B): entries of row r with key <= last B, from the sorted
    // buckets; needed only when last B < last A_r <= maxkey
    uint32_t rank_lane = 0;
    if (lb && lastB < maxkey) {
      const uint32_t bk = bucket_of(lastB, sr, sl, scale);
      const uint32_t g = bk >> 6;
      const uint32_t bl = g * 64 + lane;
      RowCount16 rc;
      if (bl <= bk) {
        const uint32_t d = dir[bl];
        const uint32_t st = d & 0xFFFFu, n = d >> 16;
        for (uint32_t k = 0; k < n; ++k) {
          if (bl == bk && ent_key<PACKED>(ent, st + k) > lastB) break;
          rc.add(ent_mask<PACKED>(ent, masks, st + k));
        }
      }
      rank_lane = rc.totals(lane) + (lane < 8 ? samp[g * 8 + lane] : 0u);
    }
    // rank_B(last A_r) for the rows with last A_r <= last B
    const uint32_t cb = lb ? rank_rows_B<R>(B, lb, meta.last, xr, lane) : 0u;
    // lane r < R evaluates pair (row0 + r, j)
    uint32_t la = 0;
    uint64_t x = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (lane == (uint32_t)r) {
        la = lr[r];
        x = xr[r];
      }
    }
    uint32_t common = common_lane;
    uint32_t total;
    if (la == 0 || lb == 0) {
      common = 0;
      total = 0;
    } else if (x <= lastB) {
      total = la + cb - common;
    } else {
      total = rank_lane + lb - common;
    }
    const uint32_t i = row0 + lane;
    const bool pass = (lane < nrows) && (j > i) && (total <= a.tmax) && (common >= a.cmin[total]);
    const unsigned long long mk = __ballot(pass);
    if (mk) {
      const uint32_t first = __builtin_ctzll(mk);
      unsigned long long obase = 0;
      if (lane == first) obase = atomicAdd(a.count, (unsigned long long)__popcll(mk));
      obase = __shfl(obase, first);
      if (pass) {
        const unsigned long long slot = obase + __popcll(mk & ((1ull << lane) - 1ull));
        if (slot < a.out_cap) a.out[slot] = gg_pair{i, j, common, total};
      }
    }
  }
}

template <int R>
__global__ __launch_bounds__(kTableThreads, 1) void pairs_table_kernel(PairsTableLaunch a) {
  extern __shared__ __align__(16) uint8_t smem[];
  TableMeta& meta = *reinterpret_cast<TableMeta*>(smem);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(smem + 256);

  constexpr uint32_t G = kTile / R;  // row blocks per segment
  const uint32_t b = blockIdx.x;
  const uint32_t q = b >> 3;
  const uint32_t rb = q % G;
  const uint32_t seg_id = (q / G) * 8 + (b & 7);
  if (seg_id >= a.n_segs) return;
  const PairSeg sg = a.segs[seg_id];
  const uint32_t row0 = sg.I * kTile + rb * R;
  if (row0 >= a.n) return;
  const uint32_t c0 = max(sg.J0 * kTile, row0 + 1);
  const uint32_t c1 = min(sg.J1 * kTile, a.n);
  if (c0 >= c1) return;
  const uint32_t tid = threadIdx.x;

  if (tid == 0) {
    const uint32_t nrows = min((uint32_t)R, a.n - row0);
    uint64_t mx = 0;
    uint32_t acc = 0;
    for (int r = 0; r < 8; ++r) {
      uint32_t l = 0;
      uint64_t last = 0;
      if (r < (int)nrows) {
        l = a.lens[row0 + r];
        if (l) last = a.sketches[(uint64_t)(row0 + r) * a.stride + l - 1];
      }
      meta.len[r] = l;
      meta.last[r] = last;
      meta.pre[r] = acc;
      acc += l;
      if (l && last > mx) mx = last;
    }
    meta.pre[8] = acc;
    meta.maxkey = mx;
    const uint32_t L = mx ? 64 - __builtin_clzll(mx) : 1;
    meta.shift_r = L > 32 ? L - 32 : 0;
    meta.shift_l = L > 32 ? 0 : 32 - L;
    const uint64_t t = (uint64_t)top32(mx, meta.shift_r, meta.shift_l) + 1;  // in (2^31, 2^32]
    meta.scale = (uint32_t)(((uint64_t)kNB << 32) / t);
    meta.nrows = nrows;
    meta.packed = (mx >> 56) == 0;
  }
  for (uint32_t i = tid; i < kNB; i += kTableThreads) cnt[i] = 0;
  __syncthreads();
  if (meta.packed) table_build_and_stream<R, true>(a, smem, row0, c0, c1);
  else table_build_and_stream<R, false>(a, smem, row0, c0, c1);
}

template <int R>
hipError_t launch_table_r(const PairsTableLaunch& a, hipStream_t st) {
  const size_t lds = table_lds_bytes((uint32_t)R * a.stride);
  hipError_t e = hipFuncSetAttribute((const void*)pairs_table_kernel<R>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  constexpr uint32_t G = kTile / R;
  const uint64_t groups = (a.n_segs + 7) / 8;
  const uint64_t blocks = groups * 8 * G;
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pairs_table_kernel<R>, dim3((uint32_t)blocks), dim3(kTableThreads), lds, st, a);
  return hipGetLastError();
}

}  // namespace

uint32_t pairs_table_rows(uint32_t s) {
  uint32_t R = 8;
  while (R > 1 && R * s > kKeyCap) R >>= 1;
  return (R * s <= kKeyCap) ? R : 0;
}

hipError_t launch_pairs_table(const PairsTableLaunch& a, hipStream_t st) {
  if (a.n_segs == 0) return hipSuccess;
  switch (pairs_table_rows(a.stride)) {
    case 8: return launch_table_r<8>(a, st);
    case 4: return launch_table_r<4>(a, st);
    case 2: return launch_table_r<2>(a, st);
    case 1: return launch_table_r<1>(a, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_pairs(const PairsLaunch& a, hipStream_t st) {
  if (a.tile_end <= a.tile_begin) return hipSuccess;
  const uint64_t n = a.tile_end - a.tile_begin;
  if (n > 0x7fffffffull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pairs_merge_kernel, dim3((uint32_t)n), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

}  // namespace gg
