// Device-side FASTA parsing and 2-bit packing (the GPU
// half): the host only reads (and gunzips) files; the raw FASTA bytes of a
// batch of genomes go to the GPU in one pinned copy and are classified,
// compacted to 2-bit codes and split into runs here.
//
// Same byte semantics as the host packer (pack.cpp, restating needletail
// 0.5 parse + normalize(false) as galah's finch path uses it, src/finch.rs:47):
//   * a line that starts with '>' is a header line (it ends the previous
//     record; its bytes are no sequence);
//   * A C G T / a c g t / U u -> codes 0..3 (U as T);
//   * ' ' '\t' '\r' '\n' are dropped (they do not break a k-mer);
//   * every other byte breaks a k-mer (needletail's N).
// A run is a maximal stretch of bases with no break and no header between
// them inside one file; the host keeps the runs of >= k bases.  Packed
// positions count bases only, each genome starting on a 16-base word, so a
// run's bases are contiguous (short runs stay in the word stream and are
// never enumerated by K1).
//
// Work is split in blocks of kBlockBytes bytes that never straddle files.
// Three passes, each one coalesced read of the block, with tiny per-block
// scans on the host in between:
//   1. last '\n' of every block;
//   2. with the line-start prefix: bases per block, run starts (as if no
//      base came before the block), whether the first non-dropped byte is a
//      base, and the block's last non-dropped byte;
//   3. with those prefixes: every base's 2-bit code into its packed word
//      (assembled in LDS) and every run start.
#include "device_util.hpp"
#include "gg_internal.hpp"

namespace gg {
namespace {

constexpr int kThreads = 256;
constexpr int kPerThread = 32;
constexpr uint32_t kBlockBytes = kThreads * kPerThread;  // 8 KiB

enum : uint32_t { kCodeBreak = 4, kCodeSkip = 5 };
// byte class: ACGTU (either case) -> code, whitespace -> skip, else break
__device__ __forceinline__ uint32_t byte_class(uint32_t c) {
  const uint32_t l = c | 0x20u;
  if (l == 'a') return 0;
  if (l == 'c') return 1;
  if (l == 'g') return 2;
  if (l == 't' || l == 'u') return 3;
  if (c == ' ' || c == '\t' || c == '\r' || c == '\n') return kCodeSkip;
  return kCodeBreak;
}

// last-non-dropped-byte record: (index + 1) << 2 | kind, 0 = none;
// kind 0 = base, 1 = break or header
__device__ __forceinline__ uint64_t later(uint64_t a, uint64_t b) { return b ? b : a; }

__device__ __forceinline__ int64_t block_max_i64(int64_t v, int64_t* sh) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (int64_t)__shfl_xor((long long)v, o));
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  int64_t r = sh[0];
  for (int w = 1; w < kThreads / 64; ++w) r = max(r, sh[w]);
  __syncthreads();
  return r;
}

// exclusive scan across the block of a per-thread value with an
// associative op; returns the thread's exclusive prefix (identity for 0)
template <class T, class Op>
__device__ __forceinline__ T block_exclusive(T v, T identity, Op op, T* sh, T* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const T y = (T)__shfl_up(inc, o);
    if (lane >= o) inc = op(y, inc);
  }
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  T pre = identity;
  for (int x = 0; x < w; ++x) pre = op(pre, sh[x]);
  T all = identity;
  for (int x = 0; x < kThreads / 64; ++x) all = op(all, sh[x]);
  const T up = (T)__shfl_up(inc, 1);
  const T excl = lane ? op(pre, up) : pre;
  __syncthreads();
  if (total) *total = all;
  return excl;
}

struct BlockArgs {
  const uint8_t* raw;
  uint64_t n;
  const uint32_t* blk_file;   // [blocks] file of the block
  const uint64_t* blk_start;  // [blocks] first byte
  const uint64_t* file_start; // [files] first byte
};

// The thread's 32 bytes as two 16-byte loads (files start on 16-byte
// boundaries of the batch: the host pads each file with '\n', which parses
// as nothing); bytes past the block read as ' ' (dropped).
__device__ __forceinline__ void load_chunk(const BlockArgs& a, uint64_t b0, uint64_t b1, uint32_t (&c)[kPerThread],
                                           uint64_t& i0) {
  i0 = b0 + (uint64_t)threadIdx.x * kPerThread;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint64_t at = i0 + 16 * h;
    uint4 v = make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
    if (at < b1) v = *(const uint4*)(a.raw + at);
    const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 16; ++q) c[16 * h + q] = (x[q >> 2] >> (8 * (q & 3))) & 0xFFu;
  }
}

// pass 1: last '\n' index + 1 of each block (0 = none)
__global__ __launch_bounds__(kThreads) void parse_nl_kernel(BlockArgs a, const uint64_t* __restrict__ blk_end,
                                                           uint64_t* __restrict__ blk_nl) {
  __shared__ int64_t sh[kThreads / 64];
  const uint32_t b = blockIdx.x;
  uint32_t c[kPerThread];
  uint64_t i0;
  load_chunk(a, a.blk_start[b], blk_end[b], c, i0);
  int64_t last = 0;
#pragma unroll
  for (int j = 0; j < kPerThread; ++j)
    if (c[j] == '\n' && i0 + j < blk_end[b]) last = (int64_t)(i0 + j + 1);
  last = block_max_i64(last, sh);
  if (threadIdx.x == 0) blk_nl[b] = (uint64_t)last;
}

// The per-byte classes of one thread's chunk, given the line-start state at
// its first byte.  cls: 0..3 base, kCodeBreak (break or header), kCodeSkip.
struct ChunkClass {
  uint32_t cls[kPerThread];
};

__device__ __forceinline__ void classify(const BlockArgs& a, uint64_t fstart, uint64_t nl_before /* index+1 or 0 */,
                                         uint64_t b1, const uint32_t (&c)[kPerThread], uint64_t i0, ChunkClass& out) {
  // line start of the chunk's first byte, and whether that line is a header
  const uint64_t ls = nl_before > fstart ? nl_before : fstart;  // (<= i0)
  bool hdr = ls < a.n && a.raw[ls] == '>';
  int32_t lsr = ls == i0 ? 0 : -1;  // a line start inside the chunk, relative to i0
  const uint32_t lim = b1 > i0 ? (uint32_t)min<uint64_t>(b1 - i0, kPerThread) : 0u;  // bytes of the block in the chunk
#pragma unroll
  for (int j = 0; j < kPerThread; ++j) {
    uint32_t k;
    if ((uint32_t)j >= lim) {
      k = kCodeSkip;
    } else {
      if (j == lsr) hdr = c[j] == '>';  // (a new line began at j)
      if (c[j] == '\n') {
        k = kCodeSkip;
        lsr = j + 1;
      } else {
        k = hdr ? (uint32_t)kCodeBreak : byte_class(c[j]);
      }
    }
    out.cls[j] = k;
  }
}

// line-start prefix of each thread: the block's prefix, then the threads
// before it (max of last '\n' index + 1)
__device__ __forceinline__ uint64_t thread_nl_prefix(const uint32_t (&c)[kPerThread], uint64_t i0, uint64_t b1,
                                                     uint64_t block_pre, int64_t* sh) {
  int64_t last = 0;
#pragma unroll
  for (int j = 0; j < kPerThread; ++j)
    if (c[j] == '\n' && i0 + j < b1) last = (int64_t)(i0 + j + 1);
  auto mx = [](int64_t x, int64_t y) { return x > y ? x : y; };
  const int64_t ex = block_exclusive<int64_t>(last, 0, mx, sh, nullptr);
  return (uint64_t)(ex > (int64_t)block_pre ? ex : (int64_t)block_pre);
}

// run-start flags of one chunk given the last non-dropped byte before it
__device__ __forceinline__ uint32_t run_starts(const ChunkClass& k, uint64_t prev, uint64_t fstart, bool (&start)[kPerThread],
                                               uint64_t i0) {
  // prev: (index + 1) << 2 | kind of the last non-dropped byte before the
  // chunk (0 = none); bytes before the file do not count
  bool prev_base = prev && ((prev >> 2) - 1) >= fstart && (prev & 3u) == 0;
  uint32_t n = 0;
#pragma unroll
  for (int j = 0; j < kPerThread; ++j) {
    const uint32_t x = k.cls[j];
    start[j] = x < 4 && !prev_base;
    n += start[j];
    if (x != kCodeSkip) prev_base = x < 4;
  }
  (void)i0;
  return n;
}

__device__ __forceinline__ uint64_t thread_last_prefix(const ChunkClass& k, uint64_t i0, uint64_t block_pre,
                                                       uint64_t* sh) {
  uint64_t last = 0;
#pragma unroll
  for (int j = 0; j < kPerThread; ++j)
    if (k.cls[j] != kCodeSkip) last = ((i0 + j + 1) << 2) | (k.cls[j] < 4 ? 0u : 1u);
  auto lat = [](uint64_t x, uint64_t y) { return later(x, y); };
  const uint64_t ex = block_exclusive<uint64_t>(last, 0, lat, sh, nullptr);
  return later(block_pre, ex);
}

// pass 2: per block its bases, its run starts counted as if no base came
// before it (runs0), whether its first non-dropped byte is a base (the host
// then takes one start off when the block before ends in a base), and its
// last non-dropped byte
__global__ __launch_bounds__(kThreads) void parse_count_kernel(BlockArgs a, const uint64_t* __restrict__ blk_end,
                                                              const uint64_t* __restrict__ pre_nl,
                                                              uint64_t* __restrict__ blk_bases,
                                                              uint64_t* __restrict__ blk_runs0,
                                                              uint64_t* __restrict__ blk_first,
                                                              uint64_t* __restrict__ blk_last) {
  __shared__ int64_t shi[kThreads / 64];
  __shared__ uint64_t shu[kThreads / 64];
  const uint32_t b = blockIdx.x;
  const uint64_t b1 = blk_end[b];
  const uint64_t fstart = a.file_start[a.blk_file[b]];
  uint32_t c[kPerThread];
  uint64_t i0;
  load_chunk(a, a.blk_start[b], b1, c, i0);
  const uint64_t nlp = thread_nl_prefix(c, i0, b1, pre_nl[b], shi);
  ChunkClass k;
  classify(a, fstart, nlp, b1, c, i0, k);
  // within the block: the last non-dropped byte before this thread's chunk
  const uint64_t prev = thread_last_prefix(k, i0, 0, shu);
  bool st[kPerThread];
  uint64_t nr = run_starts(k, prev, 0, st, i0);  // (fstart 0: a byte before the chunk inside the block counts)
  uint64_t bases = 0, last = 0, first = ~0ull;  // first: (index << 2 | kind) of the chunk's first non-dropped byte
#pragma unroll
  for (int j = kPerThread - 1; j >= 0; --j)
    if (k.cls[j] != kCodeSkip) first = ((uint64_t)j << 2) | (k.cls[j] < 4 ? 0u : 1u);
#pragma unroll
  for (int j = 0; j < kPerThread; ++j) {
    if (k.cls[j] < 4) ++bases;
    if (k.cls[j] != kCodeSkip) last = ((i0 + j + 1) << 2) | (k.cls[j] < 4 ? 0u : 1u);
  }
  if (first != ~0ull) first += (uint64_t)threadIdx.x << 7;  // (block-relative index: thread * 32 + j)
  uint64_t tb, tl, tr, tf;
  auto add = [](uint64_t x, uint64_t y) { return x + y; };
  (void)block_exclusive<uint64_t>(bases, 0, add, shu, &tb);
  auto lat = [](uint64_t x, uint64_t y) { return later(x, y); };
  (void)block_exclusive<uint64_t>(last, 0, lat, shu, &tl);
  (void)block_exclusive<uint64_t>(nr, 0, add, shu, &tr);
  auto mn = [](uint64_t x, uint64_t y) { return x < y ? x : y; };
  (void)block_exclusive<uint64_t>(first, ~0ull, mn, shu, &tf);
  if (threadIdx.x == 0) {
    blk_bases[b] = tb;
    blk_last[b] = tl;
    blk_runs0[b] = tr;
    blk_first[b] = tf != ~0ull && (tf & 3u) == 0;
  }
}

// pass 3: 2-bit codes straight into the packed words (the block's words
// assembled in LDS; the first and last, which a neighbouring block may
// share, merged with atomicOr; words pre-cleared), and every run start
// (packed position)
__global__ __launch_bounds__(kThreads) void parse_emit_kernel(BlockArgs a, const uint64_t* __restrict__ blk_end,
                                                             const uint64_t* __restrict__ pre_nl,
                                                             const uint64_t* __restrict__ pre_last,
                                                             const uint64_t* __restrict__ base_off,
                                                             const uint64_t* __restrict__ run_off,
                                                             uint32_t* __restrict__ words,
                                                             uint64_t* __restrict__ starts) {
  __shared__ int64_t shi[kThreads / 64];
  __shared__ uint64_t shu[kThreads / 64];
  __shared__ uint32_t wl[kBlockBytes / 16 + 2];
  const uint32_t b = blockIdx.x;
  const uint64_t b1 = blk_end[b];
  const uint64_t fstart = a.file_start[a.blk_file[b]];
  for (uint32_t i = threadIdx.x; i < kBlockBytes / 16 + 2; i += kThreads) wl[i] = 0;
  uint32_t c[kPerThread];
  uint64_t i0;
  load_chunk(a, a.blk_start[b], b1, c, i0);
  const uint64_t nlp = thread_nl_prefix(c, i0, b1, pre_nl[b], shi);
  ChunkClass k;
  classify(a, fstart, nlp, b1, c, i0, k);
  const uint64_t prev = thread_last_prefix(k, i0, pre_last[b], shu);
  bool st[kPerThread];
  const uint64_t nr = run_starts(k, prev, fstart, st, i0);
  uint64_t nb = 0;
#pragma unroll
  for (int j = 0; j < kPerThread; ++j) nb += k.cls[j] < 4;
  auto add = [](uint64_t x, uint64_t y) { return x + y; };
  uint64_t total;
  const uint64_t p0 = base_off[b];
  const uint64_t w0 = p0 >> 4;
  uint64_t pos = p0 + block_exclusive<uint64_t>(nb, 0, add, shu, &total);
  uint64_t rr = run_off[b] + block_exclusive<uint64_t>(nr, 0, add, shu, nullptr);
  __syncthreads();  // (wl cleared)
#pragma unroll
  for (int j = 0; j < kPerThread; ++j) {
    if (k.cls[j] >= 4) continue;
    if (st[j]) starts[rr++] = pos;
    atomicOr(&wl[(uint32_t)((pos >> 4) - w0)], k.cls[j] << (30u - 2u * (uint32_t)(pos & 15u)));
    ++pos;
  }
  __syncthreads();
  if (total) {
    const uint32_t nw = (uint32_t)(((p0 + total - 1) >> 4) - w0 + 1);
    for (uint32_t i = threadIdx.x; i < nw; i += kThreads) {
      if (i == 0 || i + 1 == nw) atomicOr(&words[w0 + i], wl[i]);
      else words[w0 + i] = wl[i];
    }
  }
}

}  // namespace

hipError_t parse_batch_pass(int pass, const ParseLaunch& p, hipStream_t st) {
  BlockArgs a{p.raw, p.n_bytes, p.blk_file, p.blk_start, p.file_start};
  const dim3 grid(p.n_blocks), block(kThreads);
  switch (pass) {
    case 1:
      hipLaunchKernelGGL(parse_nl_kernel, grid, block, 0, st, a, p.blk_end, p.blk_nl);
      break;
    case 2:
      hipLaunchKernelGGL(parse_count_kernel, grid, block, 0, st, a, p.blk_end, p.pre_nl, p.blk_bases, p.blk_runs,
                         p.blk_first, p.blk_last);
      break;
    case 3:
      hipLaunchKernelGGL(parse_emit_kernel, grid, block, 0, st, a, p.blk_end, p.pre_nl, p.pre_last, p.base_off,
                         p.run_off, p.words, p.starts);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

uint32_t parse_block_bytes() { return kBlockBytes; }

}  // namespace gg
