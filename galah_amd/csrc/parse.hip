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
// Passes 2 and 3 classify a thread's 32 bytes bit-parallel (parse_core.hpp:
// masks, carry chains, compress) with two rounds of block scans each.
#include "device_util.hpp"
#include "gg_internal.hpp"
#include "parse_core.hpp"

namespace gg {
namespace {

constexpr int kThreads = 256;
constexpr int kPerThread = 32;
constexpr uint32_t kBlockBytes = kThreads * kPerThread;  // 8 KiB

__device__ __forceinline__ int64_t block_max_i64(int64_t v, int64_t* sh) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (int64_t)__shfl_xor((long long)v, o));
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  int64_t r = sh[0];
  for (int w = 1; w < kThreads / 64; ++w) r = max(r, sh[w]);
  __syncthreads();
  return r;
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

// One round of block scans over the 256 threads: an exclusive max of vm and
// an exclusive sum of vs, with both totals.  sh: [4][2], this round's own.
__device__ __forceinline__ void block_scan(uint32_t vm, uint32_t vs, uint32_t (*sh)[2], uint32_t& exm, uint32_t& exs,
                                           uint32_t& totm, uint32_t& tots) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t im = vm, is = vs;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t ym = __shfl_up(im, o), ys = __shfl_up(is, o);
    if (lane >= o) {
      im = max(im, ym);
      is += ys;
    }
  }
  const uint32_t up = __shfl_up(im, 1);
  if (lane == 63) {
    sh[w][0] = im;
    sh[w][1] = is;
  }
  __syncthreads();
  uint32_t pm = 0, ps = 0;
  totm = 0;
  tots = 0;
#pragma unroll
  for (int x = 0; x < kThreads / 64; ++x) {
    if (x < w) {
      pm = max(pm, sh[x][0]);
      ps += sh[x][1];
    }
    totm = max(totm, sh[x][0]);
    tots += sh[x][1];
  }
  exm = lane ? max(pm, up) : pm;
  exs = ps + is - vs;
}

// A thread's 32 bytes classified and placed on their lines (parse_core.hpp).
// The line-start prefix (the last '\n' before the chunk: in the threads
// before it in the block, else the block's prefix pre_nl) says whether byte
// 0 starts a line, or else whether its line is a header.  Bytes past the
// block are dropped.
struct Chunk {
  parse::Masks m;
  parse::Roles r;
  uint32_t rel;  // block-relative index of byte 0
};
__device__ __forceinline__ Chunk chunk_roles(const BlockArgs& a, uint64_t b0, uint64_t b1, uint64_t fstart,
                                             uint64_t pre_nl, uint32_t (*sh)[2]) {
  Chunk c;
  c.rel = threadIdx.x * kPerThread;
  const uint64_t i0 = b0 + c.rel;
  uint32_t w[8];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint64_t at = i0 + 16 * h;
    uint4 v = make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
    if (at < b1) v = *(const uint4*)(a.raw + at);
    w[4 * h] = v.x;
    w[4 * h + 1] = v.y;
    w[4 * h + 2] = v.z;
    w[4 * h + 3] = v.w;
  }
  const uint32_t lim = b1 > i0 ? (uint32_t)min<uint64_t>(b1 - i0, kPerThread) : 0u;
  c.m = parse::classify(w, lim);
  const uint32_t nlv = c.m.nl ? c.rel + 32u - (uint32_t)parse::clz(c.m.nl) : 0u;  // (last '\n': relative index + 1)
  uint32_t ex, exs, tm, ts;
  block_scan(nlv, 0, sh, ex, exs, tm, ts);
  const uint64_t nlp = ex ? b0 + ex : pre_nl;       // (absolute index + 1, 0: none)
  const uint64_t ls = nlp > fstart ? nlp : fstart;  // the line start of byte 0 (<= i0)
  const bool line0 = ls == i0;
  const bool hdr0 = !line0 && ls < a.n && a.raw[ls] == '>';
  c.r = parse::roles(c.m, line0, hdr0);
  return c;
}

// the chunk's last kept byte as (block-relative index + 1) << 1 | is a
// break, 0 = none (a later byte compares greater)
__device__ __forceinline__ uint32_t last_kept(const Chunk& c) {
  if (!c.r.keep) return 0;
  const uint32_t j = 31u - (uint32_t)parse::clz(c.r.keep);
  return ((c.rel + j + 1u) << 1) | ((c.r.brk >> j) & 1u);
}
__device__ __forceinline__ bool first_is_base(const Chunk& c) {
  return c.r.keep && ((c.r.base >> parse::ctz(c.r.keep)) & 1u);
}

// pass 2: per block its bases, its run starts counted as if no base came
// before it (runs0), whether its first kept byte is a base (the host then
// takes one start off when the block before ends in a base), and its last
// kept byte
__global__ __launch_bounds__(kThreads) void parse_count_kernel(BlockArgs a, const uint64_t* __restrict__ blk_end,
                                                              const uint64_t* __restrict__ pre_nl,
                                                              uint64_t* __restrict__ blk_bases,
                                                              uint64_t* __restrict__ blk_runs0,
                                                              uint64_t* __restrict__ blk_first,
                                                              uint64_t* __restrict__ blk_last) {
  __shared__ uint32_t sh1[kThreads / 64][2], sh2[kThreads / 64][2];
  __shared__ uint32_t fix, first;
  const uint32_t b = blockIdx.x;
  const uint64_t b0 = a.blk_start[b], b1 = blk_end[b];
  if (threadIdx.x == 0) {
    fix = 0;
    first = 0;
  }
  const Chunk c = chunk_roles(a, b0, b1, a.file_start[a.blk_file[b]], pre_nl[b], sh1);
  // starts counted with no base before the chunk; the chunks that begin
  // with a base after a base (earlier in the block) then count one too many
  const uint32_t nb = (uint32_t)parse::popc(c.r.base);
  const uint32_t nr = (uint32_t)parse::popc(parse::run_starts(c.r, false));
  uint32_t prev, exs, tot_last, tot;
  block_scan(last_kept(c), nb | (nr << 16), sh2, prev, exs, tot_last, tot);
  const bool fb = first_is_base(c);
  const uint64_t dm = __ballot(fb && prev && !(prev & 1u));
  if ((threadIdx.x & 63) == 0 && dm) atomicAdd(&fix, (uint32_t)__popcll(dm));
  if (fb && !prev) first = 1;  // (the chunk holding the block's first kept byte)
  __syncthreads();
  if (threadIdx.x == 0) {
    blk_bases[b] = tot & 0xFFFFu;
    blk_runs0[b] = (tot >> 16) - fix;
    blk_first[b] = first;
    blk_last[b] = tot_last ? ((b0 + (tot_last >> 1)) << 2) | (tot_last & 1u) : 0;
  }
}

// pass 3: 2-bit codes straight into the packed words (the block's words
// assembled in LDS, three atomicOr per thread at most; the first and last,
// which a neighbouring block may share, merged into global with atomicOr;
// words pre-cleared), and every run start (packed position)
__global__ __launch_bounds__(kThreads) void parse_emit_kernel(BlockArgs a, const uint64_t* __restrict__ blk_end,
                                                             const uint64_t* __restrict__ pre_nl,
                                                             const uint64_t* __restrict__ pre_last,
                                                             const uint64_t* __restrict__ base_off,
                                                             const uint64_t* __restrict__ run_off,
                                                             uint32_t* __restrict__ words,
                                                             uint64_t* __restrict__ starts) {
  __shared__ uint32_t sh1[kThreads / 64][2], sh2[kThreads / 64][2];
  __shared__ uint32_t fixw[kThreads / 64];
  __shared__ uint32_t wl[kBlockBytes / 16 + 2];
  const uint32_t b = blockIdx.x;
  const uint64_t b0 = a.blk_start[b], b1 = blk_end[b];
  const uint64_t fstart = a.file_start[a.blk_file[b]];
  for (uint32_t i = threadIdx.x; i < kBlockBytes / 16 + 2; i += kThreads) wl[i] = 0;
  const Chunk c = chunk_roles(a, b0, b1, fstart, pre_nl[b], sh1);
  const uint32_t nb = (uint32_t)parse::popc(c.r.base);
  const uint32_t starts0 = parse::run_starts(c.r, false);
  uint32_t prev, exs, tot_last, tot;
  block_scan(last_kept(c), nb | ((uint32_t)parse::popc(starts0) << 16), sh2, prev, exs, tot_last, tot);
  // the last kept byte before the chunk: in the block, else before it (in
  // the same file)
  bool prev_base;
  if (prev) {
    prev_base = !(prev & 1u);
  } else {
    const uint64_t pl = pre_last[b];
    prev_base = pl && ((pl >> 2) - 1) >= fstart && (pl & 3u) == 0;
  }
  const bool fix = prev_base && first_is_base(c);  // (one start fewer than starts0 counts)
  const uint32_t st = fix ? starts0 & (starts0 - 1u) : starts0;
  // the fixes before this chunk: ballots per wave, wave totals in LDS
  const uint64_t fm = __ballot(fix);
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  if (lane == 0) fixw[wv] = (uint32_t)__popcll(fm);
  __syncthreads();  // (also: wl cleared)
  uint32_t fix_before = (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
  for (uint32_t x = 0; x < wv; ++x) fix_before += fixw[x];
  uint64_t pos = base_off[b] + (exs & 0xFFFFu);
  uint64_t rr = run_off[b] + (exs >> 16) - fix_before;
  const uint64_t w0 = base_off[b] >> 4;
  // run starts (few per chunk)
  for (uint32_t m = st; m;) {
    const uint32_t j = (uint32_t)parse::ctz(m);
    m &= m - 1u;
    starts[rr++] = pos + (uint64_t)parse::popc(c.r.base & ((1u << j) - 1u));
  }
  if (nb) {
    const uint64_t R = parse::packed_codes(c.m, c.r.base);
    uint32_t x0, x1, x2;
    parse::place(R, (uint32_t)(pos & 15u), x0, x1, x2);
    const uint32_t k = (uint32_t)((pos >> 4) - w0);
    atomicOr(&wl[k], x0);
    if (x1) atomicOr(&wl[k + 1], x1);
    if (x2) atomicOr(&wl[k + 2], x2);
  }
  __syncthreads();
  const uint32_t total = tot & 0xFFFFu;
  if (total) {
    const uint64_t p0 = base_off[b];
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
