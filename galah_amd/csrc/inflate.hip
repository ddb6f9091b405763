// Device gzip inflate: gzip FASTA files go to the GPU compressed (PCIe and
// host memory carry ~1/3 of the text bytes, and the host threads only read
// files) and come out as the FASTA text parse.hip reads.  finch's
// sketch_files (src/finch.rs:47) reads .fna.gz through needletail / flate2;
// the host path (pack.cpp) decodes with libdeflate on the host threads.
//
// DEFLATE is serial within a stream, so the parallel units are the stream's
// blocks (zlib level 6: ~16k symbols, ~100 KB of FASTA each; a 3 Mbp genome
// has ~30 of them).  Kernels (inflate_core.hpp has the bit-level decoding):
//   inflate_search_kernel   one wave per ~4 KB chunk of compressed data: the
//                           first bit position where a dynamic block header
//                           parses (64 positions per step, one per lane)
//   inflate_decode_kernel   one wave per found start: each block's header
//                           by lane 0, its body split into 64 sub-spans
//                           decoded at once and chained by resynchronisation
//                           (inflate_core.hpp decode_span) into tokens, until
//                           landing on the next start
//   inflate_expand_kernel   one workgroup per segment, in order: token output
//                           offsets by a block scan, the bytes of each step
//                           built in LDS (back-references inside the segment
//                           copied, those before it left as pointers into
//                           the 32 KB before the segment): u16 per byte
//   inflate_resolve_kernel  one workgroup per gzip member, its segments in
//                           order: the member's last 32 KB of text in an LDS
//                           ring, so every pointer is one LDS read
//   inflate_crc_seg_kernel  CRC-32 of every 4 KB of text, one thread each
//   inflate_crc_fold_kernel per file its segments' CRCs folded with x^(8n)
//                           mod P; checked with ISIZE against the gzip
//                           trailer by the host
#include <cstdlib>
#include <cstring>

#include "device_util.hpp"
#include "gg_internal.hpp"
#include "inflate_core.hpp"

namespace gg {
namespace {

using namespace inflate;

// A lane's code-length code store (inflate_core.hpp ClCode) in LDS.
struct ClLds {
  int32_t b[kClBits + 1];
  uint8_t s[kClSyms + 1];
  uint8_t o[kClBits + 1];
  __device__ int32_t& base(int l) { return b[l]; }
  __device__ uint8_t& sym(int i) { return s[i]; }
  __device__ uint8_t& off(int l) { return o[l]; }
};

constexpr int kSearchWaves = 4;         // chunks per search workgroup (one wave each)
constexpr uint32_t kSearchStep = 4096;  // positions per step: 64 consecutive per lane
constexpr uint32_t kSearchCands = 256;  // candidates listed at most (more: the scan resumes after the last listed)
#ifndef GG_CHECK_AT  // (A/B builds: -DGG_CHECK_AT=...)
#define GG_CHECK_AT 48
#endif
constexpr uint32_t kCheckAt = GG_CHECK_AT;  // candidates that trigger a round of full checks (~1 per 1,100 positions)
#ifndef GG_CHECK_STEPS  // (A/B builds; 1,000 C2-like files: 1 step per round (round 5) 9.08 ms, 4 8.14, 8 7.91, 32 7.78)
#define GG_CHECK_STEPS 32
#endif
constexpr uint32_t kCheckSteps = GG_CHECK_STEPS;  // header-walk symbols per round of the checks' bookkeeping
constexpr uint32_t kWinWords = kSearchStep / 32 + 8;  // a step's bits plus the 160 after its first lane's last
#ifndef GG_CHK_LDS  // (A/B builds: -DGG_CHK_LDS=1, a round's stream copied to LDS first: search 7.7 -> 8.8-9.0 ms per 600 C2-like files)
#define GG_CHK_LDS 0
#endif
constexpr uint32_t kChkWords = GG_CHK_LDS ? 2048 : 1;  // the stream from a check round's first candidate on, in LDS (~48 candidates span ~1,700)

// The stream as a lane's full check reads it: words [wb, wb + nw) from the
// LDS copy (one coalesced copy per round), the rest (a walk that runs past
// it) from global memory, through a register window of three words that a
// walk moving on by a word shifts, loading the word after it -- which it
// needs a few symbols later -- so a code-length symbol waits on no stream
// read (a round of checks is one walk of a real header, ~300 dependent
// symbols long).
struct WinBits {
  const uint32_t* lds;
  const uint32_t* g;
  uint64_t wb;
  uint32_t nw;
  mutable uint64_t wi = ~0ull;  // the window's first word
  mutable uint32_t a = 0, b = 0, c = 0;
  __device__ uint32_t word(uint64_t w) const {
    const uint64_t i = w - wb;  // (w < wb wraps to the global read)
    return i < nw ? lds[i] : g[w];
  }
  __device__ uint32_t peek(uint64_t pos) const {
    const uint64_t w = pos >> 5;
    if (w != wi) {
      if (w == wi + 1) {
        a = b;
        b = c;
        c = word(w + 2);
      } else {
        a = word(w);
        b = word(w + 1);
        c = word(w + 2);
      }
      wi = w;
    }
    return __builtin_amdgcn_alignbit(b, a, (uint32_t)pos & 31u);
  }
};

// block_header_quick (inflate_core.hpp) for the 64 positions of a lane at
// once.  A[0..4]: the 160 stream bits from the lane's first position.  The
// header fields are tested as 64-bit masks over the positions (bit i of
// S(k) = stream bit i + k): BTYPE 10, HLIT and HDIST not 30 or 31; the ~22%
// of positions left get the code-length code's Kraft sum, by 7 lookups of 3
// fields in kraft3.
__device__ __forceinline__ uint64_t quick64(const uint32_t (&A)[5], const uint8_t* kraft3) {
  const uint64_t lo = (uint64_t)A[0] | ((uint64_t)A[1] << 32), hi = (uint64_t)A[2] | ((uint64_t)A[3] << 32);
  auto S = [&](int k) { return (lo >> k) | (hi << (64 - k)); };  // (1 <= k <= 12)
  uint64_t m = ~S(1) & S(2);
  m &= ~(S(4) & S(5) & S(6) & S(7));
  m &= ~(S(9) & S(10) & S(11) & S(12));
  uint64_t out = 0;
  while (m) {
    const uint32_t i = (uint32_t)__ffsll((unsigned long long)m) - 1u;
    m &= m - 1;
    // bits i + 13 .. i + 13 + 63 (HCLEN, then the code-length fields)
    const uint32_t o = i + 13, w = o >> 5, sh = o & 31u;
    const uint32_t a0 = w == 0 ? A[0] : w == 1 ? A[1] : A[2];
    const uint32_t a1 = w == 0 ? A[1] : w == 1 ? A[2] : A[3];
    const uint32_t a2 = w == 0 ? A[2] : w == 1 ? A[3] : A[4];
    const uint32_t y0 = __builtin_amdgcn_alignbit(a1, a0, sh), y1 = __builtin_amdgcn_alignbit(a2, a1, sh);
    const uint32_t hclen = (y0 & 15u) + 4u;
    uint64_t f = ((uint64_t)y0 >> 4) | ((uint64_t)y1 << 28);  // (60 bits valid)
    f &= (1ull << (3 * hclen)) - 1ull;  // (3 hclen <= 57)
    uint32_t kr = 0;
#pragma unroll
    for (int g = 0; g < 7; ++g) kr += kraft3[(uint32_t)(f >> (9 * g)) & 511u];
    if (kr == 128u) out |= 1ull << i;
  }
  return out;
}

// One wave per chunk, in steps of kSearchStep positions: the step's words
// staged in LDS, each lane filters its 64 consecutive positions from a
// 160-bit register window (quick64, ~0.1% pass) and the survivors are
// appended in order to the chunk's list in LDS.  The full checks
// (block_header_ok, one candidate per lane) run when the list is full or
// the chunk is done, so a step waits on no header walk; the first
// candidate that passes is the chunk's start.
__global__ __launch_bounds__(64 * kSearchWaves, 4) void inflate_search_kernel(InflateSearch a) {
  __shared__ uint64_t cand[kSearchWaves][kSearchCands];
  __shared__ uint32_t win[kSearchWaves][kWinWords];
  __shared__ uint32_t chk[kSearchWaves][kChkWords];
  __shared__ ClLds cls[kSearchWaves][64];
  __shared__ uint8_t kraft3[512];  // sum over 3 code-length fields of 128 >> len (0 for len 0)
  for (uint32_t i = threadIdx.x; i < 512; i += 64 * kSearchWaves) {
    uint32_t k = 0;
    for (int j = 0; j < 3; ++j) {
      const uint32_t l = (i >> (3 * j)) & 7u;
      k += l ? 128u >> l : 0u;
    }
    kraft3[i] = (uint8_t)k;
  }
  __syncthreads();
  const uint32_t wv = threadIdx.x >> 6;
  const uint32_t c = blockIdx.x * kSearchWaves + wv;
  const uint32_t lane = threadIdx.x & 63u;
  if (c >= a.n_chunks) return;
  uint64_t* cw = cand[wv];
  uint32_t* ww = win[wv];
  ClLds& cl = cls[wv][lane];
  const uint32_t f = a.chunk_file[c];
  const uint32_t* stream = a.in + a.file_word[f];
  const uint64_t b0 = a.chunk_bit0[c];
  const uint64_t b1 = min(b0 + (uint64_t)a.chunk_bits, a.file_bits[f]);
  // words a position before b1 can touch in the filter (its 128 bits; the
  // file's trailer or the batch's padding follows its deflate data)
  const uint64_t wend = (a.file_bits[f] + 31) / 32 + 5;
  uint64_t found = ~0ull;
  uint32_t nc = 0;  // candidates listed, not yet checked (uniform)
  uint64_t tp = a.prof ? clock64() : 0;
  auto phase = [&](int k) {  // (GALAHGPU_INFLATE_DEBUG: cycles per phase)
    if (a.prof) {
      const uint64_t t = clock64();
      if (lane == 0) {
        atomicAdd((unsigned long long*)&a.prof[k], (unsigned long long)(t - tp));
        atomicAdd((unsigned long long*)&a.prof[k + 2], 1ull);
      }
      tp = t;
    }
  };
  for (uint64_t s0 = b0; found == ~0ull;) {  // (uniform per wave)
    if (s0 < b1) {
      const uint64_t s1 = min(s0 + kSearchStep, b1);
      const uint64_t w0 = s0 >> 5;
      for (uint32_t i = lane; i < kWinWords; i += 64) ww[i] = w0 + i < wend ? stream[w0 + i] : 0u;
      __builtin_amdgcn_wave_barrier();
      // this lane's positions s0 + 64 lane + [0, 64)
      const uint32_t q0 = (uint32_t)(s0 & 31u) + 64u * lane;
      uint32_t A[5];
      {
        uint32_t W[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) W[k] = ww[(q0 >> 5) + k];
#pragma unroll
        for (int k = 0; k < 5; ++k) A[k] = __builtin_amdgcn_alignbit(W[k + 1], W[k], q0 & 31u);
      }
      uint64_t m = quick64(A, kraft3);
      const uint64_t p0 = s0 + 64ull * lane;
      if (p0 >= s1) m = 0;
      else if (s1 - p0 < 64) m &= (1ull << (s1 - p0)) - 1ull;
      // candidates in position order: lane-major
      const uint32_t cnt = (uint32_t)__popcll(m);
      uint32_t incl = cnt;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (lane >= (uint32_t)o) incl += y;
      }
      const uint32_t total = __shfl(incl, 63);
      uint32_t k = nc + incl - cnt;
      while (m && k < kSearchCands) {
        cw[k++] = p0 + (uint32_t)__ffsll((unsigned long long)m) - 1u;
        m &= m - 1;
      }
      __builtin_amdgcn_wave_barrier();
      if (nc + total > kSearchCands) {  // the list is full: the next step starts after its last candidate
        nc = kSearchCands;
        s0 = cw[kSearchCands - 1] + 1;
      } else {
        nc += total;
        s0 = s1;
      }
      phase(0);
      if (nc < kCheckAt && s0 < b1) continue;  // (check in groups: a start found early ends the scan)
    }
    // the full checks of the listed candidates, in order
    if (a.prof && lane == 0) atomicAdd((unsigned long long*)&a.prof[4], (unsigned long long)nc);
    WinBits wbits{chk[wv], stream, 0, 0};
    if (GG_CHK_LDS && nc) {  // the stream from the first candidate on into LDS (the words the filter may read: up to wend)
      wbits.wb = cw[0] >> 5;
      wbits.nw = wend > wbits.wb ? (uint32_t)min<uint64_t>(kChkWords, wend - wbits.wb) : 0u;
      for (uint32_t i = lane; i < wbits.nw; i += 64) chk[wv][i] = stream[wbits.wb + i];
      __builtin_amdgcn_wave_barrier();
    }
    // (each lane walks one candidate a symbol per step and takes the next
    // unclaimed one when its own is decided; done when a candidate passed
    // and none before it is still walking, or all are decided)
    {
      HeaderWalk hw;
      int mine = -1;          // the candidate this lane walks
      uint32_t next = 0;      // candidates claimed (uniform)
      uint32_t best = nc;     // the first that passed (uniform)
      for (;;) {
        const bool need = mine < 0;
        const uint64_t nm = __ballot(need);
        const uint32_t lim = min(nc, best);
        if (need) {
          const uint32_t k = next + (uint32_t)__popcll(nm & ((1ull << lane) - 1ull));
          if (k < lim) mine = hw.start(wbits, cw[k], cl) ? (int)k : -1;  // (rejected at once: the lane claims again)
        }
        next = min(lim, next + (uint32_t)__popcll(nm));
        int r = 0;
        // (up to kCheckSteps symbols per round of the wave's bookkeeping: the
        // claims, ballots and the minimum below cost more than a step, and
        // near a round's end one lane walks a real header alone)
        for (uint32_t q = 0; q < kCheckSteps && mine >= 0 && r == 0; ++q) r = hw.step(wbits, cl);
        const uint64_t pm = __ballot(r == 1);
        if (pm) {
          uint32_t b = r == 1 ? (uint32_t)mine : ~0u;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) b = min(b, (uint32_t)__shfl_xor(b, o));
          best = min(best, b);
        }
        if (r != 0) mine = -1;
        const bool pending = mine >= 0 && (uint32_t)mine < best;
        if (!__ballot(pending) && next >= min(nc, best)) break;
      }
      if (best < nc) found = cw[best];
    }
    __builtin_amdgcn_wave_barrier();
    phase(1);
    nc = 0;
    if (s0 >= b1) break;
  }
  if (lane == 0) a.start[c] = found;
}

struct LdsStore {
  uint32_t* ll;
  uint32_t* dl;
  int32_t* lb;
  int32_t* db;
  uint32_t* lc;
  uint32_t* dc;
  uint16_t* ls;
  uint8_t* ds;
  uint32_t* lf;
  uint32_t* df;
  __device__ uint32_t& lfast(int i) { return lf[i]; }
  __device__ uint32_t& dfast(int i) { return df[i]; }
  __device__ uint32_t& llim(int l) { return ll[l]; }
  __device__ uint32_t& dlim(int l) { return dl[l]; }
  __device__ int32_t& lbase(int l) { return lb[l]; }
  __device__ int32_t& dbase(int l) { return db[l]; }
  __device__ uint32_t& lcnt(int l) { return lc[l]; }
  __device__ uint32_t& dcnt(int l) { return dc[l]; }
  __device__ uint16_t& lsym(int i) { return ls[i]; }
  __device__ uint8_t& dsym(int i) { return ds[i]; }
};

constexpr uint32_t kSpanLanes = 64;  // one wave per segment, one sub-span per lane

// A lane's tokens to its scratch area, interleaved with the wave's other
// lanes (token k of lane j at p[64 k], p = the area + j): the wave's k-th
// tokens share cache lines, so a store instruction writes a few whole lines
// instead of a 16-byte piece of 64 lines, which the L2 evicted half written
// (round 5: the decode moved 6.1x its bytes), and the copy-out's loads are
// coalesced the same way.
// Tokens before `on` is set (a first decode's, before its first checkpoint:
// they are dropped) keep their index but are not stored.
struct TokSink {
  uint32_t* p;
  uint32_t cap;
  bool on;
  uint32_t k = 0;
  __device__ bool operator()(uint32_t tk) {
    if (k >= cap) return false;
    if (on) p[(size_t)k * kSpanLanes] = tk;
    ++k;
    return true;
  }
  __device__ void flush() {}
};

// A block's header read by the whole wave.  Lane 0 parses the fields and
// walks the code lengths (SeqBits) into LDS (lens); then every lane counts
// them per length by ballots, builds the canonical limits in its registers
// (tab.s.llim / dlim) and the bases, and the symbols sorted by (length, value)
// are placed in the LDS tables by ballot ranks.  Returns btype (0 stored,
// 1 fixed, 2 dynamic) or -1 for a header zlib refuses (inflate_core.hpp
// read_block_header, the same checks).
struct HeaderLds {
  uint8_t lens[kLitSyms + kDistSyms];
  uint64_t body0;
  uint32_t stored, bfinal, hlit, hdist;
  int32_t bt;
};
__device__ int wave_header(const Bits& in, uint64_t pos, LaneTables<LdsStore>& tab, ClLds& hcl, HeaderLds& H,
                           uint32_t lane) {
  for (uint32_t i = lane; i < (uint32_t)(kLitSyms + kDistSyms); i += 64) H.lens[i] = 0;
  __syncthreads();
  if (lane == 0) {
    const uint32_t h = in.peek(pos);
    int bt = (int)((h >> 1) & 3u);
    H.bfinal = h & 1u;
    H.stored = 0;
    if (bt == 0) {
      uint64_t q = (pos + 3 + 7) & ~7ull;
      const uint32_t v = in.peek(q);
      if (((v & 0xFFFFu) ^ (v >> 16)) != 0xFFFFu) bt = -1;
      H.stored = v & 0xFFFFu;
      H.body0 = q + 32;
    } else if (bt == 1) {  // fixed codes (RFC 1951 3.2.6)
      for (uint32_t i = 0; i < 288; ++i) H.lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
      for (uint32_t i = 0; i < 32; ++i) H.lens[288 + i] = 5;
      H.hlit = 288;
      H.hdist = 32;
      H.body0 = pos + 3;
    } else if (bt == 2) {
      const uint32_t hlit = ((h >> 3) & 31u) + 257u, hdist = ((h >> 8) & 31u) + 1u, hclen = ((h >> 13) & 15u) + 4u;
      H.hlit = hlit;
      H.hdist = hdist;
      SeqBits sb{Cursor{in.w}};
      sb.c.seek(pos);
      uint64_t p = pos + 17;
      ClCode cl;
      if (hlit > 286 || hdist > 30 || !read_cl_code(sb, p, hclen, cl, hcl) ||
          !walk_lengths(sb, p, cl, hcl, hlit + hdist, [&](uint32_t i, uint32_t len) {
            H.lens[i] = (uint8_t)len;
            return true;
          }))
        bt = -1;
      H.body0 = p;
    } else {
      bt = -1;
      H.body0 = pos;
    }
    H.bt = bt;
  }
  __syncthreads();
  const int bt = H.bt;
  if (bt <= 0) return bt;
  const uint32_t hlit = H.hlit, hdist = H.hdist;
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t lc[kMaxBits + 1], dc[kMaxBits + 1];
#pragma unroll
  for (int l = 0; l <= kMaxBits; ++l) lc[l] = dc[l] = 0;
  const uint32_t dlen = lane < hdist ? H.lens[hlit + lane] : 0u;
  for (uint32_t c0 = 0; c0 < hlit; c0 += 64) {
    const uint32_t len = c0 + lane < hlit ? H.lens[c0 + lane] : 0u;
#pragma unroll
    for (int l = 1; l <= kMaxBits; ++l) lc[l] += (uint32_t)__popcll(__ballot(len == (uint32_t)l));
  }
#pragma unroll
  for (int l = 1; l <= kMaxBits; ++l) dc[l] = (uint32_t)__popcll(__ballot(dlen == (uint32_t)l));
  if (H.lens[256] == 0) return -1;  // no end-of-block code
  Canon c{};
  int ml = 0;
  int r = canon_from_counts(lc, c, ml);
  if (!code_ok(r, ml, false)) return -1;
  tab.set_lit(c);
  r = canon_from_counts(dc, c, ml);
  if (!code_ok(r, ml, true)) return -1;
  tab.set_dist(c);
  // symbols sorted by (length, value): slot = first of its length + its rank
  uint32_t off[kMaxBits + 1];
  uint32_t a = 0;
#pragma unroll
  for (int l = 1; l <= kMaxBits; ++l) {
    off[l] = a;
    a += lc[l];
  }
  for (uint32_t c0 = 0; c0 < hlit; c0 += 64) {
    const uint32_t len = c0 + lane < hlit ? H.lens[c0 + lane] : 0u;
#pragma unroll
    for (int l = 1; l <= kMaxBits; ++l) {
      const uint64_t m = __ballot(len == (uint32_t)l);
      if (len == (uint32_t)l) tab.s.lsym((int)(off[l] + (uint32_t)__popcll(m & lt))) = (uint16_t)(c0 + lane);
      off[l] += (uint32_t)__popcll(m);
    }
  }
  a = 0;
#pragma unroll
  for (int l = 1; l <= kMaxBits; ++l) {
    const uint64_t m = __ballot(dlen == (uint32_t)l);
    if (dlen == (uint32_t)l) tab.s.dsym((int)(a + (uint32_t)__popcll(m & lt))) = (uint8_t)lane;
    a += (uint32_t)__popcll(m);
  }
  __syncthreads();
  for (uint32_t i = lane; i < kFastSize; i += 64) {  // the one-lookup tables of the short codes
    tab.s.lfast((int)i) = tab.fast_entry(i, false);
    tab.s.dfast((int)i) = tab.fast_entry(i, true);
  }
  __syncthreads();
  return bt;
}

// The stream read forward from the staged segment in LDS (the staged
// decode): positions are bit offsets from the staged word 0; the window is
// the three words from the current one (a peek64 at any bit offset), and the
// two words after them are read from LDS as a symbol starts, so the rotation
// after its advance (at most 48 bits: 0, 1 or 2 words) waits on no load.
struct LdsCursor {
  const uint32_t* w;  // LDS
  uint32_t pos, wi;
  uint32_t a, b, c;    // w[wi], w[wi + 1], w[wi + 2]
  __device__ void seek(uint32_t p) {
    pos = p;
    wi = p >> 5;
    a = w[wi];
    b = w[wi + 1];
    c = w[wi + 2];
  }
  __device__ uint32_t peek() const { return __builtin_amdgcn_alignbit(b, a, pos & 31u); }
  __device__ uint64_t peek64() const {
    const uint32_t sh = pos & 31u;
    return (uint64_t)__builtin_amdgcn_alignbit(b, a, sh) | ((uint64_t)__builtin_amdgcn_alignbit(c, b, sh) << 32);
  }
  // advance by n <= 48 bits, with x = w[wi + 3], y = w[wi + 4] read beforehand
  __device__ void advance(uint32_t n, uint32_t x, uint32_t y) {
    pos += n;
    const uint32_t d = (pos >> 5) - wi;
    // (masks, not selects: a select chain over the three words became an
    // indexed load from a stack copy of them)
    const uint32_t m1 = 0u - (uint32_t)(d >= 1), m2 = 0u - (uint32_t)(d >= 2);
    const uint32_t na = (a & ~m1) | (((b & ~m2) | (c & m2)) & m1);
    const uint32_t nb = (b & ~m1) | (((c & ~m2) | (x & m2)) & m1);
    const uint32_t nc = (c & ~m1) | (((x & ~m2) | (y & m2)) & m1);
    a = na;
    b = nb;
    c = nc;
    wi += d;
  }
  __device__ void skip(uint32_t n) { advance(n, w[wi + 3], w[wi + 4]); }  // (the slow paths)
  __device__ uint32_t get(uint32_t n) {
    const uint32_t v = peek() & ((1u << n) - 1u);
    skip(n);
    return v;
  }
};

// decode_span (inflate_core.hpp) for the staged decode, the same tokens,
// checkpoints, status and stop: positions relative to the staged word 0
// (start, s_nom, range_end and stop are file bit positions, base = the
// staged word 0's).  A symbol whose codes are all in the one-lookup tables
// (nearly every one) is decoded without a branch: both the literal and the
// match reading are computed (the distance lookup happens for a literal
// too) and the right one selected, so the lanes of a wave do not split on
// the symbol kind; the rest (long codes, end-of-block, invalid codes) take
// decode_span's own handling.
// kFlat (the first decode): ck is called on every symbol as ck(k, c, hit)
// and records checkpoint k only when hit; k and the next checkpoint move on
// by selects.  (With 64 lanes some lane reaches a checkpoint on nearly every
// symbol, so the branch form ran its body, and its exec-mask work, on nearly
// every symbol anyway.)
template <bool kFlat = false, class Emit, class Ck>
__device__ __forceinline__ uint32_t decode_span_lds(const uint32_t* lds, uint64_t base, uint64_t start, uint64_t s_nom,
                                    uint64_t range_end, LaneTables<LdsStore>& t, Emit&& emit, Ck&& ck, uint32_t& n,
                                    uint64_t& stop) {
  LdsCursor cur{lds};
  cur.seek((uint32_t)(start - base));
  n = 0;
  uint32_t k = 0;
  uint32_t next_ck = (uint32_t)(s_nom - base);
  const uint32_t rend = (uint32_t)(range_end - base);
  uint32_t next_stop = next_ck < rend ? next_ck : rend;
  uint32_t st = kSpanBad;
  for (;;) {
    if constexpr (kFlat) {
      if (cur.pos >= rend) {
        st = kSpanRange;
        break;
      }
      const bool hit = cur.pos >= next_ck;
      ck(k, (uint32_t)ck_pack(cur.pos - next_ck, n, 0), hit);
      k += hit ? 1u : 0u;
      next_ck += hit ? kCkBits : 0u;
    } else if (cur.pos >= next_stop) {
      if (cur.pos >= rend) {
        st = kSpanRange;
        break;
      }
      if (cur.pos >= next_ck) {
        if (!ck(k, ck_pack(cur.pos - next_ck, n, 0))) {
          st = kSpanSynced;
          break;
        }
        ++k;
        next_ck += kCkBits;
      }
      next_stop = next_ck < rend ? next_ck : rend;
    }
    const uint32_t x = cur.w[cur.wi + 3], y = cur.w[cur.wi + 4];  // (the words the advance may bring in)
    const uint64_t bb = cur.peek64();
    const uint32_t lo = (uint32_t)bb, hi = (uint32_t)(bb >> 32);
    const uint32_t e = t.s.lfast((int)(lo & (kFastSize - 1)));
    const uint32_t l1 = (e >> kFastLenShift) & 15u, lx = entry_extra(e);
    const uint32_t lenv = entry_value(e) + (__builtin_amdgcn_alignbit(hi, lo, l1) & ((1u << lx) - 1u));
    const uint32_t u = l1 + lx;  // (<= 15)
    const uint32_t de = t.s.dfast((int)(__builtin_amdgcn_alignbit(hi, lo, u) & (kFastSize - 1)));
    const uint32_t dl = (de >> kFastLenShift) & 15u, dx = entry_extra(de);
    const uint32_t distv = entry_value(de) + (__builtin_amdgcn_alignbit(hi, lo, u + dl) & ((1u << dx) - 1u));
    const uint32_t kind = entry_kind(e);
    const bool lit = kind == kEntryLit && l1 != 0;
    const bool mat = kind == kEntryLen && l1 != 0 && dl != 0 && entry_kind(de) == kEntryLen;
    if (lit || mat) {  // (the advance and the token by selects: one path for both kinds)
      const uint32_t adv = lit ? l1 : u + dl + dx;
      const uint32_t tk = lit ? entry_value(e) : tok_match(lenv, distv);
      cur.advance(adv, x, y);
      if (!emit(tk)) break;
      ++n;
      continue;
    }
    // decode_span's handling of the other symbols
    uint32_t used = l1;
    if (used == 0) {  // a long lit/len code
      const uint32_t e2 = t.lit_entry(cur);
      if (entry_kind(e2) != kEntryLen) {
        if (entry_kind(e2) == kEntryLit) {
          if (!emit(entry_value(e2))) break;
          ++n;
          continue;
        }
        if (entry_kind(e2) == kEntryEob) st = kSpanEob;
        break;
      }
      const uint32_t len = entry_value(e2) + cur.get(entry_extra(e2));
      const uint32_t d2 = t.dist_entry(cur);
      if (entry_kind(d2) != kEntryLen) break;
      const uint32_t dist = entry_value(d2) + cur.get(entry_extra(d2));
      if (!emit(tok_match(len, dist))) break;
      ++n;
      continue;
    }
    if (kind != kEntryLen) {  // end-of-block or an invalid code (a literal took the fast path)
      cur.skip(used);
      if (kind == kEntryEob) st = kSpanEob;
      break;
    }
    used += lx;
    if (dl == 0) {  // a long distance code
      cur.skip(used);
      const uint32_t d2 = t.dist_entry(cur);
      if (entry_kind(d2) != kEntryLen) break;
      const uint32_t dist = entry_value(d2) + cur.get(entry_extra(d2));
      if (!emit(tok_match(lenv, dist))) break;
      ++n;
      continue;
    }
    cur.skip(used + dl);  // an invalid distance code
    break;
  }
  stop = base + cur.pos;
  return st;
}

// n tokens from a lane's scratch (stride kSpanLanes: TokSink) to the
// segment's tokens, kCopyBatch loads in flight (a plain loop waited on each
// load in turn; with 8 in flight a window's ~85 tokens per lane still took
// ~11 waits: 16% of the decode)
#ifndef GG_COPY_BATCH  // (A/B builds: -DGG_COPY_BATCH=8)
#define GG_COPY_BATCH 32
#endif
constexpr uint32_t kCopyBatch = GG_COPY_BATCH;
// Returns the bytes the tokens stand for (the decodes count no bytes).
__device__ uint32_t copy_tokens(uint32_t* __restrict__ dst, const uint32_t* __restrict__ src, uint32_t n) {
  uint32_t i = 0, bytes = 0;
  for (; i + kCopyBatch <= n; i += kCopyBatch) {
    uint32_t v[kCopyBatch];
#pragma unroll
    for (uint32_t k = 0; k < kCopyBatch; ++k) v[k] = src[(size_t)(i + k) * kSpanLanes];
#pragma unroll
    for (uint32_t k = 0; k < kCopyBatch; ++k) {
      dst[i + k] = v[k];
      bytes += tok_len(v[k]);
    }
  }
  // the rest: all loads first, then the stores
  uint32_t v[kCopyBatch];
#pragma unroll
  for (uint32_t k = 0; k < kCopyBatch; ++k)
    if (i + k < n) v[k] = src[(size_t)(i + k) * kSpanLanes];
#pragma unroll
  for (uint32_t k = 0; k < kCopyBatch; ++k)
    if (i + k < n) {
      dst[i + k] = v[k];
      bytes += tok_len(v[k]);
    }
  return bytes;
}

// One wave per segment (a found block start up to the next one).  Per block:
// lane 0 reads the header into the wave's LDS tables; the body is split into
// up to 64 sub-spans decoded at once, each lane from the start of its span
// (usually inside a symbol) into its own scratch, recording checkpoints
// (inflate_core.hpp decode_span).  A lane whose first checkpoint is not the
// symbol start the lane before ended on decodes again from there until one
// of its checkpoints agrees with the first decode.  The right spans up to
// the one that decoded end-of-block are the block; their tokens are copied
// to the segment's tokens.
//
// Staged form (kStaged, the lanes [0, n_staged)): at each block start the
// compressed words from there are copied into LDS by the whole wave
// (coalesced, one wait; at most kStageWords: a longer body is decoded in
// windows, the next starting at the last lane's end with the same tables),
// so the header walk, the sub-span decodes and their cursor refills read LDS
// only.  Read from global memory, every cursor refill waited for its load
// (the window rotation copies the loaded registers at once), a latency of
// thousands of cycles every ~2.5 symbols.
#ifndef GG_DECODE_MIN_WAVES
#define GG_DECODE_MIN_WAVES 1
#endif
// (10 KB + the static tables ~10 KB: eight waves per CU, two per SIMD as the
// 174 VGPRs allow; a zlib -6 block of FASTA, 24-27 KB, takes three windows.
// C2 files per call: 30 KB stages (one wave per SIMD) 0.063-0.064 s, 18 KB
// 0.063-0.064, 14 KB 0.061-0.063, 10 KB 0.060-0.061.  A/B builds:
// scripts/ab_lib.sh ... -DGG_STAGE_KB=14)
#ifndef GG_STAGE_KB
#define GG_STAGE_KB 10
#endif
constexpr uint32_t kStageWords = GG_STAGE_KB * 1024 / 4;
#ifndef GG_CK_FLAT  // (A/B builds: -DGG_CK_FLAT=0, the first decode's checkpoints behind a branch)
#define GG_CK_FLAT 1
#endif
template <bool kStaged>
__global__ __launch_bounds__(kSpanLanes, GG_DECODE_MIN_WAVES) void inflate_decode_kernel(InflateDecode a) {
  extern __shared__ uint32_t stage[];  // (kStaged: kStageWords words)
  __shared__ uint32_t llm[kMaxBits + 1], dlm[kMaxBits + 1];
  __shared__ int32_t lb[kMaxBits + 1], db[kMaxBits + 1];
  __shared__ uint32_t lcn[kMaxBits + 1], dcn[kMaxBits + 1];
  __shared__ ClLds hcl;  // (lane 0's, while it reads a header)
  __shared__ HeaderLds H;
  __shared__ uint16_t ls[kLitSyms];
  __shared__ uint8_t ds[kDistSyms];
  __shared__ uint32_t lf[kFastSize], df[kFastSize];
  __shared__ uint64_t sE[kSpanLanes];
  __shared__ uint32_t sSt[kSpanLanes];
  const uint32_t j = threadIdx.x;
  const uint32_t seg = blockIdx.x + (kStaged ? 0u : a.n_staged);
  if (seg >= a.n_lanes || (kStaged && seg >= a.n_staged)) return;
  LaneTables<LdsStore> tab;
  tab.s = LdsStore{llm, dlm, lb, db, lcn, dcn, ls, ds, lf, df};
  const uint32_t f = a.lane_file[seg];
  const uint32_t* gin = a.in + a.file_word[f];
  const uint64_t limit = a.file_bits[f];
  const uint64_t end = a.lane_end[seg];  // ~0: the file's last segment (ends with the BFINAL block)
  const bool final_seg = end == ~0ull;
  Bits in{gin};
  const uint64_t seg_end = final_seg ? limit : end;
  uint64_t sbase = 0;   // (kStaged: the file bit position of stage[0])
  uint64_t slimit = 0;  // (kStaged: lanes decode up to here; their look-ahead stays in the stage)
  // (kStaged) the file's words from bit b on into LDS, at most kStageWords
  // and no further than the segment's words; `in` reads them at their file
  // positions
  auto restage = [&](uint64_t b) {
    const uint64_t w0 = b >> 5;
    const uint32_t nw = (uint32_t)min<uint64_t>(a.stage_words ? a.stage_words : kStageWords,
                                                  inflate_segment_words(b, seg_end));
    __syncthreads();  // (every lane is done with the stage before)
    for (uint32_t i = j; i < nw; i += kSpanLanes) stage[i] = gin[w0 + i];
    __syncthreads();
    in.w = stage - w0;  // (only words [w0, w0 + nw) are read)
    sbase = w0 * 32;
    slimit = min(seg_end, sbase + (uint64_t)(nw - 8) * 32);
  };
  const uint64_t t_wave = a.prof ? wall_clock64() : 0;  // (debug: the wave's wall time, for the tail)
  uint32_t* out = a.tok + a.tok_off[seg];
  const uint64_t cap = a.tok_cap[seg];
  uint32_t* scr_all = a.scr + a.scr_off[seg];
  uint64_t pos = a.lane_start[seg];  // (uniform)
  uint64_t n_out = 0, out_bytes = 0;
  uint32_t status = kDecOk, fin = 0;
  for (;;) {
    const uint64_t blk0 = pos;  // (this block's start)
    const uint64_t n_out0 = n_out, out_bytes0 = out_bytes;  // (the tokens and bytes before it)
    if (pos == end) {
      status = kDecOk;
      break;
    }
    if (pos > end || pos >= limit) {
      status = kDecOverrun;
      break;
    }
    uint64_t tp = a.prof ? clock64() : 0;  // (GALAHGPU_INFLATE_DEBUG: cycles per phase)
    auto phase = [&](int k) {
      if (a.prof) {
        const uint64_t t = clock64();
        if (j == 0) atomicAdd((unsigned long long*)&a.prof[k], (unsigned long long)(t - tp));
        tp = t;
      }
    };
    if constexpr (kStaged) restage(pos);  // (the header and the body's first window)
    const int bt = wave_header(in, pos, tab, hcl, H, j);
    phase(0);
    const uint32_t bfinal = H.bfinal;
    const uint64_t body0 = H.body0;
    if (bt < 0) {
      status = kDecBad;
      pos = body0;
      break;
    }
    if (bt == 0) {  // stored: its bytes as literal tokens
      const uint64_t stl = H.stored;
      if (body0 + 8 * stl > limit) {
        status = kDecBad;
        break;
      }
      if (n_out + stl > cap) {
        status = kDecFull;
        break;
      }
      const uint8_t* src = (const uint8_t*)gin + body0 / 8;  // (global: a stored block may pass the stage)
      for (uint64_t i = j; i < stl; i += kSpanLanes) out[n_out + i] = src[i];
      n_out += stl;
      out_bytes += stl;
      pos = body0 + 8 * stl;
    } else {
      const uint64_t span_end = seg_end;
      // windows of the body: staged, what the LDS stage holds (a body that
      // runs past it continues from the last lane's end, a symbol start,
      // with the same tables); global, the whole span at once
      uint64_t bstart = body0;
      bool more = true, stop_blk = false;
      while (more) {
      more = false;
      const uint64_t wend = kStaged ? slimit : span_end;
      uint64_t L;
      uint32_t nsub;
      span_layout(bstart, wend, kSpanLanes, L, nsub);
      const bool act = j < nsub;
      const uint64_t S = bstart + j * L;
      const uint64_t R = j + 1 == nsub ? wend : S + L;
      const uint64_t capL = span_cap(L, a.tight), ncks = span_cks(L);
      // the wave's areas, each lane's entries interleaved (stride kSpanLanes)
      uint32_t* A = scr_all + j;                                   // first decode
      uint32_t* B = scr_all + kSpanLanes * capL + j;               // second decode
      uint32_t* ck = scr_all + 2 * kSpanLanes * capL + j;  // the first decode's checkpoints (ck_pack's low word)
#define CK(k) ck[(size_t)(k) * kSpanLanes]
      // the first decode, from S
      uint32_t na = 0, nck = 0, sa = kSpanRange;
      uint64_t Ea = S;
      if (act) {
        TokSink sink{A, (uint32_t)capL, false};
        auto ck1 = [&](uint32_t k, uint64_t c) {
          if (k < ncks) {
            CK(k) = (uint32_t)c;
            nck = k + 1;
          }
          sink.on = true;  // (from the first checkpoint on the tokens are kept)
          return true;
        };
        auto ck1f = [&](uint32_t k, uint32_t c, bool hit) {  // (the same, as decode_span_lds<true> calls it)
          const bool rec = hit && k < ncks;
          if (rec) CK(k) = c;
          nck = rec ? k + 1 : nck;
          sink.on |= hit;
        };
        // (a lane after the first starts kWarmBits early, so that its decode
        // has most likely fallen into step with the true symbols by S and its
        // first checkpoint agrees with the lane before: fewer second decodes,
        // whose longest kept the whole wave waiting; its tokens before the
        // first checkpoint are dropped as before)
        const uint64_t S0 = j == 0 ? S : (S - bstart > kWarmBits ? S - kWarmBits : bstart);
        uint64_t unused_bytes = 0;
#if GG_CK_FLAT
        if constexpr (kStaged) sa = decode_span_lds<true>(stage, sbase, S0, S, R, tab, sink, ck1f, na, Ea);
#else
        if constexpr (kStaged) sa = decode_span_lds(stage, sbase, S0, S, R, tab, sink, ck1, na, Ea);
#endif
        else sa = decode_span(in, S0, S, R, tab, sink, ck1, na, unused_bytes, Ea);
        sink.flush();
      }
      phase(1);
      uint64_t first = act && nck ? S + ck_off(CK(0)) : ~0ull;
      bool redone = false;
      int synced = -1;
      uint32_t nb = 0, sb = kSpanRange;
      uint64_t Eb = 0;
      uint32_t c_end = 0;
      bool overrun = false;
      for (;;) {
        const uint64_t E = redone && synced < 0 ? Eb : Ea;
        const uint32_t st = redone && synced < 0 ? sb : sa;
        sE[j] = E;
        sSt[j] = st;
        __syncthreads();
        const uint64_t eprev = j ? sE[j - 1] : 0;
        const uint32_t sprev = j ? sSt[j - 1] : kSpanRange;
        const bool ok = act && (j == 0 || (sprev == kSpanRange && first == eprev));
        const uint64_t okb = __ballot(ok), termb = __ballot(act && st != kSpanRange);
        const uint64_t vmask = nsub >= 64 ? ~0ull : (1ull << nsub) - 1ull;
        const uint64_t notok = ~okb & vmask;
        const uint32_t c = notok ? (uint32_t)__ffsll((unsigned long long)notok) - 1u : 64u;
        const uint32_t t = termb ? (uint32_t)__ffsll((unsigned long long)termb) - 1u : 64u;
        if (t < c) {  // the chain of right spans ends with span t's end-of-block (or bad code)
          c_end = t;
          break;
        }
        if (c >= nsub) {  // every span right, none ended the block: it runs past the window
          overrun = wend == span_end;  // (past the segment: not a block boundary; else the next window)
          more = !overrun;
          c_end = nsub - 1;
          break;
        }
        __syncthreads();  // (sE / sSt read before the next round writes them)
        if (act && j >= c && !ok && sprev == kSpanRange) {
          // the second decode, from the true start, until a checkpoint agrees
          redone = true;
          synced = -1;
          first = eprev;
          TokSink sink{B, (uint32_t)capL, true};
          auto ck2 = [&](uint32_t k, uint64_t cc) {
            if (k < nck && ck_off(cc) == ck_off(CK(k))) {
              synced = (int)k;
              return false;
            }
            return true;
          };
          uint64_t unused_bytes = 0;
          if constexpr (kStaged) sb = decode_span_lds(stage, sbase, eprev, S, R, tab, sink, ck2, nb, Eb);
          else sb = decode_span(in, eprev, S, R, tab, sink, ck2, nb, unused_bytes, Eb);
          sink.flush();
        }
      }
      const uint64_t e_end = sE[c_end];
      const uint32_t st_end = sSt[c_end];
      if (overrun) {  // (the host decodes again from this block's start, the tokens before it kept)
        // a block decoded in windows has its earlier windows' tokens counted
        // already: they are dropped with the block (kept, the host's redo
        // from blk0 appended them a second time)
        status = kDecOverrun;
        pos = blk0;
        n_out = n_out0;
        out_bytes = out_bytes0;
        stop_blk = true;
        break;
      }
      if (st_end == kSpanBad) {
        status = kDecBad;
        pos = e_end;
        stop_blk = true;
        break;
      }
      phase(2);
      // this span's tokens: [p1, p1 + n1) then [p2, p2 + n2)
      const uint32_t* p1 = A;
      const uint32_t* p2 = A;
      uint32_t n1 = 0, n2 = 0;
      if (j <= c_end) {
        if (!redone) {
          const uint32_t c0 = CK(0);
          p1 = A + (size_t)ck_tok(c0) * kSpanLanes;
          n1 = na - ck_tok(c0);
        } else {
          p1 = B;
          n1 = nb;
          if (synced >= 0) {
            const uint32_t ck_s = CK(synced);
            p2 = A + (size_t)ck_tok(ck_s) * kSpanLanes;
            n2 = na - ck_tok(ck_s);
          }
        }
      }
      const uint32_t valid = n1 + n2;
      uint32_t incl = valid;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o);
        if (j >= (uint32_t)o) incl += y;
      }
      const uint32_t total = __shfl(incl, 63);
      if (n_out + total > cap) {
        status = kDecFull;
        stop_blk = true;
        break;
      }
      uint32_t* dst = out + n_out + (incl - valid);
      uint64_t tb = copy_tokens(dst, p1, n1);  // (the bytes they stand for: the decodes count none)
      tb += copy_tokens(dst + n1, p2, n2);
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) tb += __shfl_xor(tb, o);
#undef CK
      phase(3);
      if (a.prof && j == 0) {
        atomicAdd((unsigned long long*)&a.prof[4], 1ull);
        atomicAdd((unsigned long long*)&a.prof[5], (unsigned long long)total);
      }
      n_out += total;
      out_bytes += tb;
      pos = e_end;
      __syncthreads();  // (the LDS tables and spans are rewritten for the next block or window)
      if (more) {
        bstart = e_end;
        if constexpr (kStaged) restage(bstart);
      }
      }  // (windows)
      if (stop_blk) break;
    }
    if (bfinal) {
      fin = 1;
      status = final_seg ? kDecOk : kDecFinalEarly;
      break;
    }
  }
  if (a.prof && j == 0) {
    const uint64_t dt = wall_clock64() - t_wave;
    atomicMax((unsigned long long*)&a.prof[6], (unsigned long long)dt);
    atomicAdd((unsigned long long*)&a.prof[7], (unsigned long long)dt);
  }
  if (j == 0) {
    a.status[seg] = status;
    a.n_tok[seg] = n_out;
    a.out_len[seg] = out_bytes;
    a.last_end[seg] = pos;
    a.bfinal[seg] = fin;
  }
}

// One workgroup per segment, its output built in order in steps of up to
// kExpandThreads tokens / kExpandBytes bytes (this form, one token per
// thread, is the A/B alternative, GG_EXPAND_TPT=1; the default,
// inflate_expand2_kernel below, takes three tokens per thread and step and
// the same ring).  The segment's last 32 KB of
// output stay in an LDS ring in sym's form (u16 per byte: a literal, or
// kSymPtr | the position mod 32 KB of a byte before the segment), so every
// back-reference inside the segment is an LDS read: a step's bytes are
// staged (u16) as literals, pointers to before the segment (the segment
// before is not expanded yet: the resolve pass follows them), ring values,
// or kStepRef | the step byte they copy; kStepRef entries are followed
// inside the step by pointer jumping, and the step goes to sym (coalesced)
// and to the ring.  So a pointer left in sym reaches only into the 32 KB
// before the segment, as the resolve's ring index.
//
// The tokens come from global memory kTokBuf at a time into LDS.  A wave
// waits for a global load with every older global store of its own
// outstanding (one counter for both, completed in order), and the step's
// sym stores take ~25 us to complete: reading the next step's tokens from
// global memory cost ~65k cycles per step against ~11k of work
// (GALAHGPU_INFLATE_DEBUG with -DGG_EXPAND_PROF); with the LDS buffer one
// step in four waits.  (Spreading a step's bytes over the threads instead of
// its tokens measured slower: profiles/r06/expand_bytes_ab.txt.)
// 512 threads and steps of <= 4000 bytes: 80 KB of LDS, two workgroups per
// CU.  (A/B builds: scripts/ab_lib.sh with -DGG_EXPAND_THREADS=...
// -DGG_EXPAND_BYTES=..., -DGG_EXPAND_PROF: the debug line's phase cycles)
#ifndef GG_EXPAND_THREADS
#define GG_EXPAND_THREADS 512
#endif
#ifndef GG_EXPAND_BYTES
#define GG_EXPAND_BYTES 4000
#endif
constexpr int kExpandThreads = GG_EXPAND_THREADS;
constexpr uint32_t kExpandBytes = GG_EXPAND_BYTES;
constexpr uint32_t kTokBuf = 4 * kExpandThreads - 128;  // tokens held in LDS (~4 steps of FASTA; the
                                                        // total stays within 80 KB: two workgroups per CU)
constexpr uint32_t kRing = 32768;       // the DEFLATE window
constexpr uint16_t kStepRef = 0x4000u;  // step entry: the value of step byte (entry & 0x0FFF)
static_assert(kExpandBytes <= 0x1000, "step bytes are 12-bit kStepRef indices");
__global__ __launch_bounds__(kExpandThreads) void inflate_expand_kernel(InflatePlace a) {
  __shared__ uint16_t v[kExpandBytes];
  __shared__ uint16_t ring[kRing];
  __shared__ uint32_t tb[kTokBuf];
  __shared__ uint32_t s_take, s_bytes;
  __shared__ uint32_t wsum[kExpandThreads / 64];
  const uint32_t seg = blockIdx.x;
  const uint32_t tid = threadIdx.x, ln = tid & 63u, wave = tid >> 6;
  const uint32_t* tok = a.tok + a.tok_off[seg];
  const uint64_t n = a.n_tok[seg];
  const uint64_t o0 = a.lane_out[seg];                 // the segment's first text position
  const uint64_t f0 = a.file_text[a.lane_file[seg]];  // its unit's
  const uint64_t lim = o0 + a.lane_len[seg];           // (a corrupt stream's tokens may make more or fewer bytes
                                                       //  than the decode counted: nothing is written past lim)
  uint64_t base = o0;
  bool bad = false;
  uint64_t tb0 = 0, tb1 = 0;  // tokens [tb0, tb1) are in tb
#ifdef GG_EXPAND_PROF
  uint64_t tp = a.prof ? clock64() : 0;
  auto phase = [&](int k) {
    if (a.prof) {
      const uint64_t t = clock64();
      if (tid == 0) atomicAdd((unsigned long long*)&a.prof[k], (unsigned long long)(t - tp));
      tp = t;
    }
  };
#else
  auto phase = [](int) {};
#endif
  for (uint64_t t0 = 0; t0 < n;) {
    if (t0 + kExpandThreads > tb1 && tb1 < n) {  // (uniform) the buffer from t0 on
      tb0 = t0;
      tb1 = min(n, t0 + kTokBuf);
#pragma unroll
      for (uint32_t k = 0; k < (kTokBuf + kExpandThreads - 1) / kExpandThreads; ++k) {
        const uint64_t ti = t0 + tid + k * kExpandThreads;
        if (ti < tb1) tb[tid + k * kExpandThreads] = tok[ti];
      }
      __syncthreads();
    }
    const uint64_t ti = t0 + tid;
    const uint32_t tk = ti < n ? tb[(uint32_t)(ti - tb0)] : 0u;
    const uint32_t len = ti < n ? tok_len(tk) : 0u;
    uint32_t inc = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if (ln >= (uint32_t)o) inc += y;
    }
    if (ln == 63) wsum[wave] = inc;
    if (tid == 0) {
      s_take = 0;
      s_bytes = 0;
    }
    __syncthreads();
    phase(5);
    for (uint32_t w = 0; w < wave; ++w) inc += wsum[w];
    const uint32_t before = inc - len;
    const bool take = ti < n && inc <= kExpandBytes;  // (a prefix of the threads; thread 0 always)
    const uint32_t c = (uint32_t)__popcll(__ballot(take));
    const uint32_t last = __shfl(inc, c ? c - 1 : 0);  // this wave's bytes up to its last token taken
    if (c && ln == 0) {
      atomicAdd(&s_take, c);
      atomicMax(&s_bytes, last);
    }
    if (take) {
      if (!tok_is_match(tk)) {
        v[before] = (uint16_t)(tk & 0xFFu);
      } else {
        const uint32_t dist = tok_dist(tk);
        const uint64_t p = base + before;
        if (p < f0 + dist) {
          bad = true;  // a distance before the unit's first byte
          for (uint32_t k = 0; k < len; ++k) v[before + k] = (uint16_t)'\n';
        } else {
          const uint64_t src = p - dist;
          for (uint32_t k = 0; k < len; ++k) {
            const uint64_t s = src + k;
            uint16_t x;
            if (s >= base) x = (uint16_t)(kStepRef | (uint32_t)(s - base));
            else if (s < o0) x = (uint16_t)(kSymPtr | ((uint32_t)s & (kRing - 1)));
            else x = ring[(uint32_t)s & (kRing - 1)];
            v[before + k] = x;
          }
        }
      }
    }
    __syncthreads();
    const uint32_t nb = s_bytes, nt = s_take;
    phase(0);
    for (;;) {  // kStepRef entries followed inside the step (each points to an earlier byte)
#ifdef GG_EXPAND_PROF
      if (a.prof && tid == 0) atomicAdd((unsigned long long*)&a.prof[4], 1ull);
#endif
      bool more = false;
      for (uint32_t i = tid; i < nb; i += kExpandThreads) {
        const uint32_t x = v[i];
        if ((x & 0xC000u) == kStepRef) {
          const uint32_t y = v[x & 0x0FFFu];
          v[i] = (uint16_t)y;
          more |= (y & 0xC000u) == kStepRef;
        }
      }
      if (!__syncthreads_or(more)) break;
    }
    phase(1);
    const uint32_t nw = base + nb <= lim ? nb : base < lim ? (uint32_t)(lim - base) : 0u;
    for (uint32_t i = tid; i < nw; i += kExpandThreads) {
      const uint16_t x = v[i];
      a.sym[base + i] = x;
      ring[(uint32_t)(base + i) & (kRing - 1)] = x;
    }
    __syncthreads();
    phase(2);
#ifdef GG_EXPAND_PROF
    if (a.prof && tid == 0) atomicAdd((unsigned long long*)&a.prof[3], 1ull);
#endif
    base += nb;
    t0 += nt;
  }
  if (bad) atomicOr(a.flags, 1u);
  if (base != lim && tid == 0) atomicOr(a.flags, 4u);
}

#ifndef GG_EXPAND_TPT  // (A/B builds; 1,000 C2-like files: 1 token per thread 13.9 ms, 2 (6,000-byte steps) 11.1, 3 (8,000) 10.8, 4 (8,000) 12.1)
#define GG_EXPAND_TPT 3
#endif
#ifndef GG_EXPAND_TBYTES  // (the step's bytes with GG_EXPAND_TPT > 1)
#define GG_EXPAND_TBYTES 8000
#endif
#if GG_EXPAND_TPT > 1
// The expand with kTpt tokens per thread and step (steps of up to 512 kTpt
// tokens / kTBytes bytes: a third of the steps, barriers and scans per
// segment of FASTA; 13.9 -> 10.8 ms per 1,000 C2-like files,
// profiles/r06/expand_tpt_ab.txt); the tokens are prefetched into registers
// a step ahead (the LDS has no room for a token buffer next to 16 KB of step
// bytes and the 64 KB ring: 81,832 bytes, two workgroups per CU).
constexpr int kTpt = GG_EXPAND_TPT;
constexpr uint32_t kTBytes = GG_EXPAND_TBYTES;
constexpr uint16_t kStepRef2 = 0x4000u;  // step entry: the value of step byte (entry & 0x3FFF)
#ifndef GG_EXPAND_CHASE  // (A/B builds: -DGG_EXPAND_CHASE=1, plain pointer jumping)
#define GG_EXPAND_CHASE 8
#endif
constexpr int kChase = GG_EXPAND_CHASE;
#ifndef GG_EXPAND_FILL32  // (A/B builds: -DGG_EXPAND_FILL32=0, 64-bit positions and branches per byte)
#define GG_EXPAND_FILL32 1
#endif
static_assert(kTBytes <= 0x4000, "14-bit step references");
__global__ __launch_bounds__(kExpandThreads) void inflate_expand2_kernel(InflatePlace a) {
  __shared__ uint16_t v[kTBytes];
  __shared__ uint16_t ring[kRing];
  __shared__ uint32_t s_take, s_bytes;
  __shared__ uint32_t wsum[kExpandThreads / 64];
  const uint32_t seg = blockIdx.x;
  const uint32_t tid = threadIdx.x, ln = tid & 63u, wave = tid >> 6;
  const uint32_t* tok = a.tok + a.tok_off[seg];
  const uint64_t n = a.n_tok[seg];
  const uint64_t o0 = a.lane_out[seg];
  const uint64_t f0 = a.file_text[a.lane_file[seg]];
  const uint64_t lim = o0 + a.lane_len[seg];
  const uint64_t nl = n ? n - 1 : 0;
  uint64_t base = o0;
  bool bad = false;
  uint32_t nx[kTpt];
#pragma unroll
  for (int k = 0; k < kTpt; ++k) nx[k] = tok[min<uint64_t>((uint64_t)kTpt * tid + k, nl)];
  auto fill = [&](uint32_t tk, uint32_t len, uint32_t before) {
    if (!tok_is_match(tk)) {
      v[before] = (uint16_t)(tk & 0xFFu);
      return;
    }
    const uint32_t dist = tok_dist(tk);
    const uint64_t p = base + before;
    if (p < f0 + dist) {
      bad = true;
      for (uint32_t k = 0; k < len; ++k) v[before + k] = (uint16_t)'\n';
      return;
    }
#if GG_EXPAND_FILL32
    // source bytes as 32-bit offsets from the step's first byte (r >= 0: in
    // the step; r < lo: before the lane), the ring read unconditionally and
    // the entry picked by selects (the 64-bit compares and branches per byte
    // made the fill's loop mostly scalar and exec-mask work)
    const int32_t r0 = (int32_t)before - (int32_t)dist;
    const int32_t lo = -(int32_t)min<uint64_t>(base - o0, 0x10000u);
    const uint32_t b32 = (uint32_t)base;
    for (uint32_t k = 0; k < len; ++k) {
      const int32_t r = r0 + (int32_t)k;
      const uint32_t idx = (b32 + (uint32_t)r) & (kRing - 1);
      const uint32_t y = ring[idx];
      const uint32_t x = r >= 0 ? (kStepRef2 | (uint32_t)r) : r < lo ? (kSymPtr | idx) : y;
      v[before + k] = (uint16_t)x;
    }
#else
    const uint64_t src = p - dist;
    for (uint32_t k = 0; k < len; ++k) {
      const uint64_t s = src + k;
      uint16_t x;
      if (s >= base) x = (uint16_t)(kStepRef2 | (uint32_t)(s - base));
      else if (s < o0) x = (uint16_t)(kSymPtr | ((uint32_t)s & (kRing - 1)));
      else x = ring[(uint32_t)s & (kRing - 1)];
      v[before + k] = x;
    }
#endif
  };
  for (uint64_t t0 = 0; t0 < n;) {
    const uint64_t ti = t0 + (uint64_t)kTpt * tid;
    uint32_t tk[kTpt], l[kTpt];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < kTpt; ++k) {
      tk[k] = nx[k];
      l[k] = ti + k < n ? tok_len(tk[k]) : 0u;
      sum += l[k];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if (ln >= (uint32_t)o) inc += y;
    }
    if (ln == 63) wsum[wave] = inc;
    if (tid == 0) {
      s_take = 0;
      s_bytes = 0;
    }
    __syncthreads();
    for (uint32_t w = 0; w < wave; ++w) inc += wsum[w];
    uint32_t bef[kTpt];
    bool take[kTpt];
    uint32_t c = 0, mine = 0;
    {
      uint32_t at = inc - sum;
#pragma unroll
      for (int k = 0; k < kTpt; ++k) {
        bef[k] = at;
        at += l[k];
        take[k] = ti + k < n && at <= kTBytes;  // (the taken tokens are a prefix)
        c += (uint32_t)__popcll(__ballot(take[k]));
        if (take[k]) mine = at;
      }
    }
    uint32_t mx = mine;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o));
    if (c && ln == 0) {
      atomicAdd(&s_take, c);
      atomicMax(&s_bytes, mx);
    }
#pragma unroll
    for (int k = 0; k < kTpt; ++k)
      if (take[k]) fill(tk[k], l[k], bef[k]);
    __syncthreads();
    const uint32_t nb = s_bytes, nt = s_take;
    {
      const uint64_t tn = t0 + nt + (uint64_t)kTpt * tid;  // the next step's tokens (in flight during this step's LDS work)
#pragma unroll
      for (int k = 0; k < kTpt; ++k) nx[k] = tok[min(tn + k, nl)];
    }
    for (;;) {  // kStepRef entries followed inside the step (each to an earlier byte): up to
                // kChase hops per entry and round, then pointer jumping (a run of one byte,
                // dist 1, makes chains as long as the step)
      bool more = false;
      for (uint32_t i = tid; i < nb; i += kExpandThreads) {
        uint32_t x = v[i];
        if ((x & 0xC000u) == kStepRef2) {
#pragma unroll
          for (int h = 0; h < kChase && (x & 0xC000u) == kStepRef2; ++h) x = v[x & 0x3FFFu];
          v[i] = (uint16_t)x;
          more |= (x & 0xC000u) == kStepRef2;
        }
      }
      if (!__syncthreads_or(more)) break;
    }
    const uint32_t nw = base + nb <= lim ? nb : base < lim ? (uint32_t)(lim - base) : 0u;
    for (uint32_t i = tid; i < nw; i += kExpandThreads) {
      const uint16_t x = v[i];
      a.sym[base + i] = x;
      ring[(uint32_t)(base + i) & (kRing - 1)] = x;
    }
    __syncthreads();
    base += nb;
    t0 += nt;
  }
  if (bad) atomicOr(a.flags, 1u);
  if (base != lim && tid == 0) atomicOr(a.flags, 4u);
}
#endif

// One workgroup per unit (gzip member): its lanes' bytes in order, the
// unit's last 32 KB of text in an LDS ring (position & 0x7FFF).  A lane's
// pointers reach only into the 32 KB before its first byte (the expand
// followed every back-reference inside the lane), so with the ring holding
// the text before the lane every byte is final after one LDS read, and the
// lane's bytes are independent of each other: the threads go through them
// without a barrier, 16 bytes per thread and step (two 16-byte sym loads, one
// 16-byte text store).  The lane's last 32 KB go to the other ring, which
// serves the next lane.  Traffic: 2 B of sym read and 1 B of text written per
// byte (the round-5 resolve followed u32 pointers hop by hop over the whole
// batch: 3.6x its bytes).
#ifndef GG_RESOLVE_THREADS  // (A/B builds; 1,000 C2-like files: 512 x 4 groups 3.56 ms, 1024 x 2 2.52, 1024 x 4 2.56, 256 x 8 5.99)
#define GG_RESOLVE_THREADS 1024
#endif
#ifndef GG_RESOLVE_GROUPS
#define GG_RESOLVE_GROUPS 2
#endif
constexpr int kResolveThreads = GG_RESOLVE_THREADS;
constexpr int kResolveGroups = GG_RESOLVE_GROUPS;  // 16-byte groups per thread in flight (their sym loads issued together)
__global__ __launch_bounds__(kResolveThreads) void inflate_resolve_kernel(InflatePlace a) {
  __shared__ uint8_t ring[2][kRing];
  const uint32_t u = blockIdx.x, tid = threadIdx.x;
  const uint64_t u0 = a.file_text[u];
  const uint16_t* __restrict__ sym = a.sym;
  uint8_t* __restrict__ text = a.text;
  int cur = 0;
  for (uint32_t l = a.unit_lane[u]; l < a.unit_lane[u + 1]; ++l) {
    const uint64_t o0 = a.lane_out[l], o1 = o0 + a.lane_len[l];
    const uint64_t tail0 = o1 - o0 > kRing ? o1 - kRing : o0;  // from here on the bytes also go to the next ring
    const uint8_t* R = ring[cur];
    uint8_t* N = ring[cur ^ 1];
    const uint64_t g0 = o0 / 16, g1 = (o1 + 15) / 16;
    for (uint64_t gb = g0; gb < g1; gb += kResolveThreads * kResolveGroups) {
      uint4 q[kResolveGroups][2];
#pragma unroll
      for (int k = 0; k < kResolveGroups; ++k) {
        const uint64_t g = gb + tid + (uint64_t)k * kResolveThreads;
        if (g < g1) {
          q[k][0] = *(const uint4*)(sym + 16 * g);
          q[k][1] = *(const uint4*)(sym + 16 * g + 8);
        }
      }
#pragma unroll
      for (int k = 0; k < kResolveGroups; ++k) {
        const uint64_t g = gb + tid + (uint64_t)k * kResolveThreads;
        if (g >= g1) break;
        const uint32_t w[8] = {q[k][0].x, q[k][0].y, q[k][0].z, q[k][0].w, q[k][1].x, q[k][1].y, q[k][1].z, q[k][1].w};
        uint32_t out[4] = {0, 0, 0, 0};
#pragma unroll
        for (int b = 0; b < 16; ++b) {
          const uint32_t v = (w[b >> 1] >> (16 * (b & 1))) & 0xFFFFu;
          const uint32_t r = R[v & (kRing - 1)];  // (read for a literal too: the 64 reads issue without a branch or wait each)
          const uint32_t byte = v & kSymPtr ? r : v & 0xFFu;
          out[b >> 2] |= byte << (8 * (b & 3));
        }
        const uint64_t p0 = 16 * g;
        if (p0 >= o0 && p0 + 16 <= o1) {
          *(uint4*)(text + p0) = make_uint4(out[0], out[1], out[2], out[3]);
        } else {  // (a group the lane shares with the lane before or after it)
#pragma unroll
          for (int b = 0; b < 16; ++b)
            if (p0 + b >= o0 && p0 + b < o1) text[p0 + b] = (uint8_t)(out[b >> 2] >> (8 * (b & 3)));
        }
        if (p0 + 16 > tail0) {
#pragma unroll
          for (int b = 0; b < 16; ++b)
            if (p0 + b >= tail0 && p0 + b < o1) N[(p0 + b) & (kRing - 1)] = (uint8_t)(out[b >> 2] >> (8 * (b & 3)));
        }
      }
    }
    // a lane shorter than the ring: the ring's older bytes (after the unit's
    // start) carry over to the next lane
    const uint64_t keep0 = o1 > u0 + kRing ? o1 - kRing : u0;
    for (uint64_t p = keep0 + tid; p < tail0; p += kResolveThreads) N[p & (kRing - 1)] = R[p & (kRing - 1)];
    __syncthreads();
    cur ^= 1;
  }
  // a file's last unit: the padding up to the next file ('\n' parses as nothing)
  for (uint64_t i = u0 + a.unit_len[u] + tid; i < a.unit_pad[u]; i += kResolveThreads) text[i] = '\n';
}

// CRC-32 (gzip, reflected 0xEDB88320), table in LDS.
constexpr uint32_t kCrcPoly = 0xEDB88320u;
__device__ uint32_t crc_mul(uint32_t a, uint32_t b) {  // a * b mod P (reflected)
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = b & 1 ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}
__device__ uint32_t crc_x8n(uint64_t n, const uint32_t* __restrict__ x2k) {  // x^(8n) mod P
  uint32_t p = 1u << 31;  // x^0
  uint32_t k = 3;
  while (n) {
    if (n & 1) p = crc_mul(x2k[k & 63], p);
    n >>= 1;
    ++k;
  }
  return p;
}

// CRC-32 in two kernels: every kCrcSeg-byte segment of every unit on its own
// wave -- each lane the CRC (init 0: linear) of 64 contiguous bytes
// (slicing-by-8, tables in LDS, 16-byte loads), shifted past the bytes after
// it by one multiplication mod P and XORed over the wave, then the init's
// term: the segment's standard CRC-32 -- and per unit the segments folded in
// order, crc(A || B) = x^(8|B|) crc(A) ^ crc(B).  (Round 5 gave each segment
// one thread, whose 256 16-byte loads in a row a wave issued 4 KB apart:
// 1.8-1.9 ms per C2-like call.)
constexpr uint32_t kCrcSeg = kInflateCrcSeg;
static_assert(kCrcSeg == 64 * 64, "a segment is 64 bytes per lane of one wave");
constexpr int kCrcThreads = 256;
struct CrcPowers {
  uint32_t x2k[64];         // x^(2^k) mod P
  uint32_t xseg;            // x^(8 kCrcSeg) mod P
  uint32_t lane_shift[64];  // x^(8 * 64 * (63 - lane)) mod P: a full segment's lane shifted past the lanes after it
  uint32_t seg_init;        // 0xFFFFFFFF * x^(8 kCrcSeg) mod P: a full segment's init term
};
__global__ __launch_bounds__(kCrcThreads) void inflate_crc_seg_kernel(const uint8_t* __restrict__ text,
                                                                      const uint64_t* __restrict__ file_text,
                                                                      const uint64_t* __restrict__ file_len,
                                                                      const uint32_t* __restrict__ seg_first,
                                                                      uint32_t n_files, uint32_t n_segs,
                                                                      uint32_t* __restrict__ seg_crc, CrcPowers pw) {
  __shared__ uint32_t T[8][256];
  __shared__ uint32_t x2k[64];
  {
    const uint32_t i = threadIdx.x;  // (kCrcThreads == 256: one table index per thread)
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = c & 1 ? (c >> 1) ^ kCrcPoly : c >> 1;
    T[0][i] = c;
    if (i < 64) x2k[i] = pw.x2k[i];
  }
  __syncthreads();
  {  // T[t][i]: byte i followed by t zero bytes
    const uint32_t i = threadIdx.x;
    uint32_t c = T[0][i];
    for (int t = 1; t < 8; ++t) {
      c = (c >> 8) ^ T[0][c & 0xFFu];
      T[t][i] = c;
    }
  }
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = blockIdx.x * (kCrcThreads / 64) + (threadIdx.x >> 6);  // (uniform per wave)
  if (g >= n_segs) return;
  uint32_t lo = 0, hi = n_files;  // the unit: seg_first[f] <= g < seg_first[f + 1]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (seg_first[mid] <= g) lo = mid;
    else hi = mid;
  }
  const uint32_t f = lo;
  const uint64_t off = (uint64_t)(g - seg_first[f]) * kCrcSeg;
  const uint32_t len = (uint32_t)min<uint64_t>(kCrcSeg, file_len[f] - off);
  const uint8_t* p = text + file_text[f] + off;
  const uint32_t b0 = 64 * lane, b1 = min(len, b0 + 64);
  uint32_t c = 0;  // (init 0: this lane's bytes alone)
  if (b0 < len) {
    // (a file's text starts on a 16-byte boundary; a later gzip member's
    // anywhere: such a segment, and a unit's last, partly by bytes)
    if (b1 - b0 == 64 && ((uintptr_t)(p + b0) & 15u) == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = *(const uint4*)(p + b0 + 16 * q);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int h = 0; h < 4; h += 2) {
          const uint32_t a = w[h] ^ c, b = w[h + 1];
          c = T[7][a & 0xFFu] ^ T[6][(a >> 8) & 0xFFu] ^ T[5][(a >> 16) & 0xFFu] ^ T[4][a >> 24] ^ T[3][b & 0xFFu] ^
              T[2][(b >> 8) & 0xFFu] ^ T[1][(b >> 16) & 0xFFu] ^ T[0][b >> 24];
        }
      }
    } else {
      for (uint32_t i = b0; i < b1; ++i) c = T[0][(c ^ p[i]) & 0xFFu] ^ (c >> 8);
    }
    // shifted past the segment's bytes after this lane's
    c = crc_mul(len == kCrcSeg ? pw.lane_shift[lane] : crc_x8n(len - b1, x2k), c);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c ^= __shfl_xor(c, o);
  if (lane == 0) {
    const uint32_t init = len == kCrcSeg ? pw.seg_init : crc_mul(crc_x8n(len, x2k), 0xFFFFFFFFu);
    seg_crc[g] = ~(c ^ init);
  }
}

// One workgroup per file: each thread folds a contiguous run of the file's
// segments, and the file's CRC is the XOR of every run's CRC shifted past
// the bytes after it, crc(A || B) = x^(8|B|) crc(A) ^ crc(B) applied to all
// runs at once (no tree of dependent rounds).  x^(2^k) mod P comes from the
// host (a serial chain of 64 squarings each workgroup once began with).
constexpr int kFoldThreads = 256;
__global__ __launch_bounds__(kFoldThreads) void inflate_crc_fold_kernel(const uint8_t* __restrict__ text,
                                                                        const uint64_t* __restrict__ file_text,
                                                                        const uint64_t* __restrict__ file_len,
                                                                        const uint32_t* __restrict__ seg_first,
                                                                        const uint32_t* __restrict__ seg_crc,
                                                                        uint32_t n_files, uint32_t* __restrict__ crc_out,
                                                                        CrcPowers pw) {
  __shared__ uint32_t x2k[64];
  __shared__ uint32_t part[kFoldThreads / 64];
  const uint32_t tid = threadIdx.x;
  if (tid < 64) x2k[tid] = pw.x2k[tid];
  __syncthreads();
  const uint32_t f = blockIdx.x;
  const uint64_t len = file_len[f];
  const uint32_t g0 = seg_first[f], ns = seg_first[f + 1] - g0;
  const uint32_t per = (ns + kFoldThreads - 1) / kFoldThreads;
  const uint32_t a0 = min(ns, tid * per), a1 = min(ns, a0 + per);
  uint32_t crc = 0;  // of this thread's run (standard CRC-32; 0 for none)
  for (uint32_t k = a0; k < a1; ++k) {
    const uint64_t bl = min<uint64_t>(kCrcSeg, len - (uint64_t)k * kCrcSeg);
    crc = crc_mul(bl == kCrcSeg ? pw.xseg : crc_x8n(bl, x2k), crc) ^ seg_crc[g0 + k];
  }
  // shifted past the bytes of the runs after it
  const uint64_t after = a1 < ns ? len - (uint64_t)a1 * kCrcSeg : 0;
  if (crc && after) crc = crc_mul(crc_x8n(after, x2k), crc);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) crc ^= __shfl_xor(crc, o);
  if ((tid & 63u) == 0) part[tid >> 6] = crc;
  __syncthreads();
  if (tid == 0) {
    uint32_t c = 0;
    for (int w = 0; w < kFoldThreads / 64; ++w) c ^= part[w];
    crc_out[f] = c;
    crc_out[n_files + f] = len ? text[file_text[f]] : 0u;  // (the caller checks the format: FASTA starts with '>')
  }
}

// The powers the fold kernel takes, on the host (the same arithmetic).
uint32_t crc_mul_host(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (uint32_t m = 1u << 31; m; m >>= 1) {
    if (a & m) p ^= b;
    b = b & 1 ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}
const CrcPowers& crc_powers() {
  static const CrcPowers pw = [] {
    CrcPowers x{};
    uint32_t p = 1u << 30;  // x^1
    for (int k = 0; k < 64; ++k) {
      x.x2k[k] = p;
      p = crc_mul_host(p, p);
    }
    auto x8n = [&](uint64_t bytes) {  // x^(8 bytes) mod P
      uint32_t r = 1u << 31;
      uint64_t n = 8ull * bytes;
      for (int k = 0; n; ++k, n >>= 1)
        if (n & 1) r = crc_mul_host(x.x2k[k], r);
      return r;
    };
    x.xseg = x8n(kCrcSeg);
    for (int l = 0; l < 64; ++l) x.lane_shift[l] = x8n(64ull * (63 - l));
    x.seg_init = crc_mul_host(x.xseg, 0xFFFFFFFFu);
    return x;
  }();
  return pw;
}

// A staged batch from its pinned host slot to the device (launch_slot_upload:
// a DMA-engine copy; this kernel, GALAHGPU_GZ_UPLOAD=kernel, reads the
// mapped slot over PCIe -- a few workgroups, each thread with four 16-byte
// loads in flight -- and was the default until round 6, when its PCIe reads
// were found to slow the kernels running beside it).
constexpr int kUploadThreads = 256, kUploadBlocks = 64;
template <bool kNt>
__global__ __launch_bounds__(kUploadThreads) void slot_upload_kernel(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                                     uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * kUploadThreads;
  uint64_t i = (uint64_t)blockIdx.x * kUploadThreads + threadIdx.x;
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  auto ld = [&](uint64_t k) {
    if (!kNt) return src[k];
    const v4u v = __builtin_nontemporal_load((const v4u*)(src + k));
    return make_uint4(v.x, v.y, v.z, v.w);
  };
  auto st = [&](uint64_t k, uint4 v) {
    if (kNt) {
      const v4u w = {v.x, v.y, v.z, v.w};
      __builtin_nontemporal_store(w, (v4u*)(dst + k));
    } else {
      dst[k] = v;
    }
  };
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = ld(i), b = ld(i + stride), c = ld(i + 2 * stride), d = ld(i + 3 * stride);
    st(i, a);
    st(i + stride, b);
    st(i + 2 * stride, c);
    st(i + 3 * stride, d);
  }
  for (; i < n16; i += stride) st(i, ld(i));
}

}  // namespace

uint32_t inflate_stage_words() { return kStageWords; }

hipError_t launch_slot_upload(uint8_t* dst, const uint8_t* src_mapped, uint64_t bytes, hipStream_t st) {
  const uint64_t n16 = (bytes + 15) / 16;  // (both buffers are padded past bytes to a 16-byte multiple)
  if (n16 == 0) return hipSuccess;
  // A DMA-engine copy by default: the copy kernel's PCIe reads, running
  // beside the other lane's kernels, slowed the latency-bound decode ~2x
  // (a full batch's decode 1.65 ms alone, 4.5-4.8 ms beside the kernel;
  // 600 C2-like files: decode 14.0 -> 6.6 ms per call, the call 0.038 ->
  // 0.0315 s, profiles/r06/upload_ab.txt).  GALAHGPU_GZ_UPLOAD=kernel keeps the
  // kernel (GALAHGPU_GZ_UPLOAD_BLOCKS, GALAHGPU_GZ_UPLOAD_NT=1: its workgroups,
  // non-temporal accesses -- A/B knobs, read per call).
  const char* mode = getenv("GALAHGPU_GZ_UPLOAD");
  if (!(mode && strcmp(mode, "kernel") == 0)) {
    // (GALAHGPU_GZ_UPLOAD_CHUNK_MB: the copy in pieces of that size, so that
    // the lanes' small copies queued on the DMA engines behind it wait for one
    // piece at most -- an A/B knob)
    const char* ec = getenv("GALAHGPU_GZ_UPLOAD_CHUNK_MB");
    const uint64_t chunk = ec && atoi(ec) > 0 ? (uint64_t)atoi(ec) << 20 : bytes;
    for (uint64_t o = 0; o < bytes; o += chunk) {
      const hipError_t e = hipMemcpyAsync(dst + o, src_mapped + o, std::min(chunk, bytes - o), hipMemcpyHostToDevice, st);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  const char* eb = getenv("GALAHGPU_GZ_UPLOAD_BLOCKS");
  const uint64_t want = eb && atoi(eb) > 0 ? (uint64_t)atoi(eb) : (uint64_t)kUploadBlocks;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(want, (n16 + kUploadThreads - 1) / kUploadThreads);
  const char* nt = getenv("GALAHGPU_GZ_UPLOAD_NT");
  if (nt && *nt == '1')
    hipLaunchKernelGGL(slot_upload_kernel<true>, dim3(blocks), dim3(kUploadThreads), 0, st, (uint4*)dst,
                       (const uint4*)src_mapped, n16);
  else
    hipLaunchKernelGGL(slot_upload_kernel<false>, dim3(blocks), dim3(kUploadThreads), 0, st, (uint4*)dst,
                       (const uint4*)src_mapped, n16);
  return hipGetLastError();
}

hipError_t launch_inflate_search(const InflateSearch& a, hipStream_t st) {
  if (a.n_chunks == 0) return hipSuccess;
  hipLaunchKernelGGL(inflate_search_kernel, dim3((a.n_chunks + kSearchWaves - 1) / kSearchWaves),
                     dim3(64 * kSearchWaves), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_inflate_decode(const InflateDecode& a, hipStream_t st) {
  if (a.n_staged)
    hipLaunchKernelGGL(inflate_decode_kernel<true>, dim3(a.n_staged), dim3(kSpanLanes),
                       (a.stage_words ? a.stage_words : kStageWords) * 4, st, a);
  if (a.n_lanes > a.n_staged)
    hipLaunchKernelGGL(inflate_decode_kernel<false>, dim3(a.n_lanes - a.n_staged), dim3(kSpanLanes), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_inflate_expand(const InflatePlace& a, hipStream_t st) {
#if GG_EXPAND_TPT > 1
  if (a.n_lanes) hipLaunchKernelGGL(inflate_expand2_kernel, dim3(a.n_lanes), dim3(kExpandThreads), 0, st, a);
#else
  if (a.n_lanes) hipLaunchKernelGGL(inflate_expand_kernel, dim3(a.n_lanes), dim3(kExpandThreads), 0, st, a);
#endif
  return hipGetLastError();
}

hipError_t launch_inflate_resolve(const InflatePlace& a, hipStream_t st) {
  if (a.n_units) hipLaunchKernelGGL(inflate_resolve_kernel, dim3(a.n_units), dim3(kResolveThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_inflate_crc(const uint8_t* text, uint32_t n_files, const uint64_t* file_text, const uint64_t* file_len,
                              const uint32_t* seg_first, uint32_t n_segs, uint32_t* seg_crc, uint32_t* crc,
                              hipStream_t st) {
  if (n_segs)
    hipLaunchKernelGGL(inflate_crc_seg_kernel, dim3((n_segs + kCrcThreads / 64 - 1) / (kCrcThreads / 64)),
                       dim3(kCrcThreads), 0, st, text, file_text, file_len, seg_first, n_files, n_segs, seg_crc,
                       crc_powers());
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (n_files)
    hipLaunchKernelGGL(inflate_crc_fold_kernel, dim3(n_files), dim3(kFoldThreads), 0, st, text, file_text, file_len,
                       seg_first, seg_crc, n_files, crc, crc_powers());
  return hipGetLastError();
}

}  // namespace gg
