// DEFLATE (RFC 1951) decoding primitives shared by the device inflate
// (inflate.hip) and its host-side tests: one lane decodes one run of
// blocks; nothing here allocates or synchronises.
//
// The device path inflates many gzip members at once without decoding any
// stream from its start serially:
//   1. search  every ~CH compressed bytes of a stream, the first bit position
//              where a valid dynamic-block header parses (block_header_ok)
//   2. decode   one lane per found start: Huffman-decode its blocks into
//               tokens (literal byte, or match length + distance) until it
//               lands exactly on the next start; back-references are not
//               resolved here, so no lane needs the window of the lanes
//               before it
//   3. place / resolve  (inflate.hip) token output positions by prefix sums,
//               every output byte a literal or a pointer to an earlier
//               byte, pointers followed to their literal
// A search hit that is not a block boundary is never landed on by the lane
// before it (decode reports the overrun and the host drops that start), so
// the output never depends on the search being right.
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define GG_HD __host__ __device__ __forceinline__
#else
#define GG_HD inline
#endif

namespace gg {
namespace inflate {

// The DEFLATE stream of one gzip member, as 32-bit little-endian words with
// at least two words of padding after its last byte; bit positions count
// from the member's first deflate byte, LSB first (RFC 1951 3.1.1).
// (The header functions below take any reader with Bits' peek / get.)
struct Bits {
  const uint32_t* w;
  // the 32 stream bits starting at pos, the first in bit 0
  GG_HD uint32_t peek(uint64_t pos) const {
    const uint64_t i = pos >> 5;
    const uint32_t sh = (uint32_t)pos & 31u;
    const uint64_t v = ((uint64_t)w[i + 1] << 32) | w[i];
    return (uint32_t)(v >> sh);
  }
  GG_HD uint32_t get(uint64_t& pos, uint32_t n) const {  // n <= 25
    const uint32_t v = peek(pos) & ((1u << n) - 1u);
    pos += n;
    return v;
  }
};

// The same stream read forward through cached words: the symbol loop peeks
// 32 bits per symbol from registers (words a, b), and the words after them
// arrive two at a time, loaded two words before they are needed, so the
// decode waits on memory only when it outruns a load issued ~64 bits earlier
// (loading each word as the window reached it stalled every ~32 bits).
struct Cursor {
  const uint32_t* w;
  uint64_t pos;
  uint64_t wi;       // word of pos
  uint32_t a, b;     // words wi, wi + 1
  uint32_t g0, g1;   // the next words to enter the window (g0 first; `left` of them)
  uint32_t n0, n1;   // the two after those (in flight)
  uint32_t left;
  GG_HD void seek(uint64_t p) {
    pos = p;
    wi = p >> 5;
    a = w[wi];
    b = w[wi + 1];
    g0 = w[wi + 2];
    g1 = w[wi + 3];
    n0 = w[wi + 4];
    n1 = w[wi + 5];
    left = 2;
  }
  GG_HD uint32_t peek() const {
    const uint32_t sh = (uint32_t)pos & 31u;
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(b, a, sh);
#else
    return sh ? (a >> sh) | (b << (32 - sh)) : a;
#endif
  }
  GG_HD void skip(uint32_t n) {  // n <= 32
    pos += n;
    if ((pos >> 5) != wi) {
      ++wi;
      a = b;
      b = g0;
      g0 = g1;
      if (--left == 0) {  // the next two words (loaded two words ago); load the two after them
        g0 = n0;
        g1 = n1;
        n0 = w[wi + 4];
        n1 = w[wi + 5];
        left = 2;
      }
    }
  }
  GG_HD uint32_t get(uint32_t n) {  // n <= 31
    const uint32_t v = peek() & ((1u << n) - 1u);
    skip(n);
    return v;
  }
  GG_HD uint64_t peek64() const {  // the 64 stream bits from pos
    const uint32_t sh = (uint32_t)pos & 31u;
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t x0 = __builtin_amdgcn_alignbit(b, a, sh), x1 = __builtin_amdgcn_alignbit(g0, b, sh);
#else
    const uint32_t x0 = sh ? (a >> sh) | (b << (32 - sh)) : a, x1 = sh ? (b >> sh) | (g0 << (32 - sh)) : b;
#endif
    return (uint64_t)x0 | ((uint64_t)x1 << 32);
  }
  GG_HD void skip_long(uint32_t n) {  // n <= 64
    if (n > 32) {
      skip(32);
      n -= 32;
    }
    skip(n);
  }
};

// The stream read forward through a Cursor behind Bits' interface (the
// device's header walks): positions asked for go forward, a peek within the
// three cached words loads nothing (a walk through Bits waited on two loads
// per code length); a position behind the cached words starts it over.
struct SeqBits {
  mutable Cursor c;
  GG_HD uint32_t peek(uint64_t pos) const {
    int64_t d = (int64_t)(pos - (c.wi << 5));  // pos in the cached words a, b, c
    if (d < 0 || d >= 160) {
      c.seek(pos);
      d = (int64_t)(pos & 31u);
    }
    while (d >= 64) {  // the window one word on
      c.skip(32u - ((uint32_t)c.pos & 31u));
      d -= 32;
    }
    const uint32_t sh = (uint32_t)d & 31u;
    const uint32_t lo = d < 32 ? c.a : c.b, hi = d < 32 ? c.b : c.g0;  // (g0: word wi + 2)
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
    return sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
#endif
  }
  GG_HD uint32_t get(uint64_t& pos, uint32_t n) const {
    const uint32_t v = peek(pos) & ((1u << n) - 1u);
    pos += n;
    return v;
  }
};

GG_HD uint32_t rev15(uint32_t v) {  // the low 15 bits in reverse order: a left-justified 15-bit code
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_bitreverse32(v) >> 17;
#else
  uint32_t r = 0;
  for (int i = 0; i < 15; ++i) r |= ((v >> i) & 1u) << (14 - i);
  return r;
#endif
}

constexpr int kMaxBits = 15;
constexpr int kLitSyms = 288;   // lit/len alphabet (286 codable + 2 reserved)
constexpr int kDistSyms = 32;   // distance alphabet (30 codable + 2 reserved)
constexpr int kClSyms = 19;     // code-length alphabet
constexpr uint32_t kWindow = 32768;

// Canonical Huffman code (RFC 1951 3.2.2) for decoding: a left-justified
// 15-bit code x has length L = the smallest l with x < limit[l], and symbol
// sym[base[L] + (x >> (15 - L))].
struct Canon {
  uint32_t limit[kMaxBits + 1];
  int32_t base[kMaxBits + 1];
};

// Counts per length -> limits and bases.  Returns 0 complete, 1 incomplete,
// -1 over-subscribed.  max_len receives the longest length used (0: none).
GG_HD int canon_from_counts(const uint32_t (&count)[kMaxBits + 1], Canon& c, int& max_len) {
  int left = 1;
  max_len = 0;
  for (int l = 1; l <= kMaxBits; ++l) {
    left = (left << 1) - (int)count[l];
    if (left < 0) return -1;
    if (count[l]) max_len = l;
  }
  uint32_t first = 0, offs = 0;
  for (int l = 1; l <= kMaxBits; ++l) {
    c.limit[l] = (first + count[l]) << (kMaxBits - l);
    c.base[l] = (int32_t)offs - (int32_t)first;
    offs += count[l];
    first = (first + count[l]) << 1;
  }
  c.limit[0] = 0;
  c.base[0] = 0;
  return left == 0 ? 0 : 1;
}

// Length of the code whose left-justified 15 bits are x (kMaxBits + 1: no
// such code, x past an incomplete code's last one).
GG_HD int code_len(const Canon& c, uint32_t x) {
  int L = 1;
#pragma unroll
  for (int l = 1; l < kMaxBits; ++l) L += x >= c.limit[l] ? 1 : 0;
  return x >= c.limit[kMaxBits] ? kMaxBits + 1 : L;
}

// zlib's inflate_table acceptance: complete, or incomplete only when the
// longest code has length 1 (a lone symbol); no symbols at all is accepted
// for the distance code (a block without matches) and refused elsewhere.
GG_HD bool code_ok(int r, int max_len, bool allow_empty) {
  if (r < 0) return false;
  if (max_len == 0) return allow_empty;
  return r == 0 || max_len == 1;
}

// RFC 1951 3.2.5 length and distance tables
GG_HD uint32_t len_base(uint32_t i) {  // lit/len symbol 257 + i (3, 4, .., 10, 11, 13, .., 227, 258)
  if (i < 8) return 3 + i;
  if (i == 28) return 258;
  return ((4u + (i & 3u)) << ((i >> 2) - 1u)) + 3u;
}
GG_HD uint32_t len_extra(uint32_t i) { return i < 8 || i == 28 ? 0u : (i - 4) >> 2; }
GG_HD uint32_t dist_base(uint32_t d) {  // (1, 2, 3, 4, 5, 7, .., 24577)
  if (d < 4) return d + 1;
  return ((2u + (d & 1u)) << ((d >> 1) - 1u)) + 1u;
}
GG_HD uint32_t dist_extra(uint32_t d) { return d < 4 ? 0u : (d - 2) >> 1; }

constexpr uint8_t kClOrder[kClSyms] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// The code-length code of a dynamic header.  Its limits live in registers
// (indexed by constants only); the bases, the symbols sorted by (length,
// value) and a scratch row of offsets are indexed by data, so they live in
// a store (host: arrays; device: a few bytes of the lane's LDS):
//   int32_t& base(int l); uint8_t& sym(int i); uint8_t& off(int l)
constexpr int kClBits = 7;  // longest code-length code
struct ClCode {
  uint32_t limit[kClBits + 1];  // left-justified 7-bit codes below limit[l] have length <= l
  // st.base(l) for l = 1..7 as signed bytes of one register pair (|base| <
  // 128: 19 symbols, 7-bit codes), so a symbol costs one table read, not two
  // dependent ones (the search's and the decode's header walks are chains of
  // them); an array here was indexed from scratch memory
  uint64_t base8;
  GG_HD int32_t base_of(uint32_t L) const { return (int32_t)(int8_t)(uint8_t)(base8 >> (8 * L)); }
};
struct ClArrays {
  int32_t b[kClBits + 1];
  uint8_t s[kClSyms + 1];
  uint8_t o[kClBits + 1];
  int32_t& base(int l) { return b[l]; }
  uint8_t& sym(int i) { return s[i]; }
  uint8_t& off(int l) { return o[l]; }
};

// The length of code-length symbol s, from the header's HCLEN + 4 fields
// (3 bits each, in kClOrder) packed into f.
constexpr uint8_t kClField[kClSyms] = {3, 17, 15, 13, 11, 9, 7, 5, 4, 6, 8, 10, 12, 14, 16, 18, 0, 1, 2};
GG_HD uint32_t cl_len(uint64_t f, uint32_t hclen, int s) {
  return kClField[s] < hclen ? (uint32_t)(f >> (3 * kClField[s])) & 7u : 0u;
}

// The code-length code at pos (pos + 17 of the header; hclen = HCLEN + 4);
// false if it is not complete (zlib refuses an incomplete code-length code).
// pos is moved past its fields.
template <class ClS, class B>
GG_HD bool read_cl_code(const B& in, uint64_t& pos, uint32_t hclen, ClCode& cl, ClS& st) {
  const uint64_t f = (uint64_t)in.peek(pos) | ((uint64_t)in.peek(pos + 32) << 32);
  pos += 3 * hclen;
  uint32_t count[kClBits + 1];
#pragma unroll
  for (int l = 0; l <= kClBits; ++l) count[l] = 0;
#pragma unroll
  for (int s = 0; s < kClSyms; ++s) {
    const uint32_t l = cl_len(f, hclen, s);
#pragma unroll
    for (int m = 1; m <= kClBits; ++m) count[m] += l == (uint32_t)m ? 1u : 0u;
  }
  int left = 1;
  uint32_t first = 0, offs = 0;
  uint64_t base8 = 0;
#pragma unroll
  for (int l = 1; l <= kClBits; ++l) {
    left = (left << 1) - (int)count[l];
    cl.limit[l] = (first + count[l]) << (kClBits - l);
    st.base(l) = (int32_t)offs - (int32_t)first;
    base8 |= (uint64_t)(uint8_t)(int8_t)((int32_t)offs - (int32_t)first) << (8 * l);
    st.off(l) = (uint8_t)offs;
    offs += count[l];
    first = (first + count[l]) << 1;
  }
  cl.limit[0] = 0;
  cl.base8 = base8;
  if (left != 0) return false;  // incomplete or over-subscribed
#pragma unroll
  for (int s = 0; s < kClSyms; ++s) {
    const uint32_t l = cl_len(f, hclen, s);
    if (l) {
      const uint8_t o = st.off((int)l);
      st.sym(o) = (uint8_t)s;
      st.off((int)l) = (uint8_t)(o + 1);
    }
  }
  return true;
}

template <class ClS, class B>
GG_HD int decode_cl_sym(const B& in, uint64_t& pos, const ClCode& cl, ClS& st) {
  const uint32_t x = rev15(in.peek(pos)) >> (kMaxBits - kClBits);  // left-justified 7 bits
  int L = 1;
#pragma unroll
  for (int l = 1; l < kClBits; ++l) L += x >= cl.limit[l] ? 1 : 0;
  if (x >= cl.limit[kClBits]) return -1;
  pos += (uint32_t)L;
  return st.sym(cl.base_of((uint32_t)L) + (int)(x >> (kClBits - L)));
}

// Walks the lit/len + distance code lengths of a dynamic header (after the
// code-length code), calling f(symbol index, length) for each nonzero
// length (f returns false to stop: the walk then fails); false on a
// malformed sequence.
template <class ClS, class F, class B>
GG_HD bool walk_lengths(const B& in, uint64_t& pos, const ClCode& cl, ClS& st, uint32_t n, F&& f) {
  uint32_t i = 0, prev = 0;
  while (i < n) {
    const int s = decode_cl_sym(in, pos, cl, st);
    if (s < 0) return false;
    if (s < 16) {
      if (s && !f(i, (uint32_t)s)) return false;
      prev = (uint32_t)s;
      ++i;
      continue;
    }
    uint32_t rep, val = 0;
    if (s == 16) {
      if (i == 0) return false;
      rep = 3 + in.get(pos, 2);
      val = prev;
    } else if (s == 17) {
      rep = 3 + in.get(pos, 3);
    } else {
      rep = 11 + in.get(pos, 7);
    }
    if (i + rep > n) return false;
    if (val)
      for (uint32_t r = 0; r < rep; ++r)
        if (!f(i + r, val)) return false;
    i += rep;
    if (s != 16) prev = 0;
  }
  return true;
}

// The search's first filter, from registers only: BTYPE 10 (dynamic), HLIT
// and HDIST in range, and a complete code-length code (its Kraft sum over
// the 3-bit lengths, sum 2^(7 - len) = 128).  Passes ~0.1% of the
// positions of a zlib stream.
template <class B>
GG_HD bool block_header_quick(const B& in, uint64_t pos) {
  const uint32_t h = in.peek(pos);
  if (((h >> 1) & 3u) != 2u) return false;  // BTYPE 10: dynamic Huffman
  if (((h >> 3) & 31u) > 29u || ((h >> 8) & 31u) > 29u) return false;  // HLIT <= 286, HDIST <= 30
  const uint32_t hclen = ((h >> 13) & 15u) + 4u;
  const uint64_t f = (uint64_t)in.peek(pos + 17) | ((uint64_t)in.peek(pos + 49) << 32);
  uint32_t kraft = 0;
#pragma unroll
  for (uint32_t i = 0; i < (uint32_t)kClSyms; ++i) {
    const uint32_t l = (uint32_t)(f >> (3 * i)) & 7u;
    kraft += (i < hclen && l) ? 128u >> l : 0u;
  }
  return kraft == 128u;
}

// Is there a valid dynamic-block header at pos?  (The search's test: a
// complete code-length code, length sequence in range, an end-of-block
// code, lit/len and distance codes zlib accepts -- complete, or a single
// code of length 1, or, for distances, none.)  The codes are judged by
// their Kraft sums as the lengths are walked (in units of 2^-15; an
// over-subscribed code stops the walk: most positions that pass the quick
// filter fail within a few dozen lengths), with no table built.  On
// success pos is moved past the header.
template <class ClS, class B>
GG_HD bool block_header_ok(const B& in, uint64_t& pos, ClS& st) {
  if (!block_header_quick(in, pos)) return false;
  const uint32_t h = in.peek(pos);
  const uint32_t hlit = ((h >> 3) & 31u) + 257u, hdist = ((h >> 8) & 31u) + 1u, hclen = ((h >> 13) & 15u) + 4u;
  uint64_t p = pos + 17;
  ClCode cl;
  if (!read_cl_code(in, p, hclen, cl, st)) return false;
  bool eob = false;
  uint32_t kl = 0, kd = 0, nd = 0, ml = 0, md = 0;
  if (!walk_lengths(in, p, cl, st, hlit + hdist, [&](uint32_t i, uint32_t len) {
        if (i < hlit) {
          eob |= i == 256;
          kl += 1u << (kMaxBits - len);
          ml = len > ml ? len : ml;
          return kl <= (1u << kMaxBits);
        }
        kd += 1u << (kMaxBits - len);
        ++nd;
        md = len > md ? len : md;
        return kd <= (1u << kMaxBits);
      }))
    return false;
  if (!eob) return false;
  // (code_ok: complete, or incomplete with its longest code of length 1)
  if (kl != (1u << kMaxBits) && ml != 1) return false;
  if (nd && kd != (1u << kMaxBits) && md != 1) return false;
  pos = p;
  return true;
}

// block_header_ok as a walk of one code-length symbol per step, so that the
// lanes of a wave can each walk a different candidate and take the next one
// as soon as theirs is decided (the search's checks; a wave-wide round of
// block_header_ok lasts as long as its longest walk).  start() reads the
// fields and the code-length code (false: rejected already); step() returns
// 0 (more), 1 (a valid header) or -1 (rejected).  A repeat code's lengths
// are added at once: the Kraft sums only grow, so the verdict is
// block_header_ok's.
struct HeaderWalk {
  uint64_t pos;
  ClCode cl;
  uint32_t i, n, hlit, prev;
  uint32_t kl, kd, nd, ml, md;
  bool eob;

  template <class ClS, class B>
  GG_HD bool start(const B& in, uint64_t p, ClS& st) {
    if (!block_header_quick(in, p)) return false;
    const uint32_t h = in.peek(p);
    hlit = ((h >> 3) & 31u) + 257u;
    n = hlit + ((h >> 8) & 31u) + 1u;
    pos = p + 17;
    if (!read_cl_code(in, pos, ((h >> 13) & 15u) + 4u, cl, st)) return false;
    i = prev = kl = kd = nd = ml = md = 0;
    eob = false;
    return true;
  }
  GG_HD void add(uint32_t len, uint32_t rep) {  // lengths i .. i + rep - 1 = len (> 0)
    const uint32_t rl = i < hlit ? (rep < hlit - i ? rep : hlit - i) : 0u, rd = rep - rl;
    if (rl) {
      kl += rl << (kMaxBits - len);
      ml = len > ml ? len : ml;
      eob |= i <= 256u && 256u < i + rl;
    }
    if (rd) {
      kd += rd << (kMaxBits - len);
      nd += rd;
      md = len > md ? len : md;
    }
  }
  template <class ClS, class B>
  GG_HD int step(const B& in, ClS& st) {
    const uint32_t x = in.peek(pos);
    const uint32_t y = rev15(x) >> (kMaxBits - kClBits);  // left-justified 7 bits
    if (y >= cl.limit[kClBits]) return -1;
    uint32_t L = 1;
#pragma unroll
    for (int l = 1; l < kClBits; ++l) L += y >= cl.limit[l] ? 1u : 0u;
    const int s = st.sym(cl.base_of(L) + (int)(y >> (kClBits - L)));
    pos += L;
    if (s < 16) {
      if (s) add((uint32_t)s, 1);
      prev = (uint32_t)s;
      ++i;
    } else {
      const uint32_t e = x >> L;  // (the repeat's extra bits follow the code)
      uint32_t rep, val = 0;
      if (s == 16) {
        if (i == 0) return -1;
        rep = 3 + (e & 3u);
        pos += 2;
        val = prev;
      } else if (s == 17) {
        rep = 3 + (e & 7u);
        pos += 3;
      } else {
        rep = 11 + (e & 127u);
        pos += 7;
      }
      if (i + rep > n) return -1;
      if (val) add(val, rep);
      i += rep;
      if (s != 16) prev = 0;
    }
    if (kl > (1u << kMaxBits) || kd > (1u << kMaxBits)) return -1;
    if (i < n) return 0;
    if (!eob) return -1;
    if (kl != (1u << kMaxBits) && ml != 1) return -1;
    if (nd && kd != (1u << kMaxBits) && md != 1) return -1;
    return 1;
  }
};

// One lane's tables for its current block, in the Store (host: arrays;
// device: LDS): the limits (only the long codes past the one-lookup tables
// read them), the bases, the symbols sorted by (length, value) and the
// per-length counts a header read keeps:
//   uint32_t& llim(int), dlim(int); int32_t& lbase(int), dbase(int);
//   uint32_t& lcnt(int), dcnt(int); uint16_t& lsym(int); uint8_t& dsym(int)
// Decode entries: the value in bits 0..15 (a literal byte, a length base or
// a distance base), its extra bits in 16..19, the code length in 20..23
// (fast tables only; 0 = not in the table), the kind in 24..25.
#ifndef GG_FAST_BITS  // (A/B builds: -DGG_FAST_BITS=9)
#define GG_FAST_BITS 10
#endif
constexpr int kFastBits = GG_FAST_BITS;
constexpr uint32_t kFastSize = 1u << kFastBits;
constexpr int kFastLenShift = 20;
constexpr uint32_t kFastLenMask = 15u << kFastLenShift;
enum EntryKind : uint32_t { kEntryLit = 0, kEntryLen = 1, kEntryEob = 2, kEntryInvalid = 3 };
constexpr uint32_t kEntryBad = kEntryInvalid << 24;
GG_HD uint32_t entry_kind(uint32_t e) { return e >> 24; }
GG_HD uint32_t entry_value(uint32_t e) { return e & 0xFFFFu; }
GG_HD uint32_t entry_extra(uint32_t e) { return (e >> 16) & 15u; }
GG_HD uint32_t lit_value(int sy) {  // lit/len symbol -> entry (without its code length)
  if (sy < 256) return (uint32_t)sy;
  if (sy == 256) return kEntryEob << 24;
  const uint32_t li = (uint32_t)sy - 257u;
  if (li >= 29) return kEntryBad;
  return (kEntryLen << 24) | (len_extra(li) << 16) | len_base(li);
}
GG_HD uint32_t dist_value(int d) {  // distance symbol -> entry
  if (d >= 30) return kEntryBad;
  return (kEntryLen << 24) | (dist_extra((uint32_t)d) << 16) | dist_base((uint32_t)d);
}

template <class Store>
struct LaneTables {
  Store s;
  GG_HD void set_lit(const Canon& c) {
#pragma unroll
    for (int l = 0; l <= kMaxBits; ++l) {
      s.llim(l) = c.limit[l];
      s.lbase(l) = c.base[l];
    }
  }
  GG_HD void set_dist(const Canon& c) {
#pragma unroll
    for (int l = 0; l <= kMaxBits; ++l) {
      s.dlim(l) = c.limit[l];
      s.dbase(l) = c.base[l];
    }
  }
  // A symbol as a table entry (fast_entry): codes of <= kFastBits bits in
  // one lookup of the next kFastBits stream bits, longer ones by the limits.
  // The entry is consumed from the cursor.
  template <class Cur>
  GG_HD uint32_t lit_entry(Cur& cur) {
    const uint32_t e = s.lfast(cur.peek() & (kFastSize - 1));
    if (e & kFastLenMask) {
      cur.skip((e >> kFastLenShift) & 15u);
      return e;
    }
    const int sy = lit(cur);
    return sy < 0 ? kEntryBad : lit_value(sy);
  }
  template <class Cur>
  GG_HD uint32_t dist_entry(Cur& cur) {
    const uint32_t e = s.dfast(cur.peek() & (kFastSize - 1));
    if (e & kFastLenMask) {
      cur.skip((e >> kFastLenShift) & 15u);
      return e;
    }
    const int d = dist(cur);
    return d < 0 ? kEntryBad : dist_value(d);
  }
  // The fast entry of the kFastBits stream bits i (LSB first) for the lit/len
  // (dist = false) or distance code: 0 when the code there is longer.
  GG_HD uint32_t fast_entry(uint32_t i, bool dist_code) {
    const uint32_t x = rev15(i);  // (bits past the kFastBits read as 0)
    int L = 1;  // the smallest l with x < limit[l] (15: none below 15)
#pragma unroll
    for (int l = 1; l < kMaxBits; ++l) L += x >= (dist_code ? s.dlim(l) : s.llim(l)) ? 1 : 0;
    if (L > kFastBits) return 0;
    Store& st = s;
    const uint32_t v = dist_code ? dist_value(st.dsym(st.dbase(L) + (int)(x >> (kMaxBits - L))))
                                 : lit_value(st.lsym(st.lbase(L) + (int)(x >> (kMaxBits - L))));
    return v | ((uint32_t)L << kFastLenShift);
  }
  GG_HD void build_fast() {  // (serially; the device builds them with its wave)
    for (uint32_t i = 0; i < kFastSize; ++i) {
      s.lfast((int)i) = fast_entry(i, false);
      s.dfast((int)i) = fast_entry(i, true);
    }
  }
  template <class Cur>
  GG_HD int lit(Cur& cur) {
    const uint32_t x = rev15(cur.peek());
    int L = 1;
#pragma unroll
    for (int l = 1; l < kMaxBits; ++l) L += x >= s.llim(l) ? 1 : 0;
    if (x >= s.llim(kMaxBits)) return -1;
    cur.skip((uint32_t)L);
    return s.lsym(s.lbase(L) + (int)(x >> (kMaxBits - L)));
  }
  template <class Cur>
  GG_HD int dist(Cur& cur) {
    const uint32_t x = rev15(cur.peek());
    int L = 1;
#pragma unroll
    for (int l = 1; l < kMaxBits; ++l) L += x >= s.dlim(l) ? 1 : 0;
    if (x >= s.dlim(kMaxBits)) return -1;
    cur.skip((uint32_t)L);
    return s.dsym(s.dbase(L) + (int)(x >> (kMaxBits - L)));
  }
};

// Host store: plain arrays.  (lcnt / dcnt: counts per length, then the
// next slot per length, while a header is read.)
struct ArrayStore {
  uint32_t ll[kMaxBits + 1], dl[kMaxBits + 1];
  int32_t lb[kMaxBits + 1], db[kMaxBits + 1];
  uint32_t lc[kMaxBits + 1], dc[kMaxBits + 1];
  uint16_t ls[kLitSyms];
  uint8_t ds[kDistSyms];
  uint32_t lf[kFastSize], df[kFastSize];
  uint32_t& lfast(int i) { return lf[i]; }
  uint32_t& dfast(int i) { return df[i]; }
  uint32_t& llim(int l) { return ll[l]; }
  uint32_t& dlim(int l) { return dl[l]; }
  int32_t& lbase(int l) { return lb[l]; }
  int32_t& dbase(int l) { return db[l]; }
  uint32_t& lcnt(int l) { return lc[l]; }
  uint32_t& dcnt(int l) { return dc[l]; }
  uint16_t& lsym(int i) { return ls[i]; }
  uint8_t& dsym(int i) { return ds[i]; }
};

// Reads the block header at pos and builds the lane's tables.  Returns
// btype (0 stored, 1 fixed, 2 dynamic) or -1 on a malformed header; bfinal
// receives the BFINAL bit.  For a stored block pos ends at its first data
// byte and stored_len receives LEN.
template <class Store, class ClS>
GG_HD int read_block_header(const Bits& in, uint64_t& pos, LaneTables<Store>& t, ClS& cls, uint32_t& bfinal,
                            uint32_t& stored_len) {
  const uint32_t h = in.peek(pos);
  bfinal = h & 1u;
  const uint32_t btype = (h >> 1) & 3u;
  if (btype == 0) {
    pos = (pos + 3 + 7) & ~7ull;
    const uint32_t v = in.peek(pos);
    const uint32_t len = v & 0xFFFFu, nlen = v >> 16;
    if ((len ^ nlen) != 0xFFFFu) return -1;
    pos += 32;
    stored_len = len;
    return 0;
  }
  uint32_t lc[kMaxBits + 1], dc[kMaxBits + 1];  // (indexed by constants only)
#pragma unroll
  for (int l = 0; l <= kMaxBits; ++l) lc[l] = dc[l] = 0;
  int ml = 0;
  Canon c{};
  if (btype == 1) {  // fixed codes (RFC 1951 3.2.6)
    pos += 3;
    lc[7] = 24;
    lc[8] = 152;
    lc[9] = 112;
    dc[5] = 32;
    canon_from_counts(lc, c, ml);
    t.set_lit(c);
    canon_from_counts(dc, c, ml);
    t.set_dist(c);
    uint32_t o7 = 0, o8 = 24, o9 = 176;
    for (uint32_t sy = 0; sy < (uint32_t)kLitSyms; ++sy) {
      if (sy <= 143) t.s.lsym((int)o8++) = (uint16_t)sy;
      else if (sy <= 255) t.s.lsym((int)o9++) = (uint16_t)sy;
      else if (sy <= 279) t.s.lsym((int)o7++) = (uint16_t)sy;
      else t.s.lsym((int)o8++) = (uint16_t)sy;
    }
    for (uint32_t d = 0; d < (uint32_t)kDistSyms; ++d) t.s.dsym((int)d) = (uint8_t)d;
    t.build_fast();
    return 1;
  }
  if (btype != 2) return -1;
  const uint32_t hlit = ((h >> 3) & 31u) + 257u, hdist = ((h >> 8) & 31u) + 1u, hclen = ((h >> 13) & 15u) + 4u;
  if (hlit > 286 || hdist > 30) return -1;
  uint64_t p = pos + 17;
  ClCode cl;
  if (!read_cl_code(in, p, hclen, cl, cls)) return -1;
  const uint64_t lens_at = p;
  bool eob = false;
  // pass 1: counts per length (in the store: indexed by data)
#pragma unroll
  for (int l = 0; l <= kMaxBits; ++l) t.s.lcnt(l) = t.s.dcnt(l) = 0;
  if (!walk_lengths(in, p, cl, cls, hlit + hdist, [&](uint32_t i, uint32_t len) {
        if (i < hlit) {
          t.s.lcnt((int)len) += 1;
          eob |= i == 256;
        } else {
          t.s.dcnt((int)len) += 1;
        }
        return true;
      }))
    return -1;
  if (!eob) return -1;
#pragma unroll
  for (int l = 1; l <= kMaxBits; ++l) {
    lc[l] = t.s.lcnt(l);
    dc[l] = t.s.dcnt(l);
  }
  int r = canon_from_counts(lc, c, ml);
  if (!code_ok(r, ml, false)) return -1;
  t.set_lit(c);
  r = canon_from_counts(dc, c, ml);
  if (!code_ok(r, ml, true)) return -1;
  t.set_dist(c);
  // pass 2: symbols sorted by (length, value) (the lengths are walked again
  // instead of being stored); lcnt / dcnt become each length's next slot
  uint32_t a = 0, b = 0;
#pragma unroll
  for (int l = 1; l <= kMaxBits; ++l) {
    t.s.lcnt(l) = a;
    t.s.dcnt(l) = b;
    a += lc[l];
    b += dc[l];
  }
  uint64_t q = lens_at;
  walk_lengths(in, q, cl, cls, hlit + hdist, [&](uint32_t i, uint32_t len) {
    if (i < hlit) t.s.lsym((int)t.s.lcnt((int)len)++) = (uint16_t)i;
    else t.s.dsym((int)t.s.dcnt((int)len)++) = (uint8_t)(i - hlit);
    return true;
  });
  t.build_fast();
  pos = p;
  return 2;
}

// Token: a literal byte (bit 31 clear) or a match, bit 31 set, length in
// bits 15..23 (3..258), distance - 1 in bits 0..14.
GG_HD uint32_t tok_match(uint32_t len, uint32_t dist) { return 0x80000000u | (len << 15) | (dist - 1u); }
GG_HD bool tok_is_match(uint32_t t) { return (t >> 31) != 0; }
GG_HD uint32_t tok_len(uint32_t t) { return tok_is_match(t) ? (t >> 15) & 0x1FFu : 1u; }
GG_HD uint32_t tok_dist(uint32_t t) { return (t & 0x7FFFu) + 1u; }

enum DecodeStatus : uint32_t {
  kDecOk = 0,          // landed on `end` (or ended the stream with BFINAL when end = ~0)
  kDecOverrun = 1,     // passed `end` without landing on it: `end` is not a block boundary
  kDecBad = 2,         // malformed data
  kDecFull = 3,        // token capacity exceeded
  kDecFinalEarly = 4,  // the stream's last block ended before `end`
};

// Decodes blocks from pos until a block ends exactly at `end` (~0: until
// the BFINAL block), writing tokens through emit(t) (returns false when
// full).  out_len receives the bytes the tokens stand for, last_end the bit
// position after the last decoded block.
template <class Store, class ClS, class Emit>
GG_HD uint32_t decode_blocks(const Bits& in, uint64_t pos, uint64_t end, uint64_t limit_bits, LaneTables<Store>& t,
                             ClS& cls, Emit&& emit, uint64_t& out_len, uint64_t& last_end, uint32_t& bfinal_seen) {
  out_len = 0;
  bfinal_seen = 0;
  last_end = pos;
  for (;;) {
    if (pos == end) {
      last_end = pos;
      return kDecOk;
    }
    if (pos > end || pos >= limit_bits) {
      last_end = pos;
      return kDecOverrun;
    }
    uint32_t bfinal = 0, stored = 0;
    const int bt = read_block_header(in, pos, t, cls, bfinal, stored);
    if (bt < 0) {
      last_end = pos;
      return kDecBad;
    }
    if (bt == 0) {
      for (uint32_t i = 0; i < stored; ++i)
        if (!emit(in.get(pos, 8))) return kDecFull;
      out_len += stored;
    } else {
      Cursor cur{in.w};
      cur.seek(pos);
      for (;;) {
        if (cur.pos >= limit_bits) {
          last_end = cur.pos;
          return kDecBad;
        }
        const uint32_t e = t.lit_entry(cur);
        const uint32_t kind = entry_kind(e);
        if (kind == kEntryLit) {
          if (!emit(entry_value(e))) return kDecFull;
          out_len += 1;
          continue;
        }
        if (kind == kEntryEob) break;
        if (kind != kEntryLen) {
          last_end = cur.pos;
          return kDecBad;
        }
        const uint32_t len = entry_value(e) + cur.get(entry_extra(e));
        const uint32_t de = t.dist_entry(cur);
        if (entry_kind(de) != kEntryLen) {
          last_end = cur.pos;
          return kDecBad;
        }
        const uint32_t dist = entry_value(de) + cur.get(entry_extra(de));
        if (!emit(tok_match(len, dist))) return kDecFull;
        out_len += len;
      }
      pos = cur.pos;
    }
    if (bfinal) {
      bfinal_seen = 1;
      last_end = pos;
      return end == ~0ull ? kDecOk : kDecFinalEarly;
    }
  }
}

// One sub-span of a block body, decoded speculatively.  The device splits a
// block's body [body0, span_end) into up to 64 sub-spans of L bits, one
// lane each, all decoded at once with the block's tables, each from its
// span's start S (usually inside a symbol) until the first symbol start at
// or past its span's end R (or the end-of-block symbol, or an invalid code).
//
// Chaining.  Decoding is deterministic from a symbol start, and a decode
// begun inside a symbol falls onto the true symbol starts after a while
// (a median of ~150 bits on FASTA; a few never do within a span).  The
// decode records checkpoints: for k = 0, 1, ..., the first symbol start at
// or after S + 64k, with the tokens and bytes emitted before it.  The lane
// before ends at E, the true first symbol start at or after S:
//   - checkpoint 0 at E: this lane was right from its start (its tokens
//     before E dropped);
//   - otherwise the lane decodes again from E, comparing each of its
//     checkpoints with the first decode's: at the first that agrees both
//     decodes are on the same symbol start, so the second stops there and
//     the first decode's tokens from that checkpoint on complete it.
// Each such round makes the first lane not yet right right, and one round
// almost always fixes all of them.
enum SpanStatus : uint32_t {
  kSpanRange = 0,   // reached range_end (stop: the first symbol start >= range_end)
  kSpanEob = 1,     // decoded the end-of-block symbol (stop: the bit after it)
  kSpanBad = 2,     // an invalid code or length/distance symbol
  kSpanSynced = 3,  // ck() returned false at a checkpoint (stop: that symbol start)
};
constexpr uint32_t kCkBits = 64;  // checkpoint spacing: > the longest symbol (15 + 5 + 15 + 13 bits)

// A checkpoint: its symbol start's offset past S + 64k (< 64), the tokens
// before it (24 bits) and the bytes they stand for (32 bits).
GG_HD uint64_t ck_pack(uint32_t off, uint32_t n, uint64_t bytes) {
  return (uint64_t)off | ((uint64_t)n << 8) | (bytes << 32);
}
GG_HD uint32_t ck_off(uint64_t c) { return (uint32_t)c & 0xFFu; }
GG_HD uint32_t ck_tok(uint64_t c) { return (uint32_t)(c >> 8) & 0xFFFFFFu; }
GG_HD uint64_t ck_bytes(uint64_t c) { return c >> 32; }

// Decodes from start; ck(k, c) is called at the first symbol start at or
// after s_nom + 64k for every k (c = ck_pack of it; a symbol start before
// s_nom has no checkpoint) and stops the decode when it returns false.
// n and bytes receive the tokens emitted and the bytes they stand for,
// stop the bit position where decoding stopped.
template <class Store, class Emit, class Ck>
GG_HD uint32_t decode_span(const Bits& in, uint64_t start, uint64_t s_nom, uint64_t range_end, LaneTables<Store>& t,
                           Emit&& emit, Ck&& ck, uint32_t& n, uint64_t& bytes, uint64_t& stop) {
  Cursor cur{in.w};
  cur.seek(start);
  n = 0;
  bytes = 0;
  uint32_t k = 0;
  uint64_t next_ck = s_nom;
  uint64_t next_stop = next_ck < range_end ? next_ck : range_end;  // (one compare per symbol)
  for (;;) {
    if (cur.pos >= next_stop) {
      if (cur.pos >= range_end) {
        stop = cur.pos;
        return kSpanRange;
      }
      if (cur.pos >= next_ck) {  // (a symbol is shorter than kCkBits: one checkpoint at most)
        if (!ck(k, ck_pack((uint32_t)(cur.pos - next_ck), n, bytes))) {
          stop = cur.pos;
          return kSpanSynced;
        }
        ++k;
        next_ck += kCkBits;
      }
      next_stop = next_ck < range_end ? next_ck : range_end;
    }
    // one token from 64 peeked bits: the lit/len code and, for a length,
    // its extra bits, the distance code and its extra bits (<= 10 + 5 + 10
    // + 13 bits through the one-lookup tables); longer codes take the
    // limits (lit_entry / dist_entry)
    const uint64_t bb = cur.peek64();
    uint32_t e = t.s.lfast((int)(bb & (kFastSize - 1)));
    uint32_t used = (e >> kFastLenShift) & 15u;
    if (used == 0) {  // a long lit/len code
      e = t.lit_entry(cur);
      if (entry_kind(e) != kEntryLen) {
        if (entry_kind(e) == kEntryLit) {
          if (!emit(entry_value(e))) break;
          ++n;
          bytes += 1;
          continue;
        }
        if (entry_kind(e) == kEntryEob) {
          stop = cur.pos;
          return kSpanEob;
        }
        break;
      }
      const uint32_t len = entry_value(e) + cur.get(entry_extra(e));
      const uint32_t de = t.dist_entry(cur);
      if (entry_kind(de) != kEntryLen) break;
      const uint32_t dist = entry_value(de) + cur.get(entry_extra(de));
      if (!emit(tok_match(len, dist))) break;
      ++n;
      bytes += len;
      continue;
    }
    const uint32_t kind = entry_kind(e);
    if (kind == kEntryLit) {
      cur.skip(used);
      if (!emit(entry_value(e))) break;
      ++n;
      bytes += 1;
      continue;
    }
    if (kind != kEntryLen) {
      if (kind == kEntryEob) {
        cur.skip(used);
        stop = cur.pos;
        return kSpanEob;
      }
      cur.skip(used);
      break;
    }
    const uint32_t lx = entry_extra(e);
    const uint32_t len = entry_value(e) + ((uint32_t)(bb >> used) & ((1u << lx) - 1u));
    used += lx;
    const uint32_t de = t.s.dfast((int)((bb >> used) & (kFastSize - 1)));
    const uint32_t dl = (de >> kFastLenShift) & 15u;
    uint32_t dist;
    if (dl == 0) {  // a long distance code
      cur.skip(used);
      const uint32_t d2 = t.dist_entry(cur);
      if (entry_kind(d2) != kEntryLen) break;
      dist = entry_value(d2) + cur.get(entry_extra(d2));
    } else {
      if (entry_kind(de) != kEntryLen) {
        cur.skip(used + dl);
        break;
      }
      used += dl;
      const uint32_t dx = entry_extra(de);
      dist = entry_value(de) + ((uint32_t)(bb >> used) & ((1u << dx) - 1u));
      cur.skip_long(used + dx);
    }
    if (!emit(tok_match(len, dist))) break;
    ++n;
    bytes += len;
  }
  stop = cur.pos;
  return kSpanBad;
}

// Sub-span layout of a block body [body0, span_end): nsub lanes of L bits
// (at least kMinSpanBits each); the last lane runs to span_end.
constexpr uint64_t kMinSpanBits = 256;
GG_HD void span_layout(uint64_t body0, uint64_t span_end, uint32_t max_lanes, uint64_t& L, uint32_t& nsub) {
  const uint64_t bits = span_end > body0 ? span_end - body0 : 0;
  L = (bits + max_lanes - 1) / max_lanes;
  if (L < kMinSpanBits) L = kMinSpanBits;
  nsub = (uint32_t)((bits + L - 1) / L);
  if (nsub == 0) nsub = 1;
}

// Per lane of a segment's decode: two token areas (the first decode, the
// second) of span_cap(L) tokens each -- a decode of [S - kWarmBits, R + 48)
// emits at most one token per bit -- and span_cks(L) checkpoints (u32: the
// low word of ck_pack; the device decode counts no bytes).
#ifndef GG_DECODE_WARM_BITS  // (A/B builds: scripts/ab_lib.sh ... -DGG_DECODE_WARM_BITS=0)
#define GG_DECODE_WARM_BITS 256
#endif
constexpr uint64_t kWarmBits = GG_DECODE_WARM_BITS;  // a lane's first decode starts this far before its span
// tight: a quarter of that plus 64 (FASTA streams emit ~0.08 tokens per
// bit; a decode that fills a tight area fails its batch's first attempt,
// which is then decoded again with full areas: inflate_host.cpp)
GG_HD uint64_t span_cap(uint64_t L, bool tight = false) {
  const uint64_t bits = L + kWarmBits + kCkBits;
  return ((tight ? bits / 4 + 64 : bits) + 3) / 4 * 4;
}
GG_HD uint64_t span_cks(uint64_t L) { return (L / kCkBits + 4) & ~1ull; }  // (even: areas stay 16-byte aligned)
GG_HD uint64_t span_words(uint64_t L, bool tight = false) { return 2 * span_cap(L, tight) + span_cks(L); }  // (u32 words, even)
// Scratch words the device decode of a segment of seg_bits bits needs (L
// as span_layout makes it for the segment's longest possible body, or for
// the longest window of window_bits when the segment is decoded in windows
// of at most that many bits).
GG_HD uint64_t decode_scratch(uint64_t seg_bits, uint64_t window_bits = ~0ull, bool tight = false) {
  uint64_t L;
  uint32_t nsub;
  span_layout(0, seg_bits < window_bits ? seg_bits : window_bits, 64, L, nsub);
  return 64 * span_words(L, tight);
}

}  // namespace inflate
}  // namespace gg
