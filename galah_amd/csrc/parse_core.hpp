// Bit-parallel FASTA classification for the device parser (parse.hip), host
// and device.  A thread owns 32 consecutive bytes of a block; everything the
// three parse passes need from them is computed as 32-bit masks (bit j =
// byte j) instead of byte by byte:
//   * the bytes are transposed so that word q holds bytes q, q+8, q+16,
//     q+24 (byte_perm), then each word is classified with two byte lookups
//     (byte_perm as an 8-entry table on the low 3 bits) and an exact
//     zero-byte test: A C G T U (either case) -> base + 2-bit code,
//     ' ' '\t' '\r' '\n' -> skip, '\n' and '>' flagged for the line logic;
//   * per-byte flags are gathered into natural-order masks by shifts;
//   * header lines, the state carried across skipped bytes and run starts
//     are carry chains (fill: Kogge-Stone over 32 bits);
//   * the bases' 2-bit codes are compacted (compress, Hacker's Delight 7-4)
//     into one 64-bit value, first base in the top bits (the packed word
//     order of pack.cpp).
// Byte semantics are pack.cpp's (restating needletail 0.5 + normalize(false)
// as galah's finch path uses it, src/finch.rs:47); tests/cpp/test_parse_core
// checks every function here against a byte-by-byte restatement.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define GG_PC_FN __host__ __device__ __forceinline__
#else
#define GG_PC_FN inline
#endif

namespace gg {
namespace parse {

// v_perm_b32: byte i of the result = byte sel.byte[i] of {hi (bytes 4-7), lo
// (bytes 0-3)} (selectors 0..7 only here)
GG_PC_FN uint32_t byte_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(hi, lo, sel);
#else
  const uint64_t d = ((uint64_t)hi << 32) | lo;
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) r |= (uint32_t)((d >> (8 * ((sel >> (8 * i)) & 7u))) & 0xFFu) << (8 * i);
  return r;
#endif
}
GG_PC_FN int popc(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popc(x);
#else
  return __builtin_popcount(x);
#endif
}
GG_PC_FN int clz(uint32_t x) {  // (x != 0)
#if defined(__HIP_DEVICE_COMPILE__)
  return __clz((int)x);
#else
  return __builtin_clz(x);
#endif
}
GG_PC_FN int ctz(uint32_t x) {  // (x != 0)
#if defined(__HIP_DEVICE_COMPILE__)
  return __ffs((int)x) - 1;
#else
  return __builtin_ctz(x);
#endif
}
GG_PC_FN uint32_t brev(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __brev(x);
#else
  x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
  x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
  x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
  x = ((x >> 8) & 0x00FF00FFu) | ((x & 0x00FF00FFu) << 8);
  return (x >> 16) | (x << 16);
#endif
}

// 0x80 in every zero byte of y, 0 elsewhere (exact)
GG_PC_FN uint32_t zero_bytes(uint32_t y) { return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u; }

// the 32 bytes' masks
struct Masks {
  uint32_t base;  // A C G T U, either case (before header lines are taken out)
  uint32_t skip;  // ' ' '\t' '\r' '\n'
  uint32_t past;  // bytes past the block (dropped)
  uint32_t nl;    // '\n'
  uint32_t gt;    // '>'
  uint32_t c0, c1;  // the base's 2-bit code (A 0, C 1, G 2, T/U 3), bits 0 and 1
};

// w[q]: bytes 4q .. 4q+3 of the thread's 32 (little-endian); lim: bytes of
// the block among them (the rest read as skip)
GG_PC_FN Masks classify(const uint32_t (&w)[8], uint32_t lim) {
  // transpose: t[q] = bytes q, q+8, q+16, q+24
  uint32_t t[8];
#pragma unroll
  for (int h = 0; h < 2; ++h) {  // h = 0: words 0 2 4 6 (bytes 0-3 of each 8), h = 1: words 1 3 5 7
    const uint32_t a = w[h], b = w[h + 2], c = w[h + 4], d = w[h + 6];
    const uint32_t p_ab = byte_perm(b, a, 0x05010400u), q_ab = byte_perm(b, a, 0x07030602u);  // a0 b0 a1 b1 | a2 b2 a3 b3
    const uint32_t p_cd = byte_perm(d, c, 0x05010400u), q_cd = byte_perm(d, c, 0x07030602u);
    t[4 * h + 0] = byte_perm(p_cd, p_ab, 0x05040100u);  // a0 b0 c0 d0
    t[4 * h + 1] = byte_perm(p_cd, p_ab, 0x07060302u);  // a1 b1 c1 d1
    t[4 * h + 2] = byte_perm(q_cd, q_ab, 0x05040100u);
    t[4 * h + 3] = byte_perm(q_cd, q_ab, 0x07060302u);
  }
  Masks m{0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint32_t x = t[q];
    // letters: l = x | 0x20, slot l & 7 -> a(1) c(3) t(4) u(5) g(7)
    const uint32_t l = x | 0x20202020u, sl = l & 0x07070707u;
    const uint32_t zl = zero_bytes(l ^ byte_perm(0x67007574u, 0x63006100u, sl));
    const uint32_t code = byte_perm(0x02000303u, 0x01000000u, sl);
    // the rest: slot x & 7 -> ' '(0) '\t'(1) '\n'(2) '\r'(5) '>'(6); kind:
    // 0x80 skip, 0x40 '\n', 0x20 '>'
    const uint32_t so = x & 0x07070707u;
    const uint32_t zo = zero_bytes(x ^ byte_perm(0x003E0D00u, 0x000A0920u, so));
    const uint32_t kind = byte_perm(0x00208000u, 0x00C08080u, so);
    const int sh = 7 - q;  // (byte q + 8k sits at bit 7 + 8k of the flags: to bit q + 8k)
    m.base |= zl >> sh;
    m.skip |= (zo & kind) >> sh;
    m.nl |= (zo & (kind << 1)) >> sh;
    m.gt |= (zo & (kind << 2)) >> sh;
    m.c0 |= ((code << 7) & 0x80808080u) >> sh;
    m.c1 |= ((code << 6) & 0x80808080u) >> sh;
  }
  const uint32_t in = lim >= 32 ? ~0u : (1u << lim) - 1u;
  m.base &= in;
  m.nl &= in;
  m.gt &= in;
  m.past = ~in;
  return m;
}

// F(j) = g(j) | p(j) & F(j - 1), F(-1) = cin
GG_PC_FN uint32_t fill(uint32_t g, uint32_t p, bool cin) {
  g |= p & (cin ? 1u : 0u);
#pragma unroll
  for (int d = 1; d < 32; d <<= 1) {
    g |= p & (g << d);
    p &= p << d;
  }
  return g;
}

// the bytes' roles once header lines are known
struct Roles {
  uint32_t base;  // a base (code in c0/c1)
  uint32_t brk;   // breaks a k-mer: any other byte, or a header line's byte ('\n' aside)
  uint32_t keep;  // not dropped: base | brk
};
// line0: byte 0 starts a line; hdr0: otherwise, the line byte 0 is on is a
// header ('>' at its start)
GG_PC_FN Roles roles(const Masks& m, bool line0, bool hdr0) {
  const uint32_t ls = (m.nl << 1) | (line0 ? 1u : 0u);  // line starts
  const uint32_t hdr = fill(ls & m.gt, ~ls, hdr0);     // bytes on header lines
  Roles r;
  r.base = m.base & ~hdr;
  const uint32_t drop = m.nl | m.past | (m.skip & ~hdr);
  r.brk = ~drop & ~r.base;
  r.keep = ~drop;
  return r;
}

// run starts: a base whose last kept byte before it is not a base (prev_base:
// the last kept byte before the 32 is a base)
GG_PC_FN uint32_t run_starts(const Roles& r, bool prev_base) {
  const uint32_t after_base = fill(r.base, ~r.keep, prev_base);  // state after byte j: the last kept byte is a base
  return r.base & ~((after_base << 1) | (prev_base ? 1u : 0u));
}

// x's bits at m's set positions, packed to the low end in order
struct Compress {
  uint32_t mv[5];
  GG_PC_FN explicit Compress(uint32_t m) {
    uint32_t mk = ~m << 1;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      uint32_t mp = mk ^ (mk << 1);
      mp ^= mp << 2;
      mp ^= mp << 4;
      mp ^= mp << 8;
      mp ^= mp << 16;
      mv[i] = mp & m;
      m = (m ^ mv[i]) | (mv[i] >> (1 << i));
      mk &= ~mp;
    }
  }
  GG_PC_FN uint32_t operator()(uint32_t x, uint32_t m0) const {
    x &= m0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const uint32_t t = x & mv[i];
      x = (x ^ t) | (t >> (1 << i));
    }
    return x;
  }
};

GG_PC_FN uint64_t spread(uint32_t x) {  // bit i -> bit 2i
  uint64_t v = x;
  v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
  v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
  v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
  v = (v | (v << 2)) & 0x3333333333333333ull;
  v = (v | (v << 1)) & 0x5555555555555555ull;
  return v;
}

// the codes of the bases in order, the first in bits 63-62 (high code bit
// first), as packed words hold them
GG_PC_FN uint64_t packed_codes(const Masks& m, uint32_t base) {
  const Compress c(base);
  const uint64_t v = spread(c(m.c1, base)) | (spread(c(m.c0, base)) << 1);  // base i: c1 at 2i, c0 at 2i + 1
  // bit-reverse: base i -> c1 at 63 - 2i, c0 at 62 - 2i
  return ((uint64_t)brev((uint32_t)v) << 32) | brev((uint32_t)(v >> 32));
}

// R (packed_codes) placed at base offset o (0..15) of a word: the three
// words it touches, in order
GG_PC_FN void place(uint64_t R, uint32_t o, uint32_t& w0, uint32_t& w1, uint32_t& w2) {
  const uint32_t s = 2 * o, hi = (uint32_t)(R >> 32), lo = (uint32_t)R;
  if (s == 0) {
    w0 = hi;
    w1 = lo;
    w2 = 0;
  } else {
    w0 = hi >> s;
    w1 = (hi << (32 - s)) | (lo >> s);
    w2 = lo << (32 - s);
  }
}

}  // namespace parse
}  // namespace gg
