// Host test of galah_amd/csrc/parse_core.hpp (the device parser's
// bit-parallel classification) against a byte-by-byte restatement of the
// same rules (pack.cpp's byte semantics: ACGTU either case -> codes, ' '
// '\t' '\r' '\n' dropped, header lines ('>' at a line start) break, any
// other byte breaks).  Random chunks over an alphabet weighted towards the
// bytes that matter, every block limit, line/header/base state at entry.
// Prints "ok <cases>" or the first mismatch; exit 1 on a mismatch.
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../galah_amd/csrc/parse_core.hpp"

using namespace gg::parse;

namespace {

struct Ref {
  uint32_t base = 0, brk = 0, keep = 0, starts = 0;
  std::vector<int> codes;  // of the bases in order
};

int byte_code(uint8_t c) {  // 0..3 base, 4 skip, 5 break
  const uint8_t l = c | 0x20;
  if (l == 'a') return 0;
  if (l == 'c') return 1;
  if (l == 'g') return 2;
  if (l == 't' || l == 'u') return 3;
  if (c == ' ' || c == '\t' || c == '\r' || c == '\n') return 4;
  return 5;
}

Ref reference(const uint8_t* c, uint32_t lim, bool line0, bool hdr0, bool prev_base) {
  Ref r;
  bool hdr = hdr0, at_line = line0, pb = prev_base;
  for (uint32_t j = 0; j < 32; ++j) {
    if (j >= lim) continue;  // dropped
    if (at_line) hdr = c[j] == '>';
    at_line = false;
    int k;
    if (c[j] == '\n') {
      k = 4;
      at_line = true;
    } else {
      k = hdr ? 5 : byte_code(c[j]);
    }
    if (k == 4) continue;
    r.keep |= 1u << j;
    if (k < 4) {
      r.base |= 1u << j;
      r.codes.push_back(k);
      if (!pb) r.starts |= 1u << j;
      pb = true;
    } else {
      r.brk |= 1u << j;
      pb = false;
    }
  }
  return r;
}

}  // namespace

int main() {
  std::mt19937_64 rng(12345);
  const char alpha[] = "ACGTACGTACGTacgtUuNn\n\n\n> \t\r*-X\xff\x00";
  const int na = (int)sizeof(alpha) - 1;
  long cases = 0;
  for (int it = 0; it < 400000; ++it) {
    uint8_t c[32];
    const int mode = it % 4;  // 0: any byte, 1: weighted alphabet, 2: DNA with newlines, 3: header-ish
    for (int j = 0; j < 32; ++j) {
      if (mode == 0) c[j] = (uint8_t)rng();
      else if (mode == 1) c[j] = (uint8_t)alpha[rng() % na];
      else if (mode == 2) c[j] = rng() % 20 == 0 ? '\n' : "ACGT"[rng() % 4];
      else c[j] = rng() % 6 == 0 ? '\n' : rng() % 5 == 0 ? '>' : (uint8_t)alpha[rng() % na];
    }
    const uint32_t lim = it % 7 == 0 ? (uint32_t)(rng() % 33) : 32;
    const bool line0 = rng() & 1, hdr0 = rng() & 1, prev_base = rng() & 1;
    uint32_t w[8];
    memcpy(w, c, 32);
    const Masks m = classify(w, lim);
    const Roles ro = roles(m, line0, hdr0);
    const uint32_t st = run_starts(ro, prev_base);
    const Ref r = reference(c, lim, line0, hdr0, prev_base);
    bool ok = ro.base == r.base && ro.brk == r.brk && ro.keep == r.keep && st == r.starts;
    const uint64_t R = packed_codes(m, ro.base);
    const int n = popc(ro.base);
    for (int i = 0; ok && i < n; ++i) ok = (int)((R >> (62 - 2 * i)) & 3u) == r.codes[i];
    if (ok && n < 32) ok = (R << (2 * n)) == 0;  // (nothing after the last base)
    // placement at every offset: the three words hold R shifted by 2 o
    for (uint32_t o = 0; ok && o < 16; ++o) {
      uint32_t w0, w1, w2;
      place(R, o, w0, w1, w2);
      for (int i = 0; ok && i < n; ++i) {
        const uint32_t p = o + (uint32_t)i, word = p >> 4;
        const uint32_t x = word == 0 ? w0 : word == 1 ? w1 : w2;
        ok = ((x >> (30 - 2 * (p & 15))) & 3u) == (uint32_t)r.codes[i];
      }
    }
    if (!ok) {
      printf("mismatch at case %d (lim %u line0 %d hdr0 %d prev_base %d): base %08x/%08x brk %08x/%08x keep %08x/%08x "
             "starts %08x/%08x\n",
             it, lim, line0, hdr0, prev_base, ro.base, r.base, ro.brk, r.brk, ro.keep, r.keep, st, r.starts);
      for (int j = 0; j < 32; ++j) printf("%02x ", c[j]);
      printf("\n");
      return 1;
    }
    ++cases;
  }
  // the compress step on its own: every mask with random values
  for (int it = 0; it < 200000; ++it) {
    const uint32_t m = (uint32_t)rng() & (uint32_t)rng() ? (uint32_t)rng() : (uint32_t)rng() | (uint32_t)rng();
    const uint32_t x = (uint32_t)rng();
    uint32_t want = 0;
    for (int j = 0, k = 0; j < 32; ++j)
      if ((m >> j) & 1u) want |= ((x >> j) & 1u) << k++;
    if (Compress(m)(x, m) != want) {
      printf("compress mismatch m %08x x %08x\n", m, x);
      return 1;
    }
  }
  printf("ok %ld\n", cases);
  return 0;
}
