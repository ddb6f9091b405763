// Host test of the DEFLATE core of the device inflate
// (galah_amd/csrc/inflate_core.hpp): every gzip file given is decoded
//   (a) serially from its first block, and
//   (b) as the device does it: block starts searched every `chunk` bytes,
//       one independent decode per start (an overrun drops the start it
//       passed), tokens placed by prefix sums and back-references followed
//       to their literals,
// and both must equal zlib's output byte for byte.  Prints one JSON line per
// file (blocks, starts found, starts dropped).  Built by tests/cpp/Makefile,
// run by tests/test_inflate.py.
#include <zlib.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../galah_amd/csrc/inflate_core.hpp"

using namespace gg::inflate;

static bool read_all(const char* path, std::vector<uint8_t>& out) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) out.insert(out.end(), buf, buf + n);
  fclose(f);
  return true;
}

static bool zlib_gunzip(const std::vector<uint8_t>& gz, std::vector<uint8_t>& out) {
  z_stream s{};
  if (inflateInit2(&s, 15 + 16) != Z_OK) return false;
  s.next_in = const_cast<uint8_t*>(gz.data());
  s.avail_in = (uInt)gz.size();
  uint8_t buf[1 << 16];
  int r;
  do {
    s.next_out = buf;
    s.avail_out = sizeof buf;
    r = inflate(&s, Z_NO_FLUSH);
    if (r != Z_OK && r != Z_STREAM_END) {
      inflateEnd(&s);
      return false;
    }
    out.insert(out.end(), buf, buf + (sizeof buf - s.avail_out));
  } while (r != Z_STREAM_END);
  inflateEnd(&s);
  return true;
}

// offset of the deflate data of the gzip member at the start of gz (RFC 1952)
static long gzip_data_offset(const std::vector<uint8_t>& gz) {
  if (gz.size() < 18 || gz[0] != 0x1f || gz[1] != 0x8b || gz[2] != 8) return -1;
  const uint8_t flg = gz[3];
  size_t p = 10;
  if (flg & 4) p += 2 + (gz[p] | (gz[p + 1] << 8));
  if (flg & 8) {
    while (p < gz.size() && gz[p]) ++p;
    ++p;
  }
  if (flg & 16) {
    while (p < gz.size() && gz[p]) ++p;
    ++p;
  }
  if (flg & 2) p += 2;
  return p < gz.size() ? (long)p : -1;
}

static void expand(const std::vector<uint32_t>& toks, std::vector<uint8_t>& out) {
  for (uint32_t t : toks) {
    if (!tok_is_match(t)) {
      out.push_back((uint8_t)t);
    } else {
      const uint32_t len = tok_len(t), dist = tok_dist(t);
      const size_t from = out.size() - dist;
      for (uint32_t i = 0; i < len; ++i) out.push_back(out[from + i]);
    }
  }
}

// The device decode of one segment [s0, end) (end ~0: the file's last),
// restated serially: per block the header, then the body's sub-spans
// decoded speculatively, chained by checkpoints in rounds (a lane not right
// from its start decodes again from the true start until it meets its
// first decode) and concatenated (inflate.hip inflate_decode_kernel).
// rounds counts second-decode rounds, redo_bits the bits they decoded.
struct SpecStats {
  size_t rounds = 0, redo_bits = 0, spans = 0, span_bits = 0, windows = 0;
};
// The staged decode's window (bits of LDS stage past its word-aligned base,
// less the look-ahead): a block body longer than that is decoded in
// windows, each from the last lane's end of the one before (0: no windows,
// the global form).
static uint64_t g_window = 0;
static uint32_t spec_segment(const Bits& in, uint64_t s0, uint64_t end, uint64_t limit, LaneTables<ArrayStore>& tab,
                             ClArrays& cla, std::vector<uint32_t>& out, uint64_t& out_len, uint64_t& last_end, uint32_t& fin,
                             SpecStats& ss) {
  const bool final_seg = end == ~0ull;
  uint64_t pos = s0;
  out_len = 0;
  fin = 0;
  for (;;) {
    if (pos == end) break;
    if (pos > end || pos >= limit) {
      last_end = pos;
      return kDecOverrun;
    }
    uint64_t q = pos;
    uint32_t bf = 0, stl = 0;
    const int bt = read_block_header(in, q, tab, cla, bf, stl);
    if (bt < 0) {
      last_end = q;
      return kDecBad;
    }
    if (bt == 0) {
      if (q + 8ull * stl > limit) return kDecBad;
      for (uint32_t i = 0; i < stl; ++i) out.push_back(((const uint8_t*)in.w)[q / 8 + i]);
      out_len += stl;
      pos = q + 8ull * stl;
    } else {
      const uint64_t span_end = final_seg ? limit : end;
      uint64_t bstart = q, wbase = pos;
      bool more = true;
      while (more) {
      more = false;
      const uint64_t wend = g_window ? std::min<uint64_t>(span_end, (wbase & ~31ull) + g_window) : span_end;
      ++ss.windows;
      uint64_t L;
      uint32_t nsub;
      span_layout(bstart, wend, 64, L, nsub);
      struct Lane {
        uint64_t S, R, first = 0, Ea = 0, Eb = 0, ba = 0, bb = 0;
        uint32_t na = 0, nb = 0, sa = 0, sb = 0, nck = 0;
        int synced = -1;
        bool redone = false;
        std::vector<uint32_t> A, B;
        std::vector<uint64_t> ck;
        uint64_t E() const { return redone && synced < 0 ? Eb : Ea; }
        uint32_t st() const { return redone && synced < 0 ? sb : sa; }
      };
      std::vector<Lane> ln(nsub);
      for (uint32_t j = 0; j < nsub; ++j) {
        Lane& x = ln[j];
        x.S = bstart + j * L;
        x.R = j + 1 == nsub ? wend : x.S + L;
        x.ck.assign(span_cks(L), 0);
        x.sa = decode_span(in, x.S, x.S, x.R, tab,
                           [&](uint32_t t) {
                             if (x.A.size() >= span_cap(L)) return false;
                             x.A.push_back(t);
                             return true;
                           },
                           [&](uint32_t k, uint64_t c) {
                             if (k < x.ck.size()) x.ck[k] = c, x.nck = k + 1;
                             return true;
                           },
                           x.na, x.ba, x.Ea);
        x.first = x.nck ? x.S + ck_off(x.ck[0]) : ~0ull;
        ss.spans += 1;
        ss.span_bits += x.R - x.S;
      }
      uint32_t c_end = 0;
      bool overrun = false;
      for (;;) {
        std::vector<bool> ok(nsub);
        uint32_t c = nsub, t = nsub;
        for (uint32_t j = 0; j < nsub; ++j) {
          ok[j] = j == 0 || (ln[j - 1].st() == kSpanRange && ln[j].first == ln[j - 1].E());
          if (!ok[j] && c == nsub) c = j;
          if (ln[j].st() != kSpanRange && t == nsub) t = j;
        }
        if (t < c) {
          c_end = t;
          break;
        }
        if (c >= nsub) {
          overrun = wend == span_end;
          more = !overrun;
          c_end = nsub - 1;
          break;
        }
        ++ss.rounds;
        std::vector<uint64_t> from(nsub, ~0ull);
        for (uint32_t j = c; j < nsub; ++j)
          if (!ok[j] && ln[j - 1].st() == kSpanRange) from[j] = ln[j - 1].E();
        for (uint32_t j = c; j < nsub; ++j) {
          if (from[j] == ~0ull) continue;
          Lane& x = ln[j];
          x.B.clear();
          x.redone = true;
          x.synced = -1;
          x.first = from[j];
          x.sb = decode_span(in, from[j], x.S, x.R, tab,
                             [&](uint32_t tk) {
                               if (x.B.size() >= span_cap(L)) return false;
                               x.B.push_back(tk);
                               return true;
                             },
                             [&](uint32_t k, uint64_t cc) {
                               if (k < x.nck && ck_off(cc) == ck_off(x.ck[k])) {
                                 x.synced = (int)k;
                                 return false;
                               }
                               return true;
                             },
                             x.nb, x.bb, x.Eb);
          ss.redo_bits += x.Eb - from[j];
        }
      }
      if (overrun) {
        last_end = ln[c_end].E();
        return kDecOverrun;
      }
      if (ln[c_end].st() == kSpanBad) {
        last_end = ln[c_end].E();
        return kDecBad;
      }
      for (uint32_t j = 0; j <= c_end; ++j) {
        const Lane& x = ln[j];
        if (!x.redone) {
          out.insert(out.end(), x.A.begin() + ck_tok(x.ck[0]), x.A.begin() + x.na);
          out_len += x.ba - ck_bytes(x.ck[0]);
        } else {
          out.insert(out.end(), x.B.begin(), x.B.begin() + x.nb);
          out_len += x.bb;
          if (x.synced >= 0) {
            out.insert(out.end(), x.A.begin() + ck_tok(x.ck[x.synced]), x.A.begin() + x.na);
            out_len += x.ba - ck_bytes(x.ck[x.synced]);
          }
        }
      }
      pos = ln[c_end].E();
      bstart = wbase = pos;
      }  // (windows)
    }
    if (bf) {
      fin = 1;
      last_end = pos;
      return final_seg ? kDecOk : kDecFinalEarly;
    }
  }
  last_end = pos;
  return kDecOk;
}

int main(int argc, char** argv) {
  int failures = 0;
  uint32_t chunk = 4096;
  int first = 1;
  for (;;) {
    if (argc > first + 1 && std::string(argv[first]) == "--chunk") {
      chunk = (uint32_t)atoi(argv[first + 1]);
      first += 2;
    } else if (argc > first + 1 && std::string(argv[first]) == "--window") {
      g_window = (uint64_t)atoll(argv[first + 1]);
      first += 2;
    } else {
      break;
    }
  }
  for (int a = first; a < argc; ++a) {
    std::vector<uint8_t> gz, want;
    if (!read_all(argv[a], gz) || !zlib_gunzip(gz, want)) {
      fprintf(stderr, "%s: unreadable\n", argv[a]);
      ++failures;
      continue;
    }
    const long off = gzip_data_offset(gz);
    const size_t nbytes = gz.size() - (size_t)off;
    std::vector<uint32_t> words((nbytes + 3) / 4 + 1024, 0);  // (a header walk may read ~4.5 kbit past the end)
    memcpy(words.data(), gz.data() + off, nbytes);
    const Bits in{words.data()};
    const uint64_t limit_bits = (uint64_t)nbytes * 8;
    LaneTables<ArrayStore> tab;
    ClArrays cla;
    // (a) serially
    std::vector<uint32_t> toks;
    uint64_t out_len = 0, last_end = 0;
    uint32_t bf = 0;
    const uint32_t st = decode_blocks(in, 0, ~0ull, limit_bits, tab, cla,
                                      [&](uint32_t t) {
                                        toks.push_back(t);
                                        return true;
                                      },
                                      out_len, last_end, bf);
    std::vector<uint8_t> got;
    expand(toks, got);
    if (st != kDecOk || got != want || out_len != want.size()) {
      fprintf(stderr, "%s: serial decode differs (status %u, %zu vs %zu bytes)\n", argv[a], st, got.size(), want.size());
      ++failures;
      continue;
    }
    // (b) as the device: starts, independent decodes, place + resolve
    std::vector<uint64_t> starts{0};
    for (uint64_t c = chunk; c < nbytes; c += chunk) {
      for (uint64_t p = c * 8; p < std::min<uint64_t>((c + chunk) * 8, limit_bits); ++p) {
        uint64_t q = p;
        SeqBits sb{Cursor{in.w}};
        sb.c.seek(p);
        uint64_t q2 = p;
        const bool ok2 = block_header_ok(sb, q2, cla);  // (the device's cursor reader)
        const bool ok1 = block_header_ok(in, q, cla);
        if (ok1 != ok2 || (ok1 && q != q2)) {
          fprintf(stderr, "%s: header check through SeqBits differs at bit %llu\n", argv[a], (unsigned long long)p);
          ++failures;
        }
        // the search's stepwise walk (HeaderWalk) gives the same verdict
        HeaderWalk hw;
        int v = hw.start(in, p, cla) ? 0 : -1;
        while (v == 0) v = hw.step(in, cla);
        if ((v == 1) != ok1) {
          fprintf(stderr, "%s: HeaderWalk differs from block_header_ok at bit %llu\n", argv[a], (unsigned long long)p);
          ++failures;
        }
        if (ok1) {
          starts.push_back(p);
          break;
        }
      }
    }
    const size_t found = starts.size();
    size_t dropped = 0;
    std::vector<std::vector<uint32_t>> part;
    std::vector<uint64_t> part_len;
    for (;;) {  // drop the starts a lane overran, until every lane lands
      part.assign(starts.size(), {});
      part_len.assign(starts.size(), 0);
      bool again = false;
      for (size_t b = 0; b < starts.size() && !again; ++b) {
        const uint64_t end = b + 1 < starts.size() ? starts[b + 1] : ~0ull;
        uint64_t ol, le;
        uint32_t fin;
        const uint32_t r = decode_blocks(in, starts[b], end, limit_bits, tab, cla,
                                         [&](uint32_t t) {
                                           part[b].push_back(t);
                                           return true;
                                         },
                                         ol, le, fin);
        part_len[b] = ol;
        if (r == kDecOverrun) {
          starts.erase(starts.begin() + (long)b + 1);
          ++dropped;
          again = true;
        } else if (r != kDecOk) {
          fprintf(stderr, "%s: lane %zu status %u\n", argv[a], b, r);
          ++failures;
          starts.clear();
          break;
        }
      }
      if (!again) break;
    }
    if (starts.empty()) continue;
    // (c) the device decode of each lane's segment: the same tokens
    SpecStats ss;
    for (size_t b = 0; b < starts.size(); ++b) {
      const uint64_t end = b + 1 < starts.size() ? starts[b + 1] : ~0ull;
      std::vector<uint32_t> t3;
      uint64_t ol, le;
      uint32_t fin;
      const uint32_t r = spec_segment(in, starts[b], end, limit_bits, tab, cla, t3, ol, le, fin, ss);
      if (r != kDecOk || t3 != part[b] || ol != part_len[b]) {
        fprintf(stderr, "%s: lane %zu: sub-span decode differs (status %u, %zu vs %zu tokens)\n", argv[a], b, r,
                t3.size(), part[b].size());
        ++failures;
        starts.clear();
        break;
      }
    }
    if (starts.empty()) continue;
    // place: every byte a literal (bit 31) or a pointer to an earlier byte
    std::vector<uint32_t> val;
    // (stats: bytes copied by matches, and the bytes the device's expand
    // leaves to the resolve pass -- a copy whose source, followed inside its
    // segment, lies before the segment -- and the 16-byte groups holding one)
    std::vector<uint8_t> marker;
    size_t match_bytes = 0;
    for (size_t b = 0; b < part.size(); ++b) {
      const size_t o0 = val.size();
      for (uint32_t t : part[b]) {
        if (!tok_is_match(t)) {
          val.push_back(0x80000000u | t);
          marker.push_back(0);
        } else {
          const uint32_t len = tok_len(t), dist = tok_dist(t);
          const size_t at = val.size();
          for (uint32_t i = 0; i < len; ++i) {
            const size_t src = at + i - dist;
            val.push_back((uint32_t)src);
            marker.push_back(src < o0 || marker[src] ? 1 : 0);
          }
          match_bytes += len;
        }
      }
    }
    size_t marker_bytes = 0, marker_groups = 0;
    for (size_t g = 0; g * 16 < marker.size(); ++g) {
      size_t m = 0;
      for (size_t i = g * 16; i < std::min(marker.size(), g * 16 + 16); ++i) m += marker[i];
      marker_bytes += m;
      marker_groups += m ? 1 : 0;
    }
    std::vector<uint8_t> got2(val.size());
    size_t max_chain = 0;
    for (size_t i = 0; i < val.size(); ++i) {
      uint32_t v = val[i];
      size_t chain = 0;
      while (!(v >> 31)) {
        v = val[v];
        ++chain;
      }
      max_chain = std::max(max_chain, chain);
      got2[i] = (uint8_t)v;
    }
    if (got2 != want) {
      fprintf(stderr, "%s: chunked decode differs\n", argv[a]);
      ++failures;
      continue;
    }
    printf("{\"file\": \"%s\", \"bytes\": %zu, \"gz_bytes\": %zu, \"starts_found\": %zu, \"starts_dropped\": %zu, "
           "\"lanes\": %zu, \"tokens\": %zu, \"max_chain\": %zu, \"redo_rounds\": %zu, \"spans\": %zu, \"span_bits\": %zu, \"redo_bits\": %zu, \"windows\": %zu, "
           "\"match_bytes\": %zu, \"marker_bytes\": %zu, \"marker_groups\": %zu}\n",
           argv[a], want.size(), gz.size(), found, dropped, starts.size(), toks.size(), max_chain, ss.rounds, ss.spans,
           ss.span_bits, ss.redo_bits, ss.windows, match_bytes, marker_bytes, marker_groups);
  }
  if (failures) {
    fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  return 0;
}
