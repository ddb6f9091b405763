// Host side of the device inflate (inflate.hip): gzip member framing (RFC
// 1952), the batch layout, and the launches with their checks.  The result
// is the FASTA text of a batch of files in device memory, laid out as
// parse_raw_batch (multi.cpp) reads it: file f at foff[f], each file
// starting on a 16-byte boundary, the gaps filled with '\n'.
//
// A batch is inflated on the device or not at all: a stream the lanes
// cannot chain, a CRC-32 or ISIZE that does not match a trailer, text that
// is not FASTA makes inflate_batch return ok = false, and the caller decodes
// the batch's files on the host (libdeflate, which also reports a corrupt
// file).  So the device path changes no result, only where the bytes are
// inflated.
//
// Files of several gzip members (needletail, behind src/finch.rs:47, reads
// concatenated members as one stream): every member is a *unit* of its own
// -- its own lanes, its own CRC-32 and ISIZE -- and the members' texts follow
// each other in the file's text.  A BGZF file's members are known from their
// headers (bgzf_members, before the batch); any other multi-member file is
// first taken as one member, and a lane that decodes a final block before
// its end marks where the member ends: when a gzip trailer and header follow
// there, the batch is planned again with that boundary (a few rounds at
// most; each finds every boundary some lane ran into).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "context.hpp"
#include "inflate_core.hpp"

namespace gg {

// One gzip member at the start of buf[0, n): its deflate data [*data_off,
// *data_off + *data_len) (up to the 8-byte trailer) and the trailer's CRC-32
// and ISIZE.  False when buf is not gzip (CM 8) or too short.  Whether the
// deflate stream ends exactly at the trailer (one member) is checked after
// decoding.
bool gzip_header(const uint8_t* buf, size_t n, uint64_t file_size, size_t* data_off) {
  if (n < 10 || file_size < 18 || buf[0] != 0x1f || buf[1] != 0x8b || buf[2] != 8) return false;
  const uint8_t flg = buf[3];
  if (flg & 0xE0) return false;  // reserved bits
  size_t p = 10;
  if (flg & 4) {
    if (p + 2 > n) return false;
    p += 2 + (size_t)(buf[p] | (buf[p + 1] << 8));
  }
  for (int f : {8, 16})
    if (flg & f) {
      while (p < n && buf[p]) ++p;
      ++p;
    }
  if (flg & 2) p += 2;
  if (p > n || p + 8 > file_size) return false;
  *data_off = p;
  return true;
}

bool gzip_member(const uint8_t* buf, size_t n, size_t* data_off, size_t* data_len, uint32_t* isize, uint32_t* crc) {
  size_t p;
  if (!gzip_header(buf, n, n, &p)) return false;
  *data_off = p;
  *data_len = n - 8 - p;
  *crc = (uint32_t)buf[n - 8] | ((uint32_t)buf[n - 7] << 8) | ((uint32_t)buf[n - 6] << 16) | ((uint32_t)buf[n - 5] << 24);
  *isize = (uint32_t)buf[n - 4] | ((uint32_t)buf[n - 3] << 8) | ((uint32_t)buf[n - 2] << 16) | ((uint32_t)buf[n - 1] << 24);
  return true;
}

// A BGZF member's size from the 'BC' subfield of its FEXTRA field (SAM/BAM
// specification 4.1): 0 when there is none.
uint64_t bgzf_member_size(const uint8_t* b, uint64_t n) {
  if (n < 18 || b[0] != 0x1f || b[1] != 0x8b || b[2] != 8 || !(b[3] & 4)) return 0;
  const uint64_t xlen = (uint64_t)b[10] | ((uint64_t)b[11] << 8);
  if (12 + xlen > n) return 0;
  for (uint64_t q = 12; q + 4 <= 12 + xlen;) {
    const uint64_t slen = (uint64_t)b[q + 2] | ((uint64_t)b[q + 3] << 8);
    if (b[q] == 'B' && b[q + 1] == 'C' && slen == 2 && q + 6 <= 12 + xlen)
      return ((uint64_t)b[q + 4] | ((uint64_t)b[q + 5] << 8)) + 1;
    q += 4 + slen;
  }
  return 0;
}

bool bgzf_members(const uint8_t* buf, uint64_t n, uint64_t base, std::vector<GzMember>& out) {
  std::vector<GzMember> ms;
  for (uint64_t pos = 0; pos < n;) {
    const uint64_t size = bgzf_member_size(buf + pos, n - pos);
    size_t hl = 0;
    if (!size || pos + size > n || !gzip_header(buf + pos, (size_t)size, size, &hl)) return false;
    GzMember m;
    m.off = base + pos + hl;
    m.len = size - 8 - hl;
    const uint8_t* t = buf + pos + size - 8;
    m.crc = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
    m.isize = (uint32_t)t[4] | ((uint32_t)t[5] << 8) | ((uint32_t)t[6] << 16) | ((uint32_t)t[7] << 24);
    ms.push_back(m);
    pos += size;
  }
  if (ms.size() < 2) return false;  // (one member: the plain single-member path)
  out.swap(ms);
  return true;
}

namespace {
// GALAHGPU_INFLATE_DEBUG=1: why a batch went back to the host, on stderr
bool inflate_debug() {
  static const bool on = [] {
    const char* e = getenv("GALAHGPU_INFLATE_DEBUG");
    return e && *e == '1';
  }();
  return on;
}
// A scratch buffer that does not fit the device's memory hands the batch
// to the host decoder (counted like any other hand-back) instead of failing
// the call: the host path needs no device memory beyond the text.
#define GZ_SCRATCH(m, key, count, out)                                           \
  do {                                                                           \
    const hipError_t _e = scratch_t((m), (key), (count), (out));                 \
    if (_e == hipErrorOutOfMemory) {                                             \
      (void)hipGetLastError();                                                   \
      return hand_back(o, "device memory for " key, 0);                          \
    }                                                                            \
    if (_e != hipSuccess) return hip_fail((m), _e, "scratch " key);             \
  } while (0)
// Small per-batch host <-> device copies go through pinned host scratch, one
// buffer per call site: pageable copies are staged and block the calling
// thread (the parse's arrays, pinned: two-lane call 0.0475 -> 0.0456 s,
// profiles/r06/parse_pinned/).  A site's buffer is written again only after
// the stream has synchronised (every pass of a batch ends with a sync).
hipError_t h2d_pinned(gg_ctx* m, const char* key, void* dst, const void* src, size_t bytes, hipStream_t st) {
  if (!bytes) return hipSuccess;
  uint8_t* h;
  const hipError_t e = host_scratch_t(m, key, bytes, &h);
  if (e != hipSuccess) return e;
  memcpy(h, src, bytes);
  return hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, st);
}
template <class T>
hipError_t d2h_pinned(gg_ctx* m, const char* key, T** out, const T* src, size_t count, hipStream_t st) {
  const hipError_t e = host_scratch_t(m, key, std::max<size_t>(count, 1), out);
  if (e != hipSuccess || !count) return e;
  return hipMemcpyAsync(*out, src, count * sizeof(T), hipMemcpyDeviceToHost, st);
}

// search granularity: the first block start of every chunk is found (48 KB
// scans ~1/4 of the bits, 16 KB ~2/3: C2 files 0.072 -> 0.064 s per call; a
// zlib -6 block of FASTA is ~25-27 KB, GNU gzip's ~53 KB); a segment that
// holds several blocks is decoded block after block by one wave
// (GALAHGPU_GZ_CHUNK_KB, tuning only)
uint64_t chunk_bytes() {
  const char* e = getenv("GALAHGPU_GZ_CHUNK_KB");
  const long kb = e ? atol(e) : 0;
  return (uint64_t)(kb > 0 ? std::min(kb, 1024L) : 48L) << 10;
}
constexpr int kMaxRelaunch = 8;  // decode passes that may drop wrong starts before giving up
constexpr int kMaxPlans = 8;     // plans of a batch (member boundaries found, then full-size areas)
// Token and sub-span areas are first sized for 1/4 token per compressed bit
// (FASTA: ~0.08); a lane that fills one fails the plan, and the batch is
// planned again with areas of one token per bit (GALAHGPU_GZ_TIGHT=0: full
// areas from the start)
bool tight_first() {
  const char* e = getenv("GALAHGPU_GZ_TIGHT");
  return !(e && *e == '0');
}

enum Outcome { kInflated, kHandBack, kReplan, kRetryFull };
Outcome hand_back_(const char* why, uint32_t f) {
  if (inflate_debug()) fprintf(stderr, "[inflate] batch handed back to the host: %s (unit %u of the batch)\n", why, f);
  return kHandBack;
}
#define hand_back(o, why, f) (*(o) = hand_back_((why), (f)), GG_OK)

// A unit: one gzip member of file `file`, its deflate data from bit b0 to
// bit b1 of the file's words (file_word), CRC-32 and ISIZE from its trailer.
struct Unit {
  uint32_t file;
  uint64_t b0, b1;
  uint32_t isize, crc;
  bool first, last;  // the file's first / last member
};

// One plan of a batch: search, decode, expand, resolve, CRC of its units.
// *o: kInflated (text in *d_text), kHandBack, kReplan (fl gained member
// boundaries found by the decode), kRetryFull (a tight area filled).
gg_status inflate_plan(gg_ctx* m, const uint8_t* h_in, uint64_t in_bytes, std::vector<InflateFile>& fl, bool tight,
                       uint8_t* d_in, uint8_t** d_text, std::vector<uint64_t>& foff, Outcome* o) {
  *o = kHandBack;
  hipStream_t st = m->stream;
  const auto t_start = std::chrono::steady_clock::now();
  auto stamp = [&](const char* what) {
    if (inflate_debug())
      fprintf(stderr, "[inflate] %-22s %8.3f ms\n", what,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
  };
  const uint32_t nf = (uint32_t)fl.size();
  std::vector<Unit> units;
  for (uint32_t f = 0; f < nf; ++f) {
    const InflateFile& x = fl[f];
    if (!x.gz) continue;
    if (x.members.empty()) {
      units.push_back(Unit{f, 0, x.data_len * 8, x.isize, x.crc, true, true});
      continue;
    }
    for (size_t k = 0; k < x.members.size(); ++k) {
      const GzMember& g = x.members[k];
      const uint64_t b0 = (g.off - x.data_off) * 8;
      units.push_back(Unit{f, b0, b0 + g.len * 8, g.isize, g.crc, k == 0, k + 1 == x.members.size()});
    }
  }
  const uint32_t nu = (uint32_t)units.size();
  std::vector<uint64_t> fword(nu), fbits(nu);
  std::vector<uint32_t> chunk_file;
  std::vector<uint64_t> chunk_bit0;
  std::vector<uint32_t> first_chunk(nu + 1, 0);
  const uint64_t kChunkBits = chunk_bytes() * 8;
  for (uint32_t u = 0; u < nu; ++u) {
    fword[u] = fl[units[u].file].data_off / 4;
    fbits[u] = units[u].b1;
    first_chunk[u] = (uint32_t)chunk_file.size();
    for (uint64_t c = units[u].b0 + kChunkBits; c < units[u].b1; c += kChunkBits) {
      chunk_file.push_back(u);
      chunk_bit0.push_back(c);
    }
  }
  first_chunk[nu] = (uint32_t)chunk_file.size();
  const uint32_t nc = (uint32_t)chunk_file.size();
  uint64_t *d_fword, *d_fbits, *d_cbit0, *d_start;
  uint32_t* d_cfile;
  GG_HIP(m, scratch_t(m, "gz_fword", std::max(nu, 1u), &d_fword));
  GG_HIP(m, scratch_t(m, "gz_fbits", std::max(nu, 1u), &d_fbits));
  GG_HIP(m, scratch_t(m, "gz_cfile", std::max(nc, 1u), &d_cfile));
  GG_HIP(m, scratch_t(m, "gz_cbit0", std::max(nc, 1u), &d_cbit0));
  GG_HIP(m, scratch_t(m, "gz_start", std::max(nc, 1u), &d_start));
  if (nu) {
    GG_HIP(m, h2d_pinned(m, "h_fword", d_fword, fword.data(), nu * sizeof(uint64_t), st));
    GG_HIP(m, h2d_pinned(m, "h_fbits", d_fbits, fbits.data(), nu * sizeof(uint64_t), st));
  }
  uint64_t* start = nullptr;
  if (nc) {
    GG_HIP(m, h2d_pinned(m, "h_cfile", d_cfile, chunk_file.data(), nc * sizeof(uint32_t), st));
    GG_HIP(m, h2d_pinned(m, "h_cbit0", d_cbit0, chunk_bit0.data(), nc * sizeof(uint64_t), st));
    InflateSearch s;
    s.in = (const uint32_t*)d_in;
    s.file_word = d_fword;
    s.file_bits = d_fbits;
    s.chunk_file = d_cfile;
    s.chunk_bit0 = d_cbit0;
    s.chunk_bits = (uint32_t)kChunkBits;
    s.n_chunks = nc;
    s.start = d_start;
    uint64_t* d_sprof = nullptr;
    if (inflate_debug()) {
      GG_HIP(m, scratch_t(m, "gz_sprof", 8, &d_sprof));
      GG_HIP(m, hipMemsetAsync(d_sprof, 0, 8 * sizeof(uint64_t), st));
      s.prof = d_sprof;
    }
    uint64_t gz_in = 0;
    for (const Unit& u : units) gz_in += (u.b1 - u.b0) / 8;
    GG_HIP(m, timed_launch(m, GG_KERNEL_INFLATE_SEARCH, gz_in, st, [&] { return launch_inflate_search(s, st); }));
    if (d_sprof) {
      uint64_t pr[8];
      GG_HIP(m, hipStreamSynchronize(st));
      GG_HIP(m, hipMemcpy(pr, d_sprof, sizeof pr, hipMemcpyDeviceToHost));
      fprintf(stderr, "[inflate] search: %u chunks; per chunk: %.1f steps (%.0f cycles each), %.1f check rounds "
              "(%.0f cycles each), %.1f candidates\n", nc, pr[2] / (double)nc, pr[0] / (double)std::max<uint64_t>(pr[2], 1),
              pr[3] / (double)nc, pr[1] / (double)std::max<uint64_t>(pr[3], 1), pr[4] / (double)nc);
    }
    GG_HIP(m, d2h_pinned(m, "h_start", &start, (const uint64_t*)d_start, nc, st));
  }
  GG_HIP(m, hipStreamSynchronize(st));
  stamp("copy + search");
  // lanes per unit: the member's first bit and every block start found
  std::vector<std::vector<uint64_t>> starts(nu);
  for (uint32_t u = 0; u < nu; ++u) {
    starts[u].push_back(units[u].b0);
    for (uint32_t c = first_chunk[u]; c < first_chunk[u + 1]; ++c)
      if (start[c] != ~0ull && start[c] > starts[u].back()) starts[u].push_back(start[c]);
  }
  // GALAHGPU_TEST_FAKE_STARTS=1 (tests): a false start midway (odd bit)
  // between every two starts found, not a block boundary but a lane of its
  // own, so that every lane before one runs past it and absorbs it
  {
    const char* fe = getenv("GALAHGPU_TEST_FAKE_STARTS");
    if (fe && *fe == '1')
      for (auto& v : starts) {
        std::vector<uint64_t> w;
        for (size_t i = 0; i < v.size(); ++i) {
          w.push_back(v[i]);
          if (i + 1 < v.size() && v[i + 1] - v[i] > 4096) w.push_back(((v[i] + v[i + 1]) / 2) | 1u);
        }
        v.swap(w);
      }
  }
  if (inflate_debug()) {
    size_t ns = 0;
    for (const auto& v : starts) ns += v.size();
    fprintf(stderr, "[inflate] %u files, %u units, %u chunks, %zu starts%s\n", nf, nu, nc, ns, tight ? "" : " (full areas)");
  }
  // the staged decode reads a segment in LDS windows of at most this many
  // bits: its sub-span areas are sized for one window (GALAHGPU_DECODE_GLOBAL=1:
  // the global-memory form, A/B only, decodes a segment's body at once)
  const char* gdec = getenv("GALAHGPU_DECODE_GLOBAL");
  const bool global_only = gdec && *gdec == '1';
  uint32_t stage_words = 0;
  {  // GALAHGPU_TEST_STAGE_KB (tests): a smaller LDS stage, so blocks take several windows
    const char* se = getenv("GALAHGPU_TEST_STAGE_KB");
    const int kb = se && *se ? atoi(se) : 0;
    stage_words = kb >= 1 && kb <= 30 ? (uint32_t)kb * 256u : 0u;
  }
  const uint64_t window_bits = global_only ? ~0ull : ((uint64_t)(stage_words ? stage_words : inflate_stage_words()) - 8) * 32;
  // one lane (a wave of the decode kernel) per start: [start, end) up to the
  // next start (~0: the unit's last lane), its tokens in a region of the
  // token buffer, its sub-span areas in the scratch
  struct Lane {
    uint32_t unit;
    uint64_t start, end, tok_off, cap, scr_off;
    uint64_t n_tok = 0, out_len = 0, last_end = 0;
    uint64_t done_tok = 0, done_out = 0;  // tokens and bytes of the blocks before `start` (a resumed lane)
    uint32_t status = 0, bfin = 0;
    bool redo = true, alive = true;
  };
  std::vector<Lane> lanes;
  uint64_t toks = 0, scr = 0;
  for (uint32_t u = 0; u < nu; ++u)
    for (size_t i = 0; i < starts[u].size(); ++i) {
      const uint64_t s0 = starts[u][i];
      const uint64_t e = i + 1 < starts[u].size() ? starts[u][i + 1] : ~0ull;
      // every symbol takes >= 1 bit: one token per bit bounds every lane
      // (literal-heavy DNA blocks reach ~0.5 tokens per bit; C2's FASTA
      // ~0.08); the tight plan reserves a quarter of that
      const uint64_t bits = (e == ~0ull ? fbits[u] : e) - s0;
      const uint64_t cap = tight ? std::min<uint64_t>(bits + 64, bits / 4 + 4096) : bits + 64;
      Lane ln{u, s0, e, toks, cap, scr};
      lanes.push_back(ln);
      toks += (cap + 3) / 4 * 4;
      scr += inflate::decode_scratch(bits, window_bits, tight);
    }
  // Unit u's deflate stream ended (a final block) at bit `end` before the
  // unit's end: when a gzip trailer and another member's header follow at
  // the next byte, the file's member there is split in two (true).
  auto split_member = [&](uint32_t ui, uint64_t end) {
    const Unit& u = units[ui];
    InflateFile& F = fl[u.file];
    const uint64_t q = (end + 7) / 8;  // (bytes from the file's data_off: the trailer)
    const uint64_t uend = u.b1 / 8;
    size_t hl = 0;
    const uint64_t at = F.data_off + q + 8;  // the next member's header, in the batch
    if (q + 8 + 18 > uend || at >= in_bytes ||
        !gzip_header(h_in + at, (size_t)std::min<uint64_t>(in_bytes - at, uend - q - 8), uend - q - 8, &hl))
      return false;
    if (F.members.empty()) F.members.push_back(GzMember{F.data_off, F.data_len, F.isize, F.crc});
    for (size_t k = 0; k < F.members.size(); ++k) {
      GzMember& g = F.members[k];
      const uint64_t a0 = g.off, a1 = g.off + g.len, cut = F.data_off + q;
      if (cut <= a0 || cut + 8 + hl >= a1) continue;
      const uint8_t* t = h_in + cut;
      GzMember head{a0, cut - a0, 0, 0};
      head.crc = (uint32_t)t[0] | ((uint32_t)t[1] << 8) | ((uint32_t)t[2] << 16) | ((uint32_t)t[3] << 24);
      head.isize = (uint32_t)t[4] | ((uint32_t)t[5] << 8) | ((uint32_t)t[6] << 16) | ((uint32_t)t[7] << 24);
      GzMember tail{cut + 8 + hl, a1 - (cut + 8 + hl), g.isize, g.crc};
      g = head;
      F.members.insert(F.members.begin() + (long)k + 1, tail);
      return true;
    }
    return false;
  };
  uint32_t *d_tok = nullptr, *d_scr = nullptr;
  GZ_SCRATCH(m, "gz_tok", std::max<uint64_t>(toks, 4), &d_tok);
  GZ_SCRATCH(m, "gz_scr", std::max<uint64_t>(scr, 4), &d_scr);
  m->gz_scratch_bytes = std::max<uint64_t>(m->gz_scratch_bytes, 4 * (toks + scr));
  for (int pass = 0;; ++pass) {
    std::vector<uint32_t> redo;
    for (uint32_t l = 0; l < (uint32_t)lanes.size(); ++l)
      if (lanes[l].alive && lanes[l].redo) redo.push_back(l);
    const uint32_t nl = (uint32_t)redo.size();
    if (nl == 0) break;
    const uint32_t n_staged = global_only ? 0u : nl;
    if (pass >= kMaxRelaunch) return hand_back(o, "block starts did not chain", 0);
    // the lanes to decode: 6 arrays of nl u64 (unit, start, end, tok_off, cap, scr_off)
    std::vector<uint64_t> arg((size_t)nl * 6);
    for (uint32_t k = 0; k < nl; ++k) {
      const Lane& x = lanes[redo[k]];
      arg[k] = x.unit;
      arg[nl + k] = x.start;
      arg[2 * (size_t)nl + k] = x.end;
      arg[3 * (size_t)nl + k] = x.tok_off + x.done_tok;
      arg[4 * (size_t)nl + k] = x.cap - x.done_tok;
      arg[5 * (size_t)nl + k] = x.scr_off;
    }
    uint64_t *d_arg, *d_res;
    uint32_t* d_lfile;
    GG_HIP(m, scratch_t(m, "gz_larg", arg.size(), &d_arg));
    GG_HIP(m, scratch_t(m, "gz_lfile", nl, &d_lfile));
    // results contiguous: n_tok, out_len, last_end (u64), then status, bfinal (u32)
    GG_HIP(m, scratch_t(m, "gz_res", (size_t)nl * 4, &d_res));
    std::vector<uint32_t> lf(nl);
    for (uint32_t k = 0; k < nl; ++k) lf[k] = lanes[redo[k]].unit;
    GG_HIP(m, h2d_pinned(m, "h_larg", d_arg, arg.data(), arg.size() * sizeof(uint64_t), st));
    GG_HIP(m, h2d_pinned(m, "h_lfile", d_lfile, lf.data(), nl * sizeof(uint32_t), st));
    InflateDecode d;
    d.in = (const uint32_t*)d_in;
    d.file_word = d_fword;
    d.file_bits = d_fbits;
    d.lane_file = d_lfile;
    d.lane_start = d_arg + nl;
    d.lane_end = d_arg + 2 * (size_t)nl;
    d.n_lanes = nl;
    d.n_staged = n_staged;
    d.stage_words = stage_words;
    d.tight = tight ? 1u : 0u;
    d.tok = d_tok;
    d.tok_off = d_arg + 3 * (size_t)nl;
    d.tok_cap = d_arg + 4 * (size_t)nl;
    d.scr = d_scr;
    d.scr_off = d_arg + 5 * (size_t)nl;
    d.n_tok = d_res;
    d.out_len = d_res + nl;
    d.last_end = d_res + 2 * (size_t)nl;
    d.status = (uint32_t*)(d_res + 3 * (size_t)nl);
    d.bfinal = d.status + nl;
    uint64_t* d_prof = nullptr;
    if (inflate_debug()) {
      GG_HIP(m, scratch_t(m, "gz_prof", 8, &d_prof));
      GG_HIP(m, hipMemsetAsync(d_prof, 0, 8 * sizeof(uint64_t), st));
      d.prof = d_prof;
    }
    const size_t timed_at = m->timed.size();
    GG_HIP(m, timed_launch(m, GG_KERNEL_INFLATE_DECODE, 0, st, [&] { return launch_inflate_decode(d, st); }));
    if (d_prof) {
      uint64_t pr[8];
      GG_HIP(m, hipStreamSynchronize(st));
      GG_HIP(m, hipMemcpy(pr, d_prof, sizeof pr, hipMemcpyDeviceToHost));
      const double nb = (double)std::max<uint64_t>(pr[4], 1);
      int wc_khz = 0;
      (void)hipDeviceGetAttribute(&wc_khz, hipDeviceAttributeWallClockRate, m->device);
      const double us = wc_khz > 0 ? 1e3 / wc_khz : 0.0;  // (wall_clock64 ticks to microseconds)
      fprintf(stderr, "[inflate] decode: %u lanes, %llu blocks, %.0f tokens/block; cycles per block: header %.0f, "
              "first decode %.0f, resync %.0f, copy %.0f; wave wall mean %.1f us, max %.1f us\n", nl,
              (unsigned long long)pr[4], pr[5] / nb, pr[0] / nb, pr[1] / nb, pr[2] / nb, pr[3] / nb,
              pr[7] * us / std::max(nl, 1u), pr[6] * us);
    }
    uint64_t* res;
    GG_HIP(m, d2h_pinned(m, "h_res", &res, (const uint64_t*)d_res, (size_t)nl * 4, st));
    GG_HIP(m, hipStreamSynchronize(st));
    stamp("decode pass");
    const uint32_t* r32 = (const uint32_t*)(res + 3 * (size_t)nl);
    if (timed_at < m->timed.size()) {  // (timing: the work of a decode pass is the tokens its lanes wrote)
      uint64_t toks_out = 0;
      for (uint32_t k = 0; k < nl; ++k) toks_out += res[k];
      m->timed[timed_at].work = toks_out;
    }
    for (uint32_t k = 0; k < nl; ++k) {
      Lane& x = lanes[redo[k]];
      x.n_tok = x.done_tok + res[k];
      x.out_len = x.done_out + res[nl + k];
      x.last_end = res[2 * (size_t)nl + k];
      x.status = r32[k];
      x.bfin = r32[nl + k];
      x.redo = false;
    }
    // a member boundary: a lane (not its unit's last) that decoded a final
    // block, followed, at the next byte, by a gzip trailer and another
    // member's header -- the file is planned again with the member split
    // there (the lanes' other results are of no use then)
    bool split = false;
    for (uint32_t l = 0; l < (uint32_t)lanes.size(); ++l) {
      const Lane& x = lanes[l];
      if (x.alive && !x.redo && x.status == inflate::kDecFinalEarly) split |= split_member(x.unit, x.last_end);
    }
    if (split) {
      *o = kReplan;
      return GG_OK;
    }
    // a lane that passed the next start without landing on it: that start is
    // not a block boundary -- the lane takes the next lane's range and token
    // region (they follow its own) and is decoded again, alone, from the
    // start of the block that ran past (last_end), its earlier blocks' tokens
    // kept (and its scratch, which the next lane's follows).  A failed lane
    // right after a lane set to decode again waits for that lane's next pass:
    // its start may be a false one the lane before will run past and absorb
    // (two false starts in a row), and is only confirmed when that lane ends
    // on it.
    bool prev_redo = false;
    uint32_t prev_unit = ~0u;
    for (uint32_t l = 0; l < (uint32_t)lanes.size(); ++l) {
      Lane& x = lanes[l];
      if (!x.alive) continue;
      const bool after_redo = prev_redo && prev_unit == x.unit;
      prev_unit = x.unit;
      prev_redo = x.redo;
      if (x.redo) continue;
      uint32_t nx = l + 1;
      while (nx < lanes.size() && !lanes[nx].alive) ++nx;
      const bool has_next = nx < lanes.size() && lanes[nx].unit == x.unit;
      if (x.status == inflate::kDecOverrun && has_next) {
        Lane& y = lanes[nx];
        x.done_tok = x.n_tok;
        x.done_out = x.out_len;
        x.start = x.last_end;
        x.end = y.end;
        x.cap = y.tok_off + y.cap - x.tok_off;
        x.redo = true;
        y.alive = false;
        prev_redo = true;
      } else if (x.status != inflate::kDecOk && !after_redo) {
        // a tight area filled (or garbage): once more with full areas; else
        // malformed / a member this plan cannot place: the host path
        if (tight && (x.status == inflate::kDecFull || x.status == inflate::kDecBad)) {
          if (inflate_debug()) fprintf(stderr, "[inflate] lane status %u in a tight plan: full areas\n", x.status);
          *o = kRetryFull;
          return GG_OK;
        }
        return hand_back(o, x.status == inflate::kDecFull ? "token capacity"
                            : x.status == inflate::kDecFinalEarly ? "stream ended early (no member header after it)"
                                                                  : "malformed stream", x.unit);
      }
    }
  }
  std::vector<Lane> live;
  for (const Lane& x : lanes)
    if (x.alive) live.push_back(x);
  // every unit: its last lane decoded the final block, ending at its
  // trailer, and the output length agrees with ISIZE
  std::vector<uint64_t> ulen(nu, 0), lane_out(live.size());
  for (size_t l = 0; l < live.size(); ++l) {
    const uint32_t u = live[l].unit;
    lane_out[l] = ulen[u];
    ulen[u] += live[l].out_len;
    if (l + 1 == live.size() || live[l + 1].unit != u) {
      if (live[l].bfin && (live[l].last_end + 7) / 8 < units[u].b1 / 8 && split_member(u, live[l].last_end)) {
        *o = kReplan;  // (the unit's last lane ran into a member boundary)
        return GG_OK;
      }
      if (!live[l].bfin || (live[l].last_end + 7) / 8 != units[u].b1 / 8) return hand_back(o, "member end", u);
      if ((uint32_t)ulen[u] != units[u].isize) return hand_back(o, "ISIZE", u);
    }
  }
  // text: each file's members one after the other, every file on a 16-byte
  // boundary (the gaps '\n')
  std::vector<uint64_t> flen(nf, 0), utext(nu);
  for (uint32_t u = 0; u < nu; ++u) {
    utext[u] = flen[units[u].file];  // (relative to the file's text until foff is known)
    flen[units[u].file] += ulen[u];
  }
  for (uint32_t f = 0; f < nf; ++f)
    if (!fl[f].gz) flen[f] = fl[f].data_len;
  foff.assign(nf + 1, 0);
  for (uint32_t f = 0; f < nf; ++f) foff[f + 1] = foff[f] + (flen[f] + 15) / 16 * 16;
  const uint64_t text_len = foff[nf];
  if (text_len >= (1ull << 30)) return hand_back(o, "batch text over 1 GiB", 0);  // (30-bit expand pointers)
  for (uint32_t u = 0; u < nu; ++u) utext[u] += foff[units[u].file];
  for (size_t l = 0; l < lane_out.size(); ++l) lane_out[l] += utext[live[l].unit];
  uint32_t *d_flags, *d_crc, *d_lfile, *d_ulane;
  uint16_t* d_sym;
  uint64_t *d_lout, *d_ftext, *d_flen, *d_upad;
  GZ_SCRATCH(m, "gz_sym", text_len + 16, &d_sym);
  m->gz_scratch_bytes = std::max<uint64_t>(m->gz_scratch_bytes, 4 * (toks + scr) + 3 * text_len);
  // (tests: GALAHGPU_TEST_POISON_VAL=<u16> fills sym with that value first --
  // what a previous batch or another allocation left there -- and no result
  // may change: the resolve reads sym only where the expand wrote it)
  const char* poison = getenv("GALAHGPU_TEST_POISON_VAL");
  if (poison && *poison && text_len)
    GG_HIP(m, hipMemsetD16Async(d_sym, (unsigned short)strtoul(poison, nullptr, 0), text_len, st));
  GG_HIP(m, scratch_t(m, "stage_text", std::max<uint64_t>(text_len, 16) + 16, d_text));
  // per live lane: text position, token offset, token count, bytes (u64),
  // then its unit (u32)
  const size_t NL = std::max<size_t>(live.size(), 1);
  GG_HIP(m, scratch_t(m, "gz_lout", 4 * NL + (NL + 1) / 2, &d_lout));
  d_lfile = (uint32_t*)(d_lout + 4 * NL);
  // per unit: text position, bytes, end of the padding after it (a file's
  // last unit: the next file's start; else 0) (u64), then its first lane (u32)
  const uint32_t NU = std::max(nu, 1u);
  GG_HIP(m, scratch_t(m, "gz_ftext", 3 * (size_t)NU + 1 + (NU + 2) / 2, &d_ftext));
  d_flen = d_ftext + NU;
  d_upad = d_ftext + 2 * (size_t)NU;
  d_ulane = (uint32_t*)(d_ftext + 3 * (size_t)NU + 1);
  GG_HIP(m, scratch_t(m, "gz_flags", 2 * (size_t)NU + 1, &d_flags));
  d_crc = d_flags + 1;
  for (uint32_t f = 0; f < nf; ++f)  // (plain files: their text is copied in after the resolve; until then
    if (!fl[f].gz && foff[f + 1] > foff[f])  //  no byte of theirs may send the resolve to val)
      GG_HIP(m, hipMemsetAsync(*d_text + foff[f], '\n', foff[f + 1] - foff[f], st));
  GG_HIP(m, hipMemsetAsync(d_flags, 0, sizeof(uint32_t), st));
  std::vector<uint64_t> ftext(3 * (size_t)NU + 1 + (NU + 2) / 2, 0);
  uint32_t* ulane = (uint32_t*)(ftext.data() + 3 * (size_t)NU + 1);
  for (uint32_t u = 0; u < nu; ++u) {
    ftext[u] = utext[u];
    ftext[NU + u] = ulen[u];
    ftext[2 * (size_t)NU + u] = units[u].last ? foff[units[u].file + 1] : 0;
  }
  for (size_t l = live.size(); l-- > 0;) ulane[live[l].unit] = (uint32_t)l;  // (every unit has a lane)
  ulane[nu] = (uint32_t)live.size();
  GG_HIP(m, h2d_pinned(m, "h_ftext", d_ftext, ftext.data(), ftext.size() * sizeof(uint64_t), st));
  std::vector<uint64_t> lv(4 * NL + (NL + 1) / 2, 0);
  for (size_t l = 0; l < live.size(); ++l) {
    lv[l] = lane_out[l];
    lv[NL + l] = live[l].tok_off;
    lv[2 * NL + l] = live[l].n_tok;
    lv[3 * NL + l] = live[l].out_len;
    ((uint32_t*)(lv.data() + 4 * NL))[l] = live[l].unit;
  }
  GG_HIP(m, h2d_pinned(m, "h_lout", d_lout, lv.data(), lv.size() * sizeof(uint64_t), st));
  InflatePlace p;
  p.tok = d_tok;
  p.tok_off = d_lout + NL;
  p.n_tok = d_lout + 2 * NL;
  p.lane_len = d_lout + 3 * NL;
  p.lane_file = d_lfile;
  p.lane_out = d_lout;
  p.file_text = d_ftext;
  p.unit_len = d_flen;
  p.unit_pad = d_upad;
  p.unit_lane = d_ulane;
  p.n_lanes = (uint32_t)live.size();
  p.n_units = nu;
  p.text = *d_text;
  p.sym = d_sym;
  p.flags = d_flags;
  std::vector<uint32_t> seg_first(nu + 1, 0);
  for (uint32_t u = 0; u < nu; ++u) seg_first[u + 1] = seg_first[u] + (uint32_t)((ulen[u] + kInflateCrcSeg - 1) / kInflateCrcSeg);
  const uint32_t nseg = seg_first[nu];
  uint32_t *d_sfirst, *d_scrc;
  GG_HIP(m, scratch_t(m, "gz_sfirst", nu + 1, &d_sfirst));
  GG_HIP(m, scratch_t(m, "gz_scrc", std::max(nseg, 1u), &d_scrc));
  GG_HIP(m, h2d_pinned(m, "h_sfirst", d_sfirst, seg_first.data(), (nu + 1) * sizeof(uint32_t), st));
  uint64_t* d_eprof = nullptr;
  if (inflate_debug()) {
    GG_HIP(m, scratch_t(m, "gz_eprof", 8, &d_eprof));
    GG_HIP(m, hipMemsetAsync(d_eprof, 0, 8 * sizeof(uint64_t), st));
    p.prof = d_eprof;
  }
  GG_HIP(m, timed_launch(m, GG_KERNEL_INFLATE_EXPAND, text_len, st, [&] { return launch_inflate_expand(p, st); }));
  if (d_eprof) {
    uint64_t pr[8];
    GG_HIP(m, hipStreamSynchronize(st));
    GG_HIP(m, hipMemcpy(pr, d_eprof, sizeof pr, hipMemcpyDeviceToHost));
    const double ns = (double)std::max<uint64_t>(pr[3], 1);
    fprintf(stderr, "[inflate] expand: %zu lanes, %.1f steps each, %.2f pointer rounds per step; cycles per step: "
            "token wait + scan %.0f, fill %.0f, pointer rounds %.0f, write-out %.0f\n", live.size(),
            pr[3] / (double)std::max<size_t>(live.size(), 1), pr[4] / ns, pr[5] / ns, pr[0] / ns, pr[1] / ns, pr[2] / ns);
  }
  GG_HIP(m, timed_launch(m, GG_KERNEL_INFLATE_RESOLVE, text_len, st, [&] { return launch_inflate_resolve(p, st); }));
  GG_HIP(m, timed_launch(m, GG_KERNEL_INFLATE_CRC, text_len, st, [&] {
    return launch_inflate_crc(*d_text, nu, d_ftext, d_flen, d_sfirst, nseg, d_scrc, d_crc, st);
  }));
  // plain files (not gzip) go into their place as they are
  for (uint32_t f = 0; f < nf; ++f)
    if (!fl[f].gz && fl[f].data_len)
      GG_HIP(m, hipMemcpyAsync(*d_text + foff[f], d_in + fl[f].data_off, fl[f].data_len, hipMemcpyDeviceToDevice, st));
  // flags, then per unit its CRC-32 and its first byte
  uint32_t* chk;
  GG_HIP(m, d2h_pinned(m, "h_chk", &chk, (const uint32_t*)d_flags, 2 * (size_t)nu + 1, st));
  GG_HIP(m, hipStreamSynchronize(st));
  stamp("expand + resolve + crc");
  if (chk[0])
    return hand_back(o, chk[0] & 1 ? "distance before the member's start" : "token bytes disagree with the decode's count",
                     0);
  // every gzip file's text starts with '>' (FASTQ, an empty file, anything
  // else: the host path, which reads it or reports it): its first byte is
  // that of its first member with any text
  std::vector<uint8_t> seen(nf, 0);
  for (uint32_t u = 0; u < nu; ++u) {
    if (chk[1 + u] != units[u].crc) return hand_back(o, "CRC-32", u);
    const uint32_t f = units[u].file;
    if (!seen[f] && ulen[u]) {
      if (chk[1 + nu + u] != '>') return hand_back(o, "not FASTA", u);
      seen[f] = 1;
    }
    if (units[u].last && !seen[f]) return hand_back(o, "empty file", u);
  }
  *o = kInflated;
  return GG_OK;
}
#undef hand_back
}  // namespace

// files[f]: the deflate data of a gzip file (gz = true; data_off is 4-byte
// aligned in h_in, isize/crc from its trailer, or its members) or plain
// text (gz = false).
gg_status inflate_batch(gg_ctx* m, const uint8_t* h_in, uint64_t in_bytes, const std::vector<InflateFile>& files,
                        uint8_t** d_text, std::vector<uint64_t>& foff, bool* ok, uint8_t* d_in) {
  *ok = false;
  hipStream_t st = m->stream;
  // the batch on the device (+ padding that readers past the last file's
  // end touch: a cursor's 3 words ahead, a header walk of a corrupt stream,
  // at most 316 code lengths of <= 14 bits)
  if (!d_in) {
    GG_HIP(m, scratch_t(m, "gz_in", in_bytes + kInflatePad, &d_in));
    if (in_bytes) GG_HIP(m, hipMemcpyAsync(d_in, h_in, in_bytes, hipMemcpyHostToDevice, st));
  }
  GG_HIP(m, hipMemsetAsync(d_in + in_bytes, 0, kInflatePad, st));
  std::vector<InflateFile> fl(files);  // (member boundaries found by the decode are added here)
  bool tight = tight_first();
  for (int plan = 0; plan < kMaxPlans; ++plan) {
    Outcome o = kHandBack;
    const gg_status s = inflate_plan(m, h_in, in_bytes, fl, tight, d_in, d_text, foff, &o);
    if (s != GG_OK) return s;
    if (o == kInflated) {
      *ok = true;
      return GG_OK;
    }
    if (o == kHandBack) return GG_OK;
    if (o == kRetryFull) {
      if (!tight) return GG_OK;
      tight = false;
      ++m->gz_full_plans;
    }
    if (o == kReplan) ++m->gz_member_plans;
  }
  if (inflate_debug()) fprintf(stderr, "[inflate] batch handed back to the host: too many plans\n");
  return GG_OK;
}

}  // namespace gg
