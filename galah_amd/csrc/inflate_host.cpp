// Host side of the device inflate (inflate.hip): gzip member framing (RFC
// 1952), the batch layout, and the launches with their checks.  The result
// is the FASTA text of a batch of files in device memory, laid out as
// parse_raw_batch (multi.cpp) reads it: file f at foff[f], each file
// starting on a 16-byte boundary, the gaps filled with '\n'.
//
// A batch is inflated on the device or not at all: a member this path does
// not take (a file of several members, a stream the lanes cannot chain, a
// CRC-32 or ISIZE that does not match the trailer) makes inflate_batch
// return ok = false, and the caller decodes the batch's files on the host
// (libdeflate, which also reports a corrupt file).  So the device path
// changes no result, only where the bytes are inflated.
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

namespace {
// GALAHGPU_INFLATE_DEBUG=1: why a batch went back to the host, on stderr
bool inflate_debug() {
  static const bool on = [] {
    const char* e = getenv("GALAHGPU_INFLATE_DEBUG");
    return e && *e == '1';
  }();
  return on;
}
gg_status hand_back(const char* why, uint32_t f) {
  if (inflate_debug()) fprintf(stderr, "[inflate] batch handed back to the host: %s (file %u of the batch)\n", why, f);
  return GG_OK;
}
// A scratch buffer that does not fit the device's memory hands the batch
// to the host decoder (counted like any other hand-back) instead of failing
// the call: the host path needs no device memory beyond the text.
#define GZ_SCRATCH(m, key, count, out)                                           \
  do {                                                                           \
    const hipError_t _e = scratch_t((m), (key), (count), (out));                 \
    if (_e == hipErrorOutOfMemory) {                                             \
      (void)hipGetLastError();                                                   \
      return hand_back("device memory for " key, 0);                             \
    }                                                                            \
    if (_e != hipSuccess) return hip_fail((m), _e, "scratch " key);             \
  } while (0)
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
constexpr int kMaxRelaunch = 8;         // decode passes that may drop wrong starts before giving up
}  // namespace

// files[f]: the deflate data of a gzip file (gz = true; data_off is 4-byte
// aligned in h_in, isize/crc from its trailer) or plain text (gz = false).
gg_status inflate_batch(gg_ctx* m, const uint8_t* h_in, uint64_t in_bytes, const std::vector<InflateFile>& files,
                        uint8_t** d_text, std::vector<uint64_t>& foff, bool* ok, uint8_t* d_in) {
  *ok = false;
  hipStream_t st = m->stream;
  // GALAHGPU_INFLATE_DEBUG=1: wall time of each stage (host + device), on stderr
  const auto t_start = std::chrono::steady_clock::now();
  auto stamp = [&](const char* what) {
    if (inflate_debug())
      fprintf(stderr, "[inflate] %-22s %8.3f ms\n", what,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count());
  };
  const uint32_t nf = (uint32_t)files.size();
  // the batch on the device (+ padding that readers past the last file's
  // end touch: a cursor's 3 words ahead, a header walk of a corrupt stream,
  // at most 316 code lengths of <= 14 bits)
  if (!d_in) {
    GG_HIP(m, scratch_t(m, "gz_in", in_bytes + kInflatePad, &d_in));
    if (in_bytes) GG_HIP(m, hipMemcpyAsync(d_in, h_in, in_bytes, hipMemcpyHostToDevice, st));
  }
  GG_HIP(m, hipMemsetAsync(d_in + in_bytes, 0, kInflatePad, st));
  std::vector<uint64_t> fword(nf), fbits(nf);
  std::vector<uint32_t> chunk_file;
  std::vector<uint64_t> chunk_bit0;
  std::vector<uint32_t> first_chunk(nf + 1, 0);
  const uint64_t kChunkBytes = chunk_bytes();
  for (uint32_t f = 0; f < nf; ++f) {
    fword[f] = files[f].data_off / 4;
    fbits[f] = files[f].gz ? files[f].data_len * 8 : 0;
    first_chunk[f] = (uint32_t)chunk_file.size();
    if (files[f].gz)
      for (uint64_t c = kChunkBytes; c < files[f].data_len; c += kChunkBytes) {
        chunk_file.push_back(f);
        chunk_bit0.push_back(c * 8);
      }
  }
  first_chunk[nf] = (uint32_t)chunk_file.size();
  const uint32_t nc = (uint32_t)chunk_file.size();
  uint64_t *d_fword, *d_fbits, *d_cbit0, *d_start;
  uint32_t* d_cfile;
  GG_HIP(m, scratch_t(m, "gz_fword", std::max(nf, 1u), &d_fword));
  GG_HIP(m, scratch_t(m, "gz_fbits", std::max(nf, 1u), &d_fbits));
  GG_HIP(m, scratch_t(m, "gz_cfile", std::max(nc, 1u), &d_cfile));
  GG_HIP(m, scratch_t(m, "gz_cbit0", std::max(nc, 1u), &d_cbit0));
  GG_HIP(m, scratch_t(m, "gz_start", std::max(nc, 1u), &d_start));
  GG_HIP(m, hipMemcpyAsync(d_fword, fword.data(), nf * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  GG_HIP(m, hipMemcpyAsync(d_fbits, fbits.data(), nf * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  std::vector<uint64_t> start(nc);
  if (nc) {
    GG_HIP(m, hipMemcpyAsync(d_cfile, chunk_file.data(), nc * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    GG_HIP(m, hipMemcpyAsync(d_cbit0, chunk_bit0.data(), nc * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    InflateSearch s;
    s.in = (const uint32_t*)d_in;
    s.file_word = d_fword;
    s.file_bits = d_fbits;
    s.chunk_file = d_cfile;
    s.chunk_bit0 = d_cbit0;
    s.chunk_bits = kChunkBytes * 8;
    s.n_chunks = nc;
    s.start = d_start;
    uint64_t* d_sprof = nullptr;
    if (inflate_debug()) {
      GG_HIP(m, scratch_t(m, "gz_sprof", 8, &d_sprof));
      GG_HIP(m, hipMemsetAsync(d_sprof, 0, 8 * sizeof(uint64_t), st));
      s.prof = d_sprof;
    }
    uint64_t gz_in = 0;
    for (uint32_t f = 0; f < nf; ++f) gz_in += files[f].gz ? files[f].data_len : 0;
    GG_HIP(m, timed_launch(m, GG_KERNEL_INFLATE_SEARCH, gz_in, st, [&] { return launch_inflate_search(s, st); }));
    if (d_sprof) {
      uint64_t pr[8];
      GG_HIP(m, hipStreamSynchronize(st));
      GG_HIP(m, hipMemcpy(pr, d_sprof, sizeof pr, hipMemcpyDeviceToHost));
      fprintf(stderr, "[inflate] search: %u chunks; per chunk: %.1f steps (%.0f cycles each), %.1f check rounds "
              "(%.0f cycles each), %.1f candidates\n", nc, pr[2] / (double)nc, pr[0] / (double)std::max<uint64_t>(pr[2], 1),
              pr[3] / (double)nc, pr[1] / (double)std::max<uint64_t>(pr[3], 1), pr[4] / (double)nc);
    }
    GG_HIP(m, hipMemcpyAsync(start.data(), d_start, nc * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  }
  GG_HIP(m, hipStreamSynchronize(st));
  stamp("copy + search");
  // lanes per file: the stream's first bit and every block start found
  std::vector<std::vector<uint64_t>> starts(nf);
  for (uint32_t f = 0; f < nf; ++f) {
    if (!files[f].gz) continue;
    starts[f].push_back(0);
    for (uint32_t c = first_chunk[f]; c < first_chunk[f + 1]; ++c)
      if (start[c] != ~0ull && start[c] > starts[f].back()) starts[f].push_back(start[c]);
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
    fprintf(stderr, "[inflate] %u files, %u chunks, %zu starts\n", nf, nc, ns);
  }
  // one lane (a wave of the decode kernel) per start: [start, end) up to the
  // next start (~0: the file's last lane), its tokens in a region of the
  // token buffer sized one per bit, its scratch likewise
  struct Lane {
    uint32_t file;
    uint64_t start, end, tok_off, cap, scr_off;
    uint64_t n_tok = 0, out_len = 0, last_end = 0;
    uint64_t done_tok = 0, done_out = 0;  // tokens and bytes of the blocks before `start` (a resumed lane)
    uint32_t status = 0, bfin = 0;
    bool redo = true, alive = true;
  };
  std::vector<Lane> lanes;
  uint64_t toks = 0, scr = 0;
  for (uint32_t f = 0; f < nf; ++f)
    for (size_t i = 0; i < starts[f].size(); ++i) {
      const uint64_t s0 = starts[f][i];
      const uint64_t e = i + 1 < starts[f].size() ? starts[f][i + 1] : ~0ull;
      // every symbol takes >= 1 bit: one token per bit bounds every lane
      // (literal-heavy DNA blocks reach ~0.5 tokens per bit)
      const uint64_t bits = (e == ~0ull ? fbits[f] : e) - s0;
      Lane ln{f, s0, e, toks, bits + 64, scr};
      lanes.push_back(ln);
      toks += (bits + 64 + 3) / 4 * 4;
      scr += inflate::decode_scratch(bits);
    }
  uint32_t *d_tok = nullptr, *d_scr = nullptr;
  GZ_SCRATCH(m, "gz_tok", std::max<uint64_t>(toks, 4), &d_tok);
  GZ_SCRATCH(m, "gz_scr", std::max<uint64_t>(scr, 4), &d_scr);
  for (int pass = 0;; ++pass) {
    std::vector<uint32_t> redo;
    for (uint32_t l = 0; l < (uint32_t)lanes.size(); ++l)
      if (lanes[l].alive && lanes[l].redo) redo.push_back(l);
    const uint32_t nl = (uint32_t)redo.size();
    if (nl == 0) break;
    // every lane takes the staged (LDS) decode, which stages a long segment
    // in windows (GALAHGPU_DECODE_GLOBAL=1: the global-memory form, A/B only)
    const char* gdec = getenv("GALAHGPU_DECODE_GLOBAL");
    const bool global_only = gdec && *gdec == '1';
    const uint32_t n_staged = global_only ? 0u : nl;
    if (pass >= kMaxRelaunch) return hand_back("block starts did not chain", 0);  // (ok = false)
    // the lanes to decode: 6 arrays of nl u64 (file, start, end, tok_off, cap, scr_off)
    std::vector<uint64_t> arg((size_t)nl * 6);
    for (uint32_t k = 0; k < nl; ++k) {
      const Lane& x = lanes[redo[k]];
      arg[k] = x.file;
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
    for (uint32_t k = 0; k < nl; ++k) lf[k] = lanes[redo[k]].file;
    GG_HIP(m, hipMemcpyAsync(d_arg, arg.data(), arg.size() * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    GG_HIP(m, hipMemcpyAsync(d_lfile, lf.data(), nl * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    InflateDecode d;
    d.in = (const uint32_t*)d_in;
    d.file_word = d_fword;
    d.file_bits = d_fbits;
    d.lane_file = d_lfile;
    d.lane_start = d_arg + nl;
    d.lane_end = d_arg + 2 * (size_t)nl;
    d.n_lanes = nl;
    d.n_staged = n_staged;
    {  // GALAHGPU_TEST_STAGE_KB (tests): a smaller LDS stage, so blocks take several windows
      const char* se = getenv("GALAHGPU_TEST_STAGE_KB");
      const int kb = se && *se ? atoi(se) : 0;
      d.stage_words = kb >= 1 && kb <= 30 ? (uint32_t)kb * 256u : 0u;
    }
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
      fprintf(stderr, "[inflate] decode: %u lanes, %llu blocks, %.0f tokens/block; cycles per block: header %.0f, "
              "first decode %.0f, resync %.0f, copy %.0f\n", nl, (unsigned long long)pr[4], pr[5] / nb, pr[0] / nb,
              pr[1] / nb, pr[2] / nb, pr[3] / nb);
    }
    std::vector<uint64_t> res((size_t)nl * 4);
    GG_HIP(m, hipMemcpyAsync(res.data(), d_res, res.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    GG_HIP(m, hipStreamSynchronize(st));
    stamp("decode pass");
    const uint32_t* r32 = (const uint32_t*)(res.data() + 3 * (size_t)nl);
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
    uint32_t prev_file = ~0u;
    for (uint32_t l = 0; l < (uint32_t)lanes.size(); ++l) {
      Lane& x = lanes[l];
      if (!x.alive) continue;
      const bool after_redo = prev_redo && prev_file == x.file;
      prev_file = x.file;
      prev_redo = x.redo;
      if (x.redo) continue;
      uint32_t nx = l + 1;
      while (nx < lanes.size() && !lanes[nx].alive) ++nx;
      const bool has_next = nx < lanes.size() && lanes[nx].file == x.file;
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
      } else if (x.status != inflate::kDecOk && !after_redo) {  // malformed / full / a second member: host path
        return hand_back(x.status == inflate::kDecFull ? "token capacity"
                         : x.status == inflate::kDecFinalEarly ? "stream ended early (several members?)"
                                                               : "malformed stream", x.file);
      }
    }
  }
  std::vector<Lane> live;
  for (const Lane& x : lanes)
    if (x.alive) live.push_back(x);
  // every file: its last lane decoded the final block, ending at the trailer
  // (one member), and the output length agrees with ISIZE
  std::vector<uint64_t> flen(nf, 0), lane_out(live.size());
  for (size_t l = 0; l < live.size(); ++l) {
    const uint32_t f = live[l].file;
    lane_out[l] = flen[f];
    flen[f] += live[l].out_len;
    if (l + 1 == live.size() || live[l + 1].file != f) {
      if (!live[l].bfin || (live[l].last_end + 7) / 8 != files[f].data_len) return hand_back("not one member", f);
      if ((uint32_t)flen[f] != files[f].isize) return hand_back("ISIZE", f);
    }
  }
  for (uint32_t f = 0; f < nf; ++f)
    if (!files[f].gz) flen[f] = files[f].data_len;
  foff.assign(nf + 1, 0);
  for (uint32_t f = 0; f < nf; ++f) foff[f + 1] = foff[f] + (flen[f] + 15) / 16 * 16;
  const uint64_t text_len = foff[nf];
  if (text_len >= (1ull << 30)) return hand_back("batch text over 1 GiB", 0);  // (30-bit expand pointers)
  for (size_t l = 0; l < lane_out.size(); ++l) lane_out[l] += foff[live[l].file];
  uint32_t *d_val, *d_flags, *d_crc, *d_lfile;
  uint64_t *d_lout, *d_ftext, *d_flen;
  GZ_SCRATCH(m, "gz_val", std::max<uint64_t>(text_len, 1), &d_val);
  // (tests: GALAHGPU_TEST_POISON_VAL=<u32> fills val with that word first --
  // what a previous batch or another allocation left there -- and no result
  // may change: the resolve reads val only where the expand wrote it)
  const char* poison = getenv("GALAHGPU_TEST_POISON_VAL");
  if (poison && *poison && text_len)
    GG_HIP(m, hipMemsetD32Async(d_val, (int)strtoul(poison, nullptr, 0), text_len, st));
  GG_HIP(m, scratch_t(m, "stage_text", std::max<uint64_t>(text_len, 16) + 16, d_text));
  // per live lane: text position, token offset, token count, end of the
  // padding after it (its file's last lane: the next file's start; else 0)
  // (u64), then its file (u32)
  const size_t NL = std::max<size_t>(live.size(), 1);
  GG_HIP(m, scratch_t(m, "gz_lout", 5 * NL + (NL + 1) / 2, &d_lout));
  d_lfile = (uint32_t*)(d_lout + 5 * NL);
  GG_HIP(m, scratch_t(m, "gz_ftext", 2 * (size_t)nf + 1, &d_ftext));
  d_flen = d_ftext + nf;
  GG_HIP(m, scratch_t(m, "gz_flags", 2 * (size_t)nf + 1, &d_flags));
  d_crc = d_flags + 1;
  for (uint32_t f = 0; f < nf; ++f)  // (plain files: their text is copied in after the resolve; until then
    if (!files[f].gz && foff[f + 1] > foff[f])  //  no byte of theirs may send the resolve to val)
      GG_HIP(m, hipMemsetAsync(*d_text + foff[f], '\n', foff[f + 1] - foff[f], st));
  GG_HIP(m, hipMemsetAsync(d_flags, 0, sizeof(uint32_t), st));
  std::vector<uint64_t> ftext(2 * (size_t)nf);
  for (uint32_t f = 0; f < nf; ++f) {
    ftext[f] = foff[f];
    ftext[nf + f] = flen[f];
  }
  GG_HIP(m, hipMemcpyAsync(d_ftext, ftext.data(), ftext.size() * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  std::vector<uint64_t> lv(5 * NL + (NL + 1) / 2, 0);
  for (size_t l = 0; l < live.size(); ++l) {
    lv[l] = lane_out[l];
    lv[NL + l] = live[l].tok_off;
    lv[2 * NL + l] = live[l].n_tok;
    if (l + 1 == live.size() || live[l + 1].file != live[l].file) lv[3 * NL + l] = foff[live[l].file + 1];
    lv[4 * NL + l] = live[l].out_len;
    ((uint32_t*)(lv.data() + 5 * NL))[l] = live[l].file;
  }
  GG_HIP(m, hipMemcpyAsync(d_lout, lv.data(), lv.size() * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  InflatePlace p;
  p.tok = d_tok;
  p.tok_off = d_lout + NL;
  p.n_tok = d_lout + 2 * NL;
  p.lane_pad = d_lout + 3 * NL;
  p.lane_len = d_lout + 4 * NL;
  p.lane_file = d_lfile;
  p.lane_out = d_lout;
  p.file_text = d_ftext;
  p.n_lanes = (uint32_t)live.size();
  p.text = *d_text;
  p.val = d_val;
  p.flags = d_flags;
  std::vector<uint32_t> seg_first(nf + 1, 0);
  for (uint32_t f = 0; f < nf; ++f) seg_first[f + 1] = seg_first[f] + (uint32_t)((flen[f] + kInflateCrcSeg - 1) / kInflateCrcSeg);
  const uint32_t nseg = seg_first[nf];
  uint32_t *d_sfirst, *d_scrc;
  GG_HIP(m, scratch_t(m, "gz_sfirst", nf + 1, &d_sfirst));
  GG_HIP(m, scratch_t(m, "gz_scrc", std::max(nseg, 1u), &d_scrc));
  GG_HIP(m, hipMemcpyAsync(d_sfirst, seg_first.data(), (nf + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  GG_HIP(m, timed_launch(m, GG_KERNEL_INFLATE_EXPAND, text_len, st, [&] { return launch_inflate_expand(p, st); }));
  GG_HIP(m, timed_launch(m, GG_KERNEL_INFLATE_RESOLVE, text_len, st,
                         [&] { return launch_inflate_resolve(p, text_len, st); }));
  GG_HIP(m, timed_launch(m, GG_KERNEL_INFLATE_CRC, text_len, st, [&] {
    return launch_inflate_crc(*d_text, nf, d_ftext, d_flen, d_sfirst, nseg, d_scrc, d_crc, st);
  }));
  // plain files (not gzip) go into their place as they are
  for (uint32_t f = 0; f < nf; ++f)
    if (!files[f].gz && files[f].data_len)
      GG_HIP(m, hipMemcpyAsync(*d_text + foff[f], d_in + files[f].data_off, files[f].data_len,
                               hipMemcpyDeviceToDevice, st));
  // flags, then per file its CRC-32 and its first byte
  std::vector<uint32_t> chk(2 * (size_t)nf + 1);
  GG_HIP(m, hipMemcpyAsync(chk.data(), d_flags, chk.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  GG_HIP(m, hipStreamSynchronize(st));
  stamp("expand + resolve + crc");
  if (chk[0])
    return hand_back(chk[0] & 1   ? "distance before the file start"
                     : chk[0] & 4 ? "token bytes disagree with the decode's count"
                                  : "pointer chain",
                     0);
  for (uint32_t f = 0; f < nf; ++f)
    if (files[f].gz && (chk[1 + f] != files[f].crc || chk[1 + nf + f] != '>'))  // (FASTQ, malformed: the host path)
      return hand_back(chk[1 + f] != files[f].crc ? "CRC-32" : "not FASTA", f);
  *ok = true;
  return GG_OK;
}

}  // namespace gg
