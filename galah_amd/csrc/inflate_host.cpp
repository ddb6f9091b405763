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
bool gzip_member(const uint8_t* buf, size_t n, size_t* data_off, size_t* data_len, uint32_t* isize, uint32_t* crc) {
  if (n < 18 || buf[0] != 0x1f || buf[1] != 0x8b || buf[2] != 8) return false;
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
  if (p + 8 > n) return false;
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
constexpr uint32_t kChunkBytes = 4096;  // search granularity: a zlib -6 block of FASTA is ~25-30 KB
constexpr int kMaxRelaunch = 8;         // decode passes that may drop wrong starts before giving up
}  // namespace

// files[f]: the deflate data of a gzip file (gz = true; data_off is 4-byte
// aligned in h_in, isize/crc from its trailer) or plain text (gz = false).
gg_status inflate_batch(gg_ctx* m, const uint8_t* h_in, uint64_t in_bytes, const std::vector<InflateFile>& files,
                        uint8_t** d_text, std::vector<uint64_t>& foff, bool* ok) {
  *ok = false;
  hipStream_t st = m->stream;
  const uint32_t nf = (uint32_t)files.size();
  // the batch on the device (+ padding the cursors read past a file's end)
  uint8_t* d_in;
  const uint64_t in_alloc = (in_bytes + 15) / 16 * 16 + 64;
  GG_HIP(m, scratch_t(m, "gz_in", in_alloc, &d_in));
  GG_HIP(m, hipMemsetAsync(d_in + in_bytes, 0, in_alloc - in_bytes, st));
  if (in_bytes) GG_HIP(m, hipMemcpyAsync(d_in, h_in, in_bytes, hipMemcpyHostToDevice, st));
  std::vector<uint64_t> fword(nf), fbits(nf);
  std::vector<uint32_t> chunk_file;
  std::vector<uint64_t> chunk_bit0;
  std::vector<uint32_t> first_chunk(nf + 1, 0);
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
    GG_HIP(m, launch_inflate_search(s, st));
    GG_HIP(m, hipMemcpyAsync(start.data(), d_start, nc * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  }
  GG_HIP(m, hipStreamSynchronize(st));
  // lanes per file: the stream's first bit and every block start found
  std::vector<std::vector<uint64_t>> starts(nf);
  for (uint32_t f = 0; f < nf; ++f) {
    if (!files[f].gz) continue;
    starts[f].push_back(0);
    for (uint32_t c = first_chunk[f]; c < first_chunk[f + 1]; ++c)
      if (start[c] != ~0ull && start[c] > starts[f].back()) starts[f].push_back(start[c]);
  }
  std::vector<uint32_t> lane_file, status, bfin;
  std::vector<uint64_t> lane_start, lane_end, tok_off, tok_cap, scr_off, n_tok, out_len, last_end;
  uint32_t *d_lfile = nullptr, *d_tok = nullptr, *d_scr = nullptr;
  uint64_t *d_toff = nullptr, *d_res = nullptr;
  for (int pass = 0;; ++pass) {
    if (pass >= kMaxRelaunch) return hand_back("block starts did not chain", 0);  // (ok = false)
    lane_file.clear();
    lane_start.clear();
    lane_end.clear();
    tok_off.clear();
    tok_cap.clear();
    scr_off.clear();
    uint64_t toks = 0, scr = 0;
    for (uint32_t f = 0; f < nf; ++f)
      for (size_t i = 0; i < starts[f].size(); ++i) {
        const uint64_t s0 = starts[f][i];
        const uint64_t e = i + 1 < starts[f].size() ? starts[f][i + 1] : ~0ull;
        // every symbol takes >= 1 bit: one token per bit bounds every lane
        // (literal-heavy DNA blocks reach ~0.5 tokens per bit)
        const uint64_t bits = (e == ~0ull ? fbits[f] : e) - s0;
        const uint64_t cap = bits + 64;
        lane_file.push_back(f);
        lane_start.push_back(s0);
        lane_end.push_back(e);
        tok_off.push_back(toks);
        tok_cap.push_back(cap);
        scr_off.push_back(scr);
        toks += (cap + 3) / 4 * 4;
        scr += inflate::decode_scratch(bits);
      }
    const uint32_t nl = (uint32_t)lane_file.size();
    if (nl == 0) break;
    uint32_t *d_status, *d_bfin;
    uint64_t *d_lstart, *d_lend, *d_tcap, *d_soff;
    GG_HIP(m, scratch_t(m, "gz_lfile", nl, &d_lfile));
    GG_HIP(m, scratch_t(m, "gz_lstart", nl, &d_lstart));
    GG_HIP(m, scratch_t(m, "gz_lend", nl, &d_lend));
    GG_HIP(m, scratch_t(m, "gz_toff", nl, &d_toff));
    GG_HIP(m, scratch_t(m, "gz_tcap", nl, &d_tcap));
    GG_HIP(m, scratch_t(m, "gz_soff", nl, &d_soff));
    GG_HIP(m, scratch_t(m, "gz_tok", std::max<uint64_t>(toks, 4), &d_tok));
    GG_HIP(m, scratch_t(m, "gz_scr", std::max<uint64_t>(scr, 4), &d_scr));
    // results contiguous: n_tok, out_len, last_end (u64), then status, bfinal (u32)
    GG_HIP(m, scratch_t(m, "gz_res", (size_t)nl * 4, &d_res));
    d_status = (uint32_t*)(d_res + 3 * (size_t)nl);
    d_bfin = d_status + nl;
    GG_HIP(m, hipMemcpyAsync(d_lfile, lane_file.data(), nl * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    GG_HIP(m, hipMemcpyAsync(d_lstart, lane_start.data(), nl * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    GG_HIP(m, hipMemcpyAsync(d_lend, lane_end.data(), nl * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    GG_HIP(m, hipMemcpyAsync(d_toff, tok_off.data(), nl * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    GG_HIP(m, hipMemcpyAsync(d_tcap, tok_cap.data(), nl * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    GG_HIP(m, hipMemcpyAsync(d_soff, scr_off.data(), nl * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    InflateDecode d;
    d.in = (const uint32_t*)d_in;
    d.file_word = d_fword;
    d.file_bits = d_fbits;
    d.lane_file = d_lfile;
    d.lane_start = d_lstart;
    d.lane_end = d_lend;
    d.n_lanes = nl;
    d.tok = d_tok;
    d.tok_off = d_toff;
    d.tok_cap = d_tcap;
    d.scr = d_scr;
    d.scr_off = d_soff;
    d.n_tok = d_res;
    d.out_len = d_res + nl;
    d.last_end = d_res + 2 * (size_t)nl;
    d.status = d_status;
    d.bfinal = d_bfin;
    GG_HIP(m, launch_inflate_decode(d, st));
    std::vector<uint64_t> res((size_t)nl * 4);
    GG_HIP(m, hipMemcpyAsync(res.data(), d_res, res.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    GG_HIP(m, hipStreamSynchronize(st));
    n_tok.assign(res.begin(), res.begin() + nl);
    out_len.assign(res.begin() + nl, res.begin() + 2 * nl);
    last_end.assign(res.begin() + 2 * nl, res.begin() + 3 * nl);
    const uint32_t* r32 = (const uint32_t*)(res.data() + 3 * (size_t)nl);
    status.assign(r32, r32 + nl);
    bfin.assign(r32 + nl, r32 + 2 * nl);
    // a lane that passed the next start without landing on it: that start is
    // not a block boundary -- dropped, and the batch decoded again
    bool again = false;
    uint32_t l = 0;
    for (uint32_t f = 0; f < nf; ++f) {
      std::vector<uint64_t> keep;
      bool drop_next = false;
      for (size_t i = 0; i < starts[f].size(); ++i, ++l) {
        if (drop_next) {
          drop_next = false;
          again = true;
          continue;
        }
        keep.push_back(starts[f][i]);
        if (status[l] == inflate::kDecOverrun && i + 1 < starts[f].size()) drop_next = true;
        else if (status[l] != inflate::kDecOk)  // malformed / full / a second member: host path
          return hand_back(status[l] == inflate::kDecFull ? "token capacity"
                           : status[l] == inflate::kDecFinalEarly ? "stream ended early (several members?)"
                                                                  : "malformed stream", f);
      }
      starts[f].swap(keep);
    }
    if (!again) break;
  }
  // every file: its last lane decoded the final block, ending at the trailer
  // (one member), and the output length agrees with ISIZE
  std::vector<uint64_t> flen(nf, 0), lane_out(lane_file.size());
  {
    uint32_t l = 0;
    for (uint32_t f = 0; f < nf; ++f) {
      if (!files[f].gz) {
        flen[f] = files[f].data_len;
        continue;
      }
      for (size_t i = 0; i < starts[f].size(); ++i, ++l) {
        lane_out[l] = flen[f];
        flen[f] += out_len[l];
        if (i + 1 == starts[f].size()) {
          if (!bfin[l] || (last_end[l] + 7) / 8 != files[f].data_len) return hand_back("not one member", f);
        }
      }
      if ((uint32_t)flen[f] != files[f].isize) return hand_back("ISIZE", f);
    }
  }
  foff.assign(nf + 1, 0);
  for (uint32_t f = 0; f < nf; ++f) foff[f + 1] = foff[f] + (flen[f] + 15) / 16 * 16;
  const uint64_t text_len = foff[nf];
  if (text_len >= (1ull << 30)) return hand_back("batch text over 1 GiB", 0);  // (30-bit expand pointers)
  for (size_t l = 0; l < lane_out.size(); ++l) lane_out[l] += foff[lane_file[l]];
  uint32_t *d_val, *d_flags, *d_crc;
  uint64_t *d_lout, *d_ftext, *d_flen;
  GG_HIP(m, scratch_t(m, "gz_val", std::max<uint64_t>(text_len, 1), &d_val));
  GG_HIP(m, scratch_t(m, "stage_text", std::max<uint64_t>(text_len, 16) + 16, d_text));
  GG_HIP(m, scratch_t(m, "gz_lout", std::max<size_t>(lane_out.size(), 1), &d_lout));
  GG_HIP(m, scratch_t(m, "gz_ftext", 2 * (size_t)nf + 1, &d_ftext));
  d_flen = d_ftext + nf;
  GG_HIP(m, scratch_t(m, "gz_flags", 2 * (size_t)nf + 1, &d_flags));
  d_crc = d_flags + 1;
  GG_HIP(m, hipMemsetD32Async((hipDeviceptr_t)d_val, 0x80000000u | '\n', text_len, st));
  GG_HIP(m, hipMemsetAsync(d_flags, 0, sizeof(uint32_t), st));
  std::vector<uint64_t> ftext(2 * (size_t)nf);
  for (uint32_t f = 0; f < nf; ++f) {
    ftext[f] = foff[f];
    ftext[nf + f] = flen[f];
  }
  GG_HIP(m, hipMemcpyAsync(d_ftext, ftext.data(), ftext.size() * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  if (!lane_out.empty())
    GG_HIP(m, hipMemcpyAsync(d_lout, lane_out.data(), lane_out.size() * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  InflatePlace p;
  p.tok = d_tok;
  p.tok_off = d_toff;
  p.n_tok = d_res;
  p.lane_file = d_lfile;
  p.lane_out = d_lout;
  p.file_text = d_ftext;
  p.n_lanes = (uint32_t)lane_out.size();
  p.val = d_val;
  p.flags = d_flags;
  std::vector<uint32_t> seg_first(nf + 1, 0);
  for (uint32_t f = 0; f < nf; ++f) seg_first[f + 1] = seg_first[f] + (uint32_t)((flen[f] + kInflateCrcSeg - 1) / kInflateCrcSeg);
  const uint32_t nseg = seg_first[nf];
  uint32_t *d_sfirst, *d_scrc;
  GG_HIP(m, scratch_t(m, "gz_sfirst", nf + 1, &d_sfirst));
  GG_HIP(m, scratch_t(m, "gz_scrc", std::max(nseg, 1u), &d_scrc));
  GG_HIP(m, hipMemcpyAsync(d_sfirst, seg_first.data(), (nf + 1) * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  GG_HIP(m, launch_inflate_place(p, text_len, *d_text, nf, d_ftext, d_flen, d_sfirst, nseg, d_scrc, d_crc, st));
  // plain files (not gzip) go into their place as they are
  for (uint32_t f = 0; f < nf; ++f)
    if (!files[f].gz && files[f].data_len)
      GG_HIP(m, hipMemcpyAsync(*d_text + foff[f], d_in + files[f].data_off, files[f].data_len,
                               hipMemcpyDeviceToDevice, st));
  // flags, then per file its CRC-32 and its first byte
  std::vector<uint32_t> chk(2 * (size_t)nf + 1);
  GG_HIP(m, hipMemcpyAsync(chk.data(), d_flags, chk.size() * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  GG_HIP(m, hipStreamSynchronize(st));
  if (chk[0]) return hand_back(chk[0] & 1 ? "distance before the file start" : "pointer chain", 0);
  for (uint32_t f = 0; f < nf; ++f)
    if (files[f].gz && (chk[1 + f] != files[f].crc || chk[1 + nf + f] != '>'))  // (FASTQ, malformed: the host path)
      return hand_back(chk[1 + f] != files[f].crc ? "CRC-32" : "not FASTA", f);
  *ok = true;
  return GG_OK;
}

}  // namespace gg
