// Host-side ingest: FASTA/FASTQ (plain or gzip) -> 2-bit packed ACGT runs.
//
// Replaces the byte-level front half of finch::sketch_files as galah calls
// it (src/finch.rs:47): needletail 0.5 parse_fastx_file, per-record
// normalize(false) and the "all k bytes in {A,C,G,T}" window test of
// canonical_kmers.  After this step a k-mer exists exactly at the positions
// [base, base + len - k] of each run, which is what kernel K1 enumerates.
//
// needletail normalize(false) byte map restated:
//   A C G T         -> kept                 a c g    -> upper case
//   t u U           -> T                    ' ' \t \r \n -> dropped (do not
//   everything else -> 'N' (breaks a k-mer)                 break a k-mer)
//
// Each genome starts on a 16-base word boundary so files can be packed on
// separate threads and concatenated with a memcpy.
#include <dlfcn.h>
#include <sched.h>
#include <smmintrin.h>
#include <tmmintrin.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gg_internal.hpp"

namespace gg {
namespace {

enum : uint8_t { kBreak = 4, kSkip = 5 };

struct ByteClass {
  uint8_t t[256];
  ByteClass() {
    for (int i = 0; i < 256; ++i) t[i] = kBreak;
    t['A'] = t['a'] = 0;
    t['C'] = t['c'] = 1;
    t['G'] = t['g'] = 2;
    t['T'] = t['t'] = t['U'] = t['u'] = 3;
    t[' '] = t['\t'] = t['\r'] = t['\n'] = kSkip;
  }
};
const ByteClass kClass;

// 16 bytes -> their 2-bit codes (A0 C1 G2 T3, U as T; first byte in bits
// 31..30) and the mask of the bytes that are A/C/G/T/U in either case (bit b
// = byte b; codes of other bytes are garbage).  ((c >> 1) ^ (c >> 2)) & 3
// maps exactly those ten letters to their codes.
__attribute__((target("sse4.1"))) inline uint32_t pack16(const uint8_t* p, uint32_t* word) {
  const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(p));
  const __m128i v = _mm_or_si128(c, _mm_set1_epi8(0x20));  // lower case
  __m128i ok = _mm_cmpeq_epi8(v, _mm_set1_epi8('a'));
  ok = _mm_or_si128(ok, _mm_cmpeq_epi8(v, _mm_set1_epi8('c')));
  ok = _mm_or_si128(ok, _mm_cmpeq_epi8(v, _mm_set1_epi8('g')));
  ok = _mm_or_si128(ok, _mm_cmpeq_epi8(v, _mm_set1_epi8('t')));
  ok = _mm_or_si128(ok, _mm_cmpeq_epi8(v, _mm_set1_epi8('u')));
  const __m128i code = _mm_and_si128(_mm_xor_si128(_mm_srli_epi16(c, 1), _mm_srli_epi16(c, 2)), _mm_set1_epi8(3));
  // pairs -> 4-bit, quads -> 8-bit (base 0 most significant)
  const __m128i q2 = _mm_maddubs_epi16(code, _mm_set1_epi16(0x0104));  // 4 * even + odd
  const __m128i q4 = _mm_madd_epi16(q2, _mm_set1_epi32(0x00010010));   // 16 * lo + hi
  const __m128i b = _mm_packus_epi16(_mm_packus_epi32(q4, q4), _mm_setzero_si128());
  *word = __builtin_bswap32((uint32_t)_mm_cvtsi128_si32(b));
  return (uint32_t)_mm_movemask_epi8(ok);
}

// Packs the runs of ONE genome; bases start at word 0 of its own buffer.
struct GenomePacker {
  int k;
  std::vector<uint8_t> text;  // raw streams: the FASTA text (parse.hip)
  std::vector<uint32_t> words;
  std::vector<gg_run> runs;  // base relative to this genome's first word
  uint64_t n_bases = 0;
  uint32_t cur = 0;
  uint32_t fill = 0;  // bases in cur
  uint64_t run_start = 0;
  bool in_run = false;

  explicit GenomePacker(int k_) : k(k_) {}

  inline void push(uint32_t c) {
    cur |= c << (30 - 2 * fill);
    if (++fill == 16) {
      words.push_back(cur);
      cur = 0;
      fill = 0;
    }
    ++n_bases;
  }

  // Drop bases back to `to` (a run shorter than k).
  void truncate(uint64_t to) {
    if (to == n_bases) return;
    const uint64_t w = to >> 4;
    const uint32_t f = (uint32_t)(to & 15);
    uint32_t word = (w < words.size()) ? words[w] : cur;
    words.resize(w);
    cur = f ? (word & (~0u << (32 - 2 * f))) : 0;
    fill = f;
    n_bases = to;
  }

  inline void end_run() {
    if (!in_run) return;
    in_run = false;
    const uint64_t len = n_bases - run_start;
    if (len < (uint64_t)k) {
      truncate(run_start);
    } else {
      runs.push_back(gg_run{0u, (uint32_t)len, run_start});
    }
  }

  // The first j (1..15) bases of word (MSB-first 2-bit codes; the rest of
  // word is ignored).
  inline void push_n(uint32_t word, uint32_t j) {
    if (!in_run) {
      in_run = true;
      run_start = n_bases;
    }
    word &= ~0u << (32 - 2 * j);
    if (fill == 0) {
      cur = word;
      fill = j;
    } else {
      cur |= word >> (2 * fill);
      const uint32_t nf = fill + j;
      if (nf >= 16) {
        words.push_back(cur);
        cur = nf > 16 ? word << (32 - 2 * fill) : 0u;
        fill = nf - 16;
      } else {
        fill = nf;
      }
    }
    n_bases += j;
  }

  // 16 bases at once (word = their MSB-first 2-bit codes).
  inline void push16(uint32_t word) {
    if (!in_run) {
      in_run = true;
      run_start = n_bases;
    }
    if (fill == 0) {
      words.push_back(word);
    } else {
      words.push_back(cur | (word >> (2 * fill)));
      cur = word << (32 - 2 * fill);
    }
    n_bases += 16;
  }

  // One record's sequence bytes (may contain line breaks).  16 bytes at a
  // time: all bases (the common case) in one step; otherwise the bases
  // before the first other byte in one step, then that byte (a line break
  // of a 60-column file costs one step, not one per byte up to it).
  void add_sequence(const uint8_t* p, size_t n) {
    size_t i = 0;
    while (i < n) {
      uint32_t word;
      if (i + 16 <= n) {
        const uint32_t m = pack16(p + i, &word);
        if (m == 0xFFFFu) {
          push16(word);
          i += 16;
          continue;
        }
        const uint32_t j = (uint32_t)__builtin_ctz(~m);  // leading bases
        if (j) {
          push_n(word, j);
          i += j;
        }
        if (kClass.t[p[i]] == kBreak) end_run();  // (else whitespace: skipped)
        ++i;
        continue;
      }
      const uint8_t c = kClass.t[p[i]];
      if (c < 4) {
        if (!in_run) {
          in_run = true;
          run_start = n_bases;
        }
        push(c);
      } else if (c == kBreak) {
        end_run();
      }
      ++i;
    }
  }
  void end_record() { end_run(); }

  void finish() {
    end_run();
    if (fill) {
      words.push_back(cur);
      cur = 0;
      fill = 0;
    }
  }
};

// libdeflate (whole-buffer DEFLATE, 2-3x zlib's inflate speed) is resolved
// at run time from the system library when it is installed; gzip input
// falls back to zlib's gzread otherwise.  Only the four entry points below
// are used (libdeflate >= 1.0 ABI).
struct Deflate {
  using AllocFn = void* (*)();
  using FreeFn = void (*)(void*);
  using GzipFn = int (*)(void*, const void*, size_t, void*, size_t, size_t*, size_t*);
  AllocFn alloc = nullptr;
  FreeFn free_ = nullptr;
  GzipFn gzip = nullptr;
  bool ok = false;
  Deflate() {
    if (const char* off = getenv("GALAHGPU_NO_LIBDEFLATE"); off && *off == '1') return;
    void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    alloc = (AllocFn)dlsym(h, "libdeflate_alloc_decompressor");
    free_ = (FreeFn)dlsym(h, "libdeflate_free_decompressor");
    gzip = (GzipFn)dlsym(h, "libdeflate_gzip_decompress_ex");
    ok = alloc && free_ && gzip;
  }
};
const Deflate& deflate_lib() {
  static const Deflate d;
  return d;
}

bool read_raw(const char* path, std::vector<uint8_t>& raw, std::string& err) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    err = std::string("could not open ") + path;
    return false;
  }
  raw.clear();
  if (fseek(f, 0, SEEK_END) == 0) {
    const long n = ftell(f);
    if (n > 0) raw.reserve((size_t)n);
    fseek(f, 0, SEEK_SET);
  }
  uint8_t tmp[1 << 16];
  size_t got;
  while ((got = fread(tmp, 1, sizeof tmp, f)) > 0) raw.insert(raw.end(), tmp, tmp + got);
  const bool bad = ferror(f);
  fclose(f);
  if (bad) {
    err = std::string("read error in ") + path;
    return false;
  }
  return true;
}

// gzip members (concatenated, as bgzip writes them) with libdeflate.
bool gunzip_libdeflate(const std::vector<uint8_t>& raw, std::vector<uint8_t>& buf, const char* path,
                       std::string& err) {
  const Deflate& lib = deflate_lib();
  void* d = lib.alloc();
  if (!d) {
    err = "libdeflate: out of memory";
    return false;
  }
  size_t in = 0, out = 0;
  buf.resize(std::max<size_t>(raw.size() * 4, 1 << 16));
  bool ok = true;
  while (in < raw.size()) {
    if (raw.size() - in < 18) break;  // trailing garbage shorter than a member
    size_t used_in = 0, used_out = 0;
    const int r = lib.gzip(d, raw.data() + in, raw.size() - in, buf.data() + out, buf.size() - out, &used_in, &used_out);
    if (r == 3) {  // LIBDEFLATE_INSUFFICIENT_SPACE
      buf.resize(buf.size() * 2);
      continue;
    }
    if (r != 0) {
      err = std::string("gzip decode error in ") + path;
      ok = false;
      break;
    }
    in += used_in;
    out += used_out;
  }
  lib.free_(d);
  buf.resize(out);
  return ok;
}

// gzip members with zlib (no libdeflate on the system).
bool gunzip_zlib(const std::vector<uint8_t>& raw, std::vector<uint8_t>& buf, const char* path, std::string& err) {
  z_stream zs{};
  if (inflateInit2(&zs, 15 + 32) != Z_OK) {
    err = "zlib: out of memory";
    return false;
  }
  zs.next_in = const_cast<uint8_t*>(raw.data());
  zs.avail_in = (uInt)raw.size();
  buf.resize(std::max<size_t>(raw.size() * 4, 1 << 16));
  size_t out = 0;
  for (;;) {
    if (out == buf.size()) buf.resize(buf.size() * 2);
    zs.next_out = buf.data() + out;
    zs.avail_out = (uInt)std::min<size_t>(buf.size() - out, 1u << 30);
    const uInt room = zs.avail_out;
    const int r = inflate(&zs, Z_NO_FLUSH);
    out += room - zs.avail_out;
    if (r == Z_STREAM_END) {
      if (zs.avail_in < 18) break;  // (trailing bytes shorter than a member)
      inflateReset(&zs);  // the next member
      continue;
    }
    if ((r != Z_OK && r != Z_BUF_ERROR) || (r == Z_BUF_ERROR && zs.avail_in == 0)) {
      inflateEnd(&zs);
      err = std::string("gzip decode error in ") + path;
      return false;
    }
  }
  buf.resize(out);
  inflateEnd(&zs);
  return true;
}

// bzip2 and xz, the other compressions needletail 0.5 reads by their magic
// bytes (finch's parser behind src/finch.rs:47; needletail source absent:
// parity unpinned).  libbz2 / liblzma are loaded at run time, as libdeflate
// is, through their stable C ABIs (the image has the libraries, not their
// headers); concatenated streams are all decoded, as for gzip members.
struct Bz2Lib {  // bz_stream of bzlib.h 1.0
  struct Stream {
    char* next_in;
    unsigned int avail_in, total_in_lo32, total_in_hi32;
    char* next_out;
    unsigned int avail_out, total_out_lo32, total_out_hi32;
    void* state;
    void* (*bzalloc)(void*, int, int);
    void (*bzfree)(void*, void*);
    void* opaque;
  };
  int (*init)(Stream*, int, int) = nullptr;
  int (*run)(Stream*) = nullptr;
  int (*end)(Stream*) = nullptr;
  bool ok = false;
  Bz2Lib() {
    void* h = dlopen("libbz2.so.1.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("libbz2.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    init = (int (*)(Stream*, int, int))dlsym(h, "BZ2_bzDecompressInit");
    run = (int (*)(Stream*))dlsym(h, "BZ2_bzDecompress");
    end = (int (*)(Stream*))dlsym(h, "BZ2_bzDecompressEnd");
    ok = init && run && end;
  }
};
struct XzLib {  // lzma_stream of liblzma 5 (its leading fields; the rest zeroed, LZMA_STREAM_INIT)
  struct Stream {
    const uint8_t* next_in;
    size_t avail_in;
    uint64_t total_in;
    uint8_t* next_out;
    size_t avail_out;
    uint64_t total_out;
    uint8_t rest[256];
  };
  int (*decoder)(Stream*, uint64_t, uint32_t) = nullptr;
  int (*code)(Stream*, int) = nullptr;
  void (*end)(Stream*) = nullptr;
  bool ok = false;
  XzLib() {
    void* h = dlopen("liblzma.so.5", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    decoder = (int (*)(Stream*, uint64_t, uint32_t))dlsym(h, "lzma_stream_decoder");
    code = (int (*)(Stream*, int))dlsym(h, "lzma_code");
    end = (void (*)(Stream*))dlsym(h, "lzma_end");
    ok = decoder && code && end;
  }
};

bool is_gzip(const uint8_t* b, size_t n) { return n >= 2 && b[0] == 0x1f && b[1] == 0x8b; }
bool is_bzip2(const uint8_t* b, size_t n) { return n >= 4 && b[0] == 'B' && b[1] == 'Z' && b[2] == 'h' && b[3] >= '1' && b[3] <= '9'; }
bool is_xz(const uint8_t* b, size_t n) {
  return n >= 6 && b[0] == 0xFD && b[1] == '7' && b[2] == 'z' && b[3] == 'X' && b[4] == 'Z' && b[5] == 0;
}

bool bunzip2(const std::vector<uint8_t>& raw, std::vector<uint8_t>& buf, const char* path, std::string& err) {
  static const Bz2Lib lib;
  if (!lib.ok) {
    err = std::string("bzip2 file but libbz2 is not available: ") + path;
    return false;
  }
  buf.resize(std::max<size_t>(raw.size() * 4, 1 << 16));
  size_t in = 0, out = 0;
  while (in < raw.size()) {
    Bz2Lib::Stream s{};
    if (lib.init(&s, 0, 0) != 0) {
      err = "libbz2: out of memory";
      return false;
    }
    int r = 0;
    for (;;) {  // one stream
      if (out == buf.size()) buf.resize(buf.size() * 2);
      const unsigned int ai = (unsigned int)std::min<size_t>(raw.size() - in, 1u << 30);
      const unsigned int ao = (unsigned int)std::min<size_t>(buf.size() - out, 1u << 30);
      s.next_in = (char*)raw.data() + in;
      s.avail_in = ai;
      s.next_out = (char*)buf.data() + out;
      s.avail_out = ao;
      r = lib.run(&s);
      in += ai - s.avail_in;
      out += ao - s.avail_out;
      if (r != 0) break;  // BZ_OK (0): more; BZ_STREAM_END (4) or an error
      if (s.avail_in == ai && s.avail_out == ao) break;  // no progress: truncated
    }
    lib.end(&s);
    if (r != 4) {
      err = std::string("bzip2 decode error in ") + path;
      return false;
    }
    if (raw.size() - in < 4 || !is_bzip2(raw.data() + in, raw.size() - in)) break;  // (trailing bytes)
  }
  buf.resize(out);
  return true;
}

bool unxz(const std::vector<uint8_t>& raw, std::vector<uint8_t>& buf, const char* path, std::string& err) {
  static const XzLib lib;
  if (!lib.ok) {
    err = std::string("xz file but liblzma is not available: ") + path;
    return false;
  }
  XzLib::Stream s{};
  if (lib.decoder(&s, ~0ull, 0x08 /* LZMA_CONCATENATED */) != 0) {
    err = "liblzma: out of memory";
    return false;
  }
  buf.resize(std::max<size_t>(raw.size() * 4, 1 << 16));
  size_t out = 0;
  s.next_in = raw.data();
  s.avail_in = raw.size();
  int r;
  for (;;) {
    if (out == buf.size()) buf.resize(buf.size() * 2);
    s.next_out = buf.data() + out;
    s.avail_out = buf.size() - out;
    const size_t ao = s.avail_out;
    r = lib.code(&s, 3 /* LZMA_FINISH */);
    out += ao - s.avail_out;
    if (r != 0) break;  // LZMA_OK (0): more; LZMA_STREAM_END (1) or an error
  }
  lib.end(&s);
  buf.resize(out);
  if (r != 1) {
    err = std::string("xz decode error in ") + path;
    return false;
  }
  return true;
}

// A bzip2 or xz file (its first bytes): read whole and decoded in memory
// rather than through zlib's gzread.
bool compressed_not_gzip(const char* path) {
  uint8_t h[6] = {0};
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  const size_t got = fread(h, 1, sizeof h, f);
  fclose(f);
  return is_bzip2(h, got) || is_xz(h, got);
}

// A file's bytes decompressed by their magic (gzip members, bzip2 or xz
// streams; anything else is taken as plain text).
bool decompress_bytes(std::vector<uint8_t>& raw, std::vector<uint8_t>& buf, const char* path, std::string& err) {
  if (is_gzip(raw.data(), raw.size())) {
    if (deflate_lib().ok) return gunzip_libdeflate(raw, buf, path, err);
    return gunzip_zlib(raw, buf, path, err);
  }
  if (is_bzip2(raw.data(), raw.size())) return bunzip2(raw, buf, path, err);
  if (is_xz(raw.data(), raw.size())) return unxz(raw, buf, path, err);
  buf.swap(raw);
  return true;
}

bool read_file(const char* path, std::vector<uint8_t>& buf, std::string& err) {
  const bool gz_lib = deflate_lib().ok;
  if (gz_lib || compressed_not_gzip(path)) {
    std::vector<uint8_t> raw;
    if (!read_raw(path, raw, err)) return false;
    return decompress_bytes(raw, buf, path, err);
  }
  gzFile f = gzopen(path, "rb");
  if (!f) {
    err = std::string("could not open ") + path;
    return false;
  }
  gzbuffer(f, 1 << 20);
  buf.clear();
  size_t len = 0;
  size_t cap = 1 << 22;
  buf.resize(cap);
  for (;;) {
    if (len == cap) {
      cap *= 2;
      buf.resize(cap);
    }
    const size_t want = std::min<size_t>(cap - len, 1u << 30);
    const int got = gzread(f, buf.data() + len, (unsigned)want);
    if (got < 0) {
      int zerr = 0;
      err = std::string("read error in ") + path + ": " + gzerror(f, &zerr);
      gzclose(f);
      return false;
    }
    if (got == 0) break;
    len += (size_t)got;
  }
  gzclose(f);
  buf.resize(len);
  return true;
}

// Parses FASTA ('>') or FASTQ ('@') as needletail 0.5 does for well-formed
// files; anything else is a format error (galah: "Failed to sketch genomes
// with finch", src/finch.rs:50).
gg_status pack_buffer(const uint8_t* d, size_t n, const char* name,
                      GenomePacker& gp, std::string& err) {
  if (n == 0 || (d[0] != '>' && d[0] != '@')) {
    err = std::string("not a FASTA/FASTQ file: ") + name;
    return GG_ERR_FORMAT;
  }
  size_t i = 0;
  while (i < n) {
    const uint8_t tag = d[i];
    if (tag != '>' && tag != '@') {
      err = std::string("malformed record in ") + name;
      return GG_ERR_FORMAT;
    }
    const uint8_t* nl = (const uint8_t*)memchr(d + i, '\n', n - i);
    i = nl ? (size_t)(nl - d) + 1 : n;  // skip header line
    if (tag == '>') {
      size_t start = i;
      // sequence runs until a line that starts with '>'
      while (i < n) {
        if (d[i] == '>') break;
        const uint8_t* e = (const uint8_t*)memchr(d + i, '\n', n - i);
        i = e ? (size_t)(e - d) + 1 : n;
      }
      gp.add_sequence(d + start, i - start);
      gp.end_record();
    } else {
      const uint8_t* e = (const uint8_t*)memchr(d + i, '\n', n - i);
      const size_t end = e ? (size_t)(e - d) : n;
      gp.add_sequence(d + i, end - i);
      gp.end_record();
      i = e ? end + 1 : n;
      for (int skip = 0; skip < 2 && i < n; ++skip) {  // '+' line, quality line
        const uint8_t* q = (const uint8_t*)memchr(d + i, '\n', n - i);
        i = q ? (size_t)(q - d) + 1 : n;
      }
    }
  }
  return GG_OK;
}

// Raw streams: the text the device parser reads.  A file that starts with
// '>' is FASTA to its end (pack_buffer splits records only at lines that
// start with '>'), so it goes as is; one that starts with '@' is walked as
// pack_buffer walks it and every record becomes ">\n" + its sequence bytes.
gg_status raw_text(std::vector<uint8_t>& buf, const char* name, std::vector<uint8_t>& text, std::string& err) {
  const size_t n = buf.size();
  const uint8_t* d = buf.data();
  if (n == 0 || (d[0] != '>' && d[0] != '@')) {
    err = std::string("not a FASTA/FASTQ file: ") + name;
    return GG_ERR_FORMAT;
  }
  if (d[0] == '>') {
    text.swap(buf);
    return GG_OK;
  }
  text.clear();
  text.reserve(n / 2 + 16);
  size_t i = 0;
  while (i < n) {
    const uint8_t tag = d[i];
    if (tag != '>' && tag != '@') {
      err = std::string("malformed record in ") + name;
      return GG_ERR_FORMAT;
    }
    const uint8_t* nl = (const uint8_t*)memchr(d + i, '\n', n - i);
    i = nl ? (size_t)(nl - d) + 1 : n;
    size_t start = i, end;
    if (tag == '>') {
      while (i < n) {
        if (d[i] == '>') break;
        const uint8_t* e = (const uint8_t*)memchr(d + i, '\n', n - i);
        i = e ? (size_t)(e - d) + 1 : n;
      }
      end = i;
    } else {
      const uint8_t* e = (const uint8_t*)memchr(d + i, '\n', n - i);
      end = e ? (size_t)(e - d) : n;
      i = e ? end + 1 : n;
      for (int skip = 0; skip < 2 && i < n; ++skip) {
        const uint8_t* q = (const uint8_t*)memchr(d + i, '\n', n - i);
        i = q ? (size_t)(q - d) + 1 : n;
      }
    }
    text.push_back('>');
    text.push_back('\n');
    text.insert(text.end(), d + start, d + end);
    text.push_back('\n');
  }
  return GG_OK;
}

gg_packed* assemble(std::vector<std::unique_ptr<GenomePacker>>& gps) {
  const uint32_t ng = (uint32_t)gps.size();
  uint64_t n_words = 0, n_runs = 0;
  for (auto& g : gps) {
    n_words += g->words.size();
    n_runs += g->runs.size();
  }
  gg_packed* p = (gg_packed*)calloc(1, sizeof(gg_packed));
  if (!p) return nullptr;
  p->words = (uint32_t*)malloc(std::max<uint64_t>(n_words, 1) * sizeof(uint32_t));
  p->runs = (gg_run*)malloc(std::max<uint64_t>(n_runs, 1) * sizeof(gg_run));
  p->genome_kmers = (uint64_t*)calloc(std::max<uint32_t>(ng, 1), sizeof(uint64_t));
  if (!p->words || !p->runs || !p->genome_kmers) {
    gg_packed_free(p);
    return nullptr;
  }
  uint64_t wo = 0, ro = 0;
  for (uint32_t g = 0; g < ng; ++g) {
    GenomePacker& gp = *gps[g];
    if (!gp.words.empty())
      memcpy(p->words + wo, gp.words.data(), gp.words.size() * sizeof(uint32_t));
    uint64_t kmers = 0;
    for (const gg_run& r : gp.runs) {
      p->runs[ro++] = gg_run{g, r.len, r.base + wo * 16};
      kmers += (uint64_t)r.len - (uint64_t)gp.k + 1;
    }
    p->genome_kmers[g] = kmers;
    wo += gp.words.size();
  }
  p->n_words = n_words;
  p->n_bases = n_words * 16;
  p->n_runs = n_runs;
  p->n_genomes = ng;
  return p;
}

// Threads for n_threads <= 0: GALAHGPU_THREADS, else OMP_NUM_THREADS, else
// the CPUs this process may run on (affinity mask; hardware_concurrency()
// counts the whole machine).
int default_threads() {
  for (const char* var : {"GALAHGPU_THREADS", "OMP_NUM_THREADS"}) {
    if (const char* v = getenv(var)) {
      const int t = atoi(v);
      if (t > 0) return t;
    }
  }
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof set, &set) == 0) return std::max(1, CPU_COUNT(&set));
  return (int)std::max(1u, std::thread::hardware_concurrency());
}

}  // namespace

int ingest_threads(int n_threads) { return n_threads > 0 ? n_threads : default_threads(); }

// ---------------------------------------------------------------------------
// PackStream: files packed on a worker pool, handed to consumers genome by
// genome with bounded host memory (see gg_internal.hpp).
// ---------------------------------------------------------------------------
struct PackStream::Impl {
  const char* const* paths;
  uint32_t n;
  int k;
  uint64_t budget;
  bool stamping = false;
  bool raw = false;
  std::vector<FileStamp> stamps;
  std::mutex mu;
  std::condition_variable cv_done;   // a genome finished packing
  std::condition_variable cv_space;  // in-flight bytes dropped / abort
  std::vector<std::unique_ptr<GenomePacker>> g;
  std::vector<uint8_t> state;  // 0 pending, 1 packing, 2 ready, 3 released
  std::vector<gg_status> st;
  std::vector<std::string> err;
  uint32_t next = 0;      // next file index a worker takes
  uint32_t frontier = 0;  // lowest index not yet released
  uint64_t inflight = 0;  // bytes of packed, unreleased genomes
  bool stop = false;
  std::vector<std::thread> workers;

  void work() {
    std::vector<uint8_t> buf;
    for (;;) {
      uint32_t i;
      {
        std::unique_lock<std::mutex> lk(mu);
        // the genome every consumer waits for next is always taken, so
        // waiting for space here cannot starve a consumer
        cv_space.wait(lk, [&] { return stop || next >= n || inflight < budget || next <= frontier; });
        if (stop || next >= n) return;
        i = next++;
        state[i] = 1;
      }
      auto gp = std::make_unique<GenomePacker>(k);
      gg_status s = GG_OK;
      std::string e;
      if (stamping) file_stamp(paths[i], &stamps[i]);
      if (!paths[i]) {
        s = GG_ERR_INVALID_ARG;
        e = "null path";
      } else if (!read_file(paths[i], buf, e)) {
        s = GG_ERR_IO;
      } else if (raw) {
        s = raw_text(buf, paths[i], gp->text, e);
      } else {
        s = pack_buffer(buf.data(), buf.size(), paths[i], *gp, e);
        gp->finish();
      }
      if (buf.capacity() > (256u << 20)) std::vector<uint8_t>().swap(buf);  // do not pin a huge buffer
      {
        std::lock_guard<std::mutex> lk(mu);
        inflight += gp->words.size() * sizeof(uint32_t) + gp->runs.size() * sizeof(gg_run) + gp->text.size();
        g[i] = std::move(gp);
        st[i] = s;
        err[i] = std::move(e);
        state[i] = 2;
      }
      cv_done.notify_all();
    }
  }
};

PackStream::PackStream(const char* const* paths, uint32_t n, int k, int n_threads, uint64_t budget_bytes,
                       bool stamp_files, bool raw)
    : p_(new Impl()) {
  Impl& m = *p_;
  m.stamping = stamp_files;
  m.raw = raw;
  m.stamps.resize(stamp_files ? n : 0);
  m.paths = paths;
  m.n = n;
  m.k = k;
  m.budget = std::max<uint64_t>(budget_bytes, 1);
  m.g.resize(n);
  m.state.assign(n, 0);
  m.st.assign(n, GG_OK);
  m.err.resize(n);
  const int t = (int)std::min<uint32_t>((uint32_t)ingest_threads(n_threads), std::max(1u, n));
  for (int w = 0; w < t; ++w) m.workers.emplace_back([this] { p_->work(); });
}

PackStream::~PackStream() {
  abort();
  for (auto& t : p_->workers)
    if (t.joinable()) t.join();
}

void PackStream::abort() {
  {
    std::lock_guard<std::mutex> lk(p_->mu);
    p_->stop = true;
  }
  p_->cv_space.notify_all();
  p_->cv_done.notify_all();
}

gg_status PackStream::get(uint32_t i, const std::vector<uint32_t>** words, const std::vector<gg_run>** runs,
                          std::string* err) {
  Impl& m = *p_;
  std::unique_lock<std::mutex> lk(m.mu);
  m.cv_done.wait(lk, [&] { return m.state[i] >= 2 || (m.stop && m.state[i] == 0); });
  if (m.state[i] < 2) {
    if (err) *err = "ingest aborted";
    return GG_ERR_INTERNAL;
  }
  if (m.st[i] != GG_OK) {
    if (err) *err = m.err[i];
    return m.st[i];
  }
  *words = &m.g[i]->words;
  *runs = &m.g[i]->runs;
  return GG_OK;
}

gg_status PackStream::get_raw(uint32_t i, const std::vector<uint8_t>** text, std::string* err) {
  Impl& m = *p_;
  std::unique_lock<std::mutex> lk(m.mu);
  m.cv_done.wait(lk, [&] { return m.state[i] >= 2 || (m.stop && m.state[i] == 0); });
  if (m.state[i] < 2) {
    if (err) *err = "ingest aborted";
    return GG_ERR_INTERNAL;
  }
  if (m.st[i] != GG_OK) {
    if (err) *err = m.err[i];
    return m.st[i];
  }
  *text = &m.g[i]->text;
  return GG_OK;
}

gg_status host_text_from_bytes(std::vector<uint8_t>& bytes, const char* name, std::vector<uint8_t>& text,
                               std::string& err) {
  std::vector<uint8_t> buf;
  if (!decompress_bytes(bytes, buf, name, err)) return GG_ERR_IO;
  return raw_text(buf, name, text, err);
}

FileStamp PackStream::stamp(uint32_t i) {
  std::lock_guard<std::mutex> lk(p_->mu);
  return p_->stamping ? p_->stamps[i] : FileStamp{};
}

void PackStream::release(uint32_t i) {
  Impl& m = *p_;
  {
    std::lock_guard<std::mutex> lk(m.mu);
    if (m.state[i] != 2) return;
    m.inflight -= m.g[i]->words.size() * sizeof(uint32_t) + m.g[i]->runs.size() * sizeof(gg_run) + m.g[i]->text.size();
    m.g[i].reset();
    m.state[i] = 3;
    while (m.frontier < m.n && m.state[m.frontier] == 3) ++m.frontier;
  }
  m.cv_space.notify_all();
}

gg_status PackStream::first_error(std::string* err) {
  Impl& m = *p_;
  abort();
  for (auto& t : m.workers)
    if (t.joinable()) t.join();
  for (uint32_t i = 0; i < m.n; ++i)
    if (m.state[i] == 2 && m.st[i] != GG_OK) {
      if (err) *err = m.err[i];
      return m.st[i];
    }
  return GG_OK;
}

}  // namespace gg

using namespace gg;

extern "C" gg_status gg_pack_files(const char* const* paths, uint32_t n_paths,
                                   int kmer_length, int n_threads,
                                   gg_packed** out) {
  if (!out || (n_paths && !paths) || kmer_length < 1 || kmer_length > 32) {
    set_thread_error("gg_pack_files: invalid argument");
    return GG_ERR_INVALID_ARG;
  }
  *out = nullptr;
  std::vector<std::unique_ptr<GenomePacker>> gps(n_paths);
  std::vector<gg_status> st(n_paths, GG_OK);
  std::vector<std::string> errs(n_paths);
  if (n_threads <= 0) n_threads = default_threads();
  n_threads = (int)std::min<uint32_t>((uint32_t)n_threads, std::max(1u, n_paths));
  std::atomic<uint32_t> next{0};
  auto worker = [&]() {
    std::vector<uint8_t> buf;
    for (;;) {
      const uint32_t i = next.fetch_add(1);
      if (i >= n_paths) break;
      gps[i].reset(new GenomePacker(kmer_length));
      if (!paths[i]) {
        st[i] = GG_ERR_INVALID_ARG;
        errs[i] = "null path";
        continue;
      }
      if (!read_file(paths[i], buf, errs[i])) {
        st[i] = GG_ERR_IO;
        continue;
      }
      st[i] = pack_buffer(buf.data(), buf.size(), paths[i], *gps[i], errs[i]);
      gps[i]->finish();
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < n_threads; ++t) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();
  for (uint32_t i = 0; i < n_paths; ++i) {
    if (st[i] != GG_OK) {
      set_thread_error(errs[i]);
      return st[i];
    }
  }
  gg_packed* p = assemble(gps);
  if (!p) {
    set_thread_error("gg_pack_files: out of host memory");
    return GG_ERR_OUT_OF_MEMORY;
  }
  *out = p;
  return GG_OK;
}

extern "C" gg_status gg_pack_records(const uint8_t* const* seqs,
                                     const uint64_t* lens,
                                     const uint32_t* genome_of_record,
                                     uint64_t n_records, uint32_t n_genomes,
                                     int kmer_length, gg_packed** out) {
  if (!out || kmer_length < 1 || kmer_length > 32 ||
      (n_records && (!seqs || !lens || !genome_of_record))) {
    set_thread_error("gg_pack_records: invalid argument");
    return GG_ERR_INVALID_ARG;
  }
  *out = nullptr;
  std::vector<std::unique_ptr<GenomePacker>> gps(n_genomes);
  for (uint32_t g = 0; g < n_genomes; ++g) gps[g].reset(new GenomePacker(kmer_length));
  uint32_t prev = 0;
  for (uint64_t r = 0; r < n_records; ++r) {
    const uint32_t g = genome_of_record[r];
    if (g >= n_genomes || g < prev) {
      set_thread_error("gg_pack_records: records must be grouped by non-decreasing genome < n_genomes");
      return GG_ERR_INVALID_ARG;
    }
    prev = g;
    gps[g]->add_sequence(seqs[r], (size_t)lens[r]);
    gps[g]->end_record();
  }
  for (auto& g : gps) g->finish();
  gg_packed* p = assemble(gps);
  if (!p) {
    set_thread_error("gg_pack_records: out of host memory");
    return GG_ERR_OUT_OF_MEMORY;
  }
  *out = p;
  return GG_OK;
}

extern "C" void gg_packed_free(gg_packed* p) {
  if (!p) return;
  free(p->words);
  free(p->runs);
  free(p->genome_kmers);
  free(p);
}
