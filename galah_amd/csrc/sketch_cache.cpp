// On-disk sketch cache: per-genome bottom-s sketches
// keyed by the genome file's identity, so repeated galah runs over the same
// FASTA files skip ingest and kernel K1 for every genome already sketched.
//
// galah itself never caches sketches (src/finch.rs:47 sketches every file on
// every call); finch can serialise sketches but galah does not use it.  The
// cache therefore changes no result: a hit returns exactly the sketch K1
// would compute, because
//   * an entry is used only if the file's resolved path, size and mtime (ns)
//     and the sketch parameters k and seed match, and its checksum verifies;
//   * a bottom-s sketch holds the min(s, #distinct) smallest distinct hashes,
//     so an entry computed with sketch size S >= s serves s as its prefix
//     of min(len, s) hashes (finch's process_post_filter truncation).
//
// Layout: <dir>/<fnv1a64(resolved path) as 16 hex>.k<k>.ggsk, one file per
// (genome file, k), written to a temporary name and renamed into place
// (readers never see a partial entry; concurrent writers of the same entry
// leave one complete copy).
//
//   offset size
//        0    8  magic "GGSKETCH"
//        8    4  version (1)
//       12    4  k
//       16    8  hash seed
//       24    4  sketch size the entry was computed with (S)
//       28    4  len = number of hashes stored (<= S)
//       32    8  genome file size (bytes)
//       40    8  genome file mtime (ns since the epoch)
//       48    4  path length P
//       52    4  reserved (0)
//       56    8  fnv1a64 over the path bytes and the hashes
//       64    P  resolved path (no terminator)
//     64+P  8*len hashes, ascending, little-endian u64
#include <errno.h>
#include <stdlib.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "gg_internal.hpp"

namespace gg {
namespace {

constexpr char kMagic[8] = {'G', 'G', 'S', 'K', 'E', 'T', 'C', 'H'};
constexpr uint32_t kVersion = 1;

struct CacheHeader {
  char magic[8];
  uint32_t version;
  uint32_t k;
  uint64_t seed;
  uint32_t sketch_size;
  uint32_t len;
  uint64_t file_size;
  int64_t mtime_ns;
  uint32_t path_len;
  uint32_t reserved;
  uint64_t checksum;
};
static_assert(sizeof(CacheHeader) == 64, "cache header layout");

uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
  const unsigned char* b = (const unsigned char*)p;
  for (size_t i = 0; i < n; ++i) {
    h ^= b[i];
    h *= 0x100000001b3ull;
  }
  return h;
}
constexpr uint64_t kFnvBasis = 0xcbf29ce484222325ull;

struct FileId {
  std::string path;  // resolved
  uint64_t size = 0;
  int64_t mtime_ns = 0;
};

bool file_id(const char* path, FileId& id) {
  struct stat st;
  if (stat(path, &st) != 0) return false;
  char* rp = realpath(path, nullptr);
  id.path = rp ? rp : path;
  free(rp);
  id.size = (uint64_t)st.st_size;
  id.mtime_ns = (int64_t)st.st_mtim.tv_sec * 1000000000ll + st.st_mtim.tv_nsec;
  return true;
}

std::string entry_path(const char* dir, const FileId& id, int k) {
  char name[64];
  snprintf(name, sizeof name, "/%016llx.k%d.ggsk",
           (unsigned long long)fnv1a(kFnvBasis, id.path.data(), id.path.size()), k);
  return std::string(dir) + name;
}

// mkdir -p
bool make_dirs(const std::string& dir) {
  if (dir.empty()) return false;
  std::string cur;
  size_t pos = 0;
  while (pos != std::string::npos) {
    pos = dir.find('/', pos + 1);
    cur = dir.substr(0, pos);
    if (cur.empty()) continue;
    if (mkdir(cur.c_str(), 0777) != 0 && errno != EEXIST) return false;
  }
  struct stat st;
  return stat(dir.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

// 1 = hit, 0 = miss (absent, stale, other parameters or corrupt)
int load_entry(const char* dir, const char* path, int k, uint32_t s, uint64_t seed,
               uint64_t* out, uint32_t* out_len) {
  FileId id;
  if (!file_id(path, id)) return 0;
  const std::string ep = entry_path(dir, id, k);
  FILE* f = fopen(ep.c_str(), "rb");
  if (!f) return 0;
  CacheHeader h;
  int hit = 0;
  if (fread(&h, sizeof h, 1, f) == 1 && memcmp(h.magic, kMagic, 8) == 0 && h.version == kVersion &&
      h.k == (uint32_t)k && h.seed == seed && h.sketch_size >= s && h.len <= h.sketch_size &&
      h.file_size == id.size && h.mtime_ns == id.mtime_ns && h.path_len == id.path.size()) {
    std::string p(h.path_len, '\0');
    std::vector<uint64_t> hs(h.len);
    if (fread(&p[0], 1, h.path_len, f) == h.path_len && p == id.path &&
        (h.len == 0 || fread(hs.data(), sizeof(uint64_t), h.len, f) == h.len)) {
      uint64_t c = fnv1a(kFnvBasis, p.data(), p.size());
      c = fnv1a(c, hs.data(), hs.size() * sizeof(uint64_t));
      if (c == h.checksum) {
        const uint32_t m = std::min<uint32_t>(h.len, s);
        if (m) memcpy(out, hs.data(), m * sizeof(uint64_t));
        *out_len = m;
        hit = 1;
      }
    }
  }
  fclose(f);
  return hit;
}

gg_status store_entry(const char* dir, const char* path, int k, uint32_t s, uint64_t seed,
                      const uint64_t* hashes, uint32_t len, const FileStamp* before) {
  FileId id;
  if (!file_id(path, id)) {
    set_thread_error(std::string("sketch cache: cannot stat ") + path);
    return GG_ERR_IO;
  }
  // the file was stamped before it was read: if it changed since, the
  // sketch may belong to the old contents and must not be filed under the
  // new size and mtime
  if (before && (!before->ok || before->size != id.size || before->mtime_ns != id.mtime_ns)) {
    set_thread_error(std::string("sketch cache: ") + path + " changed while it was sketched; not stored");
    return GG_ERR_IO;
  }
  if (!make_dirs(dir)) {
    set_thread_error(std::string("sketch cache: cannot create directory ") + dir);
    return GG_ERR_IO;
  }
  CacheHeader h;
  memset(&h, 0, sizeof h);
  memcpy(h.magic, kMagic, 8);
  h.version = kVersion;
  h.k = (uint32_t)k;
  h.seed = seed;
  h.sketch_size = s;
  h.len = len;
  h.file_size = id.size;
  h.mtime_ns = id.mtime_ns;
  h.path_len = (uint32_t)id.path.size();
  uint64_t c = fnv1a(kFnvBasis, id.path.data(), id.path.size());
  h.checksum = fnv1a(c, hashes, (size_t)len * sizeof(uint64_t));
  const std::string ep = entry_path(dir, id, k);
  char tmp_suffix[64];
  snprintf(tmp_suffix, sizeof tmp_suffix, ".tmp.%d.%zx", (int)getpid(),
           std::hash<std::thread::id>()(std::this_thread::get_id()));
  const std::string tmp = ep + tmp_suffix;
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) {
    set_thread_error("sketch cache: cannot write " + tmp);
    return GG_ERR_IO;
  }
  bool ok = fwrite(&h, sizeof h, 1, f) == 1 &&
            fwrite(id.path.data(), 1, id.path.size(), f) == id.path.size() &&
            (len == 0 || fwrite(hashes, sizeof(uint64_t), len, f) == len);
  ok = (fclose(f) == 0) && ok;
  if (!ok || rename(tmp.c_str(), ep.c_str()) != 0) {
    unlink(tmp.c_str());
    set_thread_error("sketch cache: cannot write " + ep);
    return GG_ERR_IO;
  }
  return GG_OK;
}

}  // namespace

// Look up every path (on a few threads: entries are small files); rows of
// misses are left untouched and flagged 0 in hit[].
void cache_load_many(const char* dir, const char* const* paths, uint32_t n, int k, uint32_t s,
                     uint64_t seed, uint64_t* rows, uint32_t* lens, uint8_t* hit) {
  const uint32_t T = std::max(1u, std::min<uint32_t>(8, n / 64 + 1));
  auto work = [&](uint32_t t) {
    for (uint32_t i = t; i < n; i += T)
      hit[i] = (uint8_t)load_entry(dir, paths[i], k, s, seed, rows + (size_t)i * s, lens + i);
  };
  std::vector<std::thread> th;
  for (uint32_t t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
}

gg_status cache_store(const char* dir, const char* path, int k, uint32_t s, uint64_t seed,
                      const uint64_t* hashes, uint32_t len, const FileStamp* before) {
  return store_entry(dir, path, k, s, seed, hashes, len, before);
}

bool file_stamp(const char* path, FileStamp* out) {
  struct stat st;
  out->ok = path && stat(path, &st) == 0;
  out->size = out->ok ? (uint64_t)st.st_size : 0;
  out->mtime_ns = out->ok ? (int64_t)st.st_mtim.tv_sec * 1000000000ll + st.st_mtim.tv_nsec : 0;
  return out->ok;
}

}  // namespace gg

extern "C" {

gg_status gg_sketch_cache_load(const char* cache_dir, const char* path, int kmer_length,
                               uint32_t sketch_size, uint64_t hash_seed, uint64_t* out_hashes,
                               uint32_t* out_len, int* hit) {
  if (!cache_dir || !path || !out_len || !hit || (sketch_size && !out_hashes) || kmer_length < 1 ||
      kmer_length > 32 || sketch_size == 0) {
    gg::set_thread_error("gg_sketch_cache_load: invalid argument");
    return GG_ERR_INVALID_ARG;
  }
  *out_len = 0;
  *hit = gg::load_entry(cache_dir, path, kmer_length, sketch_size, hash_seed, out_hashes, out_len);
  return GG_OK;
}

gg_status gg_sketch_cache_store(const char* cache_dir, const char* path, int kmer_length,
                                uint32_t sketch_size, uint64_t hash_seed, const uint64_t* hashes,
                                uint32_t len) {
  if (!cache_dir || !path || (len && !hashes) || len > sketch_size || kmer_length < 1 ||
      kmer_length > 32 || sketch_size == 0) {
    gg::set_thread_error("gg_sketch_cache_store: invalid argument");
    return GG_ERR_INVALID_ARG;
  }
  for (uint32_t i = 1; i < len; ++i)
    if (hashes[i - 1] >= hashes[i]) {
      gg::set_thread_error("gg_sketch_cache_store: hashes must be strictly ascending");
      return GG_ERR_INVALID_ARG;
    }
  return gg::store_entry(cache_dir, path, kmer_length, sketch_size, hash_seed, hashes, len, nullptr);
}

}  // extern "C"
