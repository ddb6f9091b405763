// Pure host decode time of a set of gzip files: read + libdeflate gunzip on
// T threads, nothing else (no parsing, no packing) -- the floor that
// gg_precluster_files' streamed ingest is compared with.
//   g++ -O2 -std=c++17 scripts/gunzip_probe.cpp -o scripts/gunzip_probe -ldl -lpthread
//   scripts/gunzip_probe <threads> file.gz...
#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <thread>
#include <vector>

using AllocFn = void* (*)();
using FreeFn = void (*)(void*);
using GzipFn = int (*)(void*, const void*, size_t, void*, size_t, size_t*, size_t*);

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s threads file.gz...\n", argv[0]);
    return 2;
  }
  void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    std::fprintf(stderr, "libdeflate.so.0 not found\n");
    return 1;
  }
  auto alloc = (AllocFn)dlsym(h, "libdeflate_alloc_decompressor");
  auto free_ = (FreeFn)dlsym(h, "libdeflate_free_decompressor");
  auto gzip = (GzipFn)dlsym(h, "libdeflate_gzip_decompress_ex");
  if (!alloc || !free_ || !gzip) return 1;
  const int T = std::max(1, atoi(argv[1]));
  const int n = argc - 2;
  std::atomic<int> next{0};
  std::atomic<uint64_t> out_bytes{0}, in_bytes{0};
  std::atomic<int> errors{0};
  const auto t0 = std::chrono::steady_clock::now();
  auto work = [&] {
    void* d = alloc();
    std::vector<uint8_t> raw;
    std::unique_ptr<uint8_t[]> buf;
    size_t cap = 0;
    for (int i; (i = next.fetch_add(1)) < n;) {
      FILE* f = std::fopen(argv[2 + i], "rb");
      if (!f) {
        ++errors;
        continue;
      }
      std::fseek(f, 0, SEEK_END);
      const long sz = std::ftell(f);
      std::fseek(f, 0, SEEK_SET);
      raw.resize(sz > 0 ? (size_t)sz : 0);
      const size_t got = std::fread(raw.data(), 1, raw.size(), f);
      std::fclose(f);
      if (got != raw.size() || got < 18) {
        ++errors;
        continue;
      }
      // ISIZE (uncompressed size mod 2^32) of the last member
      const size_t isz = (size_t)raw[got - 4] | ((size_t)raw[got - 3] << 8) | ((size_t)raw[got - 2] << 16) |
                         ((size_t)raw[got - 1] << 24);
      size_t in = 0, out = 0, want = std::max(isz + 64, got * 4);
      if (want > cap) {
        buf.reset(new uint8_t[want]);
        cap = want;
      }
      while (in + 18 <= got) {
        size_t ui = 0, uo = 0;
        const int r = gzip(d, raw.data() + in, got - in, buf.get() + out, cap - out, &ui, &uo);
        if (r == 3) {  // grow, keeping what is decoded
          std::unique_ptr<uint8_t[]> b2(new uint8_t[cap * 2]);
          std::copy(buf.get(), buf.get() + out, b2.get());
          buf.swap(b2);
          cap *= 2;
          continue;
        }
        if (r != 0) {
          ++errors;
          break;
        }
        in += ui;
        out += uo;
      }
      in_bytes += got;
      out_bytes += out;
    }
    free_(d);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("{\"files\": %d, \"threads\": %d, \"decode_s\": %.4f, \"in_bytes\": %llu, \"out_bytes\": %llu, "
              "\"out_GBps\": %.3f, \"errors\": %d}\n",
              n, T, s, (unsigned long long)in_bytes.load(), (unsigned long long)out_bytes.load(),
              out_bytes.load() / s / 1e9, errors.load());
  return errors.load() ? 1 : 0;
}
