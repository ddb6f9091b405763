// Host-only test of the streamed ingest (gg::PackStream, galah_amd/csrc/pack.cpp)
// that gg_precluster_files / gg_sketch_files run on: compiled from the
// library's own host sources with g++, no GPU needed.
//   usage: test_pack_stream <fasta files...>   (exit status 0 = pass)
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../galah_amd/csrc/gg_internal.hpp"

namespace gg {
thread_local std::string g_err;
void set_thread_error(const std::string& msg) { g_err = msg; }
}  // namespace gg

#define CHECK(x)                                                  \
  do {                                                            \
    if (!(x)) {                                                   \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #x); \
      return 1;                                                   \
    }                                                             \
  } while (0)

// Genome g of a gg_packed as (words, runs relative to the genome's first word).
static void genome_of(const gg_packed* p, uint32_t g, std::vector<uint32_t>& w, std::vector<gg_run>& r) {
  w.clear();
  r.clear();
  uint64_t lo = ~0ull, hi = 0;
  for (uint64_t i = 0; i < p->n_runs; ++i)
    if (p->runs[i].genome == g) {
      lo = std::min<uint64_t>(lo, p->runs[i].base / 16);
      hi = std::max<uint64_t>(hi, (p->runs[i].base + p->runs[i].len + 15) / 16);
    }
  if (lo == ~0ull) return;
  w.assign(p->words + lo, p->words + hi);
  for (uint64_t i = 0; i < p->n_runs; ++i)
    if (p->runs[i].genome == g) r.push_back(gg_run{0, p->runs[i].len, p->runs[i].base - lo * 16});
}

// Consume every genome of paths with `consumers` threads taking chunks of
// `chunk` indices; compare with gg_pack_files.
static int consume_all(const std::vector<const char*>& paths, const gg_packed* ref, int threads, uint64_t budget,
                       int consumers, uint32_t chunk) {
  gg::PackStream st(paths.data(), (uint32_t)paths.size(), 21, threads, budget, true);
  std::mutex mu;
  uint32_t cursor = 0;
  std::atomic<int> bad{0};
  auto work = [&]() {
    std::vector<uint32_t> w;
    std::vector<gg_run> r;
    for (;;) {
      uint32_t b0, b1;
      {
        std::lock_guard<std::mutex> lk(mu);
        if (cursor >= paths.size()) return;
        b0 = cursor;
        b1 = std::min<uint32_t>((uint32_t)paths.size(), b0 + chunk);
        cursor = b1;
      }
      for (uint32_t i = b0; i < b1; ++i) {
        const std::vector<uint32_t>* words;
        const std::vector<gg_run>* runs;
        std::string err;
        if (st.get(i, &words, &runs, &err) != GG_OK) {
          bad++;
          return;
        }
        genome_of(ref, i, w, r);
        // the stream's words may extend past the last run (bases of runs < k)
        bool same = r.size() == runs->size() && words->size() >= w.size() &&
                    std::equal(w.begin(), w.end(), words->begin());
        for (size_t q = 0; same && q < r.size(); ++q)
          same = r[q].len == (*runs)[q].len && r[q].base == (*runs)[q].base;
        if (!same || !st.stamp(i).ok) bad++;
        st.release(i);
      }
    }
  };
  std::vector<std::thread> th;
  for (int c = 0; c < consumers; ++c) th.emplace_back(work);
  for (auto& t : th) t.join();
  std::string err;
  if (st.first_error(&err) != GG_OK) bad++;
  return bad.load();
}

int main(int argc, char** argv) {
  std::vector<const char*> paths(argv + 1, argv + argc);
  CHECK(paths.size() >= 8);
  gg_packed* ref = nullptr;
  CHECK(gg_pack_files(paths.data(), (uint32_t)paths.size(), 21, 1, &ref) == GG_OK);
  // one consumer, generous budget; several consumers with a 1-byte budget
  // (workers then pack only the genome at the release frontier), chunks of
  // 1 and 3, 1 and 4 packing threads
  CHECK(consume_all(paths, ref, 4, 1ull << 30, 1, 32) == 0);
  CHECK(consume_all(paths, ref, 4, 1, 3, 3) == 0);
  CHECK(consume_all(paths, ref, 1, 1, 2, 1) == 0);
  CHECK(consume_all(paths, ref, 7, 1000, 4, 2) == 0);
  gg_packed_free(ref);

  // errors: the lowest failing index is reported, whatever the consumer met
  {
    std::vector<const char*> bad = paths;
    bad.insert(bad.begin() + 5, "/nonexistent/missing_a.fna");
    bad.insert(bad.begin() + 2, "/nonexistent/missing_b.fna");
    gg::PackStream st(bad.data(), (uint32_t)bad.size(), 21, 3, 1, false);
    const std::vector<uint32_t>* w;
    const std::vector<gg_run>* r;
    std::string err;
    uint32_t i = 0;
    gg_status s = GG_OK;
    for (; i < bad.size(); ++i) {
      s = st.get(i, &w, &r, &err);
      if (s != GG_OK) break;
      st.release(i);
    }
    CHECK(i == 2 && s == GG_ERR_IO);
    st.abort();
    CHECK(st.first_error(&err) == GG_ERR_IO);
    CHECK(err.find("missing_b") != std::string::npos);
  }
  // abort wakes a consumer waiting for a genome no worker will take
  {
    gg::PackStream st(paths.data(), (uint32_t)paths.size(), 21, 1, 1, false);
    std::atomic<int> rc{-1};
    std::thread waiter([&]() {
      const std::vector<uint32_t>* w;
      const std::vector<gg_run>* r;
      std::string err;
      rc = st.get((uint32_t)paths.size() - 1, &w, &r, &err);  // never released: budget blocks the workers
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(200));
    st.abort();
    waiter.join();
    CHECK(rc.load() == GG_ERR_INTERNAL || rc.load() == GG_OK);
  }
  std::printf("ok\n");
  return 0;
}
