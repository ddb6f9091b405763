// galah_finch.hpp -- C++ mirror of galah's finch precluster interface over
// the C ABI of libgalahgpu.so (galahgpu.h).  Header-only.
//
//   reference (AroneyS/galah @ 2024-12-18)               here
//   src/lib.rs:23-27   trait PreclusterDistanceFinder     galah::PreclusterDistanceFinder
//   src/finch.rs:4-24  struct FinchPreclusterer           galah::FinchPreclusterer
//   src/finch.rs:26-75 finch::distances(...)              galah::finch_distances(...)
//   src/sorted_pair_genome_distance_cache.rs:4-59         galah::SortedPairGenomeDistanceCache
//   src/cluster_argument_parsing.rs:1160-1182             galah::parse_percentage
//
// Errors: the reference panics ("Failed to sketch genomes with finch",
// src/finch.rs:50); here the same message is thrown as std::runtime_error.
#pragma once

#include <algorithm>
#include <charconv>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <map>
#include <optional>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "galahgpu.h"

namespace galah {

// src/sorted_pair_genome_distance_cache.rs: BTreeMap<(usize,usize), Option<f32>>
// with keys normalised to (min, max).
class SortedPairGenomeDistanceCache {
 public:
  using Key = std::pair<size_t, size_t>;

  void insert(Key ids, std::optional<float> distance) { internal_[norm(ids)] = distance; }
  // Option<&Option<f32>>: nullptr when absent
  const std::optional<float>* get(Key ids) const {
    auto it = internal_.find(norm(ids));
    return it == internal_.end() ? nullptr : &it->second;
  }
  bool contains_key(Key ids) const { return internal_.count(norm(ids)) != 0; }
  // :47-58
  SortedPairGenomeDistanceCache transform_ids(const std::vector<size_t>& input_ids) const {
    SortedPairGenomeDistanceCache out;
    for (size_t i = 0; i < input_ids.size(); ++i)
      for (size_t j = i + 1; j < input_ids.size(); ++j)
        if (const auto* v = get({input_ids[i], input_ids[j]})) out.insert({i, j}, *v);
    return out;
  }
  size_t size() const { return internal_.size(); }
  const std::map<Key, std::optional<float>>& internal() const { return internal_; }
  bool operator==(const SortedPairGenomeDistanceCache& o) const { return internal_ == o.internal_; }

 private:
  static Key norm(Key k) { return k.first < k.second ? k : Key{k.second, k.first}; }
  std::map<Key, std::optional<float>> internal_;
};

// src/lib.rs:23-27
class PreclusterDistanceFinder {
 public:
  virtual ~PreclusterDistanceFinder() = default;
  virtual SortedPairGenomeDistanceCache distances(const std::vector<std::string>& genome_fasta_paths) = 0;
  virtual const char* method_name() const = 0;
};

// CAP:1160-1182 (the --precluster-ani value)
inline float parse_percentage(float value) {
  float out = 0.f;
  if (gg_parse_percentage(value, &out) != GG_OK) throw std::invalid_argument(gg_thread_last_error());
  return out;
}

// rayon's global pool, which galah builds with --threads threads
// (CAP:408-412, default 1); finch_distances reads its size the way the Rust
// body in INTEGRATION.md calls rayon::current_num_threads().  0 = unset: the
// machine's CPUs, rayon's own default.
inline int& rayon_pool_slot() {
  static int n = 0;
  return n;
}
inline void set_num_threads(int n) { rayon_pool_slot() = n > 0 ? n : 0; }
inline int current_num_threads() {
  const int n = rayon_pool_slot();
  return n > 0 ? n : (int)std::max(1u, std::thread::hardware_concurrency());
}

// galah's info! log (env_logger, shown at the default level): the two lines
// of src/finch.rs:46,48 plus one line from the library (gg_info_line: device
// count, phase times, fallbacks).  The sink is replaceable (tests capture it);
// the default writes to stderr as env_logger would.
inline std::function<void(const std::string&)>& info_sink() {
  static std::function<void(const std::string&)> sink = [](const std::string& line) {
    std::fprintf(stderr, "[INFO] %s\n", line.c_str());
  };
  return sink;
}
inline void info(const std::string& line) {
  if (info_sink()) info_sink()(line);
}

// galah's debug! log: unset (the default level, info) logs nothing; set, it
// receives src/finch.rs:65-68's line for every compared pair.
inline std::function<void(const std::string&)>& debug_sink() {
  static std::function<void(const std::string&)> sink;
  return sink;
}

// Rust's `{}` of an f64: the shortest digits that read back the same value,
// fixed notation (1.0 -> "1", 1e-7 -> "0.0000001")
inline std::string rust_f64(double x) {
  char buf[400];
  const auto r = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::fixed);
  return std::string(buf, r.ptr);
}

namespace detail {
// sketch + all pairs + threshold on an existing context; takes ownership of ctx
inline SortedPairGenomeDistanceCache distances_on(gg_ctx* ctx, const std::vector<std::string>& paths, float min_ani,
                                                  int kmer_length) {
  if (!ctx)
    throw std::runtime_error(std::string("Failed to sketch genomes with finch: ") + gg_thread_last_error());
  gg_set_host_threads(ctx, current_num_threads());
  std::vector<const char*> c_paths;
  for (const auto& p : paths) c_paths.push_back(p.c_str());
  gg_pair* pairs = nullptr;
  float* ani = nullptr;
  uint64_t n = 0;
  info("Sketching MinHash representations of each genome with finch ..");  // src/finch.rs:46
  // at debug level every compared pair is logged (src/finch.rs:65-68): the
  // library streams all N (N - 1) / 2 of them in row blocks, in the
  // reference's loop order, while the returned pairs are those >= min_ani
  struct Each {
    const std::vector<std::string>* paths;
    int k;
    static int sink(void* user, const gg_pair* p, uint64_t n) {
      const Each* e = (const Each*)user;
      for (uint64_t x = 0; x < n; ++x)
        debug_sink()("Comparing " + (*e->paths)[p[x].i] + " and " + (*e->paths)[p[x].j] + ", distance " +
                     rust_f64(gg_ani_f64(p[x].common, p[x].total, e->k)));
      return 0;
    }
  } each{&paths, kmer_length};
  const gg_status st = debug_sink()
                           ? gg_precluster_files_each(ctx, c_paths.data(), (uint32_t)c_paths.size(), min_ani, nullptr,
                                                      &Each::sink, &each, &pairs, &ani, &n, nullptr)
                           : gg_precluster_files(ctx, c_paths.data(), (uint32_t)c_paths.size(), min_ani, &pairs, &ani,
                                                 &n);
  if (st != GG_OK) {
    std::string msg = gg_last_error(ctx);
    gg_destroy(ctx);
    throw std::runtime_error("Failed to sketch genomes with finch: " + msg);  // src/finch.rs:50
  }
  info("Finished sketching genomes");  // src/finch.rs:48 (sketches and pairs come from one call here)
  char line[1024];
  if (gg_info_line(ctx, line, sizeof line) == GG_OK) info(line);
  SortedPairGenomeDistanceCache cache;
  for (uint64_t i = 0; i < n; ++i) cache.insert({pairs[i].i, pairs[i].j}, ani[i]);  // src/finch.rs:70
  gg_free(pairs);
  gg_free(ani);
  gg_destroy(ctx);
  return cache;
}
}  // namespace detail

// src/finch.rs:26-75 on the GPU, same arguments: sketch (K1), all pairs (K2),
// keep ani >= min_ani.  Every visible GPU (or GALAHGPU_DEVICES), as galah's
// one distances() call would use them; file ingest on current_num_threads().
inline SortedPairGenomeDistanceCache finch_distances(const std::vector<std::string>& paths, float min_ani,
                                                     size_t num_kmers, uint8_t kmer_length) {
  gg_status st = GG_OK;
  return detail::distances_on(gg_create_multi(kmer_length, (uint32_t)num_kmers, 0, nullptr, 0, &st), paths, min_ani,
                              kmer_length);
}

// The same on one HIP device (ordinal; -1 = the current device).
inline SortedPairGenomeDistanceCache finch_distances(const std::vector<std::string>& paths, float min_ani,
                                                     size_t num_kmers, uint8_t kmer_length, int device) {
  gg_status st = GG_OK;
  return detail::distances_on(gg_create(kmer_length, (uint32_t)num_kmers, 0, device, &st), paths, min_ani, kmer_length);
}

// The same on a list of HIP ordinals (repeats allowed: several members on one GPU).
inline SortedPairGenomeDistanceCache finch_distances_on(const std::vector<int>& devices,
                                                        const std::vector<std::string>& paths, float min_ani,
                                                        size_t num_kmers, uint8_t kmer_length) {
  gg_status st = GG_OK;
  return detail::distances_on(
      gg_create_multi(kmer_length, (uint32_t)num_kmers, 0, devices.data(), (uint32_t)devices.size(), &st), paths,
      min_ani, kmer_length);
}

// src/finch.rs:4-24
class FinchPreclusterer : public PreclusterDistanceFinder {
 public:
  FinchPreclusterer(float min_ani, size_t num_kmers = 1000, uint8_t kmer_length = 21)
      : min_ani(min_ani), num_kmers(num_kmers), kmer_length(kmer_length) {}
  SortedPairGenomeDistanceCache distances(const std::vector<std::string>& paths) override {
    return finch_distances(paths, min_ani, num_kmers, kmer_length);
  }
  const char* method_name() const override { return "finch"; }

  float min_ani;  // fraction, not percentage
  size_t num_kmers;
  uint8_t kmer_length;
};

}  // namespace galah
