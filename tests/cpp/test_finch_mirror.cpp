// C++ mirror of the reference's own finch tests, through galah_finch.hpp
// and libgalahgpu.so.  Built by tests/cpp/Makefile, run by
// tests/test_cpp_mirror.py.
//   src/finch.rs:85-107                              test_hello_world
//   src/sorted_pair_genome_distance_cache.rs:69-114  transform tests
// argv[1] = directory holding set1/1mbp.fna.gz and set1/500kb.fna.gz
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "galah_finch.hpp"

static int failures = 0;
#define CHECK(cond)                                                 \
  do {                                                              \
    if (!(cond)) {                                                  \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                   \
    }                                                               \
  } while (0)

static void test_transform_hello_world() {
  galah::SortedPairGenomeDistanceCache cache;
  cache.insert({1, 2}, 0.99f);
  CHECK(cache.transform_ids({0, 3}).size() == 0);
  auto t = cache.transform_ids({1, 2});
  CHECK(t.size() == 1 && t.get({0, 1}) && **t.get({0, 1}) == 0.99f);
  CHECK(cache.transform_ids({1, 3}).size() == 0);
}

static void test_transform_multiple() {
  galah::SortedPairGenomeDistanceCache cache;
  cache.insert({1, 2}, 0.99f);
  cache.insert({4, 1}, 0.98f);
  CHECK(cache.contains_key({1, 4}));
  auto t = cache.transform_ids({1, 2, 4});
  CHECK(t.size() == 2 && **t.get({0, 1}) == 0.99f && **t.get({0, 2}) == 0.98f);
  CHECK(**cache.transform_ids({1, 4}).get({0, 1}) == 0.98f);
}

static void test_parse_percentage() {
  CHECK(galah::parse_percentage(90.0f) == 90.0f / 100.0f);
  CHECK(galah::parse_percentage(0.9f) == 0.9f);
  bool threw = false;
  try {
    galah::parse_percentage(101.0f);
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);
}

static void test_hello_world(const std::string& dir) {
  const std::vector<std::string> paths = {dir + "/set1/1mbp.fna.gz", dir + "/set1/500kb.fna.gz"};
  // galah builds rayon's global pool from --threads before clustering
  // (CAP:408-412); distances() reads its size
  galah::set_num_threads(2);
  CHECK(galah::current_num_threads() == 2);
  galah::FinchPreclusterer p(0.9f, 1000, 21);
  CHECK(std::strcmp(p.method_name(), "finch") == 0);
  std::vector<std::string> log;
  galah::info_sink() = [&](const std::string& line) { log.push_back(line); };
  auto d1 = p.distances(paths);
  // src/finch.rs:46,48 and the library's one line (device count, phases, fallbacks)
  CHECK(log.size() == 3);
  CHECK(log.size() == 3 && log[0] == "Sketching MinHash representations of each genome with finch ..");
  CHECK(log.size() == 3 && log[1] == "Finished sketching genomes");
  CHECK(log.size() == 3 && log[2].rfind("galahgpu: ", 0) == 0 && log[2].find("device(s)") != std::string::npos &&
        log[2].find("fallbacks: index->gate 0, index full sort 0, host-staged peer copies 0") != std::string::npos);
  galah::info_sink() = nullptr;
  galah::SortedPairGenomeDistanceCache e1;
  e1.insert({0, 1}, 0.9808188f);
  CHECK(d1 == e1);
  // debug level (src/finch.rs:65-68): the compared pair logged with its f64
  // distance, the same cache
  std::vector<std::string> dbg;
  galah::debug_sink() = [&](const std::string& line) { dbg.push_back(line); };
  auto d3 = p.distances(paths);
  galah::debug_sink() = nullptr;
  CHECK(d3 == e1);
  CHECK(dbg.size() == 1 && dbg[0] == "Comparing " + paths[0] + " and " + paths[1] + ", distance " +
                                         galah::rust_f64(gg_ani_f64(502, 1000, 21)));
  CHECK(galah::rust_f64(1.0) == "1" && galah::rust_f64(0.0) == "0" && galah::rust_f64(1e-7) == "0.0000001" &&
        galah::rust_f64(0.5) == "0.5");
  auto d2 = galah::finch_distances(paths, 0.99f, 1000, 21);
  CHECK(d2.size() == 0);
  // one device by ordinal, and two members of device 0
  CHECK(galah::finch_distances(paths, 0.9f, 1000, 21, 0) == e1);
  CHECK(galah::finch_distances_on({0, 0}, paths, 0.9f, 1000, 21) == e1);
  galah::set_num_threads(0);
  bool threw = false;
  try {
    galah::finch_distances({dir + "/does_not_exist.fna"}, 0.9f, 1000, 21);
  } catch (const std::runtime_error& e) {
    threw = std::string(e.what()).rfind("Failed to sketch genomes with finch", 0) == 0;
  }
  CHECK(threw);
}

int main(int argc, char** argv) {
  test_transform_hello_world();
  test_transform_multiple();
  test_parse_percentage();
  if (argc > 1) test_hello_world(argv[1]);
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("ok\n");
  return 0;
}
