// Host runtime: what galah does with the pair set right after distances()
// (SURVEY.md 8(f) rows 1 and 3).
//
//   src/clusterer.rs:409-431  partition_sketches: a DisjointSetVec over the
//     genome indices, joined for every (i, j) the cache contains -- an
//     O(N^2) contains_key scan, 5e9 BTreeMap lookups at 100k genomes.
//   src/clusterer.rs:45-57    the sets, each sorted ascending, ordered by
//     size descending (sort_unstable_by_key(Reverse(len))).
//   src/clusterer.rs:70 + src/sorted_pair_genome_distance_cache.rs:47-58
//     transform_ids: the sub-cache of one precluster, ids renumbered by
//     position in the precluster -- O(m^2) get() per precluster.
//
// Here both are linear in the sparse pair list: union-find with union by
// size and path halving over the passing pairs (single linkage does not
// depend on the order joins happen in, so the sets equal the reference's),
// then one counting sort of the genomes into their sets and one of the
// pairs into their precluster.
//
// Order among preclusters of equal size: ascending by smallest member.  The
// reference leaves it to DisjointSetVec::sets() and an unstable sort; every
// consumer in galah (src/clusterer.rs:66-123) treats preclusters
// independently, and its final cluster list is assembled in rayon completion
// order, so no output of galah depends on it.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <vector>

#include "gg_internal.hpp"

namespace gg {
namespace {

struct UnionFind {
  std::vector<uint32_t> parent, size;
  explicit UnionFind(uint32_t n) : parent(n), size(n, 1) { std::iota(parent.begin(), parent.end(), 0u); }
  uint32_t find(uint32_t x) {
    while (parent[x] != x) {
      parent[x] = parent[parent[x]];  // path halving
      x = parent[x];
    }
    return x;
  }
  void join(uint32_t a, uint32_t b) {
    a = find(a);
    b = find(b);
    if (a == b) return;
    if (size[a] < size[b]) std::swap(a, b);
    parent[b] = a;
    size[a] += size[b];
  }
};

}  // namespace
}  // namespace gg

using namespace gg;

extern "C" gg_status gg_partition_preclusters(uint32_t n_genomes, const gg_pair* pairs, uint64_t n_pairs,
                                              uint32_t* members, uint32_t* offsets, uint32_t* n_sets) {
  if ((n_pairs && !pairs) || !offsets || (n_genomes && !members) || !n_sets) {
    set_thread_error("gg_partition_preclusters: null argument");
    return GG_ERR_INVALID_ARG;
  }
  for (uint64_t p = 0; p < n_pairs; ++p) {
    if (pairs[p].i >= n_genomes || pairs[p].j >= n_genomes) {
      set_thread_error("gg_partition_preclusters: pair index out of range");
      return GG_ERR_INVALID_ARG;
    }
  }
  *n_sets = 0;
  offsets[0] = 0;
  if (n_genomes == 0) return GG_OK;
  UnionFind uf(n_genomes);
  for (uint64_t p = 0; p < n_pairs; ++p) uf.join(pairs[p].i, pairs[p].j);

  // sets numbered in order of their smallest member (genomes visited ascending)
  std::vector<uint32_t> set_of_root(n_genomes, UINT32_MAX);
  std::vector<uint32_t> set_size;
  std::vector<uint32_t> label(n_genomes);
  for (uint32_t g = 0; g < n_genomes; ++g) {
    const uint32_t r = uf.find(g);
    if (set_of_root[r] == UINT32_MAX) {
      set_of_root[r] = (uint32_t)set_size.size();
      set_size.push_back(0);
    }
    label[g] = set_of_root[r];
    ++set_size[label[g]];
  }
  const uint32_t ns = (uint32_t)set_size.size();
  // size descending; the stable sort keeps smallest-member order among ties
  std::vector<uint32_t> order(ns);
  std::iota(order.begin(), order.end(), 0u);
  std::stable_sort(order.begin(), order.end(),
                   [&](uint32_t a, uint32_t b) { return set_size[a] > set_size[b]; });
  std::vector<uint32_t> rank(ns);
  for (uint32_t r = 0; r < ns; ++r) rank[order[r]] = r;
  for (uint32_t r = 0; r < ns; ++r) offsets[r + 1] = offsets[r] + set_size[order[r]];
  std::vector<uint32_t> fill(offsets, offsets + ns);
  for (uint32_t g = 0; g < n_genomes; ++g) members[fill[rank[label[g]]]++] = g;  // ascending in a set
  *n_sets = ns;
  return GG_OK;
}

extern "C" gg_status gg_precluster_pairs(uint32_t n_genomes, const gg_pair* pairs, uint64_t n_pairs,
                                         const uint32_t* members, const uint32_t* offsets, uint32_t n_sets,
                                         gg_local_pair* out, uint64_t* pair_offsets) {
  if ((n_pairs && (!pairs || !out)) || (n_sets && (!members || !offsets)) || !pair_offsets) {
    set_thread_error("gg_precluster_pairs: null argument");
    return GG_ERR_INVALID_ARG;
  }
  // genome -> (precluster, position inside it)
  std::vector<uint32_t> set_of(n_genomes, UINT32_MAX), pos(n_genomes, 0);
  for (uint32_t s = 0; s < n_sets; ++s) {
    if (offsets[s + 1] < offsets[s] || offsets[s + 1] > n_genomes) {
      set_thread_error("gg_precluster_pairs: bad offsets");
      return GG_ERR_INVALID_ARG;
    }
    for (uint32_t m = offsets[s]; m < offsets[s + 1]; ++m) {
      const uint32_t g = members[m];
      if (g >= n_genomes || set_of[g] != UINT32_MAX) {
        set_thread_error("gg_precluster_pairs: members are not a partition of the genomes");
        return GG_ERR_INVALID_ARG;
      }
      set_of[g] = s;
      pos[g] = m - offsets[s];
    }
  }
  std::vector<uint64_t> cnt((size_t)n_sets + 1, 0);
  for (uint64_t p = 0; p < n_pairs; ++p) {
    const uint32_t i = pairs[p].i, j = pairs[p].j;
    if (i >= n_genomes || j >= n_genomes || set_of[i] == UINT32_MAX || set_of[i] != set_of[j]) {
      set_thread_error("gg_precluster_pairs: pair is not inside one precluster");
      return GG_ERR_INVALID_ARG;
    }
    ++cnt[set_of[i] + 1];
  }
  for (uint32_t s = 0; s < n_sets; ++s) cnt[s + 1] += cnt[s];
  std::memcpy(pair_offsets, cnt.data(), ((size_t)n_sets + 1) * sizeof(uint64_t));
  for (uint64_t p = 0; p < n_pairs; ++p) {
    const uint32_t i = pairs[p].i, j = pairs[p].j, s = set_of[i];
    const uint32_t a = pos[i], b = pos[j];
    // transform_ids inserts (i, j) keyed (min, max) by position
    out[cnt[s]++] = gg_local_pair{s, std::min(a, b), std::max(a, b), (uint32_t)p};
  }
  for (uint32_t s = 0; s < n_sets; ++s) {
    std::sort(out + pair_offsets[s], out + pair_offsets[s + 1],
              [](const gg_local_pair& x, const gg_local_pair& y) { return x.i != y.i ? x.i < y.i : x.j < y.j; });
  }
  return GG_OK;
}
