// Host runtime of libgalahgpu.so: context, device memory, the retry loop of
// the bottom-s selection, the cmin threshold table, tile partitioning and
// the C ABI declared in include/galahgpu.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "context.hpp"


namespace gg {

thread_local std::string g_thread_err;

void set_thread_error(const std::string& msg) { g_thread_err = msg; }

gg_status fail(gg_ctx* c, gg_status st, const std::string& msg) {
  if (c) c->err = msg;
  set_thread_error(msg);
  return st;
}

gg_status hip_fail(gg_ctx* c, hipError_t e, const char* what) {
  return fail(c, e == hipErrorOutOfMemory ? GG_ERR_OUT_OF_MEMORY : GG_ERR_HIP,
              std::string(what) + ": " + hipGetErrorString(e));
}

hipError_t scratch(gg_ctx* c, const char* key, size_t bytes, void** out) {
  auto& e = c->scratch[key];
  if (e.second < bytes) {
    // a buffer that grows again grows by a quarter at least: batches of
    // slightly different sizes (the device-inflate batches are cut at a file
    // boundary) would otherwise reallocate it call after call, and hipFree
    // waits for every stream of the device
    const size_t grown = e.second ? e.second + e.second / 4 : 0;
    const auto t0 = std::chrono::steady_clock::now();
    struct Tally {  // (the regrowth's wall time, gg_info_line: a hipFree waits for the device)
      gg_ctx* c;
      std::chrono::steady_clock::time_point t0;
      ~Tally() {
        ++c->scratch_regrows;
        c->scratch_regrow_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      }
    } tally{c, t0};
    if (e.first) {
      hipError_t err = hipFree(e.first);
      if (err != hipSuccess) return err;
      e.first = nullptr;
      e.second = 0;
    }
    size_t want = std::max<size_t>(std::max(std::max(bytes, grown), (size_t)((double)bytes * c->scratch_hint)), 256);
    hipError_t err = hipMalloc(&e.first, want);
    if (err == hipErrorOutOfMemory && want > bytes) {  // (no room for the headroom: just what is asked)
      (void)hipGetLastError();
      want = std::max<size_t>(bytes, 256);
      err = hipMalloc(&e.first, want);
    }
    if (err != hipSuccess) {
      e.first = nullptr;
      return err;
    }
    e.second = want;
  }
  *out = e.first;
  return hipSuccess;
}

hipError_t host_scratch(gg_ctx* c, const char* key, size_t bytes, void** out) {
  auto& e = c->host_scratch[key];
  if (e.second < bytes) {
    struct Tally {
      gg_ctx* c;
      std::chrono::steady_clock::time_point t0;
      ~Tally() {
        ++c->scratch_regrows;
        c->scratch_regrow_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      }
    } tally{c, std::chrono::steady_clock::now()};
    if (e.first) {
      hipError_t err = hipHostFree(e.first);
      if (err != hipSuccess) return err;
      e.first = nullptr;
      e.second = 0;
    }
    // (sized by scratch_hint like scratch(): a later, larger batch of the
    // call does not regrow it)
    size_t want = std::max<size_t>(std::max(bytes, (size_t)((double)bytes * c->scratch_hint)), 4096);
    hipError_t err = hipHostMalloc(&e.first, want, hipHostMallocDefault);
    if (err != hipSuccess) return err;
    e.second = want;
  }
  *out = e.first;
  return hipSuccess;
}

hipError_t pinned(gg_ctx* c, size_t bytes, void** out) {
  if (c->pinned_bytes < bytes) {
    if (c->pinned) {
      hipError_t err = hipHostFree(c->pinned);
      if (err != hipSuccess) return err;
      c->pinned = nullptr;
      c->pinned_bytes = 0;
    }
    const size_t want = std::max<size_t>(bytes, 1 << 20);
    hipError_t err = hipHostMalloc(&c->pinned, want, hipHostMallocDefault);
    if (err != hipSuccess) return err;
    c->pinned_bytes = want;
  }
  *out = c->pinned;
  return hipSuccess;
}

hipEvent_t take_event(gg_ctx* c) {
  if (!c->spare_events.empty()) {
    hipEvent_t e = c->spare_events.back();
    c->spare_events.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

namespace {

// Number of pairs (i < j < n) in tiles [tb, te).
// (O(tile rows): tile row I holds tiles (I, J), J = I .. nb - 1, numbered
// from t0(I); the tiles of [tb, te) in it are J in [Ja, Jb))
uint64_t pairs_in_tiles(uint32_t n, uint64_t tb, uint64_t te) {
  const uint64_t nb = (n + GG_PAIR_TILE - 1) / GG_PAIR_TILE;
  uint64_t t0 = 0, acc = 0;
  for (uint64_t I = 0; I < nb && t0 < te; ++I) {
    const uint64_t row_tiles = nb - I, t1 = t0 + row_tiles;
    const uint64_t a = std::max(t0, tb), b = std::min(t1, te);
    if (a < b) {
      const uint64_t Ja = I + (a - t0), Jb = I + (b - t0);
      const uint64_t ri = std::min<uint64_t>(GG_PAIR_TILE, n - I * GG_PAIR_TILE);
      if (Ja == I) acc += ri * (ri - 1) / 2;  // the diagonal tile
      const uint64_t c0 = std::max(Ja, I + 1) * GG_PAIR_TILE, c1 = std::min<uint64_t>(Jb * GG_PAIR_TILE, n);
      if (c1 > c0) acc += ri * (c1 - c0);
    }
    t0 = t1;
  }
  return acc;
}

inline double rust_min(double a, double b) {
  if (std::isnan(a)) return b;
  if (std::isnan(b)) return a;
  return a < b ? a : b;
}
inline double rust_max(double a, double b) {
  if (std::isnan(a)) return b;
  if (std::isnan(b)) return a;
  return a > b ? a : b;
}

// Bottom-s selection geometry (see sketch.hip header).
struct SketchGeom {
  uint32_t limit;      // max distinct candidates per genome
  uint32_t sort_pow2;  // LDS sort size (>= limit)
  uint32_t cap_log2;   // per-genome set capacity = 2 * sort_pow2
  double over;         // expected candidates = over * s
};

SketchGeom sketch_geom(uint32_t s) {
  SketchGeom g;
  // ~1.6 s candidates expected at s = 1000 (sd ~ 40): the set never reaches
  // the limit and the LDS sort never exceeds 2048 entries
  g.limit = std::min<uint32_t>(kSortCap, std::max<uint32_t>(2 * s, 64));
  g.sort_pow2 = 1;
  while (g.sort_pow2 < g.limit) g.sort_pow2 <<= 1;
  g.cap_log2 = 1;
  while ((1u << g.cap_log2) < 2 * g.sort_pow2) ++g.cap_log2;
  g.over = std::min(2.0, 0.8 * (double)g.limit / (double)s);
  // GALAHGPU_TAU_OVER overrides the oversampling for A/B runs (any value
  // gives the same sketches: too few candidates or an overflow only moves tau)
  static const double over_env = [] {
    const char* e = getenv("GALAHGPU_TAU_OVER");
    return e && *e ? atof(e) : 0.0;
  }();
  if (over_env > 0.0) g.over = std::min(over_env, 0.95 * (double)g.limit / (double)s);
  return g;
}

// (the same expression as the one-batch path's first_pass_kernel)
uint64_t initial_tau(uint64_t nk, uint32_t s, double over) { return first_tau(nk, over * (double)s); }

struct TauSearch {
  uint64_t tau;
  uint64_t lo = 0;  // largest tau known to give fewer than s distinct
  uint64_t hi = 0;  // smallest tau known to overflow
  bool lo_known = false;
  bool hi_known = false;
  int steps = 0;
};

// Moves tau after a failed pass.  Exactness does not depend on where tau
// ends up, only on every distinct hash <= tau being collected.  Returns
// false when the search cannot continue (cannot happen for limit > s + 1:
// the distinct count below tau grows by one value at a time).
bool advance_tau(TauSearch& t, uint32_t status) {
  if (++t.steps > 130) return false;
  if (status == kSketchRetryLarger) {
    t.lo = t.tau;
    t.lo_known = true;
    if (t.hi_known) t.tau = t.lo + (t.hi - t.lo) / 2;
    else t.tau = (t.tau > kEmpty / 4) ? kEmpty : t.tau * 4 + 3;
  } else {
    t.hi = t.tau;
    t.hi_known = true;
    t.tau = t.lo + (t.hi - t.lo) / 2;
  }
  if (t.lo_known && t.hi_known && t.hi - t.lo <= 1) return false;
  return true;
}

// f(t, begin, end) over T contiguous chunks of [0, n) on T threads.
template <class F>
void parallel_chunks(uint64_t n, int T, F&& f) {
  if (T <= 1 || n < 2) {
    f(0, (uint64_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back([&, t] { f(t, n * t / T, n * (t + 1) / T); });
  f(0, (uint64_t)0, n / T);
  for (auto& x : th) x.join();
}

}  // namespace

// The status and message for the first bad run of a table (check_runs, and
// the device check in sketch_core).
// Device whose memory p points into, or -1 for host memory (a pointer HIP
// does not know is host memory).
int device_of(const void* p) {
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // (clears the sticky error of an unknown host pointer)
    return -1;
  }
  return at.type == hipMemoryTypeDevice ? at.device : -1;
}

gg_status run_error(gg_ctx* c, const gg_run* runs, uint64_t first_bad, uint32_t n_genomes) {
  const gg_run& x = runs[first_bad];
  const uint32_t prev = first_bad ? runs[first_bad - 1].genome : 0u;
  if (x.genome >= n_genomes || x.genome < prev)
    return fail(c, GG_ERR_INVALID_ARG, "runs must be grouped by non-decreasing genome < n_genomes");
  if (x.len < (uint32_t)c->k) return fail(c, GG_ERR_INVALID_ARG, "run shorter than k");
  return fail(c, GG_ERR_INVALID_ARG, "run extends past the packed words");
}

gg_status check_runs(gg_ctx* c, const gg_run* runs, uint64_t n_runs, uint32_t n_genomes, uint64_t n_words) {
  if (n_runs && !runs) return fail(c, GG_ERR_INVALID_ARG, "null run table");
  const int T = n_runs >= (1u << 18) ? std::max(1, std::min(16, ingest_threads(c->host_threads))) : 1;
  const uint32_t k = (uint32_t)c->k;
  std::vector<uint64_t> bad(T, ~0ull);
  parallel_chunks(n_runs, T, [&](int t, uint64_t b, uint64_t e) {
    for (uint64_t r = b; r < e; ++r) {
      const gg_run& x = runs[r];
      const uint32_t prev = r ? runs[r - 1].genome : 0u;
      if (x.genome >= n_genomes || x.genome < prev || x.len < k || x.base + x.len > n_words * 16ull ||
          x.base + x.len < x.base) {
        bad[t] = r;
        return;
      }
    }
  });
  const uint64_t first_bad = *std::min_element(bad.begin(), bad.end());
  if (first_bad == ~0ull) return GG_OK;
  return run_error(c, runs, first_bad, n_genomes);
}

// GALAHGPU_HOST_PROFILE=1: per-stage host wall times of sketch_core on stderr
struct HostProf {
  bool on;
  std::chrono::steady_clock::time_point t;
  HostProf() : on(getenv("GALAHGPU_HOST_PROFILE") != nullptr), t(std::chrono::steady_clock::now()) {}
  void mark(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    fprintf(stderr, "[sketch_core] %-24s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};

gg_status sketch_core(gg_ctx* c, const uint32_t* d_words, uint64_t n_words, const gg_run* runs,
                      uint64_t n_runs, uint32_t n_genomes, uint64_t* d_out, uint32_t* d_lens,
                      const uint32_t* d_row_of, hipStream_t st) {
  HostProf hp;
  if (n_genomes == 0) {
    if (n_runs) return fail(c, GG_ERR_INVALID_ARG, "runs must be grouped by non-decreasing genome < n_genomes");
    return GG_OK;
  }
  const uint32_t seg = (uint32_t)sketch_segment_len(c->k);
  if (n_runs && !runs) return fail(c, GG_ERR_INVALID_ARG, "null run table");
  const SketchGeom geom = sketch_geom(c->s);
  const uint64_t cap = 1ull << geom.cap_log2;
  // genomes per batch: tables limited to ~4 GiB (GALAHGPU_K1_MAX_BATCH,
  // tests only: smaller batches, so the multi-batch path runs on small inputs)
  uint64_t batch_cap = (4ull << 30) / (cap * sizeof(uint64_t));
  if (const char* e = getenv("GALAHGPU_K1_MAX_BATCH"))
    if (*e && atoi(e) > 0) batch_cap = std::min<uint64_t>(batch_cap, (uint64_t)atoi(e));
  const uint32_t max_batch = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n_genomes, batch_cap));

  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, c->device);
  // K1 grid: many small workgroups per CU (112; each thread then owns ~60
  // segments at C3) so the dispatcher balances the tail.  At 8 per CU the
  // grid was 8 waves per SIMD against an occupancy of 7 (68 VGPRs) and the
  // last eighth of the work ran as a second, thin round (C3 K1: 56.7 ms at
  // 8, 54.4 at 14, 52.5 at 56, 52.2 at 112, 52.5 at 448).
  // A smaller launch (an ingest batch of ~200 genomes) takes fewer: each
  // workgroup first fills its LDS tables, and at 112 per CU a thread of a
  // 200 x 3 Mbp batch owned ~2 segments (1,000 C2-like files: K1 6.73 ms at
  // 112 per CU, 5.78 at 28, 5.74 at 14, 5.93 at 7; profiles/r06/k1_grid_ab.txt):
  // ~15 segments per thread, in multiples of 7 per CU (the occupancy),
  // between 14 and 112.  GALAHGPU_K1_WG_PER_CU overrides it for A/B runs.
  static const int wg_env = [] {
    const char* e = getenv("GALAHGPU_K1_WG_PER_CU");
    return e && *e ? std::max(1, atoi(e)) : 0;
  }();
  int wg_per_cu = wg_env;
  if (!wg_per_cu) {
    const double segs = (double)n_words * 16.0 / (double)seg;  // (an upper bound: runs shorter than k hold none)
    const double per = segs / (15.0 * 256.0 * std::max(1, n_cu));
    wg_per_cu = std::min(112, std::max(14, 7 * (int)std::ceil(per / 7.0)));
  }
  const int grid = std::max(1, n_cu) * wg_per_cu;

  uint64_t* d_table;
  uint32_t *d_flags, *d_count, *d_status, *d_slot_list, *d_slot_genome;
  uint64_t* d_tau;
  GG_HIP(c, scratch_t(c, "table", (size_t)max_batch * cap, &d_table));
  GG_HIP(c, scratch_t(c, "flags", max_batch, &d_flags));
  GG_HIP(c, scratch_t(c, "cand_count", max_batch, &d_count));
  GG_HIP(c, scratch_t(c, "slot_list", max_batch, &d_slot_list));
  GG_HIP(c, scratch_t(c, "slot_genome", max_batch, &d_slot_genome));
  // what the host reads back, contiguous on the device and in pinned host
  // memory (one DMA per pass): the run index (bad run, per genome first run,
  // first segment and k-mers), then tau and status per batch slot
  const size_t ng1 = (size_t)n_genomes + 1;
  const size_t rb_ix = 1 + 3 * ng1, rb_u64 = rb_ix + max_batch + (max_batch + 1) / 2;
  uint64_t *d_rb, *h_rb;
  GG_HIP(c, scratch_t(c, "readback", rb_u64, &d_rb));
  GG_HIP(c, host_scratch_t(c, "readback", rb_u64, &h_rb));
  d_tau = d_rb + rb_ix;
  d_status = reinterpret_cast<uint32_t*>(d_rb + rb_ix + max_batch);
  const uint32_t* h_status = reinterpret_cast<const uint32_t*>(h_rb + rb_ix + max_batch);

  // every slot starts a call in append mode with an empty list (count 0,
  // flags 0); the finalize leaves its slots so, so only new buffers are
  // cleared (the table itself needs no clearing: a list is [0, count), and a
  // slot's set is cleared by the finalize that switches it to set mode)
  const uint32_t nb0 = std::min(n_genomes, max_batch);
  const size_t batch_bytes = (size_t)nb0 * cap * sizeof(uint64_t);
  if (c->clean_table != d_table || c->clean_table_bytes < batch_bytes) {
    GG_HIP(c, hipMemsetAsync(d_flags, 0, nb0 * sizeof(uint32_t), st));
    GG_HIP(c, hipMemsetAsync(d_count, 0, nb0 * sizeof(uint32_t), st));
  }
  // (dirty until every batch's finalize has run; an error return leaves it so)
  c->clean_table = nullptr;
  c->clean_table_bytes = 0;
  if (!c->copy_stream) {
    GG_HIP(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    GG_HIP(c, hipEventCreateWithFlags(&c->copy_done, hipEventDisableTiming));
  }
  // the run table goes to the device once and is checked and indexed there
  // (runindex.hip); the host keeps per genome its first run, k-mer count and
  // first segment
  gg_run* d_all_runs;
  uint64_t *d_rs, *d_sc;
  uint64_t* d_ix = d_rb;  // bad, gr, grs, nk
  void* d_ix_tmp;
  GG_HIP(c, scratch_t(c, "runs_all", std::max<uint64_t>(n_runs, 1), &d_all_runs));
  GG_HIP(c, scratch_t(c, "run_sstart", n_runs + 1, &d_rs));
  GG_HIP(c, scratch_t(c, "run_segs", n_runs + 1, &d_sc));
  const size_t ix_tmp = run_index_tmp_bytes(n_runs);
  GG_HIP(c, scratch(c, "run_index_tmp", std::max<size_t>(ix_tmp, 16), &d_ix_tmp));
  // A run table already in this device's memory is indexed where it lies
  // (another device's is copied peer to peer); the host mirror of a device
  // table is made only if a retry pass or an error message needs it.
  const int runs_dev = n_runs ? device_of(runs) : -1;
  std::vector<gg_run> runs_mirror;
  auto host_runs = [&]() -> const gg_run* {
    if (runs_dev < 0) return runs;
    if (runs_mirror.empty()) {
      runs_mirror.resize(n_runs);
      if (hipMemcpy(runs_mirror.data(), runs, n_runs * sizeof(gg_run), hipMemcpyDefault) != hipSuccess)
        return nullptr;
    }
    return runs_mirror.data();
  };
  if (runs_dev == c->device) {
    d_all_runs = const_cast<gg_run*>(runs);
  } else {
    if (n_runs && runs_dev < 0) {  // (a host table through pinned scratch: a pageable copy blocks this thread)
      gg_run* h_runs;
      GG_HIP(c, host_scratch_t(c, "runs_h2d", n_runs, &h_runs));
      memcpy(h_runs, runs, n_runs * sizeof(gg_run));
      GG_HIP(c, hipMemcpyAsync(d_all_runs, h_runs, n_runs * sizeof(gg_run), hipMemcpyHostToDevice, c->copy_stream));
    } else if (n_runs) {
      GG_HIP(c, hipMemcpyAsync(d_all_runs, runs, n_runs * sizeof(gg_run), hipMemcpyDefault, c->copy_stream));
    }
    GG_HIP(c, hipEventRecord(c->copy_done, c->copy_stream));
    GG_HIP(c, hipStreamWaitEvent(st, c->copy_done, 0));
  }
  RunIndexDev xd;
  xd.runs = d_all_runs;
  xd.n_runs = n_runs;
  xd.n_genomes = n_genomes;
  xd.n_words = n_words;
  xd.k = c->k;
  xd.seg = seg;
  xd.bad = d_ix;
  xd.sc = d_sc;
  xd.rs = d_rs;
  xd.gr = d_ix + 1;
  xd.grs = d_ix + 1 + ng1;
  xd.nk = d_ix + 1 + 2 * ng1;
  xd.tmp = d_ix_tmp;
  xd.tmp_bytes = ix_tmp;
  GG_HIP(c, launch_run_index(xd, st));
  // One batch (every BASELINE config): its first pass is queued behind the
  // run index with no host round trip (tau and the slot maps computed on the
  // device, K1 reading its segment count there and skipping a bad table);
  // the host reads the index, the pass's status and the taus afterwards.
  const bool one_batch = n_genomes <= max_batch;
  size_t k1_timed = SIZE_MAX;
  if (one_batch) {
    GG_HIP(c, launch_first_pass(xd.nk, n_genomes, geom.over * (double)c->s, d_tau, d_slot_genome, d_slot_list, st));
    SketchLaunch a;
    a.words = d_words;
    a.n_words = n_words;
    a.runs = d_all_runs;
    a.run_sstart = d_rs;
    a.slot_genome0 = 0;
    a.n_runs = (uint32_t)n_runs;
    a.seg0 = 0;
    a.n_segs = 0;
    a.n_segs_dev = d_rs + n_runs;
    a.bad_dev = d_ix;
    a.tau = d_tau;
    a.table = d_table;
    a.cap_log2 = geom.cap_log2;
    a.flags = d_flags;
    a.count = d_count;
    a.seed = c->seed;
    if (c->timing) k1_timed = c->timed.size();
    GG_HIP(c, timed_launch(c, GG_KERNEL_SKETCH, 0, st, [&] { return launch_sketch_candidates(c->k, a, grid, st); }));
    GG_HIP(c, timed_launch(c, GG_KERNEL_FINALIZE, n_genomes, st, [&] {
      return launch_sketch_finalize(d_slot_list, n_genomes, d_slot_genome, d_tau, d_table, geom.cap_log2, d_flags,
                                    c->s, geom.sort_pow2, d_row_of, d_out, d_lens, d_status, d_count, st, d_ix);
    }));
  }
  // the index, and in one batch the first pass's taus and status (one batch:
  // max_batch = n_genomes, so the three are one contiguous read)
  GG_HIP(c, hipMemcpyAsync(h_rb, d_rb, (one_batch ? rb_u64 : rb_ix) * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  GG_HIP(c, hipStreamSynchronize(st));
  std::vector<uint64_t> hix(h_rb, h_rb + rb_ix);
  std::vector<uint32_t> status0;
  std::vector<uint64_t> tau0;
  if (one_batch) {
    tau0.assign(h_rb + rb_ix, h_rb + rb_ix + n_genomes);
    status0.assign(h_status, h_status + n_genomes);
  }
  if (hix[0] != ~0ull) {
    const gg_run* hr = host_runs();
    if (!hr) return fail(c, GG_ERR_HIP, "copying the run table to the host failed");
    return run_error(c, hr, hix[0], n_genomes);
  }
  const uint64_t* gr = hix.data() + 1;
  const uint64_t* grs = hix.data() + 1 + ng1;
  const uint64_t* nk = hix.data() + 1 + 2 * ng1;
  if (k1_timed < c->timed.size()) {  // (the k-mers of the first pass, known now)
    uint64_t kall = 0;
    for (uint32_t g = 0; g < n_genomes; ++g) kall += nk[g];
    c->timed[k1_timed].work = kall;
  }
  hp.mark("index runs (device)");
  for (uint32_t g0 = 0; g0 < n_genomes; g0 += max_batch) {
    const uint32_t g1 = std::min(n_genomes, g0 + max_batch);
    const uint32_t nb = g1 - g0;
    std::vector<TauSearch> ts(nb);
    std::vector<uint8_t> set_mode(nb, 0);  // slots the finalize switched to set mode (kSketchRetrySet)
    std::vector<uint64_t> h_tau(nb);
    std::vector<uint32_t> h_slot_genome(nb), h_slot_list(nb);
    for (uint32_t i = 0; i < nb; ++i) {
      ts[i].tau = one_batch ? tau0[i] : initial_tau(nk[g0 + i], c->s, geom.over);
      h_tau[i] = ts[i].tau;
      h_slot_genome[i] = g0 + i;
      h_slot_list[i] = i;
    }
    if (!one_batch)
      GG_HIP(c, hipMemcpyAsync(d_slot_genome, h_slot_genome.data(), nb * sizeof(uint32_t),
                               hipMemcpyHostToDevice, st));
    hp.mark("initial tau");

    // active genome slots for this pass
    std::vector<uint32_t> active = h_slot_list;
    for (int pass = 0; !active.empty(); ++pass) {
      if (pass > 200) return fail(c, GG_ERR_INTERNAL, "bottom-s threshold search did not converge");
      if (pass == 0 && one_batch) {  // (queued above)
        std::vector<uint32_t> next;
        for (uint32_t slot : active) {
          if (status0[slot] == kSketchOk) continue;
          if (status0[slot] == kSketchRetrySet) {  // the same tau, in set mode
            set_mode[slot] = 1;
            ++c->fallbacks[GG_FALLBACK_SKETCH_SET];
            next.push_back(slot);
            continue;
          }
          if (!advance_tau(ts[slot], status0[slot]))
            return fail(c, GG_ERR_INTERNAL, "bottom-s threshold search failed");
          h_tau[slot] = ts[slot].tau;
          next.push_back(slot);
        }
        active.swap(next);
        if (!active.empty()) ++c->fallbacks[GG_FALLBACK_SKETCH_RETRY];  // (a retry pass follows)
        continue;
      }
      // run table for the active genomes: on the first pass the batch's
      // slice of the uploaded table and its device index, on retries the
      // subset's runs and segment starts, built here and uploaded.  K1
      // segments never straddle runs: run r owns segments [rs[r], rs[r + 1]),
      // ceil(k-mers / seg) of them, so every lane of a wave hashes exactly one
      // piece per segment (a segment across a run boundary made its wave run
      // the hashing loop twice: +30% VALU at C5, where runs are ~10 kb).
      const bool all = active.size() == nb;
      const gg_run* d_run_src = d_all_runs + gr[g0];
      const uint64_t* d_rs_src = d_rs + gr[g0];
      uint64_t nr = gr[g0 + nb] - gr[g0];
      uint64_t seg0 = grs[g0], sacc = grs[g0 + nb] - grs[g0];
      uint64_t kacc = 0;
      if (!all) {
        const gg_run* runs_h = host_runs();
        if (!runs_h) return fail(c, GG_ERR_HIP, "copying the run table to the host failed");
        std::vector<gg_run> sub;
        for (uint32_t slot : active)
          for (uint64_t r = gr[g0 + slot]; r < gr[g0 + slot + 1]; ++r) sub.push_back(runs_h[r]);
        nr = sub.size();
        std::vector<uint64_t>& sub_rs = c->sstart_host;
        sub_rs.resize(nr + 1);
        uint64_t acc = 0;
        for (uint64_t r = 0; r < nr; ++r) {
          sub_rs[r] = acc;
          acc += (sub[r].len - (uint32_t)c->k + 1 + seg - 1) / seg;
        }
        sub_rs[nr] = acc;
        seg0 = 0;
        sacc = acc;
        for (uint32_t slot : active) kacc += nk[g0 + slot];
        gg_run* d_sub;
        uint64_t* d_sub_rs;
        GG_HIP(c, scratch_t(c, "runs_sub", std::max<size_t>(nr, 1), &d_sub));
        GG_HIP(c, scratch_t(c, "run_sstart_sub", nr + 1, &d_sub_rs));
        if (nr) GG_HIP(c, hipMemcpyAsync(d_sub, sub.data(), nr * sizeof(gg_run), hipMemcpyHostToDevice, st));
        GG_HIP(c, hipMemcpyAsync(d_sub_rs, sub_rs.data(), (nr + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
        GG_HIP(c, hipStreamSynchronize(st));  // (sub goes out of scope)
        d_run_src = d_sub;
        d_rs_src = d_sub_rs;
      } else {
        for (uint32_t i = 0; i < nb; ++i) kacc += nk[g0 + i];
      }
      hp.mark("segment starts");
      GG_HIP(c, hipMemcpyAsync(d_tau, h_tau.data(), nb * sizeof(uint64_t), hipMemcpyHostToDevice, st));
      GG_HIP(c, hipMemcpyAsync(d_slot_list, active.data(), active.size() * sizeof(uint32_t),
                               hipMemcpyHostToDevice, st));
      hp.mark("H2D runs/starts");
      // (the sets of batch 0 were cleared above if they needed it; every
      // later pass and batch finds the sets its slots use emptied by the
      // previous finalize)
      SketchLaunch a;
      a.words = d_words;
      a.n_words = n_words;
      a.runs = d_run_src;
      a.run_sstart = d_rs_src;
      a.slot_genome0 = g0;
      a.n_runs = (uint32_t)nr;
      a.seg0 = seg0;
      a.n_segs = sacc;
      a.tau = d_tau;
      a.table = d_table;
      a.cap_log2 = geom.cap_log2;
      a.flags = d_flags;
      a.count = d_count;
      a.any_set_mode = 0;
      for (uint32_t slot : active) a.any_set_mode |= set_mode[slot];
      a.seed = c->seed;
      const int g = (int)std::min<uint64_t>((uint64_t)grid, std::max<uint64_t>(1, (sacc + 255) / 256));
      GG_HIP(c, timed_launch(c, GG_KERNEL_SKETCH, kacc, st,
                             [&] { return launch_sketch_candidates(c->k, a, g, st); }));
      GG_HIP(c, timed_launch(c, GG_KERNEL_FINALIZE, active.size(), st, [&] {
        return launch_sketch_finalize(d_slot_list, (uint32_t)active.size(), d_slot_genome, d_tau,
                                      d_table, geom.cap_log2, d_flags, c->s,
                                      geom.sort_pow2, d_row_of, d_out, d_lens, d_status, d_count, st);
      }));
      hp.mark("enqueue K1 + finalize");
      GG_HIP(c, hipMemcpyAsync(const_cast<uint32_t*>(h_status), d_status, nb * sizeof(uint32_t),
                               hipMemcpyDeviceToHost, st));
      GG_HIP(c, hipStreamSynchronize(st));
      const std::vector<uint32_t> status(h_status, h_status + nb);
      hp.mark("wait (GPU)");
      std::vector<uint32_t> next;
      for (uint32_t slot : active) {
        if (status[slot] == kSketchOk) continue;
        if (status[slot] == kSketchRetrySet) {  // the same tau, in set mode
          set_mode[slot] = 1;
          ++c->fallbacks[GG_FALLBACK_SKETCH_SET];
          next.push_back(slot);
          continue;
        }
        if (!advance_tau(ts[slot], status[slot]))
          return fail(c, GG_ERR_INTERNAL, "bottom-s threshold search failed");
        h_tau[slot] = ts[slot].tau;
        next.push_back(slot);
      }
      active.swap(next);
      if (!active.empty()) ++c->fallbacks[GG_FALLBACK_SKETCH_RETRY];
    }
  }
  c->clean_table = d_table;
  c->clean_table_bytes = batch_bytes;
  return GG_OK;
}

namespace {

gg_status ensure_cmin(gg_ctx* c, float min_ani, uint32_t** d_cmin, uint32_t** d_sufmin, hipStream_t st) {
  const uint32_t tmax = 2 * c->s;
  GG_HIP(c, scratch_t(c, "cmin", 2 * (tmax + 1), d_cmin));
  *d_sufmin = *d_cmin + (tmax + 1);
  if (c->cmin_key != min_ani || c->cmin_host.size() != tmax + 1) {
    c->cmin_host = build_cmin(c->s, c->k, min_ani);
    // sufmin[t] = min(cmin[t..tmax]): a lower bound of cmin[total] for any
    // total >= t (the gate kernel's candidate test)
    c->sufmin_host.assign(tmax + 1, 0xFFFFFFFFu);
    uint32_t m = 0xFFFFFFFFu;
    for (uint32_t t = tmax + 1; t-- > 0;) {
      m = std::min(m, c->cmin_host[t]);
      c->sufmin_host[t] = m;
    }
    c->cmin_key = min_ani;
  }
  GG_HIP(c, hipMemcpyAsync(*d_cmin, c->cmin_host.data(), (tmax + 1) * sizeof(uint32_t),
                           hipMemcpyHostToDevice, st));
  GG_HIP(c, hipMemcpyAsync(*d_sufmin, c->sufmin_host.data(), (tmax + 1) * sizeof(uint32_t),
                           hipMemcpyHostToDevice, st));
  return GG_OK;
}

#if defined(GG_XCHECK)
// Work items of the table kernels: runs of <= seg_tiles column tiles of one
// tile row, inside tiles [tb, te).
void build_segments(std::vector<PairSeg>& segs, uint64_t nb, uint64_t tb, uint64_t te, uint32_t seg_tiles) {
  segs.clear();
  uint64_t t = 0;
  for (uint64_t I = 0; I < nb && t < te; ++I) {
    const uint64_t first = t, last = t + (nb - I);
    const uint64_t lo = std::max(first, tb), hi = std::min(last, te);
    for (uint64_t x = lo; x < hi; x += seg_tiles) {
      const uint64_t y = std::min(hi, x + seg_tiles);
      segs.push_back(PairSeg{(uint32_t)I, (uint32_t)(I + (x - first)), (uint32_t)(I + (y - first)), 0});
    }
    t = last;
  }
}
#endif

// Gate kernel (pairs_gate.hip): tables for the tile rows of [tb, te), then
// the column stream.  Work items are (tile row, row block, column segment)
// with segments aligned to absolute multiples of kGateSegTiles column
// tiles, ordered column-segment-major, and dealt to blockIdx so that runs
// of kGateXcdRun consecutive items land on one XCD (blockIdx mod 8 under
// round-robin dispatch): the workgroups resident on an XCD then stream the
// same columns through its L2.
gg_status pairs_gate(gg_ctx* c, const uint64_t* d_sk, const uint32_t* d_lens, uint32_t n, uint64_t nb,
                     uint64_t tb, uint64_t te, const uint32_t* d_cmin, const uint32_t* d_sufmin, gg_pair* d_out,
                     uint64_t cap, uint64_t* d_count, uint64_t work, hipStream_t st) {
  constexpr uint32_t kGateXcdRun = 64;  // ~ workgroups resident per XCD (32 CUs x 2)
  const GateParams gp = gate_params(c->s);
  if (gp.cap > 65535u || c->s > kMaxSketch)
    return fail(c, GG_ERR_INTERNAL, "gate kernel: R * s exceeds its 16-bit positions");
  std::vector<PairSeg> items;
  uint32_t I0 = UINT32_MAX, I1 = 0;
  {
    uint64_t t = 0;
    for (uint64_t I = 0; I < nb && t < te; ++I) {
      const uint64_t first = t, last = t + (nb - I);
      const uint64_t lo = std::max(first, tb), hi = std::min(last, te);
      t = last;
      if (lo >= hi) continue;
      I0 = std::min<uint32_t>(I0, (uint32_t)I);
      I1 = std::max<uint32_t>(I1, (uint32_t)I);
      uint64_t J = I + (lo - first);
      const uint64_t Jend = I + (hi - first);
      while (J < Jend) {
        const uint64_t Jn = std::min<uint64_t>(Jend, (J / kGateSegTiles + 1) * kGateSegTiles);
        for (uint32_t rb = 0; rb < gp.G; ++rb)
          if (I * GG_PAIR_TILE + rb * gp.R < n)
            items.push_back(PairSeg{(uint32_t)I, (uint32_t)J, (uint32_t)Jn, rb});
        J = Jn;
      }
    }
  }
  if (items.empty()) return GG_OK;
  std::stable_sort(items.begin(), items.end(), [](const PairSeg& x, const PairSeg& y) {
    return x.J0 / kGateSegTiles < y.J0 / kGateSegTiles;
  });
  const uint64_t per = 8ull * kGateXcdRun;
  const uint64_t n_blocks = (items.size() + per - 1) / per * per;
  if (n_blocks > 0x7fffffffull) return fail(c, GG_ERR_INVALID_ARG, "too many pair work items");
  c->seg_host.assign(n_blocks, PairSeg{UINT32_MAX, 0, 0, 0});
  for (uint64_t k = 0; k < items.size(); ++k) {
    const uint64_t run = k / kGateXcdRun;
    const uint64_t b = (run / 8) * per + (k % kGateXcdRun) * 8 + run % 8;
    c->seg_host[b] = items[k];
  }
  PairSeg* d_items;
  GG_HIP(c, scratch_t(c, "pair_segs", c->seg_host.size(), &d_items));
  GG_HIP(c, hipMemcpyAsync(d_items, c->seg_host.data(), c->seg_host.size() * sizeof(PairSeg),
                           hipMemcpyHostToDevice, st));
  GateBuildLaunch bl;
  bl.sketches = d_sk;
  bl.lens = d_lens;
  bl.n = n;
  bl.stride = c->s;
  bl.tile_row0 = I0;
  bl.n_blocks = (I1 - I0 + 1) * gp.G;
  bl.p = gp;
  GG_HIP(c, scratch_t(c, "gate_tables", (size_t)bl.n_blocks * gp.block_bytes, &bl.tables));
  GG_HIP(c, scratch_t(c, "gate_lo32", (size_t)n * c->s, &bl.lo32));
  GateLaunch g;
  g.sketches = d_sk;
  g.lens = d_lens;
  g.n = n;
  g.stride = c->s;
  g.items = d_items;
  g.n_items = (uint32_t)n_blocks;
  g.tile_row0 = I0;
  g.p = gp;
  g.tables = bl.tables;
  g.lo32 = bl.lo32;
  g.cmin = d_cmin;
  g.sufmin = d_sufmin;
  g.tmax = 2 * c->s;
  g.zero_passes = c->sufmin_host[0] == 0;
  g.out = d_out;
  g.out_cap = cap;
  g.count = (unsigned long long*)d_count;
  GG_HIP(c, timed_launch(c, GG_KERNEL_PAIRS, work, st, [&] {
    hipError_t e = launch_gate_build(bl, st);
    return e != hipSuccess ? e : launch_pairs_gate(g, st);
  }));
  return GG_OK;
}

// Inverted-index K2 (pairs_index.hip) over tiles [tb, te).  *used = false
// when the index path does not apply (a hash shared by more than kMaxRun
// sketches, or a row whose partners overflow the LDS map at 2^16 partner
// classes); the output count is then as before the call and the caller runs
// the gate kernel.  Eligibility (no pass without a shared hash, sizes) is
// the caller's.
gg_status pairs_index(gg_ctx* c, const uint64_t* d_sk, const uint32_t* d_lens, uint32_t n, uint64_t nb,
                      uint64_t tb, uint64_t te, const uint32_t* d_cmin, const uint32_t* d_sufmin, gg_pair* d_out,
                      uint64_t cap, uint64_t* d_count, uint64_t work, hipStream_t st, bool* used, bool* costly,
                      bool weigh_cost) {
  // (runs in row order -- every build but the row-range one -- read only the
  // members after each entry; a longer run's start is found by walks that
  // grow with it, so past this the gate kernel runs instead)
  constexpr uint32_t kMaxRun = 1u << 16;
  constexpr uint64_t kBigMapRun = 1536;  // runs longer than the small partner map's fill: the large map
  *used = false;
  *costly = false;
  const uint64_t total = (uint64_t)n * c->s;
  uint32_t kbits = 1;
  while ((1u << kbits) < c->s) ++kbits;
  IndexBuild b;
  b.sketches = d_sk;
  b.lens = d_lens;
  b.n = n;
  b.stride = c->s;
  b.kbits = kbits;
  b.max_run = kMaxRun;
  GG_HIP(c, scratch_t(c, "idx_offs", std::max(n, 1u), &b.offs));
  // info (2 u64) and flags (4 u32) adjacent: one read-back
  GG_HIP(c, scratch_t(c, "idx_info", 4 + index_cost_bytes() / sizeof(uint64_t), &b.info));
  b.flags = reinterpret_cast<uint32_t*>(b.info + 2);
  b.cost = reinterpret_cast<unsigned long long*>(b.info + 4);
  GG_HIP(c, scratch_t(c, "idx_keys_in", total, &b.keys_in));
  // (+16: the super-bin sort reads keys_out as bytes and vals_in as u32 in
  // aligned groups of 16 entries up to ceil(total / 16) * 16; the split build
  // places `total` of them, so the last group's tail is in bounds whatever
  // the element widths -- ADVICE round 5)
  GG_HIP(c, scratch_t(c, "idx_keys_out", total + 16, &b.keys_out));
  GG_HIP(c, scratch_t(c, "idx_vals_in", total + 16, &b.vals_in));
  GG_HIP(c, scratch_t(c, "idx_vals_out", total, &b.vals_out));
  GG_HIP(c, scratch_t(c, "idx_runinfo", total, &b.runinfo));
  GG_HIP(c, scratch_t(c, "idx_mixed", (total + 31) / 32, &b.mixed));
  // rows of the tile rows that intersect [tb, te)
  uint64_t I0 = UINT64_MAX, I1 = 0, t = 0;
  for (uint64_t I = 0; I < nb && t < te; ++I) {
    const uint64_t first = t, last = t + (nb - I);
    t = last;
    if (std::max(first, tb) >= std::min(last, te)) continue;
    I0 = std::min(I0, I);
    I1 = std::max(I1, I + 1);
  }
  if (I0 == UINT64_MAX) {  // no tile here: nothing to index or emit
    *used = true;
    return GG_OK;
  }
  const uint32_t r0 = (uint32_t)(I0 * GG_PAIR_TILE), r1 = (uint32_t)std::min<uint64_t>(n, I1 * GG_PAIR_TILE);
  // A device that evaluates only some rows (a multi-device call) indexes only
  // the entries whose hash may occur in them (GALAHGPU_INDEX_RANGE=0: every
  // entry, as a single device does).
  static const bool range_on = [] {
    const char* e = getenv("GALAHGPU_INDEX_RANGE");
    return !(e && *e == '0');
  }();
  // (a range of more than ~40% of the rows keeps most entries anyway: the
  // filter would cost more than the smaller sort saves)
  if (range_on && (r0 > 0 || r1 < n) && 5ull * (r1 - r0) <= 2ull * n) {
    uint32_t lg = 20;
    while (lg < 30 && (1ull << lg) < 16ull * (r1 - r0) * c->s) ++lg;
    b.bloom_log2 = lg;
    b.r0 = r0;
    b.r1 = r1;
    GG_HIP(c, scratch_t(c, "idx_bloom", (size_t)1 << (lg - 5), &b.bloom));
  }
  // Bucketed build (default; GALAHGPU_INDEX_BUCKETS=0: the full 32-bit sort
  // and the run pass).  A bucket too large for LDS falls back to the full
  // build, from a fresh fill (its keys differ, and the bucket pass
  // overwrote keys_in).
  const char* be = getenv("GALAHGPU_INDEX_BUCKETS");
  b.bucket = !(be && *be == '0');
  if (b.bucket) {
    GG_HIP(c, scratch_t(c, "idx_hist", kIndexCoarse, &b.hist));
    GG_HIP(c, scratch_t(c, "idx_bbase", kIndexCoarse + 1, &b.bbase));
  }
  IndexLaunch a;
  a.sketches = d_sk;
  a.lens = d_lens;
  a.n = n;
  a.stride = c->s;
  a.kbits = kbits;
  a.row0 = r0;
  a.nb = nb;
  a.tile_begin = tb;
  a.tile_end = te;
  a.runinfo = b.runinfo;
  a.vals = b.keys_in;  // the build leaves the run members' entries there
  a.cmin = d_cmin;
  a.sufmin = d_sufmin;
  a.tmax = 2 * c->s;
  a.out = d_out;
  a.out_cap = cap;
  a.count = (unsigned long long*)d_count;
  // GALAHGPU_INDEX_MAX_SPLIT (tests): fewer partner classes per row, so the
  // overflow fallback below can be reached on small inputs
  {
    const char* e = getenv("GALAHGPU_INDEX_MAX_SPLIT");
    a.max_split_log2 = e && *e ? (uint32_t)std::min(16, std::max(0, atoi(e))) : 16u;
  }
  a.overflow = b.flags + 2;  // (zeroed by index_fill)
  // The index's cost is its pairs kernel's member reads (the run passes sum
  // them into b.cost: per entry of a shared hash, the other sketches holding
  // it); the gate kernel's, the pair count x s.  Clusters of thousands of
  // near-identical genomes make the first grow as g^2 per hash (C3 with
  // clusters of 1,000: 2.7e9 reads, index 25 ms against ~3 ms of gate), so
  // past kIndexCost x s x pairs member reads the pairs kernel emits nothing
  // and the gate kernel runs instead (GALAHGPU_INDEX_COST=<factor>, 0: never;
  // never either when the index is asked for by GALAHGPU_PAIRS_KERNEL=index)
  {
    const char* e = getenv("GALAHGPU_INDEX_COST");
    const double k = !weigh_cost ? 0.0 : e && *e ? atof(e) : 0.0;
    // (a member of a multi-device call weighs its share: the pairs of its tiles)
    const double lim = k * (double)c->s * (double)pairs_in_tiles(n, tb, te);
    a.cost = b.cost;
    a.cost_limit = k > 0 && lim < 1.8e19 ? (unsigned long long)lim : ~0ull;
  }
  // the output count before the pairs launch: restored if a row overflows
  uint64_t* d_count0;
  GG_HIP(c, scratch_t(c, "idx_count0", 1, &d_count0));
  GG_HIP(c, hipMemcpyAsync(d_count0, d_count, sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
  auto launch_pairs = [&](bool guarded) -> gg_status {
    a.build_flags = guarded ? b.flags : nullptr;
    a.ents16 = b.bucket && index_ents16(n);  // (b.bucket: the bucketed build made the index)
    GG_HIP(c, timed_launch(c, GG_KERNEL_PAIRS, work, st, [&] { return launch_index_pairs(a, r1 - r0, st); }));
    return GG_OK;
  };
  uint64_t info[2] = {0, 0};
  uint32_t kept = 0;
  uint32_t flags[4] = {0, 0, 0, 0};
  bool built = false, paired = false;
  if (b.bucket && !b.bloom) {
    // one host round trip: fill, bucketed build and the pairs kernel queued
    // back to back (every row slot is a sort item, so the sort's size is
    // known up front; the pairs kernel emits nothing if the build failed)
    const uint32_t nbb = index_bucket_bound(total);
    // split build (default; GALAHGPU_INDEX_SPLIT=0: the fill and the 16-bit
    // sort), whose super-bin sort writes the bounds of all 2^16 bucket ids
    const char* se = getenv("GALAHGPU_INDEX_SPLIT");
    const bool split = !(se && *se == '0');
    if (split) {
      GG_HIP(c, scratch_t(c, "idx_split_cnt", (size_t)256 * n + 1, &b.split_cnt));
      GG_HIP(c, scratch_t(c, "idx_split_off", (size_t)256 * n + 1, &b.split_off));
      GG_HIP(c, scratch_t(c, "idx_split_hist", (size_t)256 * 16 * 256, &b.split_hist));
    }
    b.sort_tmp_bytes = split ? index_split_tmp_bytes(n) : index_bucket_sort_tmp_bytes(total);
    GG_HIP(c, scratch(c, "idx_sort_tmp", b.sort_tmp_bytes, &b.sort_tmp));
    GG_HIP(c, scratch_t(c, "idx_bstart", split ? (size_t)65537 : (size_t)nbb + 1, &b.bstart));
    GG_HIP(c, timed_launch(c, GG_KERNEL_PAIRS_INDEX, total, st, [&] { return index_fill(b, st); }));
    GG_HIP(c, timed_launch(c, GG_KERNEL_PAIRS_INDEX, 0, st, [&] { return index_build_buckets(b, total, nbb, st); }));
    gg_status ps = launch_pairs(true);
    if (ps != GG_OK) return ps;
    uint64_t* h_if;
    GG_HIP(c, host_scratch_t(c, "idx_info", 5, &h_if));
    GG_HIP(c, hipMemcpyAsync(h_if, b.info, 5 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    GG_HIP(c, hipStreamSynchronize(st));
    memcpy(info, h_if, sizeof info);
    memcpy(flags, h_if + 2, sizeof flags);
    built = paired = flags[3] == 0;
    if (built && !flags[0] && h_if[4] > a.cost_limit) {  // (the pairs kernel emitted nothing)
      *costly = true;
      return GG_OK;
    }
  } else {
    uint32_t nbuckets = 0;
    GG_HIP(c, timed_launch(c, GG_KERNEL_PAIRS_INDEX, total, st, [&] { return index_fill(b, st); }));
    GG_HIP(c, hipMemcpyAsync(info, b.info, sizeof info, hipMemcpyDeviceToHost, st));
    if (b.bloom) GG_HIP(c, hipMemcpyAsync(&kept, b.flags + 1, sizeof kept, hipMemcpyDeviceToHost, st));
    if (b.bucket)
      GG_HIP(c, hipMemcpyAsync(&nbuckets, b.bbase + kIndexCoarse, sizeof nbuckets, hipMemcpyDeviceToHost, st));
    GG_HIP(c, hipStreamSynchronize(st));
    if (b.bucket) {  // (row-range index: its kept entries, compacted)
      b.sort_tmp_bytes = index_bucket_sort_tmp_bytes(kept);
      GG_HIP(c, scratch(c, "idx_sort_tmp", b.sort_tmp_bytes, &b.sort_tmp));
      GG_HIP(c, scratch_t(c, "idx_bstart", (size_t)nbuckets + 1, &b.bstart));
      GG_HIP(c, timed_launch(c, GG_KERNEL_PAIRS_INDEX, 0, st,
                             [&] { return index_build_buckets(b, kept, nbuckets, st); }));
      GG_HIP(c, hipMemcpyAsync(flags, b.flags, sizeof flags, hipMemcpyDeviceToHost, st));
      GG_HIP(c, hipStreamSynchronize(st));
      built = flags[3] == 0;
    }
  }
  // keys of the full build = the top 32 significant bits of each hash (the
  // low 32 bits travel with the entry): shift by the bits of the largest hash
  // beyond 32 (the row-range fill computed the same shift on the device)
  const uint64_t n_entries = b.bloom ? kept : info[0], maxh = info[1];
  uint32_t bits = 0;
  while (bits < 64 && (maxh >> bits) != 0) ++bits;
  const uint32_t sh = bits > 32 ? bits - 32 : 0;
  const uint32_t end_bit = std::max(1u, bits - sh);
  if (!built) {
    if (b.bucket) {  // refill with the full build's keys (the row-range kept count comes out the same)
      b.bucket = false;
      GG_HIP(c, timed_launch(c, GG_KERNEL_PAIRS_INDEX, 0, st, [&] { return index_fill(b, st); }));
    }
    ++c->pair_paths[GG_PATH_INDEX_FULL_SORT];
    b.sort_tmp_bytes = index_sort_tmp_bytes(n_entries, end_bit);
    GG_HIP(c, scratch(c, "idx_sort_tmp", b.sort_tmp_bytes, &b.sort_tmp));
    GG_HIP(c, timed_launch(c, GG_KERNEL_PAIRS_INDEX, 0, st,
                           [&] { return index_build(b, n_entries, sh, end_bit, st); }));
    uint64_t* h_if;
    GG_HIP(c, host_scratch_t(c, "idx_info", 6, &h_if));
    GG_HIP(c, hipMemcpyAsync(h_if, b.info, 6 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    GG_HIP(c, hipStreamSynchronize(st));
    memcpy(flags, h_if + 2, sizeof(uint32_t));
    if (!flags[0] && h_if[4] > a.cost_limit) {
      *costly = true;
      return GG_OK;
    }
    // a run longer than the partner map's fill limit (clusters of thousands
    // of near-identical genomes): rows with that many partners, which the
    // large map counts in one pass instead of several over their runs (C3
    // in clusters of 5,000: K2 429 -> 197 ms)
    a.big_map = h_if[5] > kBigMapRun;
  } else if (!paired && !flags[0]) {  // (row-range bucketed build: its cost before the pairs kernel)
    uint64_t cost[2] = {0, 0};
    GG_HIP(c, hipMemcpyAsync(cost, b.info + 4, sizeof cost, hipMemcpyDeviceToHost, st));
    GG_HIP(c, hipStreamSynchronize(st));
    if (cost[0] > a.cost_limit) {
      *costly = true;
      return GG_OK;
    }
    a.big_map = cost[1] > kBigMapRun;
  }
  if (flags[0]) return GG_OK;  // a run longer than kMaxRun (the pairs kernel, if queued, emitted nothing)
  if (!paired) {
    gg_status ps = launch_pairs(false);
    if (ps != GG_OK) return ps;
    GG_HIP(c, hipMemcpyAsync(&flags[2], b.flags + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    GG_HIP(c, hipStreamSynchronize(st));
  }
  *used = true;
  if (flags[2]) {  // a row's partners did not fit the LDS map: drop what the pairs launch emitted
    GG_HIP(c, hipMemcpyAsync(d_count, d_count0, sizeof(uint64_t), hipMemcpyDeviceToDevice, st));
    *used = false;
  }
  return GG_OK;
}

}  // namespace

gg_status pairs_core(gg_ctx* c, const uint64_t* d_sk, const uint32_t* d_lens, uint32_t n,
                     uint64_t tb, uint64_t te, float min_ani, gg_pair* d_out, uint64_t cap,
                     uint64_t* d_count, hipStream_t st) {
  uint32_t *d_cmin, *d_sufmin;
  gg_status cs = ensure_cmin(c, min_ani, &d_cmin, &d_sufmin, st);
  if (cs != GG_OK) return cs;
  const uint64_t nb = (n + GG_PAIR_TILE - 1) / GG_PAIR_TILE;
  te = std::min<uint64_t>(te, gg_pair_tiles(n));
  const uint64_t work = c->timing ? pairs_in_tiles(n, tb, te) : 0;
#if defined(GG_XCHECK)
  int kern = (c->pairs_kernel == 1 && pairs_table_rows(c->s) == 0) ? 2 : c->pairs_kernel;
#else
  // the cross-check forms (table, merge) live in pairs.hip, which only the
  // test build libgalahgpu_xcheck.so carries
  if (c->pairs_kernel == 1 || c->pairs_kernel == 2)
    return fail(c, GG_ERR_INVALID_ARG,
                "GALAHGPU_PAIRS_KERNEL=table|merge: the cross-check kernels are built into "
                "libgalahgpu_xcheck.so (tests) only");
  int kern = c->pairs_kernel;
#endif
  // auto (0) / index (4): the inverted index when no pair without a shared
  // hash can pass (min_ani > 0) and the packed (row, position) values fit
  // 32 bits; "auto" also leaves tiny sets to the gate kernel
  if (kern == 0 || kern == 4) {
    uint32_t kbits = 1;
    while ((1u << kbits) < c->s) ++kbits;
    const bool fits = (uint64_t)n * c->s < (1ull << 31) && kbits < 32 && ((uint64_t)n << kbits) <= (1ull << 32);
    if (c->sufmin_host[0] != 0 && fits && n >= 2 && (kern == 4 || n >= 512)) {
      bool used = false, costly = false;
      gg_status is = pairs_index(c, d_sk, d_lens, n, nb, tb, te, d_cmin, d_sufmin, d_out, cap, d_count, work, st,
                                 &used, &costly, kern == 0);
      if (is != GG_OK) return is;
      ++c->pair_paths[used ? GG_PATH_INDEX : GG_PATH_INDEX_ABANDONED];
      if (costly) ++c->index_costly;
      if (used) return GG_OK;
    }
    kern = 0;
  }
  ++c->pair_paths[(kern == 0 || kern == 3) ? GG_PATH_GATE : GG_PATH_OTHER];
  if (kern == 0 || kern == 3)
    return pairs_gate(c, d_sk, d_lens, n, nb, tb, te, d_cmin, d_sufmin, d_out, cap, d_count, work, st);
#if defined(GG_XCHECK)
  if (kern == 2) {
    PairsLaunch a;
    a.sketches = d_sk;
    a.lens = d_lens;
    a.n = n;
    a.stride = c->s;
    a.n_row_tiles = (uint32_t)nb;
    a.tile_begin = tb;
    a.tile_end = te;
    a.cmin = d_cmin;
    a.tmax = 2 * c->s;
    a.out = d_out;
    a.out_cap = cap;
    a.count = (unsigned long long*)d_count;
    GG_HIP(c, timed_launch(c, GG_KERNEL_PAIRS, work, st, [&] { return launch_pairs(a, st); }));
    return GG_OK;
  }
  build_segments(c->seg_host, nb, tb, te, kSegTiles);
  if (c->seg_host.empty()) return GG_OK;
  PairSeg* d_segs;
  GG_HIP(c, scratch_t(c, "pair_segs", c->seg_host.size(), &d_segs));
  GG_HIP(c, hipMemcpyAsync(d_segs, c->seg_host.data(), c->seg_host.size() * sizeof(PairSeg),
                           hipMemcpyHostToDevice, st));
  if (kern == 1) {
    PairsTableLaunch b;
    b.sketches = d_sk;
    b.lens = d_lens;
    b.n = n;
    b.stride = c->s;
    b.segs = d_segs;
    b.n_segs = (uint32_t)c->seg_host.size();
    b.cmin = d_cmin;
    b.tmax = 2 * c->s;
    b.out = d_out;
    b.out_cap = cap;
    b.count = (unsigned long long*)d_count;
    GG_HIP(c, timed_launch(c, GG_KERNEL_PAIRS, work, st, [&] { return launch_pairs_table(b, st); }));
    return GG_OK;
  }
#endif
  return GG_OK;
}

// Passing pairs of tiles [tb, te) appended to res in (i, j) order: from
// kDeviceSortPairs up to 2^31 of them sorted on the device, otherwise on
// the calling thread.
gg_status pairs_range_to_host(gg_ctx* c, const uint64_t* d_sk, const uint32_t* d_lens, uint32_t n,
                              uint64_t tb, uint64_t te, float min_ani, std::vector<gg_pair>& res,
                              hipStream_t st) {
  if (n < 2 || tb >= te) return GG_OK;
  uint64_t *d_count, *h_count;
  GG_HIP(c, scratch_t(c, "pair_count", 1, &d_count));
  GG_HIP(c, host_scratch_t(c, "pair_count", 1, &h_count));
  uint64_t cap = std::max<uint64_t>(1 << 20, (uint64_t)n * 16);
  const uint64_t all = (uint64_t)n * (n > 0 ? n - 1 : 0) / 2;
  cap = std::min<uint64_t>(cap, std::max<uint64_t>(all, 1));
  for (int attempt = 0; attempt < 2; ++attempt) {
    gg_pair* d_out;
    GG_HIP(c, scratch_t(c, "pair_out", cap, &d_out));
    GG_HIP(c, hipMemsetAsync(d_count, 0, sizeof(uint64_t), st));
    gg_status ps = pairs_core(c, d_sk, d_lens, n, tb, te, min_ani, d_out, cap, d_count, st);
    if (ps != GG_OK) return ps;
    GG_HIP(c, hipMemcpyAsync(h_count, d_count, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    GG_HIP(c, hipStreamSynchronize(st));
    const uint64_t cnt = *h_count;
    if (cnt <= cap) {
      const size_t at = res.size();
      res.resize(at + cnt);
      if (cnt < kDeviceSortPairs || cnt >= (1ull << 31)) {  // (few, or beyond the sort's int count: the host sorts)
        if (cnt) {
          GG_HIP(c, hipMemcpyAsync(res.data() + at, d_out, cnt * sizeof(gg_pair), hipMemcpyDeviceToHost, st));
          GG_HIP(c, hipStreamSynchronize(st));
          // in (i, j) order here, on the calling (member) thread: the members
          // of a multi-device call sort their parts at the same time
          std::sort(res.begin() + at, res.end(), [](const gg_pair& x, const gg_pair& y) {
            return x.i != y.i ? x.i < y.i : x.j < y.j;
          });
        }
        return GG_OK;
      }
      // many: sorted by (i, j) on the device and copied out in that order
      // (scratch: keys and sorted keys [cnt] u64, positions and sorted
      // positions [cnt] u32, the sorted pairs [cnt] x 16 B)
      uint64_t* d_kv;
      void* d_tmp;
      const size_t tmp_bytes = pair_sort_tmp_bytes(cnt, n);
      GG_HIP(c, scratch_t(c, "pair_sort_kv", 5 * cnt, &d_kv));
      GG_HIP(c, scratch(c, "pair_sort_tmp", std::max<size_t>(tmp_bytes, 16), &d_tmp));
      uint32_t* d_idx = (uint32_t*)(d_kv + 2 * cnt);
      gg_pair* d_sorted = (gg_pair*)(d_kv + 3 * cnt);
      GG_HIP(c, sort_pairs_device(d_out, cnt, n, d_kv, d_kv + cnt, d_idx, d_idx + cnt, d_sorted, d_tmp, tmp_bytes,
                                  st));
      // staged through a pinned chunk of at most kPairStage pairs (16 MiB), so
      // a long-lived context holds no page-locked memory sized by its largest
      // result
      constexpr uint64_t kPairStage = 1ull << 20;
      gg_pair* h_sorted;
      GG_HIP(c, host_scratch_t(c, "pair_sorted", std::min(cnt, kPairStage), &h_sorted));
      for (uint64_t x = 0; x < cnt; x += kPairStage) {
        const uint64_t m = std::min(kPairStage, cnt - x);
        GG_HIP(c, hipMemcpyAsync(h_sorted, d_sorted + x, m * sizeof(gg_pair), hipMemcpyDeviceToHost, st));
        GG_HIP(c, hipStreamSynchronize(st));
        memcpy(res.data() + at + x, h_sorted, m * sizeof(gg_pair));
      }
      return GG_OK;
    }
    cap = cnt;
  }
  return fail(c, GG_ERR_INTERNAL, "pair output sizing failed");
}

double ani_f64(uint32_t common, uint32_t total, int k) {
  // finch distance(): J = common/total; mash = -ln(2J/(1+J))/k clamped to
  // [0,1] with f64::min / f64::max; galah: ani = 1 - mash (src/finch.rs:56)
  const double jaccard = (double)common / (double)total;
  double d = -1.0 * std::log((2.0 * jaccard) / (1.0 + jaccard)) / (double)k;
  d = rust_max(rust_min(d, 1.0), 0.0);
  return 1.0 - d;
}

std::vector<uint32_t> build_cmin(uint32_t s, int k, float min_ani) {
  const uint32_t tmax = 2 * s;
  const double thr = (double)min_ani;  // src/finch.rs:69: min_ani as f64
  std::vector<uint32_t> cmin(tmax + 1, 0xFFFFFFFFu);
  for (uint32_t t = 0; t <= tmax; ++t) {
    const uint32_t cmax = std::min(t, s);
    if (!(ani_f64(cmax, t, k) >= thr)) continue;  // nothing passes at this total
    uint32_t lo = 0, hi = cmax;  // smallest c with ani(c,t) >= thr lies in [lo, hi]
    if (ani_f64(0, t, k) >= thr) {
      cmin[t] = 0;
      continue;
    }
    while (hi - lo > 1) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (ani_f64(mid, t, k) >= thr) hi = mid;
      else lo = mid;
    }
    cmin[t] = hi;
  }
  return cmin;
}

gg_status mark_rows_ready(gg_ctx* m) {
  if (!m->rows_ready) GG_HIP(m, hipEventCreateWithFlags(&m->rows_ready, hipEventDisableTiming));
  GG_HIP(m, hipEventRecord(m->rows_ready, m->stream));
  return GG_OK;
}

gg_ctx* lane_ctx(gg_ctx* m, size_t i) {
  if (m->lanes.size() <= i) m->lanes.resize(i + 1, nullptr);
  gg_ctx*& l = m->lanes[i];
  if (l) return l;
  gg_ctx* x = new (std::nothrow) gg_ctx();
  if (!x) return nullptr;
  x->k = m->k;
  x->s = m->s;
  x->seed = m->seed;
  x->device = m->device;
  x->pairs_kernel = m->pairs_kernel;
  x->host_threads = m->host_threads;
  if (hipSetDevice(m->device) != hipSuccess || hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking) != hipSuccess) {
    delete x;
    return nullptr;
  }
  l = x;
  return l;
}

}  // namespace gg

using namespace gg;

// ----------------------------------------------------------------------------
extern "C" {

uint32_t gg_abi_version(void) { return GG_ABI_VERSION; }

const char* gg_status_string(gg_status s) {
  switch (s) {
    case GG_OK: return "ok";
    case GG_ERR_INVALID_ARG: return "invalid argument";
    case GG_ERR_IO: return "I/O error";
    case GG_ERR_FORMAT: return "format error";
    case GG_ERR_NO_DEVICE: return "no usable gfx950 device";
    case GG_ERR_HIP: return "HIP error";
    case GG_ERR_OUT_OF_MEMORY: return "out of memory";
    case GG_ERR_INTERNAL: return "internal error";
    case GG_ERR_OUTPUT_FULL: return "output buffer full";
    case GG_ERR_CANCELLED: return "cancelled by the caller";
  }
  return "unknown status";
}

const char* gg_last_error(const gg_ctx* ctx) { return ctx ? ctx->err.c_str() : g_thread_err.c_str(); }
const char* gg_thread_last_error(void) { return g_thread_err.c_str(); }

gg_ctx* gg_create(int kmer_length, uint32_t sketch_size, uint64_t hash_seed, int device,
                  gg_status* status) {
  gg_status dummy;
  if (!status) status = &dummy;
  if (kmer_length < 1 || kmer_length > 32 || sketch_size < 1 || sketch_size > kMaxSketch) {
    *status = fail(nullptr, GG_ERR_INVALID_ARG, "kmer_length must be 1..32 and sketch_size 1..12000");
    return nullptr;
  }
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    *status = fail(nullptr, GG_ERR_NO_DEVICE, "no HIP device visible (libgalahgpu has no CPU path)");
    return nullptr;
  }
  int dev = device;
  if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (dev >= n) {
    *status = fail(nullptr, GG_ERR_NO_DEVICE, "device ordinal out of range");
    return nullptr;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess ||
      strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    *status = fail(nullptr, GG_ERR_NO_DEVICE,
                   std::string("device is not gfx950 (MI355X): ") + prop.gcnArchName);
    return nullptr;
  }
  gg_ctx* c = new (std::nothrow) gg_ctx();
  if (!c) {
    *status = fail(nullptr, GG_ERR_OUT_OF_MEMORY, "out of host memory");
    return nullptr;
  }
  c->k = kmer_length;
  c->s = sketch_size;
  c->seed = hash_seed;
  c->device = dev;
  // GALAHGPU_PAIRS_KERNEL: auto (default: the inverted index where it
  // applies, else the gate kernel), gate, index, table, merge -- for A/B
  // runs and the parity tests; results never depend on it
  const char* pk = getenv("GALAHGPU_PAIRS_KERNEL");
  c->pairs_kernel = !pk ? 0
                    : strcmp(pk, "table") == 0 ? 1
                    : strcmp(pk, "merge") == 0 ? 2
                    : strcmp(pk, "gate") == 0  ? 3
                    : strcmp(pk, "index") == 0 ? 4
                                               : 0;
  hipError_t e = hipSetDevice(dev);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  (void)e;
  if (!c->stream) {
    *status = fail(nullptr, GG_ERR_HIP, "stream creation failed");
    delete c;
    return nullptr;
  }
  *status = GG_OK;
  return c;
}

void gg_destroy(gg_ctx* ctx) {
  if (!ctx) return;
  ctx->pool.reset();  // (member threads idle between calls: joined here)
  for (gg_ctx* m : ctx->devs) gg_destroy(m);
  for (gg_ctx* l : ctx->lanes) gg_destroy(l);
  for (auto& kv : ctx->host_scratch)
    if (kv.second.first) (void)hipHostFree(kv.second.first);
  ctx->host_scratch.clear();
  if (!ctx->devs.empty()) {
    delete ctx;
    return;
  }
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (auto& kv : ctx->scratch)
    if (kv.second.first) (void)hipFree(kv.second.first);
  for (auto& t : ctx->timed) {
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  for (hipEvent_t e : ctx->spare_events) (void)hipEventDestroy(e);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  for (hipStream_t ps : ctx->peer_streams)
    if (ps) (void)hipStreamDestroy(ps);
  for (hipEvent_t e : ctx->rep_start)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->rep_done)
    if (e) (void)hipEventDestroy(e);
  if (ctx->copy_done) (void)hipEventDestroy(ctx->copy_done);
  if (ctx->rows_ready) (void)hipEventDestroy(ctx->rows_ready);
  if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
  if (ctx->pinned) (void)hipHostFree(ctx->pinned);
  for (auto& sl : ctx->gz_slot) {
    if (sl.st) (void)hipStreamSynchronize(sl.st);
    if (sl.st) (void)hipStreamDestroy(sl.st);
    if (sl.host) (void)hipHostFree(sl.host);
    if (sl.dev) (void)hipFree(sl.dev);
  }
  delete ctx;
}

int gg_device(const gg_ctx* ctx) {
  if (!ctx) return -1;
  return ctx->devs.empty() ? ctx->device : ctx->devs[0]->device;
}

static gg_status gg_sketch_device_one(gg_ctx* ctx, const uint32_t* d_words, uint64_t n_words,
                           const gg_run* runs, uint64_t n_runs, uint32_t n_genomes,
                           uint64_t* d_out, uint32_t* d_lens, void* stream) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  if ((n_runs && (!runs || !d_words)) || (n_genomes && (!d_out || !d_lens)))
    return fail(ctx, GG_ERR_INVALID_ARG, "gg_sketch_device: null buffer");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, GG_ERR_HIP, "hipSetDevice failed");
  hipStream_t st = (hipStream_t)stream;  // NULL = the default stream
  return sketch_core(ctx, d_words, n_words, runs, n_runs, n_genomes, d_out, d_lens, nullptr, st);
}

gg_status gg_sketch_device(gg_ctx* ctx, const uint32_t* d_words, uint64_t n_words,
                           const gg_run* runs, uint64_t n_runs, uint32_t n_genomes,
                           uint64_t* d_out, uint32_t* d_lens, void* stream) {
  gg_ctx* m = primary(ctx);
  const gg_status st = gg_sketch_device_one(m, d_words, n_words, runs, n_runs, n_genomes, d_out, d_lens, stream);
  if (st != GG_OK && m != ctx) ctx->err = m->err;
  return st;
}

uint64_t gg_pair_tiles(uint32_t n) {
  const uint64_t nb = (n + GG_PAIR_TILE - 1) / GG_PAIR_TILE;
  return nb * (nb + 1) / 2;
}

// First tile whose first pair index is >= target (pairs counted in tile
// enumeration order); nt when none.
static uint64_t tile_at_pair(uint32_t n, long double target) {
  const uint64_t nb = (n + GG_PAIR_TILE - 1) / GG_PAIR_TILE;
  uint64_t t = 0;
  long double acc = 0;
  for (uint64_t I = 0; I < nb; ++I) {
    const uint64_t ri = std::min<uint64_t>(GG_PAIR_TILE, n - I * GG_PAIR_TILE);
    for (uint64_t J = I; J < nb; ++J, ++t) {
      if (acc >= target) return t;
      const uint64_t cj = std::min<uint64_t>(GG_PAIR_TILE, n - J * GG_PAIR_TILE);
      acc += (I == J) ? (long double)(ri * (ri - 1) / 2) : (long double)(ri * cj);
    }
  }
  return t;
}

void gg_pair_partition(uint32_t n, uint32_t parts, uint32_t part, uint64_t* begin, uint64_t* end) {
  if (!begin || !end) return;
  const uint64_t nt = gg_pair_tiles(n);
  if (parts == 0 || part >= parts) {
    *begin = *end = nt;
    return;
  }
  const long double all = (long double)n * (long double)(n ? n - 1 : 0) / 2.0L;
  *begin = (part == 0) ? 0 : tile_at_pair(n, all * part / parts);
  *end = (part + 1 == parts) ? nt : tile_at_pair(n, all * (part + 1) / parts);
  if (*end < *begin) *end = *begin;
}

static gg_status gg_pairs_device_one(gg_ctx* ctx, const uint64_t* d_sketches, const uint32_t* d_lens,
                          uint32_t n, uint64_t tile_begin, uint64_t tile_end, float min_ani,
                          gg_pair* d_out, uint64_t out_cap, uint64_t* d_count, void* stream) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  if (n && (!d_sketches || !d_lens || !d_count || (out_cap && !d_out)))
    return fail(ctx, GG_ERR_INVALID_ARG, "gg_pairs_device: null buffer");
  if (std::isnan(min_ani)) return fail(ctx, GG_ERR_INVALID_ARG, "min_ani is NaN");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, GG_ERR_HIP, "hipSetDevice failed");
  hipStream_t st = (hipStream_t)stream;  // NULL = the default stream
  return pairs_core(ctx, d_sketches, d_lens, n, tile_begin, tile_end, min_ani, d_out, out_cap,
                    d_count, st);
}

gg_status gg_pairs_device(gg_ctx* ctx, const uint64_t* d_sketches, const uint32_t* d_lens,
                          uint32_t n, uint64_t tile_begin, uint64_t tile_end, float min_ani,
                          gg_pair* d_out, uint64_t out_cap, uint64_t* d_count, void* stream) {
  gg_ctx* m = primary(ctx);
  const gg_status st = gg_pairs_device_one(m, d_sketches, d_lens, n, tile_begin, tile_end, min_ani, d_out, out_cap, d_count, stream);
  if (st != GG_OK && m != ctx) ctx->err = m->err;
  return st;
}

double gg_ani_f64(uint32_t common, uint32_t total, int kmer_length) {
  return ani_f64(common, total, kmer_length);
}

float gg_ani_f32(uint32_t common, uint32_t total, int kmer_length) {
  return (float)ani_f64(common, total, kmer_length);
}

gg_status gg_parse_percentage(float value, float* fraction) {
  if (!fraction) return fail(nullptr, GG_ERR_INVALID_ARG, "null output");
  float p = value;
  if (p >= 1.0f && p <= 100.0f) {
    p /= 100.0f;
  } else if (!(p >= 0.0f && p <= 100.0f)) {
    char buf[96];
    snprintf(buf, sizeof buf, "Invalid percentage specified for --precluster-ani: '%g'", (double)value);
    return fail(nullptr, GG_ERR_INVALID_ARG, buf);
  }
  *fraction = p;
  return GG_OK;
}

void gg_free(void* p) { free(p); }

gg_status gg_timing_enable(gg_ctx* ctx, int on) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  for (gg_ctx* m : ctx->devs) gg_timing_enable(m, on);
  for (auto& t : ctx->timed) {
    (void)hipEventSynchronize(t.b);
    ctx->spare_events.push_back(t.a);
    ctx->spare_events.push_back(t.b);
  }
  ctx->timed.clear();
  ctx->timing = on != 0;
  return GG_OK;
}

gg_status gg_pair_paths(const gg_ctx* ctx, uint64_t* paths) {
  if (!ctx || !paths) return fail(nullptr, GG_ERR_INVALID_ARG, "gg_pair_paths: null argument");
  for (int i = 0; i < GG_PATH_COUNT; ++i) paths[i] = ctx->pair_paths[i];
  for (const gg_ctx* m : ctx->devs)
    for (int i = 0; i < GG_PATH_COUNT; ++i) paths[i] += m->pair_paths[i];
  return GG_OK;
}

gg_status gg_fallbacks(const gg_ctx* ctx, uint64_t* counts) {
  if (!ctx || !counts) return fail(nullptr, GG_ERR_INVALID_ARG, "gg_fallbacks: null argument");
  uint64_t paths[GG_PATH_COUNT];
  gg_pair_paths(ctx, paths);
  for (int i = 0; i < GG_FALLBACK_COUNT; ++i) counts[i] = ctx->fallbacks[i];
  for (const gg_ctx* m : ctx->devs)
    for (int i = 0; i < GG_FALLBACK_COUNT; ++i) counts[i] += m->fallbacks[i];
  counts[GG_FALLBACK_INDEX_TO_GATE] = paths[GG_PATH_INDEX_ABANDONED];
  counts[GG_FALLBACK_INDEX_FULL_SORT] = paths[GG_PATH_INDEX_FULL_SORT];
  return GG_OK;
}

gg_status gg_peer_links(const gg_ctx* ctx, int* links) {
  if (!ctx || !links) return fail(nullptr, GG_ERR_INVALID_ARG, "gg_peer_links: null argument");
  const size_t M = ctx->devs.empty() ? 1 : ctx->devs.size();
  for (size_t x = 0; x < M * M; ++x) links[x] = (M == 1 || x >= ctx->peer_direct.size()) ? 1 : ctx->peer_direct[x];
  return GG_OK;
}

gg_status gg_info_line(const gg_ctx* ctx, char* buf, size_t cap) {
  if (!ctx || !buf) return fail(nullptr, GG_ERR_INVALID_ARG, "gg_info_line: null argument");
  if (cap == 0) return GG_OK;
  std::string ords;
  if (ctx->devs.empty()) {
    ords = std::to_string(ctx->device);
  } else {
    for (size_t i = 0; i < ctx->devs.size(); ++i) ords += (i ? "," : "") + std::to_string(ctx->devs[i]->device);
  }
  uint64_t fb[GG_FALLBACK_COUNT];
  gg_fallbacks(ctx, fb);
  const size_t M = ctx->devs.empty() ? 1 : ctx->devs.size();
  uint64_t staged_links = 0;
  for (size_t x = 0; x < ctx->peer_direct.size(); ++x) staged_links += ctx->peer_direct[x] ? 0 : 1;
  uint64_t dev_batches = ctx->inflate_dev_batches;
  for (const gg_ctx* m : ctx->devs) dev_batches += m->inflate_dev_batches;
  char line[600];
  snprintf(line, sizeof line,
           "galahgpu: %zu device(s) [%s]; sketch %.1f ms, replicate %.2f ms, pairs %.2f ms, merge %.2f ms; "
           "fallbacks: index->gate %llu, index full sort %llu, host-staged peer copies %llu (links without peer "
           "access %llu), sketch retry passes %llu (set-mode genomes %llu), host-inflated batches %llu "
           "(device-inflated %llu)",
           M, ords.c_str(), ctx->phase_ms[GG_PHASE_SKETCH], ctx->phase_ms[GG_PHASE_REPLICATE],
           ctx->phase_ms[GG_PHASE_PAIRS], ctx->phase_ms[GG_PHASE_MERGE], (unsigned long long)fb[0],
           (unsigned long long)fb[1], (unsigned long long)fb[2], (unsigned long long)staged_links,
           (unsigned long long)fb[3], (unsigned long long)fb[5], (unsigned long long)fb[4],
           (unsigned long long)dev_batches);
  std::string out = line;
  // device inflate: batches planned again (gzip member boundaries found on
  // the device; full-size token areas after a tight one filled) and the
  // largest scratch one lane used for a batch
  uint64_t mplans = ctx->gz_member_plans, fplans = ctx->gz_full_plans, scr = ctx->gz_scratch_bytes;
  for (const gg_ctx* m : ctx->devs) {
    mplans += m->gz_member_plans;
    fplans += m->gz_full_plans;
    scr = std::max(scr, m->gz_scratch_bytes);
  }
  if (dev_batches) {
    snprintf(line, sizeof line, "; inflate replans: members %llu, full areas %llu; lane scratch %.0f MB",
             (unsigned long long)mplans, (unsigned long long)fplans, scr / 1e6);
    out += line;
  }
  // the index calls that went to the gate kernel because their member reads
  // (large clusters of near-identical genomes) outweighed its merges
  uint64_t costly = ctx->index_costly;
  for (const gg_ctx* m : ctx->devs) costly += m->index_costly;
  if (costly) {
    snprintf(line, sizeof line, "; index->gate by cost %llu", (unsigned long long)costly);
    out += line;
  }
  // device / pinned scratch buffers grown since the context was created
  // (and the wall time that took: hipFree waits for the device), its lanes'
  // included -- a call that grows one runs long
  uint64_t regrows = ctx->scratch_regrows;
  double regrow_ms = ctx->scratch_regrow_ms;
  auto add_lanes = [&](const gg_ctx* m) {
    for (const gg_ctx* l : m->lanes)
      if (l) {
        regrows += l->scratch_regrows;
        regrow_ms += l->scratch_regrow_ms;
      }
  };
  add_lanes(ctx);
  for (const gg_ctx* m : ctx->devs) {
    regrows += m->scratch_regrows;
    regrow_ms += m->scratch_regrow_ms;
    add_lanes(m);
  }
  snprintf(line, sizeof line, "; scratch regrows %llu (%.1f ms)", (unsigned long long)regrows, regrow_ms);
  out += line;
  if (ctx->devs.size() > 1) {  // (last) the device-inflated batches of each member
    out += " [";
    for (size_t i = 0; i < ctx->devs.size(); ++i)
      out += (i ? "," : "") + std::to_string(ctx->devs[i]->inflate_dev_batches);
    out += "]";
  }
  const size_t n = std::min(cap - 1, out.size());
  memcpy(buf, out.data(), n);
  buf[n] = 0;
  return GG_OK;
}

gg_status gg_timing_read(gg_ctx* ctx, int kernel, gg_kernel_stats* out) {
  if (!ctx || !out || kernel < 0 || kernel >= GG_KERNEL_COUNT)
    return fail(ctx, GG_ERR_INVALID_ARG, "gg_timing_read: bad argument");
  gg_kernel_stats s{0.0, 0, 0};
  for (gg_ctx* m : ctx->devs) {  // a multi-device context sums its members
    gg_kernel_stats x;
    const gg_status st = gg_timing_read(m, kernel, &x);
    if (st != GG_OK) return fail(ctx, st, m->err);
    s.ms += x.ms;
    s.launches += x.launches;
    s.work += x.work;
  }
  for (auto& t : ctx->timed) {
    if (t.kernel != kernel) continue;
    GG_HIP(ctx, hipEventSynchronize(t.b));
    float ms = 0.f;
    GG_HIP(ctx, hipEventElapsedTime(&ms, t.a, t.b));
    s.ms += ms;
    s.launches += 1;
    s.work += t.work;
  }
  *out = s;
  return GG_OK;
}

static gg_status gg_synth_clustered_device_one(gg_ctx* ctx, uint32_t first_genome, uint32_t n_genomes, uint32_t genome_len,
                                    uint32_t cluster_size, float max_sub_rate, uint64_t seed,
                                    uint32_t* d_words, gg_run* runs, void* stream) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  if (!d_words || !runs || genome_len % 16 || genome_len < (uint32_t)ctx->k || cluster_size == 0)
    return fail(ctx, GG_ERR_INVALID_ARG, "gg_synth_clustered_device: bad arguments");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, GG_ERR_HIP, "hipSetDevice failed");
  hipStream_t st = (hipStream_t)stream;  // NULL = the default stream
  GG_HIP(ctx, launch_synth(first_genome, n_genomes, genome_len, cluster_size, max_sub_rate, seed, d_words, st));
  for (uint32_t g = 0; g < n_genomes; ++g) runs[g] = gg_run{g, genome_len, (uint64_t)g * genome_len};
  return GG_OK;
}

gg_status gg_synth_clustered_device(gg_ctx* ctx, uint32_t first_genome, uint32_t n_genomes, uint32_t genome_len,
                                    uint32_t cluster_size, float max_sub_rate, uint64_t seed,
                                    uint32_t* d_words, gg_run* runs, void* stream) {
  gg_ctx* m = primary(ctx);
  const gg_status st = gg_synth_clustered_device_one(m, first_genome, n_genomes, genome_len, cluster_size, max_sub_rate, seed, d_words, runs, stream);
  if (st != GG_OK && m != ctx) ctx->err = m->err;
  return st;
}

static uint64_t splitmix_host(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

gg_status gg_synth_mixed_lengths(uint32_t first_genome, uint32_t n_genomes, uint32_t min_len, uint32_t max_len,
                                 uint32_t cluster_size, uint64_t seed, uint32_t* lens) {
  if ((n_genomes && !lens) || cluster_size == 0 || min_len < 64 || max_len < min_len)
    return fail(nullptr, GG_ERR_INVALID_ARG, "gg_synth_mixed_lengths: bad arguments");
  const double lo = std::log((double)min_len), hi = std::log((double)max_len);
  for (uint32_t i = 0; i < n_genomes; ++i) {
    const uint32_t cl = (first_genome + i) / cluster_size;
    const double u = (double)(splitmix_host(seed * 0x9E3779B97F4A7C15ull + cl) >> 11) * (1.0 / 9007199254740992.0);
    const uint32_t L = (uint32_t)std::exp(lo + u * (hi - lo));
    lens[i] = std::max<uint32_t>(64, std::min(max_len, L)) / 16 * 16;
  }
  return GG_OK;
}

static gg_status gg_synth_mixed_device_one(gg_ctx* ctx, uint32_t first_genome, uint32_t n_genomes, const uint32_t* lens,
                                uint32_t cluster_size, float max_sub_rate, double n_run_rate, uint64_t seed,
                                uint32_t* d_words, gg_run* runs, uint64_t runs_cap, uint64_t* n_runs, void* stream) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  if (!d_words || !lens || !n_runs || cluster_size == 0 || !(n_run_rate >= 0.0 && n_run_rate < 1.0))
    return fail(ctx, GG_ERR_INVALID_ARG, "gg_synth_mixed_device: bad arguments");
  for (uint32_t g = 0; g < n_genomes; ++g)
    if (lens[g] % 16 || lens[g] == 0) return fail(ctx, GG_ERR_INVALID_ARG, "genome lengths must be positive multiples of 16");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, GG_ERR_HIP, "hipSetDevice failed");
  hipStream_t st = (hipStream_t)stream;
  std::vector<uint64_t> woff(n_genomes + 1, 0);
  uint64_t max_words = 0;
  for (uint32_t g = 0; g < n_genomes; ++g) {
    woff[g + 1] = woff[g] + lens[g] / 16;
    max_words = std::max<uint64_t>(max_words, lens[g] / 16);
  }
  uint64_t* d_woff;
  GG_HIP(ctx, scratch_t(ctx, "synth_woff", n_genomes + 1, &d_woff));
  GG_HIP(ctx, hipMemcpyAsync(d_woff, woff.data(), (n_genomes + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  GG_HIP(ctx, launch_synth_mixed(first_genome, n_genomes, d_woff, max_words, cluster_size, max_sub_rate, seed, d_words, st));
  // N runs: geometric gaps (start probability n_run_rate per base), 1-64 bases
  uint64_t nr = 0;
  const uint32_t k = (uint32_t)ctx->k;
  for (uint32_t g = 0; g < n_genomes; ++g) {
    uint64_t state = splitmix_host(seed ^ 0x4E4E4E4Eull ^ ((uint64_t)(first_genome + g) << 20));
    auto next = [&]() { state = splitmix_host(state); return state; };
    const uint64_t L = lens[g], base0 = woff[g] * 16;
    uint64_t pos = 0;
    while (pos < L) {
      uint64_t run_end = L;
      if (n_run_rate > 0.0) {
        const double u = ((double)(next() >> 11) + 0.5) * (1.0 / 9007199254740992.0);
        const double gap = std::floor(std::log(u) / std::log1p(-n_run_rate));
        if (gap < (double)(L - pos)) run_end = pos + (uint64_t)gap;
      }
      if (run_end - pos >= k) {
        if (nr < runs_cap && runs) runs[nr] = gg_run{g, (uint32_t)(run_end - pos), base0 + pos};
        ++nr;
      }
      pos = run_end + (run_end < L ? 1 + next() % 64 : 0);
    }
  }
  *n_runs = nr;
  if (nr > runs_cap) return fail(ctx, GG_ERR_OUTPUT_FULL, "run buffer too small");
  return GG_OK;
}

gg_status gg_synth_mixed_device(gg_ctx* ctx, uint32_t first_genome, uint32_t n_genomes, const uint32_t* lens,
                                uint32_t cluster_size, float max_sub_rate, double n_run_rate, uint64_t seed,
                                uint32_t* d_words, gg_run* runs, uint64_t runs_cap, uint64_t* n_runs, void* stream) {
  gg_ctx* m = primary(ctx);
  const gg_status st = gg_synth_mixed_device_one(m, first_genome, n_genomes, lens, cluster_size, max_sub_rate, n_run_rate, seed, d_words, runs, runs_cap, n_runs, stream);
  if (st != GG_OK && m != ctx) ctx->err = m->err;
  return st;
}

}  // extern "C"
