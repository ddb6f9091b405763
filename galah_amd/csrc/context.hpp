// The context behind the C ABI (gg_ctx) and the single-device building
// blocks the entry points are made of (api.cpp), shared with the
// multi-device orchestration (multi.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gg_internal.hpp"

// One host thread per member of a multi-device context beyond the first
// (member 0 runs on the calling thread), kept for the context's life: a
// distances() call hands work to the members several times (sketch,
// replicate, pairs), and starting 7 threads each time cost ~0.5 ms per call
// at 8 devices, where a C3 step is ~7 ms.
class MemberPool {
 public:
  explicit MemberPool(size_t n) {
    for (size_t i = 1; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
  }
  ~MemberPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  size_t size() const { return th_.size() + 1; }
  // f(i) for every member i, member 0 on the calling thread; returns when all are done
  void run(const std::function<void(size_t)>& f) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &f;
      pending_ = th_.size();
      ++gen_;
    }
    cv_.notify_all();
    f(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void loop(size_t i) {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
      if (quit_) return;
      seen = gen_;
      const std::function<void(size_t)>* f = job_;
      lk.unlock();
      (*f)(i);
      lk.lock();
      if (--pending_ == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t)>* job_ = nullptr;
  size_t pending_ = 0;
  uint64_t gen_ = 0;
  bool quit_ = false;
};

// A context is either ONE device (devs empty: the fields below drive it) or
// a multi-device context whose members devs[i] are single-device contexts
// (one per entry of the device list; the same ordinal may appear more than
// once, each entry then being its own shard with its own stream).
struct gg_ctx {
  int k = 21;
  uint32_t s = 1000;
  uint64_t seed = 0;
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  // grow-only device scratch, keyed by purpose
  std::map<std::string, std::pair<void*, size_t>> scratch;
  // K1's candidate sets ("table" scratch) known empty, with their flags
  // clear, over [0, clean_table_bytes) of clean_table: the finalize kernel
  // leaves every set it reads empty, so only a new or grown buffer is cleared
  const void* clean_table = nullptr;
  size_t clean_table_bytes = 0;
  // grow-only pinned host staging buffer (streamed ingest)
  void* pinned = nullptr;
  size_t pinned_bytes = 0;
  // device-inflate staging slots (ingest_gz.cpp GzStager): batch N is inflated
  // from one while N + 1 is staged into the other by a helper thread, which
  // touches only its slot (grow-only pinned and device buffers, its stream)
  struct GzSlot {
    uint8_t* host = nullptr;      // (mapped: host_dev is its device address)
    uint8_t* host_dev = nullptr;
    size_t host_cap = 0;
    uint8_t* dev = nullptr;
    size_t dev_cap = 0;
    hipStream_t st = nullptr;
  };
  GzSlot gz_slot[2];
  // grow-only pinned host buffers keyed by purpose (small read-backs: one
  // DMA instead of a staged copy of pageable memory, ~35 us each)
  std::map<std::string, std::pair<void*, size_t>> host_scratch;
  // cached cmin table
  float cmin_key = -1.0f;
  std::vector<uint32_t> cmin_host;
  // per-kernel timing (gg_timing_enable)
  struct Timed {
    int kernel;
    hipEvent_t a, b;
    uint64_t work;
  };
  std::vector<gg::PairSeg> seg_host;
  std::vector<uint64_t> sstart_host;
  int pairs_kernel = 0;  // GALAHGPU_PAIRS_KERNEL: 0 auto, 1 table, 2 merge, 3 gate, 4 index
  std::vector<uint32_t> sufmin_host;
  bool timing = false;
  std::vector<Timed> timed;
  std::vector<hipEvent_t> spare_events;
  // multi-device context: the members (owned) and their host threads
  std::vector<gg_ctx*> devs;
  // helper contexts of this device (owned; created on first use, kept for
  // the context's life): the device-inflate ingest runs several batches at
  // once, each processing lane on its own stream with its own scratch
  // (ingest_gz.cpp); lanes[0] is unused (lane 0 is this context)
  std::vector<gg_ctx*> lanes;
  std::unique_ptr<MemberPool> pool;
  // a member's copy streams, one per peer it gathers rows from (created on
  // first use), so the copies from different peers run at once
  std::vector<hipStream_t> peer_streams;
  uint64_t pair_paths[GG_PATH_COUNT] = {};  // gg_pair_paths
  // of the index calls abandoned for the gate kernel (GG_PATH_INDEX_ABANDONED),
  // those whose member reads outweighed the gate kernel's merges (gg_info_line)
  uint64_t index_costly = 0;
  // gg_fallbacks (the two index entries are read from pair_paths)
  uint64_t fallbacks[GG_FALLBACK_COUNT] = {};
  uint64_t inflate_dev_batches = 0;  // gzip batches inflated on the device (gg_info_line)
  // device-inflate plans beyond a batch's first: member boundaries found by
  // the decode (files of several gzip members), full-size token areas after
  // a tight one filled (gg_info_line)
  uint64_t gz_member_plans = 0, gz_full_plans = 0;
  // the largest inflate scratch of a batch on this lane (tokens, sub-span
  // areas, val, text), bytes: the per-lane footprint the info line reports
  uint64_t gz_scratch_bytes = 0;
  // scratch / host-scratch buffers regrown (and the wall ms it took), gg_info_line
  uint64_t scratch_regrows = 0;
  double scratch_regrow_ms = 0;
  // a device scratch buffer that grows is allocated for this many times the
  // size asked (an ingest batch smaller than the largest the call may stage:
  // its buffers sized for that one at once, so that no later batch regrows
  // them -- a regrowth's hipFree waits for the whole device)
  double scratch_hint = 1.0;
  // multi-device context: [a * M + b] = 1 when member a reaches member b's
  // memory directly (same device, or peer access enabled), gg_peer_links
  std::vector<uint8_t> peer_direct;
  // a member's replication events, per peer: copies started / done (device
  // time of the copies, read after the pairs phase) and whether they are live
  std::vector<hipEvent_t> rep_start, rep_done;
  std::vector<char> rep_live;
  // recorded on `stream` when this member's rows of the call are final
  // (sketch phase done): the other members' replication copies wait on it
  hipEvent_t rows_ready = nullptr;
  hipStream_t copy_stream = nullptr;  // run-table uploads beside work on `stream` (sketch_core)
  hipEvent_t copy_done = nullptr;
  // host threads for file ingest (<= 0: gg_pack_files' default)
  int host_threads = 0;
  // wall-clock phases of the last fused call (GG_PHASE_*)
  double phase_ms[GG_PHASE_COUNT] = {0};
};

namespace gg {

// The member that single-device entry points use on a multi-device context.
inline gg_ctx* primary(gg_ctx* c) { return c && !c->devs.empty() ? c->devs[0] : c; }

gg_status fail(gg_ctx* c, gg_status st, const std::string& msg);
gg_status hip_fail(gg_ctx* c, hipError_t e, const char* what);

#define GG_HIP(ctx, expr)                                        \
  do {                                                           \
    hipError_t _e = (expr);                                      \
    if (_e != hipSuccess) return ::gg::hip_fail((ctx), _e, #expr); \
  } while (0)

// Grow-only device scratch buffer owned by the context.
hipError_t scratch(gg_ctx* c, const char* key, size_t bytes, void** out);
template <typename T>
hipError_t scratch_t(gg_ctx* c, const char* key, size_t count, T** out) {
  void* p = nullptr;
  hipError_t e = scratch(c, key, count * sizeof(T), &p);
  *out = (T*)p;
  return e;
}
// Grow-only pinned host buffer of the context (contents not preserved).
hipError_t pinned(gg_ctx* c, size_t bytes, void** out);
// Grow-only pinned host buffer keyed by purpose (contents not preserved).
hipError_t host_scratch(gg_ctx* c, const char* key, size_t bytes, void** out);
template <typename T>
hipError_t host_scratch_t(gg_ctx* c, const char* key, size_t count, T** out) {
  void* p = nullptr;
  hipError_t e = host_scratch(c, key, count * sizeof(T), &p);
  *out = static_cast<T*>(p);
  return e;
}

// The run-table checks sketch_core applies (genome < n_genomes and
// non-decreasing, len >= k, base + len <= 16 n_words), for callers that
// read the table before sketch_core does (gg_sketch splits it by genome).
gg_status check_runs(gg_ctx* c, const gg_run* runs, uint64_t n_runs, uint32_t n_genomes, uint64_t n_words);
// K1 over device-resident packed words; runs are host metadata with genome
// indices in [0, n_genomes).  Row g of d_out / entry g of d_lens receive
// genome g, or genome g goes to row d_row_of[g] when d_row_of (device, n_genomes
// entries) is given.  Synchronises st.
gg_status sketch_core(gg_ctx* c, const uint32_t* d_words, uint64_t n_words, const gg_run* runs,
                      uint64_t n_runs, uint32_t n_genomes, uint64_t* d_out, uint32_t* d_lens,
                      const uint32_t* d_row_of, hipStream_t st);
// K2 over tiles [tb, te) of n device sketches; appends to d_out / *d_count.
gg_status pairs_core(gg_ctx* c, const uint64_t* d_sk, const uint32_t* d_lens, uint32_t n,
                     uint64_t tb, uint64_t te, float min_ani, gg_pair* d_out, uint64_t cap,
                     uint64_t* d_count, hipStream_t st);
// K2 over tiles [tb, te), passing pairs appended to res, the appended part
// in (i, j) order.
constexpr uint64_t kDeviceSortPairs = 4096;  // pairs_range_to_host sorts this many or more on the device
gg_status pairs_range_to_host(gg_ctx* c, const uint64_t* d_sk, const uint32_t* d_lens, uint32_t n,
                              uint64_t tb, uint64_t te, float min_ani, std::vector<gg_pair>& res,
                              hipStream_t st);

// A batch of files inflated on m's device (inflate_host.cpp): h_in (pinned,
// in_bytes) holds files[f]'s bytes; *d_text receives the batch's FASTA text,
// file f at foff[f] (16-byte aligned, gaps '\n').  *ok = false (status GG_OK)
// when the device path does not take the batch: the caller decodes it on the
// host.  d_in: the batch already queued to the device on m->stream (at least
// in_bytes + kInflatePad bytes; nullptr: inflate_batch uploads h_in).
// Synchronises m->stream.
constexpr uint64_t kInflatePad = 4096;  // device bytes past a batch's last file (readers run past its end)
gg_status inflate_batch(gg_ctx* m, const uint8_t* h_in, uint64_t in_bytes, const std::vector<InflateFile>& files,
                        uint8_t** d_text, std::vector<uint64_t>& foff, bool* ok, uint8_t* d_in = nullptr);

// One batch of FASTA text already in device memory (d_text, file f at
// foff[f]) parsed on the device: 2-bit words into *d_words (scratch of m),
// runs of >= k bases (genome = file index in the batch) into runs.
// Synchronises m->stream.  (multi.cpp)
gg_status parse_raw_batch(gg_ctx* m, const uint8_t* d_text, const std::vector<uint64_t>& foff, uint32_t** d_words,
                          uint64_t* n_words, std::vector<gg_run>& runs);

// A timing event of c (a spare one, else a new one; nullptr on failure).
hipEvent_t take_event(gg_ctx* c);
// Runs `launch` (which enqueues one kernel on st); when timing is enabled
// brackets it with events recorded on the same stream (gg_timing_read).
template <typename F>
hipError_t timed_launch(gg_ctx* c, int kernel, uint64_t work, hipStream_t st, F&& launch) {
  if (!c->timing) return launch();
  hipEvent_t a = take_event(c), b = take_event(c);
  if (!a || !b) return hipErrorOutOfMemory;
  hipError_t e = hipEventRecord(a, st);
  if (e != hipSuccess) return e;
  e = launch();
  if (e != hipSuccess) return e;
  e = hipEventRecord(b, st);
  if (e != hipSuccess) return e;
  c->timed.push_back(gg_ctx::Timed{kernel, a, b, work});
  return hipSuccess;
}

// Records m->rows_ready on m->stream (after the member's sketching).
gg_status mark_rows_ready(gg_ctx* m);

// Helper context i >= 1 of single-device context m: the same device, k, s
// and seed, its own stream and scratch (api.cpp; owned by m).
gg_ctx* lane_ctx(gg_ctx* m, size_t i);

// The file list of one device-inflate ingest call, shared by every member
// and lane (ingest_gz.cpp).  Files are claimed one at a time, so each batch
// is cut at its size limits whatever the number of stagers; a claimed file
// that does not fit its batch is given back and claimed again first.
struct GzClaims {
  const char* const* paths = nullptr;  // the files to sketch (not found in the cache)
  const uint32_t* row_of = nullptr;    // their rows in the call's sketch array
  uint32_t n = 0;
  const char* cache_dir = nullptr;     // new sketches stored there (files stamped before they are read)
  std::mutex mu;
  uint32_t cursor = 0;
  std::vector<uint32_t> back;  // claimed, given back
  std::vector<uint32_t> abandoned;  // placed in a batch that was dropped undecoded
  uint32_t batches = 0;        // batches begun (the first ones are cut smaller)
  // the tail of the list cut into equal batches, a multiple of the stagers
  // (members x lanes), so that they finish together instead of the last
  // lane running a full batch alone
  uint32_t stagers = 1;
  uint64_t seen_files = 0, seen_bytes = 0;  // files staged so far, their bytes
  uint32_t tail_cap = 0;                    // files per batch from the tail on (0: not there yet)
  bool stop = false;           // no more claims: a failure
  // the failing file with the lowest index (a file that did not read, or
  // did not decode or parse on the host): the call's error, as a serial
  // reader meets it
  uint32_t err_idx = UINT32_MAX;
  gg_status err_st = GG_OK;
  std::string err_msg;
  bool claim(uint32_t* i);
  void give_back(uint32_t i);
  void abandon(const std::vector<uint32_t>& idx);
  void file_error(uint32_t i, gg_status st, const std::string& msg);
  void halt();
};
// Inflate lanes per device (GALAHGPU_GZ_LANES, default 2).
int gz_lane_count();
// Member m's share of the list: inflated, parsed and sketched on m's device
// by several lanes at once, rows into d_sk / d_len (m's [n x s] arrays);
// the rows sketched are appended to owned.  host_threads: the host threads
// this member may use (staging reads, host decodes).
gg_status gz_member_ingest(gg_ctx* m, GzClaims& cl, uint64_t* d_sk, uint32_t* d_len, int host_threads,
                           std::vector<uint32_t>& owned);
// After a file error: files given back (never read) below the failing index
// are read on the host, so the lowest failing index is reported.
void gz_settle_errors(GzClaims& cl);
// Whether a file list takes the device inflate: GALAHGPU_INFLATE=device /
// host, else when one of its first files is gzip (by its magic bytes).
bool gz_device_list(const char* const* paths, uint32_t n);

template <typename T>
T* copy_out(const std::vector<T>& v) {
  T* p = (T*)malloc(std::max<size_t>(v.size(), 1) * sizeof(T));
  if (p && !v.empty()) memcpy(p, v.data(), v.size() * sizeof(T));
  return p;
}

}  // namespace gg
