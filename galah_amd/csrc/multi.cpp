// Multi-device orchestration of the finch precluster path and the entry
// points that use every device of a context (include/galahgpu.h).
//
// galah calls FinchPreclusterer::distances once, from one thread, for all
// genomes (src/clusterer.rs:36; src/finch.rs:47 sketches every file, :53-73
// compares every pair).  Inside that one call this library drives every
// device of the context with one host thread each:
//
//   1. sketch   genomes are dealt to the devices (files: in batches pulled
//               from a shared cursor as the host threads finish packing them;
//               device-resident shards: one shard per device); K1 writes each
//               genome's row into that device's full [n x s] sketch array
//   2. gather   every device copies the rows it did not sketch from their
//               owners (hipMemcpyPeerAsync: on an MI355X node every GPU has a
//               direct xGMI link to every other, so the copies from the seven
//               peers run on seven links at once; a ring all-gather would use
//               two of them)
//   3. pairs    device d runs K2 over part d of the upper-triangle tiles
//               (equal numbers of tile rows for the inverted index, which
//               indexes only the entries its rows may share; equal pair
//               counts, gg_pair_partition, for the gate kernel); passing
//               pairs come back sparse
//   4. merge    concatenate, sort by (i, j) (SortedPairGenomeDistanceCache
//               order), f32 ANI per pair (src/finch.rs:56-70)
//
// The result never depends on the device list: every pair is evaluated by
// exactly one device on identical sketch rows.
#include <algorithm>
#include <chrono>
#include <future>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <thread>

#include "context.hpp"

namespace gg {
namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

std::vector<gg_ctx*> members(gg_ctx* c) { return c->devs.empty() ? std::vector<gg_ctx*>{c} : c->devs; }

// f(index, member) on one host thread per member (member 0 on the calling
// thread), each bound to its member's device.  The lowest failing member's
// status is returned and its message copied to c (and to the calling
// thread's error slot: gg_thread_last_error is per thread).
template <class F>
gg_status on_members(gg_ctx* c, const std::vector<gg_ctx*>& ms, F&& f) {
  std::vector<gg_status> st(ms.size(), GG_OK);
  const std::function<void(size_t)> run = [&](size_t i) {
    if (hipSetDevice(ms[i]->device) != hipSuccess) {
      st[i] = fail(ms[i], GG_ERR_HIP, "hipSetDevice failed");
      return;
    }
    st[i] = f(i, ms[i]);
  };
  if (ms.size() == 1) {
    run(0);
  } else {
    if (!c->pool || c->pool->size() != ms.size()) c->pool.reset(new MemberPool(ms.size()));
    c->pool->run(run);
  }
  for (size_t i = 0; i < ms.size(); ++i)
    if (st[i] != GG_OK) {
      if (ms[i] != c) c->err = ms[i]->err;
      set_thread_error(c->err);
      return st[i];
    }
  return GG_OK;
}

// A member's full sketch array: rows [n x s] u64 and lens [n].
struct Rows {
  uint64_t* sk = nullptr;
  uint32_t* len = nullptr;
};

gg_status member_rows(gg_ctx* m, uint32_t n, Rows* r) {
  GG_HIP(m, scratch_t(m, "mg_sk", (size_t)std::max(n, 1u) * m->s, &r->sk));
  GG_HIP(m, scratch_t(m, "mg_len", std::max(n, 1u), &r->len));
  return GG_OK;
}

// A run of consecutive rows sketched by member `owner`.
struct RowSpan {
  uint32_t row0, rows, owner;
};

// Spans of the sorted row list `rows` (all sketched by `owner`).
void spans_of(std::vector<uint32_t>& rows, uint32_t owner, std::vector<RowSpan>& out) {
  std::sort(rows.begin(), rows.end());
  for (size_t a = 0; a < rows.size();) {
    size_t b = a + 1;
    while (b < rows.size() && rows[b] == rows[b - 1] + 1) ++b;
    out.push_back(RowSpan{rows[a], (uint32_t)(b - a), owner});
    a = b;
  }
}

// Member mi copies every span it does not own from the owner's array.  The
// copies from each owner go on a stream of their own: in one stream they
// would run one after the other, and each peer is a different xGMI link (at
// 8 devices, C3's 10 MB per peer, C4's 100 MB).  Nothing here waits on the
// host: the member's compute stream waits on each peer stream's event, so
// the host thread goes straight on to queue K2 (its table uploads and the
// index build are queued behind the copies, not behind a host barrier), and
// the copies' device time is read after the pairs phase (replicate_ms).
gg_status replicate(gg_ctx* m, size_t mi, const std::vector<gg_ctx*>& ms, const std::vector<Rows>& rows,
                    const std::vector<RowSpan>& spans, const std::vector<uint8_t>& direct) {
  const size_t s = m->s, M = ms.size();
  if (m->peer_streams.size() < M) m->peer_streams.resize(M, nullptr);
  if (m->rep_start.size() < M) {
    m->rep_start.resize(M, nullptr);
    m->rep_done.resize(M, nullptr);
  }
  m->rep_live.assign(M, 0);
  for (const RowSpan& sp : spans) {
    if (sp.owner == mi) continue;
    hipStream_t& ps = m->peer_streams[sp.owner];
    if (!ps) GG_HIP(m, hipStreamCreateWithFlags(&ps, hipStreamNonBlocking));
    if (!m->rep_live[sp.owner]) {
      if (!m->rep_start[sp.owner]) {
        GG_HIP(m, hipEventCreate(&m->rep_start[sp.owner]));
        GG_HIP(m, hipEventCreate(&m->rep_done[sp.owner]));
      }
      GG_HIP(m, hipEventRecord(m->rep_start[sp.owner], ps));
      m->rep_live[sp.owner] = 1;
    }
    const gg_ctx* o = ms[sp.owner];
    if (m->rep_live[sp.owner] == 1 && o->rows_ready) {  // (the owner's rows are final on its device)
      GG_HIP(m, hipStreamWaitEvent(ps, o->rows_ready, 0));
      m->rep_live[sp.owner] = 2;
    }
    uint64_t* dsk = rows[mi].sk + (size_t)sp.row0 * s;
    const uint64_t* ssk = rows[sp.owner].sk + (size_t)sp.row0 * s;
    uint32_t* dl = rows[mi].len + sp.row0;
    const uint32_t* sl = rows[sp.owner].len + sp.row0;
    // one call for every member pair, same device included (a peer copy with
    // src == dst device is legal), so the one-GPU tests run the node's code
    GG_HIP(m, hipMemcpyPeerAsync(dsk, m->device, ssk, o->device, (size_t)sp.rows * s * sizeof(uint64_t), ps));
    GG_HIP(m, hipMemcpyPeerAsync(dl, m->device, sl, o->device, sp.rows * sizeof(uint32_t), ps));
    if (!direct.empty() && !direct[mi * M + sp.owner]) m->fallbacks[GG_FALLBACK_PEER_STAGED] += 2;
  }
  for (size_t o = 0; o < M; ++o)
    if (m->rep_live[o]) {
      GG_HIP(m, hipEventRecord(m->rep_done[o], m->peer_streams[o]));
      GG_HIP(m, hipStreamWaitEvent(m->stream, m->rep_done[o], 0));
    }
  return GG_OK;
}

// Device time of member m's last replication (first copy started to last
// copy done, per peer stream; the largest), in ms.  After the member's
// stream has been synchronised.
double replicate_ms(gg_ctx* m) {
  double worst = 0.0;
  for (size_t o = 0; o < m->rep_live.size(); ++o) {
    if (!m->rep_live[o]) continue;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, m->rep_start[o], m->rep_done[o]) == hipSuccess) worst = std::max(worst, (double)ms);
  }
  return worst;
}

bool pair_ij_less(const gg_pair& x, const gg_pair& y) { return x.i != y.i ? x.i < y.i : x.j < y.j; }

// Steps 2-4 over rows resident on every member: gather, pairs, merge.
gg_status gather_pairs_merge(gg_ctx* c, const std::vector<gg_ctx*>& ms, const std::vector<Rows>& rows,
                             const std::vector<RowSpan>& spans, uint32_t n, float min_ani,
                             std::vector<gg_pair>& res) {
  const size_t M = ms.size();
  auto t0 = Clock::now();
  std::vector<std::vector<gg_pair>> part(M);
  // Which tiles each member evaluates.  When K2 takes the inverted index
  // (min_ani > 0: a pair needs a shared hash), a member's cost is mostly
  // indexing the entries its rows may share (pairs_index.hip's row-range
  // index), so the members get equal numbers of tile rows; otherwise (the
  // gate kernel) equal numbers of pairs (gg_pair_partition).
  const uint64_t nb = (n + GG_PAIR_TILE - 1) / GG_PAIR_TILE;
  const bool by_rows = M > 1 && min_ani > 0.0f && !(min_ani != min_ani);
  auto row_tile = [&](uint64_t I) { return I * nb - I * (I - 1) / 2; };  // first tile of tile row I
  gg_status st = on_members(c, ms, [&](size_t i, gg_ctx* m) {
    uint64_t tb = 0, te = 0;
    if (by_rows) {
      tb = row_tile(nb * i / M);
      te = row_tile(nb * (i + 1) / M);
    } else {
      gg_pair_partition(n, (uint32_t)M, (uint32_t)i, &tb, &te);
    }
    // (replication queued first: K2's kernels wait for the copies on the device)
    if (M > 1 && !spans.empty()) {
      const gg_status r = replicate(m, i, ms, rows, spans, c->peer_direct);
      if (r != GG_OK) return r;
    }
    return pairs_range_to_host(m, rows[i].sk, rows[i].len, n, tb, te, min_ani, part[i], m->stream);
  });
  if (st != GG_OK) return st;
  c->phase_ms[GG_PHASE_PAIRS] = ms_since(t0);
  // replicate: the copies' device time (they ran inside the pairs phase's
  // wall time, ahead of each member's K2 kernels)
  double rep = 0.0;
  if (M > 1 && !spans.empty())
    for (gg_ctx* m : ms) rep = std::max(rep, replicate_ms(m));
  c->phase_ms[GG_PHASE_REPLICATE] = rep;
  t0 = Clock::now();
  // every member's part comes in (i, j) order (pairs_range_to_host: sorted
  // on the device, or few and sorted by the member's thread), then merged:
  // SortedPairGenomeDistanceCache order
  res.clear();
  // members given whole tile rows (the inverted index) hold disjoint,
  // increasing row ranges: their parts are already in order one after the
  // other and are concatenated; otherwise (a tile row split between members
  // by the gate kernel's partition) merged
  size_t total = 0;
  bool ordered = true;
  const gg_pair* last = nullptr;
  for (const auto& p : part) {
    if (p.empty()) continue;
    total += p.size();
    if (last && !pair_ij_less(*last, p.front())) ordered = false;
    last = &p.back();
  }
  if (ordered) {
    for (auto& p : part) {
      if (p.empty()) continue;
      if (res.empty() && p.size() == total) {
        res.swap(p);
        break;
      }
      if (res.empty()) res.reserve(total);
      res.insert(res.end(), p.begin(), p.end());
    }
  } else {
    for (auto& p : part) {
      if (res.empty()) {
        res.swap(p);
        continue;
      }
      std::vector<gg_pair> merged(res.size() + p.size());
      std::merge(res.begin(), res.end(), p.begin(), p.end(), merged.begin(), pair_ij_less);
      res.swap(merged);
    }
  }
  c->phase_ms[GG_PHASE_MERGE] = ms_since(t0);
  return GG_OK;
}

gg_status pairs_with_ani(gg_ctx* c, const std::vector<gg_pair>& res, gg_pair** pairs, float** ani,
                         uint64_t* n_out) {
  auto t0 = Clock::now();
  const size_t m = res.size();
  // the caller's arrays are filled in place (no staging vector for the ANI)
  *pairs = copy_out(res);
  *ani = (float*)malloc(std::max<size_t>(m, 1) * sizeof(float));
  if (!*pairs || !*ani) {
    free(*pairs);
    free(*ani);
    *pairs = nullptr;
    *ani = nullptr;
    return fail(c, GG_ERR_OUT_OF_MEMORY, "out of host memory");
  }
  float* a = *ani;
  // f64 log per pair (src/finch.rs:56): on several threads for large outputs
  const int T = m >= (1u << 16) ? (int)std::min<size_t>(16, std::max(1, ingest_threads(c->host_threads))) : 1;
  std::vector<std::thread> th;
  auto work = [&](int t) {
    for (size_t i = m * t / T; i < m * (t + 1) / T; ++i) a[i] = gg_ani_f32(res[i].common, res[i].total, c->k);
  };
  for (int t = 1; t < T; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  *n_out = m;
  c->phase_ms[GG_PHASE_MERGE] += ms_since(t0);
  return GG_OK;
}

// ---------------------------------------------------------------------------
// Streamed file ingest (the body of finch's sketch_files, src/finch.rs:47).
// ---------------------------------------------------------------------------
constexpr uint32_t kBatchGenomes = 32;          // genomes per K1 batch
constexpr uint64_t kBatchWords = 64ull << 20;   // or 1 Gbases of packed words, whichever first
constexpr uint64_t kBatchText = 1ull << 30;     // raw (device-parsed) batches: 1 GiB of FASTA text
// memcpy on up to T threads (staging copies of a batch into pinned memory:
// one thread moves ~10 GB/s, a batch of FASTA text is up to 1 GiB)
void parallel_copy(void* dst, const void* src, size_t bytes, int T) {
  constexpr size_t kPer = 8u << 20;
  T = (int)std::max<size_t>(1, std::min<size_t>((size_t)T, bytes / kPer));
  if (T <= 1) {
    if (bytes) memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> th;
  auto part = [&](int t) {
    const size_t a = bytes * t / T, b = bytes * (t + 1) / T;
    memcpy((uint8_t*)dst + a, (const uint8_t*)src + a, b - a);
  };
  for (int t = 1; t < T; ++t) th.emplace_back(part, t);
  part(0);
  for (auto& x : th) x.join();
}

// Where FASTA text becomes 2-bit runs: on the host threads (pack.cpp)
// unless GALAHGPU_PARSE=device (parse.hip; the host threads then only read
// and gunzip).  Measured on the MI355X box (profiles/r02_device_parse/, 128
// x 3 Mbp gzip files): 16 threads 0.039 s host vs 0.087 s device, 1 thread
// 0.494 vs 0.482 s -- the SSE packer runs ~2.5 Gbases/s per thread, gzip
// decode dominates, and the device path moves 4x the bytes (text, not 2-bit
// words) through host memory and PCIe, so the host packer stays the default.
bool device_parse() {
  const char* e = getenv("GALAHGPU_PARSE");
  return e && strcmp(e, "device") == 0;
}

}  // namespace

// One batch of FASTA text, already in device memory (d_text, files at
// foff[0..nf]), parsed on the device: 2-bit words into *d_words (scratch of
// m), runs of >= k bases (genome = file index in the batch, base = packed
// position) into runs.  Synchronises m->stream.
gg_status parse_raw_batch(gg_ctx* m, const uint8_t* d_text, const std::vector<uint64_t>& foff, uint32_t** d_words,
                          uint64_t* n_words, std::vector<gg_run>& runs) {
  hipStream_t st = m->stream;
  const uint32_t nf = (uint32_t)foff.size() - 1;
  const uint64_t bb = parse_block_bytes();
  static const bool dbg = [] {
    const char* e = getenv("GALAHGPU_INFLATE_DEBUG");
    return e && *e == '1';
  }();
  const auto t0 = Clock::now();
  auto stamp = [&](const char* what) {
    if (dbg) fprintf(stderr, "[parse] %-12s %8.3f ms\n", what, ms_since(t0));
  };
  // The block tables and every per-block array the host scans live in one
  // pinned buffer (pageable ones made each copy a staged, blocking one):
  // bstart, bend, h, h2, hr, hf, boff (nb u64 each), then bfile (nb u32).
  uint64_t n_blk = 0;
  for (uint32_t f = 0; f < nf; ++f) n_blk += (foff[f + 1] - foff[f] + bb - 1) / bb;
  const uint32_t nb = (uint32_t)n_blk;
  const size_t NBH = std::max(nb, 1u);
  uint64_t* hbuf;
  GG_HIP(m, host_scratch_t(m, "parse_host", 7 * NBH + (NBH + 1) / 2, &hbuf));
  uint64_t* bstart = hbuf;
  uint64_t* bend = hbuf + NBH;
  uint64_t* h = hbuf + 2 * NBH;
  uint64_t* h2 = hbuf + 3 * NBH;
  uint64_t* hr = hbuf + 4 * NBH;
  uint64_t* hf = hbuf + 5 * NBH;
  uint64_t* boff = hbuf + 6 * NBH;
  uint32_t* bfile = reinterpret_cast<uint32_t*>(hbuf + 7 * NBH);
  {
    uint32_t b = 0;
    for (uint32_t f = 0; f < nf; ++f)
      for (uint64_t x = foff[f]; x < foff[f + 1]; x += bb, ++b) {
        bfile[b] = f;
        bstart[b] = x;
        bend[b] = std::min(foff[f + 1], x + bb);
      }
  }
  runs.clear();
  ParseLaunch p{};
  p.raw = d_text;
  p.n_bytes = foff[nf];
  p.n_blocks = nb;
  uint64_t* blk;  // 11 arrays of nb u64: start, end, nl, pre_nl, bases, last, pre_last, runs, base_off, run_off, first
  GG_HIP(m, scratch_t(m, "parse_blk", (size_t)std::max(nb, 1u) * 11 + nf + 1, &blk));
  uint32_t* d_bfile;
  GG_HIP(m, scratch_t(m, "parse_bfile", std::max(nb, 1u), &d_bfile));
  uint64_t* d_fstart = blk + (size_t)std::max(nb, 1u) * 11;
  const size_t NB = std::max(nb, 1u);
  p.blk_file = d_bfile;
  p.blk_start = blk;
  p.blk_end = blk + NB;
  p.blk_nl = blk + 2 * NB;
  p.pre_nl = blk + 3 * NB;
  p.blk_bases = blk + 4 * NB;
  p.blk_last = blk + 5 * NB;
  p.pre_last = blk + 6 * NB;
  p.blk_runs = blk + 7 * NB;
  p.base_off = blk + 8 * NB;
  p.run_off = blk + 9 * NB;
  p.blk_first = blk + 10 * NB;
  p.file_start = d_fstart;
  if (nb) {
    GG_HIP(m, hipMemcpyAsync(d_bfile, bfile, nb * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    GG_HIP(m, hipMemcpyAsync((void*)p.blk_start, bstart, nb * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    GG_HIP(m, hipMemcpyAsync((void*)p.blk_end, bend, nb * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  }
  GG_HIP(m, hipMemcpyAsync(d_fstart, foff.data(), (nf + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  // pass 1 -> line-start prefix (last '\n' index + 1 before each block)
  std::vector<uint64_t> fbases(nf, 0), gofs(nf + 1, 0);
  uint64_t n_starts = 0;
  if (nb) {
    GG_HIP(m, timed_launch(m, GG_KERNEL_PARSE, foff[nf], st, [&] { return parse_batch_pass(1, p, st); }));
    GG_HIP(m, hipMemcpyAsync(h, p.blk_nl, nb * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    GG_HIP(m, hipStreamSynchronize(st));
    stamp("pass 1");
    uint64_t acc = 0;
    for (uint32_t b = 0; b < nb; ++b) {
      const uint64_t x = h[b];
      h[b] = acc;
      acc = std::max(acc, x);
    }
    GG_HIP(m, hipMemcpyAsync((void*)p.pre_nl, h, nb * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    // pass 2 -> bases, run starts (as if no base before), first byte a base?, last non-dropped byte
    GG_HIP(m, timed_launch(m, GG_KERNEL_PARSE, 0, st, [&] { return parse_batch_pass(2, p, st); }));
    GG_HIP(m, hipMemcpyAsync(h, p.blk_bases, nb * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    GG_HIP(m, hipMemcpyAsync(h2, p.blk_last, nb * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    GG_HIP(m, hipMemcpyAsync(hr, p.blk_runs, nb * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    GG_HIP(m, hipMemcpyAsync(hf, p.blk_first, nb * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    GG_HIP(m, hipStreamSynchronize(st));
    stamp("pass 2");
    for (uint32_t b = 0; b < nb; ++b) fbases[bfile[b]] += h[b];
    for (uint32_t f = 0; f < nf; ++f) gofs[f + 1] = gofs[f] + (fbases[f] + 15) / 16 * 16;  // genomes on words
    uint64_t cur = 0;
    uint32_t cf = ~0u;
    for (uint32_t b = 0; b < nb; ++b) {
      if (bfile[b] != cf) {
        cf = bfile[b];
        cur = gofs[cf];
      }
      boff[b] = cur;
      cur += h[b];
    }
    GG_HIP(m, hipMemcpyAsync((void*)p.base_off, boff, nb * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    // the last non-dropped byte before each block; a block whose first
    // non-dropped byte is a base continues the run of a block before it (in
    // its file) that ended in a base
    uint64_t last = 0;
    for (uint32_t b = 0; b < nb; ++b) {
      const uint64_t x = h2[b];
      h2[b] = last;
      if (x) last = x;
      const uint64_t fs = foff[bfile[b]];
      const bool prev_base = h2[b] && ((h2[b] >> 2) - 1) >= fs && (h2[b] & 3u) == 0;
      const uint64_t runs = hr[b] - (prev_base && hf[b] ? 1 : 0);
      hr[b] = n_starts;
      n_starts += runs;
    }
    GG_HIP(m, hipMemcpyAsync((void*)p.pre_last, h2, nb * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    GG_HIP(m, hipMemcpyAsync((void*)p.run_off, hr, nb * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  }
  const uint64_t total = gofs[nf];
  *n_words = total / 16;
  uint64_t* starts;
  GG_HIP(m, scratch_t(m, "parse_starts", std::max<uint64_t>(n_starts, 1), &starts));
  GG_HIP(m, scratch_t(m, "stage_words", std::max<uint64_t>(*n_words, 1), d_words));
  p.starts = starts;
  p.n_words = *n_words;
  p.words = *d_words;
  uint64_t* hs;
  GG_HIP(m, host_scratch_t(m, "parse_starts_host", std::max<uint64_t>(n_starts, 1), &hs));
  if (nb) {
    if (*n_words) GG_HIP(m, hipMemsetAsync(*d_words, 0, *n_words * sizeof(uint32_t), st));
    GG_HIP(m, timed_launch(m, GG_KERNEL_PARSE, 0, st, [&] { return parse_batch_pass(3, p, st); }));
    if (n_starts) GG_HIP(m, hipMemcpyAsync(hs, starts, n_starts * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    GG_HIP(m, hipStreamSynchronize(st));
    stamp("pass 3");
  }
  // runs: consecutive starts of one genome; a genome's last run ends at its
  // last base; keep runs of >= k bases
  uint32_t f = 0;
  for (uint64_t r = 0; r < n_starts; ++r) {
    const uint64_t a = hs[r];
    while (f + 1 < nf && a >= gofs[f + 1]) ++f;
    const uint64_t gend = gofs[f] + fbases[f];
    const uint64_t e = (r + 1 < n_starts && hs[r + 1] < gend) ? hs[r + 1] : gend;
    if (e - a >= (uint64_t)m->k) runs.push_back(gg_run{f, (uint32_t)(e - a), a});
  }
  stamp("runs");
  return GG_OK;
}

namespace {

// Sketches of paths[0..n) into every member's full array (rows[i]); spans
// receives the rows each member sketched.  Genomes with a valid entry in
// cache_dir are read from it (every member receives those rows from the
// host); the others are packed on the host threads and sketched in batches
// (each batch: pinned staging -> H2D -> K1 with a row map), and stored in
// the cache.  host_out / host_lens (optional) receive the rows.
gg_status sketch_files_members(gg_ctx* c, const std::vector<gg_ctx*>& ms, const char* const* paths, uint32_t n,
                               const char* cache_dir, std::vector<Rows>& rows, std::vector<RowSpan>& spans,
                               uint64_t* host_out, uint32_t* host_lens, uint32_t* n_cached) {
  const size_t M = ms.size();
  const uint32_t s = c->s;
  rows.assign(M, Rows{});
  spans.clear();
  if (n_cached) *n_cached = 0;
  // cache lookups (host), in chunks of paths; the rows of the entries found
  // are kept compact, in row order (host memory grows with the hits, not
  // with n * s)
  std::vector<uint8_t> hit(n, 0);
  std::vector<uint64_t> hit_rows;  // [hits * s]
  std::vector<uint32_t> hit_lens;  // [n]
  if (cache_dir) {
    hit_lens.assign(n, 0);
    constexpr uint32_t kChunk = 1024;
    std::vector<uint64_t> chunk((size_t)std::min(n, kChunk) * s);
    for (uint32_t i0 = 0; i0 < n; i0 += kChunk) {
      const uint32_t cn = std::min(kChunk, n - i0);
      cache_load_many(cache_dir, paths + i0, cn, c->k, s, c->seed, chunk.data(), hit_lens.data() + i0,
                      hit.data() + i0);
      for (uint32_t i = 0; i < cn; ++i)
        if (hit[i0 + i]) hit_rows.insert(hit_rows.end(), chunk.begin() + (size_t)i * s, chunk.begin() + (size_t)(i + 1) * s);
    }
  }
  std::vector<const char*> miss;
  std::vector<uint32_t> miss_at;
  for (uint32_t i = 0; i < n; ++i)
    if (!hit[i]) {
      miss.push_back(paths[i]);
      miss_at.push_back(i);
    }
  if (n_cached) *n_cached = n - (uint32_t)miss.size();
  std::vector<RowSpan> hit_spans;
  std::vector<uint64_t> hit_first;  // per span: its first row's index among the hits
  {
    std::vector<uint32_t> h;
    for (uint32_t i = 0; i < n; ++i)
      if (hit[i]) h.push_back(i);
    spans_of(h, 0, hit_spans);
    uint64_t before = 0;
    for (const RowSpan& sp : hit_spans) {
      hit_first.push_back(before);
      before += sp.rows;
    }
  }
  const uint32_t nm = (uint32_t)miss.size();
  // in-flight packed genomes: ~2 batches per member, at least 1 GiB
  const uint64_t budget = std::max<uint64_t>(1ull << 30, 2ull * M * kBatchWords * sizeof(uint32_t));
  const bool gz_dev = gz_device_list(miss.data(), nm);
  const bool raw = device_parse();
  // host threads per member: the host threads shared among the members
  const int copy_threads = std::max(1, std::min(16, ingest_threads(c->host_threads)) / (int)M);
  // gzip lists: ingest_gz.cpp's stagers read the files; otherwise the
  // PackStream workers read (and pack) them
  std::unique_ptr<PackStream> streamp;
  if (!gz_dev) streamp.reset(new PackStream(miss.data(), nm, c->k, c->host_threads, budget, cache_dir != nullptr, raw));
  GzClaims claims;
  claims.paths = miss.data();
  claims.row_of = miss_at.data();
  claims.n = nm;
  claims.cache_dir = cache_dir;
  claims.stagers = (uint32_t)(M * gz_lane_count());
  std::mutex cursor_mu;
  uint32_t cursor = 0;
  bool stop = false;        // a member failed: the others take no more batches
  bool file_error = false;  // ... because a file did not read or parse
  int first_fail = -1;      // member whose failure came first (not a file)
  std::vector<std::vector<uint32_t>> owned(M);

  auto body = [&](size_t mi, gg_ctx* m) -> gg_status {
    Rows& r = rows[mi];
    gg_status ms_ = member_rows(m, n, &r);
    if (ms_ != GG_OK) return ms_;
    GG_HIP(m, hipMemsetAsync(r.sk, 0, (size_t)n * s * sizeof(uint64_t), m->stream));
    GG_HIP(m, hipMemsetAsync(r.len, 0, (size_t)n * sizeof(uint32_t), m->stream));
    for (size_t hs = 0; hs < hit_spans.size(); ++hs) {  // cached rows straight from the host
      const RowSpan& sp = hit_spans[hs];
      GG_HIP(m, hipMemcpyAsync(r.sk + (size_t)sp.row0 * s, hit_rows.data() + hit_first[hs] * s,
                               (size_t)sp.rows * s * sizeof(uint64_t), hipMemcpyHostToDevice, m->stream));
      GG_HIP(m, hipMemcpyAsync(r.len + sp.row0, hit_lens.data() + sp.row0, sp.rows * sizeof(uint32_t),
                               hipMemcpyHostToDevice, m->stream));
    }
    GG_HIP(m, hipStreamSynchronize(m->stream));
    if (gz_dev) {
      const gg_status gs = gz_member_ingest(m, claims, r.sk, r.len, copy_threads, owned[mi]);
      return gs != GG_OK ? gs : mark_rows_ready(m);
    }
    PackStream& stream = *streamp;
    std::vector<gg_run> runs;
    std::vector<uint32_t> row_of;
    std::vector<uint64_t> out_rows;
    std::vector<uint32_t> out_lens;
    for (;;) {
      uint32_t b0, b1;
      {
        std::lock_guard<std::mutex> lk(cursor_mu);
        if (stop || cursor >= nm) break;
        b0 = cursor;
        b1 = std::min(nm, b0 + kBatchGenomes);
        cursor = b1;
      }
      // assemble the batch in the pinned staging buffer
      runs.clear();
      row_of.clear();
      uint64_t nw = 0;
      uint32_t g = 0;
      uint32_t* d_words = nullptr;
      if (raw) {  // FASTA text -> device parser
        std::vector<uint64_t> foff(1, 0);
        for (uint32_t i = b0; i < b1; ++i) {
          const std::vector<uint8_t>* tx;
          std::string err;
          const gg_status gs = stream.get_raw(i, &tx, &err);
          if (gs != GG_OK) {
            std::lock_guard<std::mutex> lk(cursor_mu);
            if (!stop) file_error = true;
            return fail(m, gs, err);
          }
          const uint64_t at = foff.back();
          const uint64_t padded = (tx->size() + 15) / 16 * 16;  // next file on a 16-byte boundary
          const size_t need = at + padded;
          if (need > m->pinned_bytes) {  // grow, keeping what is staged
            std::vector<uint8_t> keep((const uint8_t*)m->pinned, (const uint8_t*)m->pinned + at);
            void* stage;
            GG_HIP(m, pinned(m, std::max(need, std::min<size_t>(2 * need, kBatchText * 2)), &stage));
            if (at) memcpy(stage, keep.data(), at);
          }
          parallel_copy((uint8_t*)m->pinned + at, tx->data(), tx->size(), copy_threads);
          memset((uint8_t*)m->pinned + at + tx->size(), '\n', padded - tx->size());  // (parses as nothing)
          foff.push_back(at + padded);
          row_of.push_back(miss_at[i]);
          stream.release(i);
          if (foff.back() >= kBatchText && i + 1 < b1) {  // large genomes: cut the batch here
            std::lock_guard<std::mutex> lk(cursor_mu);
            if (cursor == b1) {
              cursor = i + 1;
              b1 = i + 1;
            }
          }
        }
        uint8_t* d_text;
        GG_HIP(m, scratch_t(m, "stage_text", std::max<uint64_t>(foff.back(), 1), &d_text));
        if (foff.back())
          GG_HIP(m, hipMemcpyAsync(d_text, m->pinned, foff.back(), hipMemcpyHostToDevice, m->stream));
        const gg_status ps = parse_raw_batch(m, d_text, foff, &d_words, &nw, runs);
        if (ps != GG_OK) return ps;
      }
      for (uint32_t i = b0; !raw && i < b1; ++i, ++g) {
        const std::vector<uint32_t>* w;
        const std::vector<gg_run>* rr;
        std::string err;
        const gg_status gs = stream.get(i, &w, &rr, &err);
        if (gs != GG_OK) {
          std::lock_guard<std::mutex> lk(cursor_mu);
          if (!stop) file_error = true;  // (an abort caused by another member is not a file error)
          return fail(m, gs, err);
        }
        void* stage;
        const size_t need = (nw + w->size()) * sizeof(uint32_t);
        if (need > m->pinned_bytes) {  // grow, keeping what is staged
          std::vector<uint32_t> keep((const uint32_t*)m->pinned, (const uint32_t*)m->pinned + nw);
          GG_HIP(m, pinned(m, std::max(need, std::min<size_t>(2 * need, kBatchWords * sizeof(uint32_t) * 2)), &stage));
          if (nw) memcpy(stage, keep.data(), nw * sizeof(uint32_t));
        }
        stage = m->pinned;
        if (!w->empty()) memcpy((uint32_t*)stage + nw, w->data(), w->size() * sizeof(uint32_t));
        for (const gg_run& x : *rr) runs.push_back(gg_run{g, x.len, x.base + nw * 16});
        row_of.push_back(miss_at[i]);
        nw += w->size();
        stream.release(i);
        if (nw >= kBatchWords && i + 1 < b1) {  // large genomes: cut the batch here, return the rest
          std::lock_guard<std::mutex> lk(cursor_mu);
          if (cursor == b1) {
            cursor = i + 1;
            b1 = i + 1;
          }
        }
      }
      const uint32_t ng = b1 - b0;
      uint32_t* d_row_of;
      if (!raw) {
        GG_HIP(m, scratch_t(m, "stage_words", std::max<uint64_t>(nw, 1), &d_words));
        if (nw) GG_HIP(m, hipMemcpyAsync(d_words, m->pinned, nw * sizeof(uint32_t), hipMemcpyHostToDevice, m->stream));
      }
      GG_HIP(m, scratch_t(m, "row_of", ng, &d_row_of));
      GG_HIP(m, hipMemcpyAsync(d_row_of, row_of.data(), ng * sizeof(uint32_t), hipMemcpyHostToDevice, m->stream));
      gg_status ks = sketch_core(m, d_words, nw, runs.data(), runs.size(), ng, r.sk, r.len, d_row_of, m->stream);
      if (ks != GG_OK) return ks;
      owned[mi].insert(owned[mi].end(), row_of.begin(), row_of.end());
      if (cache_dir) {  // store the new sketches (a failed store fails nothing)
        out_rows.resize((size_t)ng * s);
        out_lens.resize(ng);
        for (uint32_t q = 0; q < ng; ++q) {
          GG_HIP(m, hipMemcpyAsync(&out_rows[(size_t)q * s], r.sk + (size_t)row_of[q] * s, s * sizeof(uint64_t),
                                   hipMemcpyDeviceToHost, m->stream));
          GG_HIP(m, hipMemcpyAsync(&out_lens[q], r.len + row_of[q], sizeof(uint32_t), hipMemcpyDeviceToHost, m->stream));
        }
        GG_HIP(m, hipStreamSynchronize(m->stream));
        for (uint32_t q = 0; q < ng; ++q) {
          const FileStamp fs = stream.stamp(b0 + q);
          (void)cache_store(cache_dir, miss[b0 + q], c->k, s, c->seed, &out_rows[(size_t)q * s], out_lens[q], &fs);
        }
      }
    }
    return mark_rows_ready(m);
  };
  gg_status st = on_members(c, ms, [&](size_t mi, gg_ctx* m) -> gg_status {
    const gg_status r = body(mi, m);
    if (r != GG_OK) {
      {
        std::lock_guard<std::mutex> lk(cursor_mu);
        if (!file_error && first_fail < 0) first_fail = (int)mi;
        stop = true;
      }
      claims.halt();
      if (streamp) streamp->abort();  // wakes members waiting for genomes nobody will pack now
    }
    return r;
  });
  if (gz_dev) {  // a file that did not read or decode: the lowest failing index, as a serial reader meets it
    gz_settle_errors(claims);
    if (claims.err_idx != UINT32_MAX) return fail(c, claims.err_st, claims.err_msg);
  }
  if (file_error) {  // report the lowest failing file, as a serial reader would meet it
    std::string err;
    const gg_status fs = streamp->first_error(&err);
    if (fs != GG_OK) return fail(c, fs, err);
  }
  if (first_fail >= 0 && ms[first_fail]->err.size()) {
    const gg_status fs = st != GG_OK ? st : GG_ERR_INTERNAL;
    return fail(c, fs, ms[first_fail]->err);
  }
  if (st != GG_OK) return st;
  for (size_t mi = 0; mi < M; ++mi) spans_of(owned[mi], (uint32_t)mi, spans);
  if (host_out || host_lens) {
    // the caller wants the rows: every row is on its owner (or, cached, everywhere)
    std::vector<RowSpan> all = spans;
    all.insert(all.end(), hit_spans.begin(), hit_spans.end());
    for (const RowSpan& sp : all) {
      gg_ctx* o = ms[sp.owner];
      if (hipSetDevice(o->device) != hipSuccess) return fail(c, GG_ERR_HIP, "hipSetDevice failed");
      if (host_out)
        GG_HIP(c, hipMemcpyAsync(host_out + (size_t)sp.row0 * s, rows[sp.owner].sk + (size_t)sp.row0 * s,
                                 (size_t)sp.rows * s * sizeof(uint64_t), hipMemcpyDeviceToHost, o->stream));
      if (host_lens)
        GG_HIP(c, hipMemcpyAsync(host_lens + sp.row0, rows[sp.owner].len + sp.row0, sp.rows * sizeof(uint32_t),
                                 hipMemcpyDeviceToHost, o->stream));
    }
    for (gg_ctx* o : ms) {
      if (hipSetDevice(o->device) != hipSuccess) return fail(c, GG_ERR_HIP, "hipSetDevice failed");
      GG_HIP(c, hipStreamSynchronize(o->stream));
    }
  }
  return GG_OK;
}

// Direct access from device a to device b's memory: true when a == b (a
// device always reaches its own memory) or when the peer link is enabled.
// (GALAHGPU_TEST_NO_PEER=1, tests: every pair of distinct members reports
// no peer access, so one GPU runs the host-staged branch of replicate.)
bool test_no_peer() {
  const char* e = getenv("GALAHGPU_TEST_NO_PEER");
  return e && *e == '1';
}
bool enable_peer(int a, int b) {
  if (a == b) return true;
  int can = 0;
  if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can || hipSetDevice(a) != hipSuccess) return false;
  const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
  return e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
}

// Contiguous genome ranges with about equal k-mer counts, one per member.
std::vector<uint32_t> balance_genomes(const gg_run* runs, uint64_t n_runs, uint32_t n_genomes, int k, size_t M) {
  std::vector<uint64_t> per(n_genomes + 1, 0);
  for (uint64_t r = 0; r < n_runs; ++r) per[runs[r].genome + 1] += (uint64_t)runs[r].len - (uint64_t)k + 1;
  for (uint32_t g = 0; g < n_genomes; ++g) per[g + 1] += per[g];
  std::vector<uint32_t> cut(M + 1, n_genomes);
  cut[0] = 0;
  for (size_t m = 1; m < M; ++m) {
    const long double target = (long double)per[n_genomes] * m / M;
    uint32_t g = (uint32_t)(std::lower_bound(per.begin(), per.end(), (uint64_t)target) - per.begin());
    cut[m] = std::max(cut[m - 1], std::min(g, n_genomes));
  }
  return cut;
}

}  // namespace
}  // namespace gg

using namespace gg;

extern "C" {

gg_ctx* gg_create_multi(int kmer_length, uint32_t sketch_size, uint64_t hash_seed, const int* devices,
                        uint32_t n_devices, gg_status* status) {
  gg_status dummy;
  if (!status) status = &dummy;
  std::vector<int> list;
  if (devices) {
    list.assign(devices, devices + n_devices);
  } else {
    int vis = 0;
    if (hipGetDeviceCount(&vis) != hipSuccess || vis == 0) {
      *status = fail(nullptr, GG_ERR_NO_DEVICE, "no HIP device visible (libgalahgpu has no CPU path)");
      return nullptr;
    }
    const char* env = getenv("GALAHGPU_DEVICES");
    if (n_devices == 0 && env && *env) {
      for (const char* p = env; *p;) {
        char* end = nullptr;
        const long v = strtol(p, &end, 10);
        if (end == p) {
          *status = fail(nullptr, GG_ERR_INVALID_ARG, std::string("GALAHGPU_DEVICES: not a device list: ") + env);
          return nullptr;
        }
        list.push_back((int)v);
        p = (*end == ',') ? end + 1 : end;
      }
    } else {
      const int want = n_devices ? (int)n_devices : vis;
      if (want > vis) {
        *status = fail(nullptr, GG_ERR_NO_DEVICE, "fewer devices visible than requested");
        return nullptr;
      }
      for (int d = 0; d < want; ++d) list.push_back(d);
    }
  }
  if (list.empty()) {
    *status = fail(nullptr, GG_ERR_INVALID_ARG, "empty device list");
    return nullptr;
  }
  if (list.size() == 1) return gg_create(kmer_length, sketch_size, hash_seed, list[0], status);
  gg_ctx* c = new (std::nothrow) gg_ctx();
  if (!c) {
    *status = fail(nullptr, GG_ERR_OUT_OF_MEMORY, "out of host memory");
    return nullptr;
  }
  c->k = kmer_length;
  c->s = sketch_size;
  c->seed = hash_seed;
  for (int d : list) {
    if (d < 0) {
      gg_destroy(c);
      *status = fail(nullptr, GG_ERR_INVALID_ARG, "negative device ordinal in the device list");
      return nullptr;
    }
    gg_ctx* m = gg_create(kmer_length, sketch_size, hash_seed, d, status);
    if (!m) {
      const std::string e = gg_thread_last_error();
      gg_destroy(c);
      set_thread_error(e);
      return nullptr;
    }
    c->devs.push_back(m);
  }
  c->device = list[0];
  // direct xGMI peer access between every pair of members (a copy between
  // devices without it is staged through the host); the same loop runs for
  // repeated ordinals, where it is a no-op
  const size_t M = list.size();
  c->peer_direct.assign(M * M, 0);
  for (size_t a = 0; a < M; ++a)
    for (size_t b = 0; b < M; ++b)
      c->peer_direct[a * M + b] = (a == b || !test_no_peer()) && enable_peer(list[a], list[b]) ? 1 : 0;
  (void)hipSetDevice(list[0]);
  *status = GG_OK;
  return c;
}

uint32_t gg_device_count(const gg_ctx* ctx) {
  if (!ctx) return 0;
  return ctx->devs.empty() ? 1u : (uint32_t)ctx->devs.size();
}

gg_ctx* gg_device_ctx(gg_ctx* ctx, uint32_t index) {
  if (!ctx) return nullptr;
  if (ctx->devs.empty()) return index == 0 ? ctx : nullptr;
  return index < ctx->devs.size() ? ctx->devs[index] : nullptr;
}

gg_status gg_set_host_threads(gg_ctx* ctx, int n_threads) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  ctx->host_threads = n_threads > 0 ? n_threads : 0;
  for (gg_ctx* m : ctx->devs) m->host_threads = ctx->host_threads;
  return GG_OK;
}

gg_status gg_phase_times(const gg_ctx* ctx, double* ms) {
  if (!ctx || !ms) return fail(nullptr, GG_ERR_INVALID_ARG, "gg_phase_times: null argument");
  for (int i = 0; i < GG_PHASE_COUNT; ++i) ms[i] = ctx->phase_ms[i];
  return GG_OK;
}

gg_status gg_sketch(gg_ctx* ctx, const gg_packed* packed, uint64_t* out_hashes, uint32_t* out_lens) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  if (!packed || (packed->n_genomes && (!out_hashes || !out_lens)))
    return fail(ctx, GG_ERR_INVALID_ARG, "gg_sketch: null buffer");
  const uint32_t ng = packed->n_genomes;
  if (ng == 0) return GG_OK;
  const std::vector<gg_ctx*> ms = members(ctx);
  const size_t s = ctx->s;
  // the run table is split by genome below, before sketch_core sees it
  gg_status vs = check_runs(ctx, packed->runs, packed->n_runs, ng, packed->n_words);
  if (vs != GG_OK) return vs;
  if (packed->n_runs && !packed->words) return fail(ctx, GG_ERR_INVALID_ARG, "gg_sketch: null packed words");
  // contiguous genome ranges of about equal k-mer counts; each member copies
  // the packed words its range spans and sketches it
  const std::vector<uint32_t> cut = balance_genomes(packed->runs, packed->n_runs, ng, ctx->k, ms.size());
  return on_members(ctx, ms, [&](size_t mi, gg_ctx* m) -> gg_status {
    const uint32_t g0 = cut[mi], g1 = cut[mi + 1];
    if (g0 >= g1) return GG_OK;
    const gg_run* rall = packed->runs;
    const gg_run* rend = packed->runs + packed->n_runs;
    const gg_run* rb = std::lower_bound(rall, rend, g0,
                                        [](const gg_run& r, uint32_t g) { return r.genome < g; });
    const gg_run* re = std::lower_bound(rb, rend, g1,
                                        [](const gg_run& r, uint32_t g) { return r.genome < g; });
    uint64_t w0 = 0, w1 = 0;
    if (rb != re) {  // the words the range's runs touch (bases need not rise with the genome)
      w0 = ~0ull;
      for (const gg_run* r = rb; r != re; ++r) {
        w0 = std::min<uint64_t>(w0, r->base / 16);
        w1 = std::max<uint64_t>(w1, (r->base + r->len + 15) / 16);
      }
    }
    std::vector<gg_run> runs(rb, re);
    for (gg_run& r : runs) {
      r.genome -= g0;
      r.base -= w0 * 16;
    }
    uint32_t* d_words;
    uint64_t* d_out;
    uint32_t* d_lens;
    const uint32_t nl = g1 - g0;
    GG_HIP(m, scratch_t(m, "in_words", std::max<uint64_t>(w1 - w0, 1), &d_words));
    GG_HIP(m, scratch_t(m, "sk_out", (size_t)nl * s, &d_out));
    GG_HIP(m, scratch_t(m, "sk_lens", nl, &d_lens));
    if (w1 > w0)
      GG_HIP(m, hipMemcpyAsync(d_words, packed->words + w0, (w1 - w0) * sizeof(uint32_t), hipMemcpyHostToDevice,
                               m->stream));
    GG_HIP(m, hipMemsetAsync(d_out, 0, (size_t)nl * s * sizeof(uint64_t), m->stream));
    gg_status st = sketch_core(m, d_words, w1 - w0, runs.data(), runs.size(), nl, d_out, d_lens, nullptr, m->stream);
    if (st != GG_OK) return st;
    GG_HIP(m, hipMemcpyAsync(out_hashes + (size_t)g0 * s, d_out, (size_t)nl * s * sizeof(uint64_t),
                             hipMemcpyDeviceToHost, m->stream));
    GG_HIP(m, hipMemcpyAsync(out_lens + g0, d_lens, nl * sizeof(uint32_t), hipMemcpyDeviceToHost, m->stream));
    GG_HIP(m, hipStreamSynchronize(m->stream));
    return GG_OK;
  });
}

gg_status gg_pairs(gg_ctx* ctx, const uint64_t* sketches, const uint32_t* lens, uint32_t n, float min_ani,
                   gg_pair** out, uint64_t* n_out) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  if (!out || !n_out || (n && (!sketches || !lens))) return fail(ctx, GG_ERR_INVALID_ARG, "gg_pairs: null buffer");
  if (std::isnan(min_ani)) return fail(ctx, GG_ERR_INVALID_ARG, "min_ani is NaN");
  *out = nullptr;
  *n_out = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (lens[i] > ctx->s) return fail(ctx, GG_ERR_INVALID_ARG, "sketch longer than sketch_size");
  std::vector<gg_pair> res;
  if (n >= 2) {
    const std::vector<gg_ctx*> ms = members(ctx);
    std::vector<Rows> rows(ms.size());
    gg_status st = on_members(ctx, ms, [&](size_t mi, gg_ctx* m) -> gg_status {
      gg_status r = member_rows(m, n, &rows[mi]);
      if (r != GG_OK) return r;
      GG_HIP(m, hipMemcpyAsync(rows[mi].sk, sketches, (size_t)n * m->s * sizeof(uint64_t), hipMemcpyHostToDevice,
                               m->stream));
      GG_HIP(m, hipMemcpyAsync(rows[mi].len, lens, n * sizeof(uint32_t), hipMemcpyHostToDevice, m->stream));
      GG_HIP(m, hipStreamSynchronize(m->stream));
      return GG_OK;
    });
    if (st != GG_OK) return st;
    // every member holds every row: nothing to replicate
    st = gather_pairs_merge(ctx, ms, rows, {}, n, min_ani, res);
    if (st != GG_OK) return st;
  }
  *out = copy_out(res);
  if (!*out) return fail(ctx, GG_ERR_OUT_OF_MEMORY, "out of host memory");
  *n_out = res.size();
  return GG_OK;
}

gg_status gg_sketch_files(gg_ctx* ctx, const char* const* paths, uint32_t n_paths, const char* cache_dir,
                          uint64_t* out_hashes, uint32_t* out_lens, uint32_t* n_cached) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  if (n_paths && (!paths || !out_hashes || !out_lens))
    return fail(ctx, GG_ERR_INVALID_ARG, "gg_sketch_files: null argument");
  if (n_cached) *n_cached = 0;
  if (n_paths == 0) return GG_OK;
  const std::vector<gg_ctx*> ms = members(ctx);
  std::vector<Rows> rows;
  std::vector<RowSpan> spans;
  return sketch_files_members(ctx, ms, paths, n_paths, cache_dir, rows, spans, out_hashes, out_lens, n_cached);
}

gg_status gg_precluster_files_cached(gg_ctx* ctx, const char* const* paths, uint32_t n_paths, float min_ani,
                                     const char* cache_dir, gg_pair** pairs, float** ani, uint64_t* n_out,
                                     uint32_t* n_cached) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  if (!pairs || !ani || !n_out || (n_paths && !paths))
    return fail(ctx, GG_ERR_INVALID_ARG, "gg_precluster_files: null argument");
  if (std::isnan(min_ani)) return fail(ctx, GG_ERR_INVALID_ARG, "min_ani is NaN");
  *pairs = nullptr;
  *ani = nullptr;
  *n_out = 0;
  if (n_cached) *n_cached = 0;
  for (double& x : ctx->phase_ms) x = 0.0;
  const std::vector<gg_ctx*> ms = members(ctx);
  std::vector<Rows> rows;
  std::vector<RowSpan> spans;
  std::vector<gg_pair> res;
  auto t0 = Clock::now();
  // every file is read and sketched, even a lone one: a file that does not
  // parse fails the call as finch's sketch_files does (src/finch.rs:50)
  gg_status st = sketch_files_members(ctx, ms, paths, n_paths, cache_dir, rows, spans, nullptr, nullptr, n_cached);
  if (st != GG_OK) return st;
  ctx->phase_ms[GG_PHASE_SKETCH] = ms_since(t0);
  if (n_paths >= 2) {
    st = gather_pairs_merge(ctx, ms, rows, spans, n_paths, min_ani, res);
    if (st != GG_OK) return st;
  }
  return pairs_with_ani(ctx, res, pairs, ani, n_out);
}

gg_status gg_precluster_files(gg_ctx* ctx, const char* const* paths, uint32_t n_paths, float min_ani,
                              gg_pair** pairs, float** ani, uint64_t* n_out) {
  return gg_precluster_files_cached(ctx, paths, n_paths, min_ani, nullptr, pairs, ani, n_out, nullptr);
}

gg_status gg_precluster_files_each(gg_ctx* ctx, const char* const* paths, uint32_t n_paths, float min_ani,
                                   const char* cache_dir, gg_pair_sink sink, void* user, gg_pair** pairs,
                                   float** ani, uint64_t* n_out, uint32_t* n_cached) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  if (!sink || !pairs || !ani || !n_out || (n_paths && !paths))
    return fail(ctx, GG_ERR_INVALID_ARG, "gg_precluster_files_each: null argument");
  if (std::isnan(min_ani)) return fail(ctx, GG_ERR_INVALID_ARG, "min_ani is NaN");
  *pairs = nullptr;
  *ani = nullptr;
  *n_out = 0;
  if (n_cached) *n_cached = 0;
  for (double& x : ctx->phase_ms) x = 0.0;
  const std::vector<gg_ctx*> ms = members(ctx);
  std::vector<Rows> rows;
  std::vector<RowSpan> spans;
  std::vector<gg_pair> res;
  auto t0 = Clock::now();
  gg_status st = sketch_files_members(ctx, ms, paths, n_paths, cache_dir, rows, spans, nullptr, nullptr, n_cached);
  if (st != GG_OK) return st;
  ctx->phase_ms[GG_PHASE_SKETCH] = ms_since(t0);
  if (n_paths >= 2) {
    // the passing pairs as gg_precluster_files finds them (the index K2);
    // afterwards every member holds every row
    st = gather_pairs_merge(ctx, ms, rows, spans, n_paths, min_ani, res);
    if (st != GG_OK) return st;
    // every compared pair (src/finch.rs:53-68), min_ani 0 (the gate kernel
    // emits all of them), on member 0 in blocks of whole tile rows of at
    // most ~kEachPairs pairs, each sorted by (i, j): memory stays bounded by
    // a block whatever N is
    uint64_t kEachPairs = 1ull << 22;
    if (const char* e = getenv("GALAHGPU_EACH_PAIRS"))  // (tests: smaller blocks)
      if (atoll(e) > 0) kEachPairs = (uint64_t)atoll(e);
    gg_ctx* m = ms[0];
    if (hipSetDevice(m->device) != hipSuccess) return fail(ctx, GG_ERR_HIP, "hipSetDevice failed");
    const uint64_t n = n_paths, nb = (n + GG_PAIR_TILE - 1) / GG_PAIR_TILE;
    auto row_tile = [&](uint64_t I) { return I * nb - I * (I - 1) / 2; };  // first tile of tile row I
    std::vector<gg_pair> blk;
    for (uint64_t a = 0; a < nb;) {
      uint64_t b = a, cnt = 0;
      do {  // tile row b: rows [64 b, 64 b + 64) against every later genome
        const uint64_t r0 = b * GG_PAIR_TILE, r1 = std::min(n, r0 + GG_PAIR_TILE);
        for (uint64_t i = r0; i < r1; ++i) cnt += n - 1 - i;
        ++b;
      } while (b < nb && cnt < kEachPairs);
      blk.clear();
      st = pairs_range_to_host(m, rows[0].sk, rows[0].len, n_paths, row_tile(a), row_tile(b), 0.0f, blk, m->stream);
      if (st != GG_OK) {
        if (m != ctx) ctx->err = m->err;
        return st;
      }
      if (sink(user, blk.data(), blk.size()) != 0)
        return fail(ctx, GG_ERR_CANCELLED, "gg_precluster_files_each: the pair sink stopped the call");
      a = b;
    }
  }
  return pairs_with_ani(ctx, res, pairs, ani, n_out);
}

gg_status gg_precluster_shards(gg_ctx* ctx, const gg_shard* shards, float min_ani, gg_pair** pairs, float** ani,
                               uint64_t* n_out) {
  if (!ctx) return fail(nullptr, GG_ERR_INVALID_ARG, "null context");
  if (!shards || !pairs || !ani || !n_out) return fail(ctx, GG_ERR_INVALID_ARG, "gg_precluster_shards: null argument");
  if (std::isnan(min_ani)) return fail(ctx, GG_ERR_INVALID_ARG, "min_ani is NaN");
  *pairs = nullptr;
  *ani = nullptr;
  *n_out = 0;
  for (double& x : ctx->phase_ms) x = 0.0;
  const std::vector<gg_ctx*> ms = members(ctx);
  const size_t M = ms.size();
  std::vector<uint32_t> off(M + 1, 0);
  for (size_t i = 0; i < M; ++i) {
    if (shards[i].n_runs && (!shards[i].runs || !shards[i].d_words))
      return fail(ctx, GG_ERR_INVALID_ARG, "gg_precluster_shards: null shard buffer");
    if ((uint64_t)off[i] + shards[i].n_genomes > 0xFFFFFFFFull)
      return fail(ctx, GG_ERR_INVALID_ARG, "gg_precluster_shards: too many genomes");
    off[i + 1] = off[i] + shards[i].n_genomes;
  }
  const uint32_t n = off[M];
  std::vector<Rows> rows(M);
  std::vector<RowSpan> spans;
  for (size_t i = 0; i < M; ++i)
    if (shards[i].n_genomes) spans.push_back(RowSpan{off[i], shards[i].n_genomes, (uint32_t)i});
  auto t0 = Clock::now();
  gg_status st = on_members(ctx, ms, [&](size_t mi, gg_ctx* m) -> gg_status {
    gg_status r = member_rows(m, n, &rows[mi]);
    if (r != GG_OK) return r;
    const gg_shard& sh = shards[mi];
    if (sh.n_genomes == 0) return GG_OK;
    // K1 writes the shard's rows at their global offset
    const gg_status ks = sketch_core(m, sh.d_words, sh.n_words, sh.runs, sh.n_runs, sh.n_genomes,
                                     rows[mi].sk + (size_t)off[mi] * m->s, rows[mi].len + off[mi], nullptr, m->stream);
    return ks != GG_OK ? ks : mark_rows_ready(m);
  });
  if (st != GG_OK) return st;
  ctx->phase_ms[GG_PHASE_SKETCH] = ms_since(t0);
  std::vector<gg_pair> res;
  if (n >= 2) {
    st = gather_pairs_merge(ctx, ms, rows, spans, n, min_ani, res);
    if (st != GG_OK) return st;
  }
  return pairs_with_ani(ctx, res, pairs, ani, n_out);
}

}  // extern "C"
