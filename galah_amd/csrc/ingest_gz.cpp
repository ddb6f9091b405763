// Device-inflate ingest of a gzip file list: the body of finch's
// sketch_files (src/finch.rs:47) for the .fna.gz paths galah hands
// distances().  The files go to the GPU compressed, are inflated
// (inflate.hip) and parsed (parse.hip) there, and K1 sketches them; the host
// threads only read files.
//
// Per member (device), several processing lanes run at once, each with its
// own stream and scratch (lane_ctx): while one lane waits on the host side
// of a batch (the block starts, the decode results, the parse counts), the
// other's kernels keep the GPU busy, and their kernels overlap where one
// alone leaves the GPU part idle.  Each lane has a stager: while the lane
// processes batch N, a helper thread stages batch N + 1 into the lane's
// other pinned slot -- its pool of threads claims files one at a time from
// the call's shared list (GzClaims), reads each straight into its place in
// the slot (pread: no intermediate copy), and the batch goes to the slot's
// device buffer by a kernel reading the mapped slot over PCIe.  A batch is cut at its size limits (the first batches of a call
// smaller, so the GPU starts sooner); a claimed file that does not fit is
// given back and claimed again first.
//
// A batch the device inflate does not take (a stream it cannot chain, a
// CRC-32 or ISIZE that does not match, not FASTA) is decoded on the host
// threads instead (GG_FALLBACK_INFLATE_HOST): the result never depends on
// where the bytes were inflated.  Files that are not gzip are placed as
// their text (plain FASTA), or converted on the host first (FASTQ records,
// bzip2 and xz streams: pack.cpp host_text_from_bytes).
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <future>
#include <mutex>
#include <new>
#include <thread>

#include <cmath>

#include "context.hpp"

namespace gg {

bool GzClaims::claim(uint32_t* i) {
  std::lock_guard<std::mutex> lk(mu);
  if (stop) return false;
  if (!back.empty()) {  // (the lowest given-back file first)
    auto it = std::min_element(back.begin(), back.end());
    *i = *it;
    back.erase(it);
    return true;
  }
  if (cursor >= n) return false;
  *i = cursor++;
  return true;
}

void GzClaims::give_back(uint32_t i) {
  std::lock_guard<std::mutex> lk(mu);
  back.push_back(i);
}

void GzClaims::file_error(uint32_t i, gg_status st, const std::string& msg) {
  std::lock_guard<std::mutex> lk(mu);
  stop = true;
  if (i < err_idx) {
    err_idx = i;
    err_st = st;
    err_msg = msg;
  }
}

void GzClaims::abandon(const std::vector<uint32_t>& idx) {
  std::lock_guard<std::mutex> lk(mu);
  abandoned.insert(abandoned.end(), idx.begin(), idx.end());
}

void GzClaims::halt() {
  std::lock_guard<std::mutex> lk(mu);
  stop = true;
}

namespace {

using Clock = std::chrono::steady_clock;
double ms_since(Clock::time_point t0) { return std::chrono::duration<double, std::milli>(Clock::now() - t0).count(); }

bool debug() {  // GALAHGPU_INFLATE_DEBUG=1: a timeline of the batches on stderr
  static const bool on = [] {
    const char* e = getenv("GALAHGPU_INFLATE_DEBUG");
    return e && *e == '1';
  }();
  return on;
}

// device-inflate batches: up to 4096 files, 192 MiB of gzip data or 576 MiB
// of text (the inflate's parallel units are the streams' blocks, ~30 per
// 3 Mbp genome: a batch needs hundreds of files to fill the GPU)
constexpr uint32_t kBatchGenomesGz = 4096;
// (GALAHGPU_GZ_BATCH_FILES, 1..4096, read per call: fewer files per batch, so
// a test's few small files make many batches; no result depends on it)
uint32_t gz_batch_files() {
  const char* e = getenv("GALAHGPU_GZ_BATCH_FILES");
  const long x = e ? atol(e) : 0;
  return x > 0 ? (uint32_t)std::min<long>(x, kBatchGenomesGz) : kBatchGenomesGz;
}
// (GALAHGPU_GZ_BATCH_MB sets the gzip bytes per batch, the text cap follows
// at 3x, at most 960 MiB: tuning only, no result depends on it.  Device
// memory per lane: ~100 B per gzip byte of scratch (tokens and sub-span
// decodes are sized one per compressed bit), 4 B per text byte for val.)
uint64_t gz_batch_bytes() {
  static const uint64_t v = [] {
    const char* e = getenv("GALAHGPU_GZ_BATCH_MB");
    const long mb = e ? atol(e) : 0;
    return (uint64_t)(mb > 0 ? std::min(mb, 320L) : 192L) << 20;
  }();
  return v;
}
uint64_t gz_batch_text() { return std::min<uint64_t>(3 * gz_batch_bytes(), 960ull << 20); }  // (text < 1 GiB)
// processing lanes per device (GALAHGPU_GZ_LANES, 1..4, read per call;
// tuning and per-kernel timing without overlap: no result depends on it)
int gz_lanes() {
  const char* e = getenv("GALAHGPU_GZ_LANES");
  const int x = e ? atoi(e) : 0;
  return x > 0 ? std::min(x, 4) : 2;
}
// reading threads per stager (GALAHGPU_GZ_COPY_THREADS; tuning only)
int gz_stage_threads(int host_threads, int lanes) {
  const char* e = getenv("GALAHGPU_GZ_COPY_THREADS");
  const int t = e ? atoi(e) : 0;
  if (t > 0) return std::min(t, 16);
  return std::max(2, host_threads / lanes);
}

// A file opened and looked at before its place in a batch is taken.
struct Probe {
  int fd = -1;
  uint64_t size = 0;
  bool gz = false;       // gzip magic
  bool member = false;   // a gzip member whose header the device path reads
  bool bgzf = false;     // its header has BGZF's member size (bgzip): the members are walked once read
  size_t doff = 0;       // its deflate data [doff, doff + dlen)
  uint64_t dlen = 0;
  uint32_t isize = 0, crc = 0;
  bool converted = false;  // text: the file's FASTA text made on the host
  std::vector<uint8_t> text;
  FileStamp stamp;
  gg_status st = GG_OK;
  std::string err;
  Probe() = default;
  Probe(const Probe&) = delete;
  ~Probe() {
    if (fd >= 0) close(fd);
  }
};

bool pread_all(int fd, uint8_t* dst, uint64_t len, uint64_t off) {
  while (len) {
    const ssize_t got = pread(fd, dst, (size_t)std::min<uint64_t>(len, 1ull << 30), (off_t)off);
    if (got <= 0) return false;
    dst += got;
    off += (uint64_t)got;
    len -= (uint64_t)got;
  }
  return true;
}

void probe_file(const char* path, bool stamp, Probe& p) {
  if (!path) {
    p.st = GG_ERR_INVALID_ARG;
    p.err = "null path";
    return;
  }
  if (stamp) file_stamp(path, &p.stamp);
  p.fd = open(path, O_RDONLY | O_CLOEXEC);
  struct stat sb;
  if (p.fd < 0 || fstat(p.fd, &sb) != 0) {
    p.st = GG_ERR_IO;
    p.err = std::string("could not open ") + path;
    return;
  }
  p.size = (uint64_t)sb.st_size;
  uint8_t head[4096];
  const uint64_t hn = std::min<uint64_t>(p.size, sizeof head);
  if (!pread_all(p.fd, head, hn, 0)) {
    p.st = GG_ERR_IO;
    p.err = std::string("read error in ") + path;
    return;
  }
  if (hn >= 2 && head[0] == 0x1f && head[1] == 0x8b) {
    p.gz = true;
    uint8_t tail[8];
    if (gzip_header(head, (size_t)hn, p.size, &p.doff) && pread_all(p.fd, tail, 8, p.size - 8)) {
      p.member = true;
      p.dlen = p.size - 8 - p.doff;
      p.crc = (uint32_t)tail[0] | ((uint32_t)tail[1] << 8) | ((uint32_t)tail[2] << 16) | ((uint32_t)tail[3] << 24);
      p.isize = (uint32_t)tail[4] | ((uint32_t)tail[5] << 8) | ((uint32_t)tail[6] << 16) | ((uint32_t)tail[7] << 24);
      p.bgzf = bgzf_member_size(head, hn) != 0;
    }
    return;  // (a gzip file whose header this path does not read: its batch is decoded on the host)
  }
  if (hn && head[0] == '>') return;  // plain FASTA: its bytes are its text
  // anything else through the host: FASTQ records rewritten, bzip2 / xz
  // decoded, and the host path's error for what is none of these
  std::vector<uint8_t> raw(p.size);
  if (!pread_all(p.fd, raw.data(), p.size, 0)) {
    p.st = GG_ERR_IO;
    p.err = std::string("read error in ") + path;
    return;
  }
  p.st = host_text_from_bytes(raw, path, p.text, p.err);
  p.converted = true;
}

struct GzHeld {  // a file's bytes in the slot
  uint64_t pos, len;
  bool gz;
};
struct GzStaged {
  std::vector<uint32_t> idx;  // the files (indices into GzClaims::paths), in batch order
  std::vector<InflateFile> files;
  std::vector<GzHeld> held;
  std::vector<FileStamp> stamps;
  uint64_t at = 0;          // bytes staged
  bool host_only = false;   // a gzip header the device path does not read
  bool file_err = false;    // a file did not read (recorded in GzClaims)
  gg_status st = GG_OK;     // a HIP failure
  std::string err;
  double ms = 0;
  Clock::time_point t0;
  hipEvent_t up_a = nullptr, up_b = nullptr;  // (timing: the upload kernel)
};

// One lane's stager: two slots (pinned host + device buffers and an upload
// stream, in the lane context's gz_slot), batch N + 1 staged by a helper
// thread into one while the lane processes batch N from the other.
class GzStager {
 public:
  GzStager(gg_ctx* m, GzClaims& cl, int threads) : m_(m), cl_(cl), threads_(threads) {}
  ~GzStager() {
    if (next_.valid()) next_.wait();
    // a batch staged but never processed (the lane stopped on an error):
    // its files were claimed but not decoded, so a file error among them
    // is still to be found (gz_settle_errors); its timing events go
    for (int si = 0; si < 2; ++si) {
      GzStaged& g = staged_[si];
      if (si != cur_ || !consumed_) cl_.abandon(g.idx);
      drop_events(g);
    }
  }
  // The next staged batch (nullptr: no more); starts staging the one after.
  GzStaged* next() {
    bool have;
    if (next_.valid()) {
      have = next_.get();
    } else {
      have = stage(slot_, staged_[slot_]);
    }
    if (!have) {
      staged_[slot_].idx.clear();  // (nothing staged there)
      return nullptr;
    }
    cur_ = slot_;
    consumed_ = true;
    slot_ ^= 1;
    if (staged_[cur_].st == GG_OK && !staged_[cur_].file_err)
      next_ = std::async(std::launch::async, [this] {
        (void)hipSetDevice(m_->device);
        return stage(slot_, staged_[slot_]);
      });
    return &staged_[cur_];
  }
  const uint8_t* host() const { return m_->gz_slot[cur_].host; }
  uint8_t* dev() const { return m_->gz_slot[cur_].dev; }
  hipStream_t up_stream() const { return m_->gz_slot[cur_].st; }

 private:
  // Claims files and stages them into slot si until the batch is full or no
  // file is left; false when it got no file.
  static void drop_events(GzStaged& g) {
    if (g.up_a) (void)hipEventDestroy(g.up_a);
    if (g.up_b) (void)hipEventDestroy(g.up_b);
    g.up_a = g.up_b = nullptr;
  }
  bool stage(int si, GzStaged& g) {
    drop_events(g);  // (a batch left unprocessed kept its upload events)
    g = GzStaged{};
    g.t0 = Clock::now();
    int ramp;
    uint32_t max_files = gz_batch_files();
    {
      std::lock_guard<std::mutex> lk(cl_.mu);
      if (cl_.stop || (cl_.cursor >= cl_.n && cl_.back.empty())) return false;
      // the first batches of a call at 1/8, 1/4, 1/2: the device starts
      // while the full-size ones are staged
      ramp = cl_.batches < 3 ? 3 - (int)cl_.batches : 0;
      ++cl_.batches;
      // the tail: once the files left fit fewer full batches than one per
      // stager and one more, they go in k equal batches, k the stagers'
      // smallest multiple that holds them at full size
      if (!ramp && !cl_.tail_cap && cl_.seen_files && !(getenv("GALAHGPU_GZ_NO_TAIL") && *getenv("GALAHGPU_GZ_NO_TAIL") == '1')) {
        const uint64_t left = (uint64_t)(cl_.n - cl_.cursor) + cl_.back.size();
        const double full = std::max(1.0, (double)gz_batch_bytes() * cl_.seen_files / std::max<uint64_t>(1, cl_.seen_bytes));
        const uint64_t S = std::max<uint32_t>(1, cl_.stagers);
        if ((double)left < (double)(S + 1) * full) {
          const uint64_t need = (uint64_t)std::ceil((double)left / full);
          const uint64_t k = (std::max<uint64_t>(need, 1) + S - 1) / S * S;
          cl_.tail_cap = (uint32_t)std::max<uint64_t>(1, (left + k - 1) / k);
        }
      }
      if (cl_.tail_cap) max_files = std::min(max_files, cl_.tail_cap);
    }
    const uint64_t cut_gz = gz_batch_bytes() >> ramp, cut_text = gz_batch_text() >> ramp;
    gg_ctx::GzSlot& sl = m_->gz_slot[si];
    auto hip = [&](hipError_t e, const char* what) {
      if (e != hipSuccess && g.st == GG_OK) {
        g.st = e == hipErrorOutOfMemory ? GG_ERR_OUT_OF_MEMORY : GG_ERR_HIP;
        g.err = std::string(what) + ": " + hipGetErrorString(e);
      }
      return e == hipSuccess;
    };
    if (!sl.st && !hip(hipStreamCreateWithFlags(&sl.st, hipStreamNonBlocking), "hipStreamCreate")) return true;
    // room for two full batches (a larger file gets a slot of its size, alone in its batch)
    auto grow = [&](uint64_t cap) {
      if (!hip(hipStreamSynchronize(sl.st), "hipStreamSynchronize")) return false;
      if (cap > sl.host_cap) {
        if (sl.host) (void)hipHostFree(sl.host);
        sl.host = nullptr;
        sl.host_cap = 0;
        if (!hip(hipHostMalloc((void**)&sl.host, cap, hipHostMallocMapped), "hipHostMalloc")) return false;
        if (!hip(hipHostGetDevicePointer((void**)&sl.host_dev, sl.host, 0), "hipHostGetDevicePointer")) return false;
        sl.host_cap = cap;
      }
      if (cap > sl.dev_cap) {
        if (sl.dev) (void)hipFree(sl.dev);
        sl.dev = nullptr;
        sl.dev_cap = 0;
        if (!hip(hipMalloc((void**)&sl.dev, cap), "hipMalloc")) return false;
        sl.dev_cap = cap;
      }
      return true;
    };
    if (!grow(2 * gz_batch_bytes() + kInflatePad)) return true;
    std::mutex bm;
    bool full = false;
    uint64_t gz_bytes = 0, text_est = 0;
    const bool stamp = cl_.cache_dir != nullptr;
    auto worker = [&] {
      (void)hipSetDevice(m_->device);
      for (;;) {
        {
          std::lock_guard<std::mutex> lk(bm);
          if (full || g.st != GG_OK || g.file_err) return;
        }
        uint32_t i;
        if (!cl_.claim(&i)) return;
        Probe pr;
        probe_file(cl_.paths[i], stamp, pr);
        if (pr.st != GG_OK) {
          cl_.file_error(i, pr.st, pr.err);
          std::lock_guard<std::mutex> lk(bm);
          g.file_err = true;
          return;
        }
        const uint64_t len = pr.converted ? pr.text.size() : pr.size;
        const uint64_t doff = pr.member ? pr.doff : 0;
        uint64_t p;
        size_t slot_file = 0;
        {
          std::lock_guard<std::mutex> lk(bm);
          if (full || g.st != GG_OK || g.file_err) {
            cl_.give_back(i);
            return;
          }
          p = (g.at + doff + 3) / 4 * 4 - doff;  // (deflate data on a 4-byte boundary)
          const uint64_t end = p + len + 16 + kInflatePad;
          const bool fits = end <= sl.host_cap && end <= sl.dev_cap;
          if (!g.idx.empty() && (!fits || g.idx.size() >= max_files)) {
            full = true;
            cl_.give_back(i);
            return;
          }
          if (!fits && !grow(end)) {  // (an empty batch: no read in flight into the slot)
            cl_.give_back(i);
            return;
          }
          g.at = p + len;
          gz_bytes += pr.gz ? pr.size : 0;
          {
            std::lock_guard<std::mutex> lc(cl_.mu);
            ++cl_.seen_files;
            cl_.seen_bytes += pr.size;
          }
          text_est += pr.member ? pr.isize : len;
          if (gz_bytes >= cut_gz || text_est >= cut_text) full = true;
          InflateFile f;
          f.gz = pr.member;
          f.data_off = p + doff;
          f.data_len = pr.member ? pr.dlen : len;
          f.isize = pr.isize;
          f.crc = pr.crc;
          slot_file = g.files.size();
          g.idx.push_back(i);
          g.files.push_back(f);
          g.held.push_back(GzHeld{p, len, pr.gz});
          g.stamps.push_back(pr.stamp);
          if (pr.gz && !pr.member) g.host_only = true;
        }
        // (the place is this thread's: the slot does not move while the batch holds a file)
        bool ok = true;
        if (pr.converted) {
          if (len) memcpy(sl.host + p, pr.text.data(), len);
        } else {
          ok = pread_all(pr.fd, sl.host + p, len, 0);
        }
        if (!ok) {
          std::lock_guard<std::mutex> lk(bm);
          cl_.file_error(i, GG_ERR_IO, std::string("read error in ") + cl_.paths[i]);
          g.file_err = true;
        } else if (pr.bgzf) {  // bgzip: every member from its header's size field
          std::vector<GzMember> ms;
          if (bgzf_members(sl.host + p, len, p, ms)) {
            std::lock_guard<std::mutex> lk(bm);
            g.files[slot_file].members.swap(ms);
          }
        }
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads_; ++t) th.emplace_back(worker);
    worker();
    for (auto& x : th) x.join();
    // the batch to the device by a kernel reading the mapped slot (inflate.hip
    // launch_slot_upload): no DMA-engine queue for the lanes' small copies to wait behind
    if (g.st == GG_OK && !g.file_err && g.at) {
      if (m_->timing && !g.up_a) {  // (events of the consuming lane's timing, gg_timing_read)
        hip(hipEventCreate(&g.up_a), "hipEventCreate");
        hip(hipEventCreate(&g.up_b), "hipEventCreate");
      }
      if (g.up_a) hip(hipEventRecord(g.up_a, sl.st), "hipEventRecord");
      hip(launch_slot_upload(sl.dev, sl.host_dev, g.at, sl.st), "slot upload");
      if (g.up_b) hip(hipEventRecord(g.up_b, sl.st), "hipEventRecord");
    }
    g.ms = ms_since(g.t0);
    return !g.idx.empty() || g.st != GG_OK || g.file_err;
  }

  gg_ctx* m_;
  GzClaims& cl_;
  int threads_;
  GzStaged staged_[2];
  int slot_ = 0, cur_ = 0;
  bool consumed_ = false;  // staged_[cur_] was handed to the lane
  std::future<bool> next_;
};

// Inflates (or, when the device path does not take it, decodes on the host
// threads) and parses one staged batch on m's stream: 2-bit words into
// *d_words, runs into runs.
gg_status inflate_staged_batch(gg_ctx* m, GzStager& pipe, GzStaged& g, GzClaims& cl, int host_threads,
                               uint32_t** d_words, uint64_t* nw, std::vector<gg_run>& runs) {
  const auto t0 = Clock::now();
  if (g.st != GG_OK) return fail(m, g.st, g.err);
  if (g.file_err) {  // (the call reports the file's own error; the batch's other files were never decoded)
    cl.abandon(g.idx);
    return fail(m, GG_ERR_IO, "a file did not read");
  }
  if (g.up_a) {  // (the stager's upload, timed: the lane's events from here on)
    m->timed.push_back(gg_ctx::Timed{GG_KERNEL_UPLOAD, g.up_a, g.up_b, g.at});
    g.up_a = g.up_b = nullptr;
  }
  // the stream waits for the batch's copies (queued on the slot's stream)
  if (!m->copy_done) GG_HIP(m, hipEventCreateWithFlags(&m->copy_done, hipEventDisableTiming));
  GG_HIP(m, hipEventRecord(m->copy_done, pipe.up_stream()));
  GG_HIP(m, hipStreamWaitEvent(m->stream, m->copy_done, 0));
  static const Clock::time_point t_proc = Clock::now();  // (debug: times since the process's first batch)
  if (debug())
    fprintf(stderr, "[inflate] at %.3f ms: lane %p: batch of %zu files (%.1f MB) staged in %.3f ms (began at %.3f ms)\n",
            ms_since(t_proc), (void*)m, g.files.size(), g.at / 1e6, g.ms,
            std::chrono::duration<double, std::milli>(g.t0 - t_proc).count());
  uint8_t* d_text = nullptr;
  std::vector<uint64_t> foff;
  bool ok = false;
  if (!g.host_only) {
    const gg_status is = inflate_batch(m, pipe.host(), g.at, g.files, &d_text, foff, &ok, pipe.dev());
    if (is != GG_OK) return is;
  }
  if (ok) ++m->inflate_dev_batches;
  if (!ok) {  // the host decodes this batch (and reports a corrupt file)
    ++m->fallbacks[GG_FALLBACK_INFLATE_HOST];
    const size_t nf = g.files.size();
    std::vector<std::vector<uint8_t>> texts(nf);
    std::vector<gg_status> sts(nf, GG_OK);
    std::vector<std::string> errs(nf);
    std::vector<std::thread> th;
    const int T = std::max(1, std::min<int>(host_threads, (int)nf));
    auto work = [&](int t) {
      for (size_t f = (size_t)t; f < nf; f += (size_t)T) {
        const uint8_t* b = pipe.host() + g.held[f].pos;
        if (g.held[f].gz) {
          std::vector<uint8_t> gzb(b, b + g.held[f].len);
          sts[f] = host_text_from_bytes(gzb, cl.paths[g.idx[f]], texts[f], errs[f]);
        } else {
          texts[f].assign(b, b + g.held[f].len);
        }
      }
    };
    for (int t = 1; t < T; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    bool bad = false;
    for (size_t f = 0; f < nf; ++f)
      if (sts[f] != GG_OK) {
        cl.file_error(g.idx[f], sts[f], errs[f]);
        bad = true;
      }
    if (bad) return fail(m, GG_ERR_IO, "a file did not decode");  // (the call reports the file's own error)
    foff.assign(nf + 1, 0);
    for (size_t f = 0; f < nf; ++f) foff[f + 1] = foff[f] + (texts[f].size() + 15) / 16 * 16;
    std::vector<uint8_t> all(foff[nf], '\n');
    for (size_t f = 0; f < nf; ++f) memcpy(all.data() + foff[f], texts[f].data(), texts[f].size());
    GG_HIP(m, scratch_t(m, "stage_text", std::max<uint64_t>(foff[nf], 16) + 16, &d_text));
    if (foff[nf]) GG_HIP(m, hipMemcpyAsync(d_text, all.data(), foff[nf], hipMemcpyHostToDevice, m->stream));
    GG_HIP(m, hipStreamSynchronize(m->stream));
  }
  const gg_status ps = parse_raw_batch(m, d_text, foff, d_words, nw, runs);
  if (debug())
    fprintf(stderr, "[inflate] at %.3f ms: lane %p: batch inflated and parsed in %.3f ms\n", ms_since(t_proc),
            (void*)m, ms_since(t0));
  return ps;
}

// One lane: batches from its stager until none is left, each inflated,
// parsed and sketched into the member's rows.
gg_status run_lane(gg_ctx* x, GzClaims& cl, uint64_t* d_sk, uint32_t* d_len, int host_threads, int stage_threads,
                   std::mutex& owned_mu, std::vector<uint32_t>& owned) {
  const uint32_t s = x->s;
  GzStager pipe(x, cl, stage_threads);
  std::vector<gg_run> runs;
  std::vector<uint32_t> row_of;
  std::vector<uint64_t> out_rows;
  std::vector<uint32_t> out_lens;
  for (;;) {
    GzStaged* g = pipe.next();
    if (!g) break;
    runs.clear();
    uint64_t nw = 0;
    uint32_t* d_words = nullptr;
    // (scratch that grows is sized for the largest batch at once: a batch
    // cut smaller -- the ramp at a call's start, the tail -- would otherwise
    // leave it to grow again, with a device-wide wait, in a later call)
    struct Hint {
      gg_ctx* m;
      ~Hint() { m->scratch_hint = 1.0; }
    } hint{x};
    x->scratch_hint = g->at ? std::min(16.0, std::max(1.0, (double)gz_batch_bytes() / (double)g->at)) : 1.0;
    const gg_status is = inflate_staged_batch(x, pipe, *g, cl, host_threads, &d_words, &nw, runs);
    if (is != GG_OK) return is;
    const uint32_t ng = (uint32_t)g->idx.size();
    row_of.resize(ng);
    for (uint32_t q = 0; q < ng; ++q) row_of[q] = cl.row_of[g->idx[q]];
    uint32_t* d_row_of;
    uint32_t* h_row_of;  // (pinned: a pageable copy blocks this thread; sketch_core syncs before the next batch)
    GG_HIP(x, scratch_t(x, "row_of", ng, &d_row_of));
    GG_HIP(x, host_scratch_t(x, "row_of_h", std::max<uint32_t>(ng, 1), &h_row_of));
    std::copy(row_of.begin(), row_of.end(), h_row_of);
    GG_HIP(x, hipMemcpyAsync(d_row_of, h_row_of, ng * sizeof(uint32_t), hipMemcpyHostToDevice, x->stream));
    const gg_status ks = sketch_core(x, d_words, nw, runs.data(), runs.size(), ng, d_sk, d_len, d_row_of, x->stream);
    if (ks != GG_OK) return ks;
    {
      std::lock_guard<std::mutex> lk(owned_mu);
      owned.insert(owned.end(), row_of.begin(), row_of.end());
    }
    if (cl.cache_dir) {  // store the new sketches (a failed store fails nothing)
      out_rows.resize((size_t)ng * s);
      out_lens.resize(ng);
      for (uint32_t q = 0; q < ng; ++q) {
        GG_HIP(x, hipMemcpyAsync(&out_rows[(size_t)q * s], d_sk + (size_t)row_of[q] * s, s * sizeof(uint64_t),
                                 hipMemcpyDeviceToHost, x->stream));
        GG_HIP(x, hipMemcpyAsync(&out_lens[q], d_len + row_of[q], sizeof(uint32_t), hipMemcpyDeviceToHost, x->stream));
      }
      GG_HIP(x, hipStreamSynchronize(x->stream));
      for (uint32_t q = 0; q < ng; ++q)
        (void)cache_store(cl.cache_dir, cl.paths[g->idx[q]], x->k, s, x->seed, &out_rows[(size_t)q * s], out_lens[q],
                          &g->stamps[q]);
    }
  }
  return GG_OK;
}

}  // namespace

int gz_lane_count() { return gz_lanes(); }

gg_status gz_member_ingest(gg_ctx* m, GzClaims& cl, uint64_t* d_sk, uint32_t* d_len, int host_threads,
                           std::vector<uint32_t>& owned) {
  const int L = gz_lanes();
  std::vector<gg_ctx*> lanes(L, m);
  for (int l = 1; l < L; ++l) {
    lanes[l] = lane_ctx(m, (size_t)l);
    if (!lanes[l]) {
      cl.halt();
      return fail(m, GG_ERR_HIP, "helper stream creation failed");
    }
  }
  for (int l = 1; l < L; ++l) lanes[l]->timing = m->timing;
  const int per = std::max(1, host_threads / L);
  const int stage_threads = gz_stage_threads(host_threads, L);
  std::mutex owned_mu;
  std::vector<gg_status> st(L, GG_OK);
  auto lane = [&](int l) {
    if (l) (void)hipSetDevice(m->device);
    st[l] = run_lane(lanes[l], cl, d_sk, d_len, per, stage_threads, owned_mu, owned);
    if (st[l] != GG_OK) cl.halt();
  };
  std::vector<std::thread> th;
  for (int l = 1; l < L; ++l) th.emplace_back(lane, l);
  lane(0);
  for (auto& t : th) t.join();
  for (int l = 1; l < L; ++l) {  // the member's stream waits for the helpers' work; their counts are the member's
    if (st[l] == GG_OK && st[0] == GG_OK) {
      if (!lanes[l]->copy_done) GG_HIP(m, hipEventCreateWithFlags(&lanes[l]->copy_done, hipEventDisableTiming));
      GG_HIP(m, hipEventRecord(lanes[l]->copy_done, lanes[l]->stream));
      GG_HIP(m, hipStreamWaitEvent(m->stream, lanes[l]->copy_done, 0));
    }
    for (int k = 0; k < GG_FALLBACK_COUNT; ++k) {
      m->fallbacks[k] += lanes[l]->fallbacks[k];
      lanes[l]->fallbacks[k] = 0;
    }
    m->inflate_dev_batches += lanes[l]->inflate_dev_batches;
    lanes[l]->inflate_dev_batches = 0;
    m->gz_member_plans += lanes[l]->gz_member_plans;
    m->gz_full_plans += lanes[l]->gz_full_plans;
    lanes[l]->gz_member_plans = lanes[l]->gz_full_plans = 0;
    m->gz_scratch_bytes = std::max(m->gz_scratch_bytes, lanes[l]->gz_scratch_bytes);
    m->timed.insert(m->timed.end(), lanes[l]->timed.begin(), lanes[l]->timed.end());  // (the events are m's now)
    lanes[l]->timed.clear();
  }
  for (int l = 0; l < L; ++l)
    if (st[l] != GG_OK) {
      if (l) m->err = lanes[l]->err;
      return st[l];
    }
  return GG_OK;
}

void gz_settle_errors(GzClaims& cl) {
  if (cl.err_idx == UINT32_MAX) return;
  // files below the failing one that were given back, or placed in a batch
  // that was dropped before its decode (a read error elsewhere in it, or a
  // lane's prefetched batch after its lane stopped), were never checked
  std::vector<uint32_t> lower;
  for (uint32_t i : cl.back)
    if (i < cl.err_idx) lower.push_back(i);
  for (uint32_t i : cl.abandoned)
    if (i < cl.err_idx) lower.push_back(i);
  std::sort(lower.begin(), lower.end());
  lower.erase(std::unique(lower.begin(), lower.end()), lower.end());
  for (uint32_t i : lower) {  // (never read: read and decoded here, in index order)
    Probe pr;
    probe_file(cl.paths[i], false, pr);
    if (pr.st == GG_OK && pr.gz) {
      std::vector<uint8_t> raw(pr.size), text;
      if (!pread_all(pr.fd, raw.data(), pr.size, 0)) {
        pr.st = GG_ERR_IO;
        pr.err = std::string("read error in ") + cl.paths[i];
      } else {
        pr.st = host_text_from_bytes(raw, cl.paths[i], text, pr.err);
      }
    }
    if (pr.st != GG_OK) {
      cl.file_error(i, pr.st, pr.err);
      return;
    }
  }
}

bool gz_device_list(const char* const* paths, uint32_t n) {
  const char* e = getenv("GALAHGPU_INFLATE");
  if (e && strcmp(e, "device") == 0) return true;
  if (e && strcmp(e, "host") == 0) return false;
  for (uint32_t i = 0; i < std::min<uint32_t>(n, 8); ++i) {  // (by the bytes, not the name)
    if (!paths[i]) continue;
    const int fd = open(paths[i], O_RDONLY | O_CLOEXEC);
    if (fd < 0) continue;
    uint8_t h[2] = {0, 0};
    const bool gz = pread(fd, h, 2, 0) == 2 && h[0] == 0x1f && h[1] == 0x8b;
    close(fd);
    if (gz) return true;
  }
  return false;
}

}  // namespace gg
