/*
 * finch_oracle.c -- CPU restatement of galah's finch precluster path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker (and the timed
 * CPU baseline, "kind": "port") for the MI355X implementation in galah_amd/.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  Nothing in the product library links, calls or falls back to it.
 *
 * Parity pin: src/finch.rs:85-97 of the reference (set1/1mbp vs set1/500kb,
 * k=21, s=1000 -> Some(0.9808188)), src/finch.rs:99-106 (fails at 0.99) and
 * the threshold facts of src/clusterer.rs:482-612 / tests/test_cmdline.rs
 * (SURVEY.md section 4).  See tests/test_oracle_golden.py.
 *
 * What it restates (the reference itself is Rust; its arithmetic lives in
 * third-party crates that are not vendored in /root/reference, see
 * SURVEY.md section 8(c)):
 *
 *   galah  src/finch.rs:26-75      distances(): sketch all files, serial
 *                                  upper-triangle loop, ani = 1 - mash_distance
 *                                  (f64), keep iff ani >= (min_ani as f64),
 *                                  store ani as f32.
 *   galah  src/finch.rs:33-45      SketchParams::Mash{s, s, no_strict, k, seed 0},
 *                                  FilterParams{filter_on: Some(false)} (no-op).
 *   finch 0.6 sketch_files         per file: needletail parse -> per record
 *                                  MashSketcher::process -> bottom-s distinct
 *                                  hashes, ascending.
 *   needletail 0.5 normalize(false) byte map (see norm_byte below).
 *   needletail 0.5 canonical_kmers  k-mer emitted iff all k bytes in {A,C,G,T};
 *                                  canonical = (fwd < rc) ? fwd : rc, compared
 *                                  as byte slices (memcmp).
 *   murmurhash3 0.0.5              murmurhash3_x64_128(kmer_ascii, seed).0
 *   finch 0.6 MashSketcher::push   insert iff len < s or hash <= heap max, and
 *                                  hash not already present; pop max when
 *                                  len > s.
 *   finch 0.6 distance(q, r, false) / raw_distance
 *                                  two-cursor merge until EITHER list is
 *                                  exhausted; common = #equal,
 *                                  total = i + j - common,
 *                                  J = common/total,
 *                                  d = -ln(2J/(1+J))/k clamped to [0,1]
 *                                  with Rust f64::min/max NaN semantics.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

/* ------------------------------------------------------------------ */
/* murmurhash3 0.0.5: murmurhash3_x64_128(bytes, seed) -> (h1, h2)      */
/* ------------------------------------------------------------------ */
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

static inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

static inline uint64_t load_le64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

void oracle_murmur3_x64_128(const uint8_t* data, size_t len, uint64_t seed,
                            uint64_t out[2]) {
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  const size_t nblocks = len / 16;
  uint64_t h1 = seed, h2 = seed;
  for (size_t i = 0; i < nblocks; ++i) {
    uint64_t k1 = load_le64(data + 16 * i);
    uint64_t k2 = load_le64(data + 16 * i + 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* tail = data + nblocks * 16;
  uint64_t k1 = 0, k2 = 0;
  switch (len & 15) {
    case 15: k2 ^= (uint64_t)tail[14] << 48; /* fallthrough */
    case 14: k2 ^= (uint64_t)tail[13] << 40; /* fallthrough */
    case 13: k2 ^= (uint64_t)tail[12] << 32; /* fallthrough */
    case 12: k2 ^= (uint64_t)tail[11] << 24; /* fallthrough */
    case 11: k2 ^= (uint64_t)tail[10] << 16; /* fallthrough */
    case 10: k2 ^= (uint64_t)tail[9] << 8;   /* fallthrough */
    case 9:
      k2 ^= (uint64_t)tail[8];
      k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
      /* fallthrough */
    case 8: k1 ^= (uint64_t)tail[7] << 56; /* fallthrough */
    case 7: k1 ^= (uint64_t)tail[6] << 48; /* fallthrough */
    case 6: k1 ^= (uint64_t)tail[5] << 40; /* fallthrough */
    case 5: k1 ^= (uint64_t)tail[4] << 32; /* fallthrough */
    case 4: k1 ^= (uint64_t)tail[3] << 24; /* fallthrough */
    case 3: k1 ^= (uint64_t)tail[2] << 16; /* fallthrough */
    case 2: k1 ^= (uint64_t)tail[1] << 8;  /* fallthrough */
    case 1:
      k1 ^= (uint64_t)tail[0];
      k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint64_t)len;
  h2 ^= (uint64_t)len;
  h1 += h2;
  h2 += h1;
  h1 = fmix64(h1);
  h2 = fmix64(h2);
  h1 += h2;
  h2 += h1;
  out[0] = h1;
  out[1] = h2;
}

uint64_t oracle_murmur3_h1(const uint8_t* data, size_t len, uint64_t seed) {
  uint64_t o[2];
  oracle_murmur3_x64_128(data, len, seed, o);
  return o[0];
}

/* ------------------------------------------------------------------ */
/* needletail 0.5 normalize(iupac = false), byte by byte.               */
/* Returns 0 for bytes that are dropped (whitespace / line endings).    */
/* ------------------------------------------------------------------ */
static inline uint8_t norm_byte(uint8_t c) {
  switch (c) {
    case 'A': case 'C': case 'G': case 'T': return c;
    case 'a': return 'A';
    case 'c': return 'C';
    case 'g': return 'G';
    case 't': case 'u': case 'U': return 'T';
    case '.': case '~': return '-';
    case ' ': case '\t': case '\r': case '\n': return 0;
    default: return 'N';
  }
}

static inline uint8_t comp_byte(uint8_t c) {
  switch (c) {
    case 'A': return 'T';
    case 'C': return 'G';
    case 'G': return 'C';
    case 'T': return 'A';
    default: return 'N';
  }
}

/* ------------------------------------------------------------------ */
/* finch MashSketcher: bounded max-heap + membership set (bottom-s).    */
/* ------------------------------------------------------------------ */
typedef struct {
  uint32_t size;      /* s */
  uint32_t len;       /* heap entries */
  uint64_t* heap;     /* max-heap, size s+1 */
  uint64_t* set;      /* open addressing, EMPTY = 0, value stored as hash+1? */
  uint8_t* used;      /* slot occupancy */
  uint32_t set_cap;   /* power of two >= 4*(s+1) */
  uint64_t total_kmers;
} sketcher_t;

static int sketcher_init(sketcher_t* sk, uint32_t s) {
  memset(sk, 0, sizeof(*sk));
  sk->size = s;
  sk->heap = (uint64_t*)malloc(sizeof(uint64_t) * (s + 2));
  uint32_t cap = 16;
  while (cap < 4 * (s + 2)) cap <<= 1;
  sk->set_cap = cap;
  sk->set = (uint64_t*)calloc(cap, sizeof(uint64_t));
  sk->used = (uint8_t*)calloc(cap, 1);
  return (sk->heap && sk->set && sk->used) ? 0 : -1;
}

static void sketcher_free(sketcher_t* sk) {
  free(sk->heap);
  free(sk->set);
  free(sk->used);
}

static inline uint32_t set_slot(const sketcher_t* sk, uint64_t h) {
  return (uint32_t)((h * 0x9E3779B97F4A7C15ULL) >> 32) & (sk->set_cap - 1);
}

static int set_contains(const sketcher_t* sk, uint64_t h) {
  uint32_t i = set_slot(sk, h);
  while (sk->used[i]) {
    if (sk->set[i] == h) return 1;
    i = (i + 1) & (sk->set_cap - 1);
  }
  return 0;
}

static void set_insert(sketcher_t* sk, uint64_t h) {
  uint32_t i = set_slot(sk, h);
  while (sk->used[i]) i = (i + 1) & (sk->set_cap - 1);
  sk->used[i] = 1;
  sk->set[i] = h;
}

static void set_remove(sketcher_t* sk, uint64_t h) {
  /* backward-shift deletion for linear probing */
  uint32_t mask = sk->set_cap - 1;
  uint32_t i = set_slot(sk, h);
  while (sk->used[i] && sk->set[i] != h) i = (i + 1) & mask;
  if (!sk->used[i]) return;
  uint32_t j = i;
  for (;;) {
    j = (j + 1) & mask;
    if (!sk->used[j]) break;
    uint32_t home = set_slot(sk, sk->set[j]);
    /* can entry j move to i?  yes iff home is not cyclically in (i, j] */
    int in_range = (i <= j) ? (home > i && home <= j) : (home > i || home <= j);
    if (!in_range) {
      sk->set[i] = sk->set[j];
      i = j;
    }
  }
  sk->used[i] = 0;
}

static void heap_push(sketcher_t* sk, uint64_t h) {
  uint32_t i = sk->len++;
  sk->heap[i] = h;
  while (i > 0) {
    uint32_t p = (i - 1) / 2;
    if (sk->heap[p] >= sk->heap[i]) break;
    uint64_t t = sk->heap[p]; sk->heap[p] = sk->heap[i]; sk->heap[i] = t;
    i = p;
  }
}

static uint64_t heap_pop(sketcher_t* sk) {
  uint64_t top = sk->heap[0];
  sk->heap[0] = sk->heap[--sk->len];
  uint32_t i = 0;
  for (;;) {
    uint32_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < sk->len && sk->heap[l] > sk->heap[m]) m = l;
    if (r < sk->len && sk->heap[r] > sk->heap[m]) m = r;
    if (m == i) break;
    uint64_t t = sk->heap[m]; sk->heap[m] = sk->heap[i]; sk->heap[i] = t;
    i = m;
  }
  return top;
}

/* finch MashSketcher::push */
static inline void sketcher_push(sketcher_t* sk, uint64_t h) {
  sk->total_kmers++;
  if (sk->size == 0) return;
  if (sk->len >= sk->size && h > sk->heap[0]) return;
  if (set_contains(sk, h)) return; /* count bump only */
  set_insert(sk, h);
  heap_push(sk, h);
  if (sk->len > sk->size) {
    uint64_t m = heap_pop(sk);
    set_remove(sk, m);
  }
}

static int cmp_u64(const void* a, const void* b) {
  uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return (x > y) - (x < y);
}

/* to_vec(): ascending; process_post_filter: truncate(final_size) */
static uint32_t sketcher_finish(sketcher_t* sk, uint64_t* out) {
  uint32_t n = sk->len;
  memcpy(out, sk->heap, sizeof(uint64_t) * n);
  qsort(out, n, sizeof(uint64_t), cmp_u64);
  return n;
}

/* ------------------------------------------------------------------ */
/* MashSketcher::process over one record: normalize -> rc -> canonical  */
/* k-mers -> push.                                                      */
/* ------------------------------------------------------------------ */
typedef struct {
  uint8_t* norm;
  uint8_t* rc;
  size_t cap;
} recbuf_t;

static int recbuf_reserve(recbuf_t* b, size_t n) {
  if (n <= b->cap) return 0;
  size_t c = b->cap ? b->cap : 1024;
  while (c < n) c *= 2;
  uint8_t* a = (uint8_t*)realloc(b->norm, c);
  if (!a) return -1;
  b->norm = a;
  uint8_t* r = (uint8_t*)realloc(b->rc, c);
  if (!r) return -1;
  b->rc = r;
  b->cap = c;
  return 0;
}

/* raw: record sequence bytes as they appear between header lines (may
 * contain line breaks).  */
static int process_record(sketcher_t* sk, recbuf_t* rb, const uint8_t* raw,
                          size_t n, int k, uint64_t seed) {
  if (recbuf_reserve(rb, n + 1)) return -1;
  size_t m = 0;
  for (size_t i = 0; i < n; ++i) {
    uint8_t c = norm_byte(raw[i]);
    if (c) rb->norm[m++] = c;
  }
  for (size_t i = 0; i < m; ++i) rb->rc[m - 1 - i] = comp_byte(rb->norm[i]);
  if ((size_t)k > m) return 0;
  /* canonical_kmers: a k-mer at pos p exists iff norm[p..p+k) all ACGT */
  size_t good = 0; /* length of the current ACGT run ending at i */
  for (size_t i = 0; i < m; ++i) {
    uint8_t c = rb->norm[i];
    good = (c == 'A' || c == 'C' || c == 'G' || c == 'T') ? good + 1 : 0;
    if (good >= (size_t)k) {
      size_t p = i + 1 - k;
      const uint8_t* fwd = rb->norm + p;
      const uint8_t* rev = rb->rc + (m - p - k);
      const uint8_t* can = (memcmp(fwd, rev, k) < 0) ? fwd : rev;
      sketcher_push(sk, oracle_murmur3_h1(can, (size_t)k, seed));
    }
  }
  return 0;
}

/* Sketch one in-memory sequence record (no header), e.g. a synthetic
 * genome.  Returns sketch length or -1. */
int oracle_sketch_sequence(const uint8_t* seq, size_t n, int k, int s,
                           uint64_t seed, uint64_t* out) {
  sketcher_t sk;
  recbuf_t rb = {0};
  if (sketcher_init(&sk, (uint32_t)s)) return -1;
  int rc = process_record(&sk, &rb, seq, n, k, seed);
  int len = rc ? -1 : (int)sketcher_finish(&sk, out);
  sketcher_free(&sk);
  free(rb.norm);
  free(rb.rc);
  return len;
}

/* Sketch several in-memory records of one genome (k-mers never span
 * records).  recs: concatenated bytes; offs: n_recs+1 offsets. */
int oracle_sketch_records(const uint8_t* recs, const uint64_t* offs,
                          uint32_t n_recs, int k, int s, uint64_t seed,
                          uint64_t* out) {
  sketcher_t sk;
  recbuf_t rb = {0};
  if (sketcher_init(&sk, (uint32_t)s)) return -1;
  int rc = 0;
  for (uint32_t r = 0; r < n_recs && !rc; ++r)
    rc = process_record(&sk, &rb, recs + offs[r], offs[r + 1] - offs[r], k, seed);
  int len = rc ? -1 : (int)sketcher_finish(&sk, out);
  sketcher_free(&sk);
  free(rb.norm);
  free(rb.rc);
  return len;
}

/* ------------------------------------------------------------------ */
/* FASTA / FASTQ reading (needletail parse_fastx_file; gz via zlib,     */
/* gzread passes plain files through unchanged).                        */
/* ------------------------------------------------------------------ */
static int read_whole_file(const char* path, uint8_t** data, size_t* n) {
  gzFile f = gzopen(path, "rb");
  if (!f) return -1;
  size_t cap = 1 << 20, len = 0;
  uint8_t* buf = (uint8_t*)malloc(cap);
  if (!buf) { gzclose(f); return -1; }
  for (;;) {
    if (len == cap) {
      cap *= 2;
      uint8_t* nb = (uint8_t*)realloc(buf, cap);
      if (!nb) { free(buf); gzclose(f); return -1; }
      buf = nb;
    }
    int got = gzread(f, buf + len, (unsigned)(cap - len > (1u << 30) ? (1u << 30) : cap - len));
    if (got < 0) { free(buf); gzclose(f); return -1; }
    if (got == 0) break;
    len += (size_t)got;
  }
  gzclose(f);
  *data = buf;
  *n = len;
  return 0;
}

/* Sketch a FASTA/FASTQ file.  Returns sketch length, or -1 on I/O or
 * format error (finch::sketch_files -> Err -> galah panics at
 * src/finch.rs:50). */
int oracle_sketch_file(const char* path, int k, int s, uint64_t seed,
                       uint64_t* out) {
  uint8_t* data;
  size_t n;
  if (read_whole_file(path, &data, &n)) return -1;
  sketcher_t sk;
  recbuf_t rb = {0};
  if (sketcher_init(&sk, (uint32_t)s)) { free(data); return -1; }
  int err = 0;
  size_t i = 0;
  if (n > 0 && data[0] != '>' && data[0] != '@') err = 1;
  while (!err && i < n) {
    uint8_t tag = data[i];
    if (tag != '>' && tag != '@') { err = 1; break; }
    /* skip header line */
    while (i < n && data[i] != '\n') ++i;
    if (i < n) ++i;
    size_t start = i;
    if (tag == '>') {
      /* sequence lines until a line starting with '>' */
      while (i < n) {
        if (data[i] == '>' && (i == start || data[i - 1] == '\n')) break;
        ++i;
      }
      err = process_record(&sk, &rb, data + start, i - start, k, seed);
    } else {
      /* FASTQ: one sequence line, '+' line, one quality line */
      while (i < n && data[i] != '\n') ++i;
      size_t end = i;
      if (i < n) ++i;
      err = process_record(&sk, &rb, data + start, end - start, k, seed);
      while (i < n && data[i] != '\n') ++i; /* '+' line */
      if (i < n) ++i;
      while (i < n && data[i] != '\n') ++i; /* quality */
      if (i < n) ++i;
    }
  }
  int len = err ? -1 : (int)sketcher_finish(&sk, out);
  sketcher_free(&sk);
  free(rb.norm);
  free(rb.rc);
  free(data);
  return len;
}

/* finch::sketch_files: rayon par_iter over files.  Here: a pthread pool
 * of n_threads workers pulling files in order.  out is n_files * s,
 * lens is n_files; returns 0 or the (1-based) index of the first failing
 * file. */
typedef struct {
  const char* const* paths;
  uint32_t n;
  int k, s;
  uint64_t seed;
  uint64_t* out;
  int32_t* lens;
  uint32_t next;
  pthread_mutex_t mu;
} sketch_job_t;

static void* sketch_worker(void* arg) {
  sketch_job_t* j = (sketch_job_t*)arg;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    uint32_t i = j->next++;
    pthread_mutex_unlock(&j->mu);
    if (i >= j->n) break;
    j->lens[i] = oracle_sketch_file(j->paths[i], j->k, j->s, j->seed,
                                    j->out + (size_t)i * j->s);
  }
  return NULL;
}

int oracle_sketch_files(const char* const* paths, uint32_t n, int k, int s,
                        uint64_t seed, int n_threads, uint64_t* out,
                        int32_t* lens) {
  sketch_job_t job = {paths, n, k, s, seed, out, lens, 0, PTHREAD_MUTEX_INITIALIZER};
  if (n_threads < 1) n_threads = 1;
  pthread_t th[256];
  if (n_threads > 256) n_threads = 256;
  for (int t = 0; t < n_threads; ++t) pthread_create(&th[t], NULL, sketch_worker, &job);
  for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
  for (uint32_t i = 0; i < n; ++i)
    if (lens[i] < 0) return (int)i + 1;
  return 0;
}

/* ------------------------------------------------------------------ */
/* finch distance(q, r, mash_mode = false)                              */
/* ------------------------------------------------------------------ */
void oracle_raw_distance(const uint64_t* a, uint32_t na, const uint64_t* b,
                         uint32_t nb, uint64_t* common_out,
                         uint64_t* total_out) {
  uint32_t i = 0, j = 0;
  uint64_t common = 0;
  while (i < na && j < nb) {
    if (a[i] < b[j]) ++i;
    else if (a[i] > b[j]) ++j;
    else { ++common; ++i; ++j; }
  }
  *common_out = common;
  *total_out = (uint64_t)i + (uint64_t)j - common;
}

/* Rust f64::min / f64::max: if one argument is NaN the other is returned */
static inline double rust_min(double a, double b) {
  if (isnan(a)) return b;
  if (isnan(b)) return a;
  return a < b ? a : b;
}
static inline double rust_max(double a, double b) {
  if (isnan(a)) return b;
  if (isnan(b)) return a;
  return a > b ? a : b;
}

double oracle_mash_distance(uint64_t common, uint64_t total, int k) {
  double jaccard = (double)common / (double)total;
  double d = -1.0 * log((2.0 * jaccard) / (1.0 + jaccard)) / (double)k;
  return rust_max(rust_min(d, 1.0), 0.0);
}

/* src/finch.rs:56-64: distance = 1.0 - mash_distance (f64) */
double oracle_ani(uint64_t common, uint64_t total, int k) {
  return 1.0 - oracle_mash_distance(common, total, k);
}

/* src/finch.rs:53-73: serial upper-triangle loop.  sketches: n rows of
 * stride u64; lens: per-row length.  Emits passing pairs (i<j) in loop
 * order.  Returns the number of passing pairs; writes at most cap. */
uint64_t oracle_pairs(const uint64_t* sketches, const int32_t* lens,
                      uint32_t n, uint32_t stride, int k, float min_ani,
                      uint32_t* out_i, uint32_t* out_j, uint32_t* out_common,
                      uint32_t* out_total, float* out_ani, uint64_t cap) {
  uint64_t cnt = 0;
  for (uint32_t i = 0; i < n; ++i) {
    for (uint32_t j = i + 1; j < n; ++j) {
      uint64_t c, t;
      oracle_raw_distance(sketches + (size_t)i * stride, (uint32_t)lens[i],
                          sketches + (size_t)j * stride, (uint32_t)lens[j], &c, &t);
      double ani = oracle_ani(c, t, k);
      if (ani >= (double)min_ani) {
        if (cnt < cap) {
          out_i[cnt] = i; out_j[cnt] = j;
          out_common[cnt] = (uint32_t)c; out_total[cnt] = (uint32_t)t;
          out_ani[cnt] = (float)ani;
        }
        ++cnt;
      }
    }
  }
  return cnt;
}

/* All-core variant (the "fairer upper bound" CPU figure of SURVEY 8(d)):
 * rows dealt round-robin to threads, per-thread counts only. */
typedef struct {
  const uint64_t* sk;
  const int32_t* lens;
  uint32_t n, stride, tid, nth;
  int k;
  float min_ani;
  uint64_t passed;
  uint64_t checksum;
} pair_job_t;

static void* pair_worker(void* arg) {
  pair_job_t* p = (pair_job_t*)arg;
  for (uint32_t i = p->tid; i < p->n; i += p->nth) {
    for (uint32_t j = i + 1; j < p->n; ++j) {
      uint64_t c, t;
      oracle_raw_distance(p->sk + (size_t)i * p->stride, (uint32_t)p->lens[i],
                          p->sk + (size_t)j * p->stride, (uint32_t)p->lens[j], &c, &t);
      if (oracle_ani(c, t, p->k) >= (double)p->min_ani) {
        p->passed++;
        p->checksum += ((uint64_t)i * 1000003u + j) ^ (c << 32) ^ t;
      }
    }
  }
  return NULL;
}

/* (common, total) of an explicit list of pairs (pi[x], pj[x]), on n_threads
 * threads: the full-size parity tests check thousands of chosen pairs. */
typedef struct {
  const uint64_t* sk;
  const int32_t* lens;
  uint32_t stride;
  const uint32_t *pi, *pj;
  uint64_t begin, end;
  uint32_t *oc, *ot;
} list_job_t;

static void* list_worker(void* arg) {
  list_job_t* p = (list_job_t*)arg;
  for (uint64_t x = p->begin; x < p->end; ++x) {
    const uint32_t i = p->pi[x], j = p->pj[x];
    uint64_t c, t;
    oracle_raw_distance(p->sk + (size_t)i * p->stride, (uint32_t)p->lens[i],
                        p->sk + (size_t)j * p->stride, (uint32_t)p->lens[j], &c, &t);
    p->oc[x] = (uint32_t)c;
    p->ot[x] = (uint32_t)t;
  }
  return NULL;
}

void oracle_pair_list(const uint64_t* sketches, const int32_t* lens, uint32_t stride,
                      const uint32_t* pi, const uint32_t* pj, uint64_t n_pairs,
                      uint32_t* out_common, uint32_t* out_total, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  list_job_t jobs[256];
  pthread_t th[256];
  for (int t = 0; t < n_threads; ++t) {
    jobs[t] = (list_job_t){sketches, lens, stride, pi, pj, n_pairs * t / n_threads,
                           n_pairs * (t + 1) / n_threads, out_common, out_total};
    pthread_create(&th[t], NULL, list_worker, &jobs[t]);
  }
  for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
}

uint64_t oracle_pairs_parallel(const uint64_t* sketches, const int32_t* lens,
                               uint32_t n, uint32_t stride, int k,
                               float min_ani, int n_threads,
                               uint64_t* checksum) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  pair_job_t jobs[256];
  pthread_t th[256];
  for (int t = 0; t < n_threads; ++t) {
    jobs[t] = (pair_job_t){sketches, lens, n, stride, (uint32_t)t, (uint32_t)n_threads, k, min_ani, 0, 0};
    pthread_create(&th[t], NULL, pair_worker, &jobs[t]);
  }
  uint64_t tot = 0, cs = 0;
  for (int t = 0; t < n_threads; ++t) {
    pthread_join(th[t], NULL);
    tot += jobs[t].passed;
    cs += jobs[t].checksum;
  }
  if (checksum) *checksum = cs;
  return tot;
}
