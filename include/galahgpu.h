/*
 * galahgpu.h -- C ABI of libgalahgpu.so, the MI355X implementation of
 * galah's finch MinHash precluster path.
 *
 * Reference interface this replaces (file:line in AroneyS/galah @ 2024-12-18):
 *
 *   src/lib.rs:23-27          trait PreclusterDistanceFinder { distances(); method_name(); }
 *   src/finch.rs:11-24        impl PreclusterDistanceFinder for FinchPreclusterer
 *   src/finch.rs:26-75        finch::distances(paths, min_ani, num_kmers, kmer_length)
 *                             -> SortedPairGenomeDistanceCache
 *     :33-47                  finch::sketch_files (needletail parse, normalize,
 *                             canonical k-mers, murmur3, bottom-s)   -> gg_pack_* + gg_sketch*
 *     :53-73                  serial all-pairs finch::distance::distance,
 *                             ani >= min_ani as f64, insert Some(ani as f32)
 *                                                                   -> gg_pairs*
 *   src/sorted_pair_genome_distance_cache.rs:22-28   key (min,max) normalisation:
 *                             every gg_pair has i < j.
 *
 * Conventions
 *   - Every entry point returns a status code; nothing throws or aborts
 *     across the ABI.  gg_last_error(ctx) (or gg_thread_last_error() for the
 *     ctx-free host functions) describes the last failure.
 *   - Inputs are borrowed for the duration of the call.  Buffers returned
 *     through pointer-to-pointer arguments are library-owned and released
 *     with gg_free / gg_packed_free.
 *   - A context drives one HIP device (gg_create) or several
 *     (gg_create_multi: one host thread per device inside each call; sketches
 *     are replicated between the devices by peer copies over xGMI and the
 *     pair tiles are partitioned).  Calls on one context must be serialised
 *     by the caller (galah calls distances() once, from one thread:
 *     src/clusterer.rs:36).
 *   - There is NO CPU fallback: gg_create fails with GG_ERR_NO_DEVICE when
 *     no MI355X (gfx950) device is visible.
 *   - *_device entry points take device pointers on the context's device
 *     and enqueue on the given hipStream_t (passed as void*; NULL is the
 *     default stream, as in HIP); they do not synchronise unless stated.
 *     When the caller shares the process with PyTorch, torch's bundled
 *     libamdhip64 must be the one loaded (import torch first) so that
 *     streams and device pointers belong to one HIP runtime.
 */
#ifndef GALAHGPU_H
#define GALAHGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GG_ABI_VERSION 7u

typedef enum gg_status {
  GG_OK = 0,
  GG_ERR_INVALID_ARG = 1,
  GG_ERR_IO = 2,          /* file could not be opened / read */
  GG_ERR_FORMAT = 3,      /* not FASTA/FASTQ */
  GG_ERR_NO_DEVICE = 4,   /* no usable HIP device */
  GG_ERR_HIP = 5,         /* HIP runtime error */
  GG_ERR_OUT_OF_MEMORY = 6,
  GG_ERR_INTERNAL = 7,
  GG_ERR_OUTPUT_FULL = 8, /* device pair buffer too small; *count holds the need */
  GG_ERR_CANCELLED = 9    /* a caller's callback asked to stop (gg_precluster_files_each) */
} gg_status;

typedef struct gg_ctx gg_ctx;

/* One maximal stretch of A/C/G/T (after needletail normalize) inside one
 * FASTA record, at least k bases long.  Bases [base, base+len) of the
 * packed stream.  Runs of one genome are contiguous and genomes appear in
 * input order. */
typedef struct gg_run {
  uint32_t genome;
  uint32_t len;
  uint64_t base;
} gg_run;

/* One above-threshold genome pair; i < j (SortedPairGenomeDistanceCache key). */
typedef struct gg_pair {
  uint32_t i;
  uint32_t j;
  uint32_t common; /* finch raw_distance common  = |A n B|                         */
  uint32_t total;  /* finch raw_distance total   = i + j - common at first exhaustion */
} gg_pair;

/* 2-bit packed genomes: A=0 C=1 G=2 T=3, 16 bases per uint32 word, the
 * first base of a word in bits 31..30. */
typedef struct gg_packed {
  uint32_t* words;
  uint64_t n_words;
  uint64_t n_bases;
  gg_run* runs;
  uint64_t n_runs;
  uint32_t n_genomes;
  uint64_t* genome_kmers; /* per genome: number of k-mer positions (sum of len-k+1) */
} gg_packed;

/* ---- versioning / errors --------------------------------------------- */
uint32_t gg_abi_version(void);
const char* gg_status_string(gg_status s);
const char* gg_last_error(const gg_ctx* ctx);
const char* gg_thread_last_error(void);

/* ---- context ---------------------------------------------------------- */
/* kmer_length: 1..32 (galah: 21, CAP:981); sketch_size: 1..12000 (galah:
 * 1000, CAP:980); hash_seed: murmur3 seed (galah: 0, src/finch.rs:38);
 * device: HIP ordinal, or -1 for the current device. */
gg_ctx* gg_create(int kmer_length, uint32_t sketch_size, uint64_t hash_seed,
                  int device, gg_status* status);
void gg_destroy(gg_ctx* ctx);
/* HIP ordinal of the context's (first) device. */
int gg_device(const gg_ctx* ctx);

/* ---- multi-device context (SURVEY.md 8(b) n_gpus, 8(e)) ----------------- */
/* devices[0 .. n_devices): HIP ordinals, one shard each; an ordinal may
 * repeat (each entry is then its own shard with its own stream on that
 * device -- how the sharded path is exercised on one GPU).
 * devices == NULL: the first n_devices visible devices, or, for
 * n_devices == 0, the GALAHGPU_DEVICES environment variable (comma-separated
 * ordinals) when it is set and every visible device otherwise -- galah's
 * `n_gpus = 0` ("all").  One resolved device gives a plain single-device
 * context.  gg_sketch, gg_pairs, gg_sketch_files, gg_precluster_files(_cached)
 * and gg_precluster_shards use every member; the other entry points act on
 * the first member.  Results never depend on the device list. */
gg_ctx* gg_create_multi(int kmer_length, uint32_t sketch_size, uint64_t hash_seed,
                        const int* devices, uint32_t n_devices, gg_status* status);
/* Number of members (1 for a single-device context). */
uint32_t gg_device_count(const gg_ctx* ctx);
/* Member `index` as a single-device context (owned by ctx, valid until
 * gg_destroy(ctx)); ctx itself when it is a single-device context and
 * index == 0; NULL otherwise. */
gg_ctx* gg_device_ctx(gg_ctx* ctx, uint32_t index);
/* Host threads that read, gunzip and pack genome files inside
 * gg_sketch_files / gg_precluster_files(_cached): galah's --threads
 * (CAP:1327-1332).  <= 0 restores the default (GALAHGPU_THREADS, else
 * OMP_NUM_THREADS, else the CPUs of the process's affinity mask). */
gg_status gg_set_host_threads(gg_ctx* ctx, int n_threads);

/* Wall-clock phases of the last gg_precluster_files(_cached) /
 * gg_precluster_shards call on ctx, in ms: ingest + K1 (files are streamed,
 * so reading and sketching overlap), replication of the sketches between
 * devices, K2 on every device + D2H, host merge (sort by (i, j) + ANI). */
enum { GG_PHASE_SKETCH = 0, GG_PHASE_REPLICATE = 1, GG_PHASE_PAIRS = 2, GG_PHASE_MERGE = 3, GG_PHASE_COUNT = 4 };
gg_status gg_phase_times(const gg_ctx* ctx, double* ms /* [GG_PHASE_COUNT] */);

/* ---- host-side ingest: FASTA/FASTQ (plain or gz) -> 2-bit runs --------- */
/* Replaces needletail parse_fastx_file + normalize(false) + the ACGT
 * window test of canonical_kmers inside finch::sketch_files
 * (src/finch.rs:47).  Files are read on n_threads threads (<= 0: the
 * GALAHGPU_THREADS or OMP_NUM_THREADS environment variable, else the CPUs
 * in the process's affinity mask); gzip is decoded with libdeflate when the
 * system library is present, zlib otherwise. */
gg_status gg_pack_files(const char* const* paths, uint32_t n_paths,
                        int kmer_length, int n_threads, gg_packed** out);
/* In-memory records: record r (bytes seqs[r][0..lens[r]) , no header, may
 * contain line breaks) belongs to genome genome_of_record[r]; records must
 * be grouped by non-decreasing genome index. */
gg_status gg_pack_records(const uint8_t* const* seqs, const uint64_t* lens,
                          const uint32_t* genome_of_record, uint64_t n_records,
                          uint32_t n_genomes, int kmer_length, gg_packed** out);
void gg_packed_free(gg_packed* p);

/* ---- sketching (kernel K1) -------------------------------------------- */
/* Bottom-s distinct murmur3 h1 of canonical k-mers per genome, ascending;
 * bit-exact with finch's MashSketcher + process_post_filter.  out_hashes
 * is n_genomes * sketch_size (row g padded after out_lens[g]). */
gg_status gg_sketch(gg_ctx* ctx, const gg_packed* packed,
                    uint64_t* out_hashes, uint32_t* out_lens);
/* Device-resident variant: d_words / d_out / d_lens are device pointers;
 * runs is host memory (copied by the library) or device memory (a table
 * on the context's device is read in place, no copy).  Synchronises stream
 * internally (retry planning reads per-genome status). */
gg_status gg_sketch_device(gg_ctx* ctx, const uint32_t* d_words,
                           uint64_t n_words, const gg_run* runs,
                           uint64_t n_runs, uint32_t n_genomes,
                           uint64_t* d_out, uint32_t* d_lens, void* stream);

/* ---- all-pairs (kernel K2) -------------------------------------------- */
/* The pair space (i < j < n) is cut into GG_PAIR_TILE x GG_PAIR_TILE tiles
 * of the upper triangle, enumerated row-major.  Multi-GPU runs partition
 * the tile range; the union of the per-range outputs is independent of
 * the partition. */
#define GG_PAIR_TILE 64u
uint64_t gg_pair_tiles(uint32_t n);
/* Tile range [*begin, *end) of part `part` of `parts`, equal pair counts. */
void gg_pair_partition(uint32_t n, uint32_t parts, uint32_t part,
                       uint64_t* begin, uint64_t* end);

/* Host buffers in and out.  *out is library-owned (gg_free), sorted by
 * (i, j).  Pass iff ani(common,total) >= (double)min_ani, ani computed as
 * src/finch.rs:56-69 does. */
gg_status gg_pairs(gg_ctx* ctx, const uint64_t* sketches, const uint32_t* lens,
                   uint32_t n, float min_ani, gg_pair** out, uint64_t* n_out);
/* Device-resident: sketches [n x sketch_size] u64, lens [n] u32 with every
 * lens[i] <= sketch_size and row i ascending in its first lens[i] entries
 * (not checked on the device; gg_pairs checks the lengths of host input).
 * Appends passing pairs of tiles [tile_begin, tile_end) to d_out (unsorted),
 * *d_count (device u64) incremented by the number found; entries past
 * out_cap are dropped (caller compares *d_count with out_cap). Async. */
gg_status gg_pairs_device(gg_ctx* ctx, const uint64_t* d_sketches,
                          const uint32_t* d_lens, uint32_t n,
                          uint64_t tile_begin, uint64_t tile_end,
                          float min_ani, gg_pair* d_out, uint64_t out_cap,
                          uint64_t* d_count, void* stream);

/* ---- the fused FinchPreclusterer::distances body ------------------------ */
/* paths -> sorted passing pairs plus their f32 ANI (src/finch.rs:70 value).
 * Files are streamed: read, gunzipped and packed on the host threads
 * (gg_set_host_threads) while earlier batches are copied to the devices and
 * sketched; host memory stays bounded whatever the number of files. */
gg_status gg_precluster_files(gg_ctx* ctx, const char* const* paths,
                              uint32_t n_paths, float min_ani, gg_pair** pairs,
                              float** ani, uint64_t* n_out);

/* galah's debug level (src/finch.rs:65-68 logs every compared pair): the
 * same call, plus every pair i < j of the N(N-1)/2, whatever its ANI,
 * handed to sink in blocks of whole 64-genome tile rows (at most ~4M pairs
 * each, common and total set; gg_ani_f64 gives the printed distance), in
 * (i, j) order over the call, so memory stays bounded by one block.  sink
 * returns 0 to go on; anything else ends the call with GG_ERR_CANCELLED.
 * *pairs / *ani / *n_out are the pairs >= min_ani, as gg_precluster_files
 * returns them.  cache_dir as gg_precluster_files_cached (NULL: none). */
typedef int (*gg_pair_sink)(void* user, const gg_pair* pairs, uint64_t n);
gg_status gg_precluster_files_each(gg_ctx* ctx, const char* const* paths, uint32_t n_paths,
                                   float min_ani, const char* cache_dir, gg_pair_sink sink,
                                   void* user, gg_pair** pairs, float** ani, uint64_t* n_out,
                                   uint32_t* n_cached);

/* One member's shard of device-resident packed genomes for
 * gg_precluster_shards: d_words lives on that member's device, runs (host
 * memory, or device memory: read in place on that member's device) index
 * the shard's n_genomes genomes by their genome field.  The global genome
 * order is shard 0's genomes, then shard 1's, ... */
typedef struct gg_shard {
  const uint32_t* d_words;
  uint64_t n_words;
  const gg_run* runs;
  uint64_t n_runs;
  uint32_t n_genomes;
} gg_shard;
/* The fused precluster step over genomes already resident in HBM:
 * K1 on every member's shard, sketches replicated to every member (peer
 * copies), K2 over each member's share of the pair tiles (gg_pair_partition),
 * sparse results gathered and sorted by (i, j) with their f32 ANI.
 * shards has gg_device_count(ctx) entries.  Synchronous. */
gg_status gg_precluster_shards(gg_ctx* ctx, const gg_shard* shards, float min_ani, gg_pair** pairs,
                               float** ani, uint64_t* n_out);

/* ---- sketch cache --------------------------------- */
/* galah sketches every genome on every run (src/finch.rs:47); these entry
 * points keep per-genome sketches on disk so a repeated run over the same
 * files skips ingest and K1 for them.  One entry per (genome file, k) in
 * cache_dir, valid while the file's resolved path, size and mtime and the
 * hash seed are unchanged; an entry computed with sketch size S serves any
 * s <= S (bottom-s is a prefix of bottom-S).  Results are identical with and
 * without the cache.  Format: galah_amd/csrc/sketch_cache.cpp. */

/* *hit = 1 and out_hashes[0..*out_len) filled when a valid entry exists,
 * else *hit = 0 (absent, stale, other parameters or corrupt).  Host only. */
gg_status gg_sketch_cache_load(const char* cache_dir, const char* path, int kmer_length,
                               uint32_t sketch_size, uint64_t hash_seed, uint64_t* out_hashes,
                               uint32_t* out_len, int* hit);
/* Writes (atomically replaces) the entry of path; hashes strictly ascending,
 * len <= sketch_size.  Creates cache_dir when missing.  Host only. */
gg_status gg_sketch_cache_store(const char* cache_dir, const char* path, int kmer_length,
                                uint32_t sketch_size, uint64_t hash_seed, const uint64_t* hashes,
                                uint32_t len);
/* finch::sketch_files (src/finch.rs:47) for files: out_hashes is
 * n_paths * sketch_size (row padded with 0 after out_lens[g]).  cache_dir
 * may be NULL (no cache); otherwise cached genomes are read from it and
 * the rest sketched on the device and stored (a failed store does not fail
 * the call).  *n_cached (may be NULL) receives the number of cache hits. */
gg_status gg_sketch_files(gg_ctx* ctx, const char* const* paths, uint32_t n_paths,
                          const char* cache_dir, uint64_t* out_hashes, uint32_t* out_lens,
                          uint32_t* n_cached);
/* gg_precluster_files with a sketch cache directory (NULL = none). */
gg_status gg_precluster_files_cached(gg_ctx* ctx, const char* const* paths, uint32_t n_paths,
                                     float min_ani, const char* cache_dir, gg_pair** pairs,
                                     float** ani, uint64_t* n_out, uint32_t* n_cached);

/* ---- after distances(): preclusters -------- */
/* src/clusterer.rs:409-431 partition_sketches (single linkage over the
 * pairs the cache contains) + :45-57 (each set sorted ascending, sets
 * ordered by size descending; ties: by smallest member).  Linear in
 * n_pairs (union-find) instead of the reference's O(N^2) contains_key
 * scan.  pairs may be in any order.  Output is CSR: precluster s is
 * members[offsets[s] .. offsets[s+1]); members has n_genomes entries,
 * offsets n_genomes + 1 (caller-owned); *n_sets receives the count. */
gg_status gg_partition_preclusters(uint32_t n_genomes, const gg_pair* pairs,
                                   uint64_t n_pairs, uint32_t* members,
                                   uint32_t* offsets, uint32_t* n_sets);

/* One pair of a precluster's sub-cache: src/sorted_pair_genome_distance_cache.rs
 * :47-58 transform_ids(precluster members) keys it (i, j), i < j, by
 * position inside the precluster; src indexes the input pairs array (for
 * its ANI value). */
typedef struct gg_local_pair {
  uint32_t precluster;
  uint32_t i;
  uint32_t j;
  uint32_t src;
} gg_local_pair;

/* transform_ids for every precluster at once (src/clusterer.rs:70), linear
 * in n_pairs instead of O(m^2) per precluster.  Every pair must lie inside
 * one precluster (true for the partition of the same pairs).  out has
 * n_pairs entries, grouped by precluster and sorted by (i, j) inside it;
 * pair_offsets has n_sets + 1 entries. */
gg_status gg_precluster_pairs(uint32_t n_genomes, const gg_pair* pairs,
                              uint64_t n_pairs, const uint32_t* members,
                              const uint32_t* offsets, uint32_t n_sets,
                              gg_local_pair* out, uint64_t* pair_offsets);

/* ---- host arithmetic shared with the caller ---------------------------- */
/* src/finch.rs:56-64: 1 - finch mash_distance, f64, Rust NaN semantics */
double gg_ani_f64(uint32_t common, uint32_t total, int kmer_length);
/* the value galah stores: Some(ani as f32), src/finch.rs:70 */
float gg_ani_f32(uint32_t common, uint32_t total, int kmer_length);
/* CAP:1160-1182 parse_percentage applied to --precluster-ani: values in
 * [1,100] are divided by 100 in f32, [0,1) kept; else GG_ERR_INVALID_ARG. */
gg_status gg_parse_percentage(float value, float* fraction);

void gg_free(void* p);

/* ---- per-kernel timing (benchmarks) ------------------------------------ */
/* When enabled, every kernel launch of the context is bracketed by HIP
 * events recorded on the stream it is launched on.  gg_timing_read
 * synchronises on those events and returns the summed duration, the number
 * of launches and the algorithmic work units (k-mer positions for
 * GG_KERNEL_SKETCH, genomes for GG_KERNEL_FINALIZE, evaluated pairs for
 * GG_KERNEL_PAIRS; GG_KERNEL_PAIRS_INDEX is the inverted-index pair kernel's
 * sort and run pass, whose pair pass counts under GG_KERNEL_PAIRS) since the
 * last gg_timing_enable.  The device-inflate ingest of gg_precluster_files /
 * gg_sketch_files (gzip lists) times its kernels too, every lane of every
 * member: the block-start search (work: compressed bytes of the batch), the
 * sub-span decode (tokens written), the expand and the resolve (text bytes),
 * the CRC-32 (text bytes), the three parse passes (text bytes, counted on
 * the first) and the PCIe upload of each staged batch (bytes). */
enum { GG_KERNEL_SKETCH = 0, GG_KERNEL_FINALIZE = 1, GG_KERNEL_PAIRS = 2, GG_KERNEL_PAIRS_INDEX = 3,
       GG_KERNEL_INFLATE_SEARCH = 4, GG_KERNEL_INFLATE_DECODE = 5, GG_KERNEL_INFLATE_EXPAND = 6,
       GG_KERNEL_INFLATE_RESOLVE = 7, GG_KERNEL_INFLATE_CRC = 8, GG_KERNEL_PARSE = 9, GG_KERNEL_UPLOAD = 10,
       GG_KERNEL_COUNT = 11 };
typedef struct gg_kernel_stats {
  double ms;
  uint64_t launches;
  uint64_t work;
} gg_kernel_stats;
gg_status gg_timing_enable(gg_ctx* ctx, int on);
gg_status gg_timing_read(gg_ctx* ctx, int kernel, gg_kernel_stats* out);

/* ---- which pair kernel ran ---------------------------------------------- */
/* Counts since the context was created (all members of a multi-device
 * context summed), one per pair-kernel call over a tile range:
 * paths[0] the inverted index ran to completion, paths[1] the index was
 * abandoned for the gate kernel (a hash shared by more sketches than its run
 * limit, or a row's partners overflowing its map), paths[2] the gate kernel
 * ran (after an abandoned index too), paths[3] another form (table / merge,
 * GALAHGPU_PAIRS_KERNEL), paths[4] of the index calls in paths[0], those
 * whose index was built by the full 32-bit sort and run pass instead of the
 * bucketed build (a bucket too large for LDS, or GALAHGPU_INDEX_BUCKETS=0).
 * paths must hold GG_PATH_COUNT values. */
enum {
  GG_PATH_INDEX = 0,
  GG_PATH_INDEX_ABANDONED = 1,
  GG_PATH_GATE = 2,
  GG_PATH_OTHER = 3,
  GG_PATH_INDEX_FULL_SORT = 4,
  GG_PATH_COUNT = 5
};
gg_status gg_pair_paths(const gg_ctx* ctx, uint64_t* paths);

/* ---- fallbacks, peer links and one log line ---------------------------- */
/* None of these changes a result; each costs time, and galah would not see
 * it otherwise.  Counts since the context was created, members summed:
 *   GG_FALLBACK_INDEX_TO_GATE    K2 calls whose inverted index was abandoned
 *                                for the gate kernel (gg_pair_paths[1])
 *   GG_FALLBACK_INDEX_FULL_SORT  index calls rebuilt with the full 32-bit
 *                                sort after a bucket overflowed (gg_pair_paths[4])
 *   GG_FALLBACK_PEER_STAGED      sketch-row copies between two members on
 *                                different devices WITHOUT direct peer access
 *                                (the HIP runtime stages them through host
 *                                memory; see gg_peer_links)
 *   GG_FALLBACK_SKETCH_RETRY     K1 passes re-run for genomes whose first
 *                                bottom-s threshold missed (exact either way)
 *   GG_FALLBACK_INFLATE_HOST     file batches the device gzip inflate
 *                                (GALAHGPU_INFLATE=device) handed back to the
 *                                host threads (several members per file,
 *                                FASTQ, a stream it could not chain, a CRC
 *                                mismatch)
 *   GG_FALLBACK_SKETCH_SET       genomes whose candidate list outgrew its
 *                                region and were re-run in set mode (one
 *                                insert per distinct candidate; a subset of
 *                                the passes GG_FALLBACK_SKETCH_RETRY counts) */
enum {
  GG_FALLBACK_INDEX_TO_GATE = 0,
  GG_FALLBACK_INDEX_FULL_SORT = 1,
  GG_FALLBACK_PEER_STAGED = 2,
  GG_FALLBACK_SKETCH_RETRY = 3,
  GG_FALLBACK_INFLATE_HOST = 4,
  GG_FALLBACK_SKETCH_SET = 5,
  GG_FALLBACK_COUNT = 6
};
gg_status gg_fallbacks(const gg_ctx* ctx, uint64_t* counts /* [GG_FALLBACK_COUNT] */);
/* links[a * M + b] (M = gg_device_count) for members a and b: 1 when member
 * a's copies from member b go device to device (same device, or xGMI peer
 * access enabled at gg_create_multi), 0 when they are staged through host
 * memory.  A single-device context reports {1}. */
gg_status gg_peer_links(const gg_ctx* ctx, int* links /* [M * M] */);
/* One human-readable line for galah's info! log after distances(): device
 * count and ordinals, the last fused call's phase times, and the fallback
 * counts.  Writes at most cap bytes including the terminating NUL (the line
 * is cut to fit).  Returns GG_ERR_INVALID_ARG for a null ctx or buf. */
gg_status gg_info_line(const gg_ctx* ctx, char* buf, size_t cap);

/* ---- benchmark support: synthetic clustered genomes on device ---------- */
/* Genomes [first_genome, first_genome + n_genomes) of a synthetic set of
 * genomes of genome_len bases, in clusters of cluster_size consecutive
 * genomes (global index).  Member m of a cluster is the cluster root with
 * i.i.d. substitutions at rate r_m ~ U(0, max_sub_rate) (r = 0 for the
 * root itself).  Counter-based RNG: output depends only on the arguments.
 * Writes packed words (local genome g at base g*genome_len, genome_len a
 * multiple of 16) and fills runs[g] = {g, genome_len, g*genome_len} (host
 * array, local indices). */
gg_status gg_synth_clustered_device(gg_ctx* ctx, uint32_t first_genome, uint32_t n_genomes,
                                    uint32_t genome_len, uint32_t cluster_size,
                                    float max_sub_rate, uint64_t seed,
                                    uint32_t* d_words, gg_run* runs,
                                    void* stream);

/* Config C5: mixed genome lengths and N runs.  Host side,
 * deterministic in the arguments: lens[g] for genomes [first_genome,
 * first_genome + n_genomes) -- log-uniform in [min_len, max_len], rounded
 * down to a multiple of 16, shared by the members of a cluster. */
gg_status gg_synth_mixed_lengths(uint32_t first_genome, uint32_t n_genomes, uint32_t min_len,
                                 uint32_t max_len, uint32_t cluster_size, uint64_t seed,
                                 uint32_t* lens);
/* Writes the genomes (local genome g at word offset sum(lens[<g])/16) and
 * the ACGT runs between N runs: an N run starts at a base with probability
 * n_run_rate and is 1-64 bases long (those bases are excluded from every
 * run, as needletail's non-ACGT bytes break k-mers); runs shorter than k are
 * dropped.  runs has room for runs_cap entries; *n_runs receives the count
 * (GG_ERR_OUTPUT_FULL when it exceeds runs_cap). */
gg_status gg_synth_mixed_device(gg_ctx* ctx, uint32_t first_genome, uint32_t n_genomes,
                                const uint32_t* lens, uint32_t cluster_size, float max_sub_rate,
                                double n_run_rate, uint64_t seed, uint32_t* d_words, gg_run* runs,
                                uint64_t runs_cap, uint64_t* n_runs, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GALAHGPU_H */
