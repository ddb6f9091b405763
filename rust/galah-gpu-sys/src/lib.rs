//! Raw FFI declarations of libgalahgpu.so (`include/galahgpu.h`, ABI 7): the
//! MI355X finch MinHash precluster path behind galah's
//! `PreclusterDistanceFinder` (`src/lib.rs:23-27`) and `finch::distances`
//! (`src/finch.rs:26-75`).
//!
//! Every declaration mirrors the C header one to one (same names, argument
//! order and widths; `#[repr(C)]` structs with the header's field order).
//! `tests/test_rust_binding.py` parses this file and the header and checks
//! exactly that, and compares the struct layouts with `offsetof`/`sizeof` of
//! the compiled header, so the two cannot drift apart unnoticed.
//!
//! Safety: every function is `unsafe`; pointers follow the header's
//! conventions (inputs borrowed for the call, outputs released with
//! `gg_free` / `gg_packed_free`, one thread per context at a time).
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_int, c_void};

pub const GG_ABI_VERSION: u32 = 7;
pub const GG_PAIR_TILE: u32 = 64;

/// `gg_status` (a C enum: `int` wide).
pub type GgStatus = c_int;
pub const GG_OK: GgStatus = 0;
pub const GG_ERR_INVALID_ARG: GgStatus = 1;
pub const GG_ERR_IO: GgStatus = 2;
pub const GG_ERR_FORMAT: GgStatus = 3;
pub const GG_ERR_NO_DEVICE: GgStatus = 4;
pub const GG_ERR_HIP: GgStatus = 5;
pub const GG_ERR_OUT_OF_MEMORY: GgStatus = 6;
pub const GG_ERR_INTERNAL: GgStatus = 7;
pub const GG_ERR_OUTPUT_FULL: GgStatus = 8;
pub const GG_ERR_CANCELLED: GgStatus = 9;

pub const GG_PHASE_SKETCH: c_int = 0;
pub const GG_PHASE_REPLICATE: c_int = 1;
pub const GG_PHASE_PAIRS: c_int = 2;
pub const GG_PHASE_MERGE: c_int = 3;
pub const GG_PHASE_COUNT: c_int = 4;

pub const GG_KERNEL_SKETCH: c_int = 0;
pub const GG_KERNEL_FINALIZE: c_int = 1;
pub const GG_KERNEL_PAIRS: c_int = 2;
pub const GG_KERNEL_PAIRS_INDEX: c_int = 3;
pub const GG_KERNEL_INFLATE_SEARCH: c_int = 4;
pub const GG_KERNEL_INFLATE_DECODE: c_int = 5;
pub const GG_KERNEL_INFLATE_EXPAND: c_int = 6;
pub const GG_KERNEL_INFLATE_RESOLVE: c_int = 7;
pub const GG_KERNEL_INFLATE_CRC: c_int = 8;
pub const GG_KERNEL_PARSE: c_int = 9;
pub const GG_KERNEL_UPLOAD: c_int = 10;
pub const GG_KERNEL_COUNT: c_int = 11;

pub const GG_PATH_INDEX: c_int = 0;
pub const GG_PATH_INDEX_ABANDONED: c_int = 1;
pub const GG_PATH_GATE: c_int = 2;
pub const GG_PATH_OTHER: c_int = 3;
pub const GG_PATH_INDEX_FULL_SORT: c_int = 4;
pub const GG_PATH_COUNT: c_int = 5;

pub const GG_FALLBACK_INDEX_TO_GATE: c_int = 0;
pub const GG_FALLBACK_INDEX_FULL_SORT: c_int = 1;
pub const GG_FALLBACK_PEER_STAGED: c_int = 2;
pub const GG_FALLBACK_SKETCH_RETRY: c_int = 3;
pub const GG_FALLBACK_INFLATE_HOST: c_int = 4;
pub const GG_FALLBACK_SKETCH_SET: c_int = 5;
pub const GG_FALLBACK_COUNT: c_int = 6;

/// Opaque context (`gg_ctx`).
#[repr(C)]
pub struct gg_ctx {
    _private: [u8; 0],
}

/// One maximal A/C/G/T stretch of at least k bases (`gg_run`).
#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct gg_run {
    pub genome: u32,
    pub len: u32,
    pub base: u64,
}

/// One above-threshold pair, `i < j` (`gg_pair`): the
/// `SortedPairGenomeDistanceCache` key plus finch's raw counts.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct gg_pair {
    pub i: u32,
    pub j: u32,
    pub common: u32,
    pub total: u32,
}

/// 2-bit packed genomes (`gg_packed`), library-owned.
#[repr(C)]
pub struct gg_packed {
    pub words: *mut u32,
    pub n_words: u64,
    pub n_bases: u64,
    pub runs: *mut gg_run,
    pub n_runs: u64,
    pub n_genomes: u32,
    pub genome_kmers: *mut u64,
}

/// One member's device-resident shard (`gg_shard`).
#[repr(C)]
pub struct gg_shard {
    pub d_words: *const u32,
    pub n_words: u64,
    pub runs: *const gg_run,
    pub n_runs: u64,
    pub n_genomes: u32,
}

/// One pair of a precluster's sub-cache (`gg_local_pair`).
#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq, Eq)]
pub struct gg_local_pair {
    pub precluster: u32,
    pub i: u32,
    pub j: u32,
    pub src: u32,
}

/// Per-kernel timing (`gg_kernel_stats`).
#[repr(C)]
#[derive(Clone, Copy, Debug, Default, PartialEq)]
pub struct gg_kernel_stats {
    pub ms: f64,
    pub launches: u64,
    pub work: u64,
}

/// `gg_pair_sink`: a block of compared pairs; return 0 to go on.
pub type gg_pair_sink = Option<unsafe extern "C" fn(user: *mut c_void, pairs: *const gg_pair, n: u64) -> c_int>;

#[link(name = "galahgpu")]
extern "C" {
    // versioning / errors
    pub fn gg_abi_version() -> u32;
    pub fn gg_status_string(s: GgStatus) -> *const c_char;
    pub fn gg_last_error(ctx: *const gg_ctx) -> *const c_char;
    pub fn gg_thread_last_error() -> *const c_char;

    // context
    pub fn gg_create(kmer_length: c_int, sketch_size: u32, hash_seed: u64, device: c_int, status: *mut GgStatus)
        -> *mut gg_ctx;
    pub fn gg_destroy(ctx: *mut gg_ctx);
    pub fn gg_device(ctx: *const gg_ctx) -> c_int;
    pub fn gg_create_multi(kmer_length: c_int, sketch_size: u32, hash_seed: u64, devices: *const c_int,
                           n_devices: u32, status: *mut GgStatus) -> *mut gg_ctx;
    pub fn gg_device_count(ctx: *const gg_ctx) -> u32;
    pub fn gg_device_ctx(ctx: *mut gg_ctx, index: u32) -> *mut gg_ctx;
    pub fn gg_set_host_threads(ctx: *mut gg_ctx, n_threads: c_int) -> GgStatus;
    pub fn gg_phase_times(ctx: *const gg_ctx, ms: *mut f64) -> GgStatus;

    // host-side ingest
    pub fn gg_pack_files(paths: *const *const c_char, n_paths: u32, kmer_length: c_int, n_threads: c_int,
                         out: *mut *mut gg_packed) -> GgStatus;
    pub fn gg_pack_records(seqs: *const *const u8, lens: *const u64, genome_of_record: *const u32, n_records: u64,
                           n_genomes: u32, kmer_length: c_int, out: *mut *mut gg_packed) -> GgStatus;
    pub fn gg_packed_free(p: *mut gg_packed);

    // sketching (K1)
    pub fn gg_sketch(ctx: *mut gg_ctx, packed: *const gg_packed, out_hashes: *mut u64, out_lens: *mut u32)
        -> GgStatus;
    pub fn gg_sketch_device(ctx: *mut gg_ctx, d_words: *const u32, n_words: u64, runs: *const gg_run, n_runs: u64,
                            n_genomes: u32, d_out: *mut u64, d_lens: *mut u32, stream: *mut c_void) -> GgStatus;

    // all pairs (K2)
    pub fn gg_pair_tiles(n: u32) -> u64;
    pub fn gg_pair_partition(n: u32, parts: u32, part: u32, begin: *mut u64, end: *mut u64);
    pub fn gg_pairs(ctx: *mut gg_ctx, sketches: *const u64, lens: *const u32, n: u32, min_ani: f32,
                    out: *mut *mut gg_pair, n_out: *mut u64) -> GgStatus;
    pub fn gg_pairs_device(ctx: *mut gg_ctx, d_sketches: *const u64, d_lens: *const u32, n: u32, tile_begin: u64,
                           tile_end: u64, min_ani: f32, d_out: *mut gg_pair, out_cap: u64, d_count: *mut u64,
                           stream: *mut c_void) -> GgStatus;

    // the fused FinchPreclusterer::distances body
    pub fn gg_precluster_files(ctx: *mut gg_ctx, paths: *const *const c_char, n_paths: u32, min_ani: f32,
                               pairs: *mut *mut gg_pair, ani: *mut *mut f32, n_out: *mut u64) -> GgStatus;
    pub fn gg_precluster_files_each(ctx: *mut gg_ctx, paths: *const *const c_char, n_paths: u32, min_ani: f32,
                                    cache_dir: *const c_char, sink: gg_pair_sink, user: *mut c_void,
                                    pairs: *mut *mut gg_pair, ani: *mut *mut f32, n_out: *mut u64,
                                    n_cached: *mut u32) -> GgStatus;
    pub fn gg_precluster_shards(ctx: *mut gg_ctx, shards: *const gg_shard, min_ani: f32, pairs: *mut *mut gg_pair,
                                ani: *mut *mut f32, n_out: *mut u64) -> GgStatus;

    // sketch cache
    pub fn gg_sketch_cache_load(cache_dir: *const c_char, path: *const c_char, kmer_length: c_int, sketch_size: u32,
                                hash_seed: u64, out_hashes: *mut u64, out_len: *mut u32, hit: *mut c_int)
        -> GgStatus;
    pub fn gg_sketch_cache_store(cache_dir: *const c_char, path: *const c_char, kmer_length: c_int,
                                 sketch_size: u32, hash_seed: u64, hashes: *const u64, len: u32) -> GgStatus;
    pub fn gg_sketch_files(ctx: *mut gg_ctx, paths: *const *const c_char, n_paths: u32, cache_dir: *const c_char,
                           out_hashes: *mut u64, out_lens: *mut u32, n_cached: *mut u32) -> GgStatus;
    pub fn gg_precluster_files_cached(ctx: *mut gg_ctx, paths: *const *const c_char, n_paths: u32, min_ani: f32,
                                      cache_dir: *const c_char, pairs: *mut *mut gg_pair, ani: *mut *mut f32,
                                      n_out: *mut u64, n_cached: *mut u32) -> GgStatus;

    // after distances(): preclusters
    pub fn gg_partition_preclusters(n_genomes: u32, pairs: *const gg_pair, n_pairs: u64, members: *mut u32,
                                    offsets: *mut u32, n_sets: *mut u32) -> GgStatus;
    pub fn gg_precluster_pairs(n_genomes: u32, pairs: *const gg_pair, n_pairs: u64, members: *const u32,
                               offsets: *const u32, n_sets: u32, out: *mut gg_local_pair, pair_offsets: *mut u64)
        -> GgStatus;

    // host arithmetic
    pub fn gg_ani_f64(common: u32, total: u32, kmer_length: c_int) -> f64;
    pub fn gg_ani_f32(common: u32, total: u32, kmer_length: c_int) -> f32;
    pub fn gg_parse_percentage(value: f32, fraction: *mut f32) -> GgStatus;
    pub fn gg_free(p: *mut c_void);

    // timing, paths, fallbacks, peer links, log line
    pub fn gg_timing_enable(ctx: *mut gg_ctx, on: c_int) -> GgStatus;
    pub fn gg_timing_read(ctx: *mut gg_ctx, kernel: c_int, out: *mut gg_kernel_stats) -> GgStatus;
    pub fn gg_pair_paths(ctx: *const gg_ctx, paths: *mut u64) -> GgStatus;
    pub fn gg_fallbacks(ctx: *const gg_ctx, counts: *mut u64) -> GgStatus;
    pub fn gg_peer_links(ctx: *const gg_ctx, links: *mut c_int) -> GgStatus;
    pub fn gg_info_line(ctx: *const gg_ctx, buf: *mut c_char, cap: usize) -> GgStatus;

    // benchmark support
    pub fn gg_synth_clustered_device(ctx: *mut gg_ctx, first_genome: u32, n_genomes: u32, genome_len: u32,
                                     cluster_size: u32, max_sub_rate: f32, seed: u64, d_words: *mut u32,
                                     runs: *mut gg_run, stream: *mut c_void) -> GgStatus;
    pub fn gg_synth_mixed_lengths(first_genome: u32, n_genomes: u32, min_len: u32, max_len: u32, cluster_size: u32,
                                  seed: u64, lens: *mut u32) -> GgStatus;
    pub fn gg_synth_mixed_device(ctx: *mut gg_ctx, first_genome: u32, n_genomes: u32, lens: *const u32,
                                 cluster_size: u32, max_sub_rate: f32, n_run_rate: f64, seed: u64, d_words: *mut u32,
                                 runs: *mut gg_run, runs_cap: u64, n_runs: *mut u64, stream: *mut c_void)
        -> GgStatus;
}
