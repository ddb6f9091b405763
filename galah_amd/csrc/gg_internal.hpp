// Internal declarations shared by the host runtime (api.cpp, pack.cpp) and
// the kernels (sketch.hip, pairs.hip, synth.hip) of libgalahgpu.so.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "../../include/galahgpu.h"

namespace gg {

constexpr uint64_t kEmpty = ~0ull;  // empty hash-set slot; also the largest hash

// Per-genome sketch status written by the finalize kernel.
enum SketchStatus : uint32_t {
  kSketchOk = 0,
  kSketchRetryLarger = 1,   // fewer than s distinct hashes <= tau, tau < 2^64-1
  kSketchRetrySmaller = 2,  // candidate set overflowed its limit
  kSketchRetrySet = 3,      // the candidate list (append mode) held more than the finalize sorts
                            // (duplicates count there): the same tau again in set mode
};

// flags[] bits
constexpr uint32_t kFlagOverflow = 1u;
constexpr uint32_t kFlagSawMax = 2u;
constexpr uint32_t kFlagSetMode = 4u;  // the slot collects its candidates in a hash set (K1 inserts
                                       // with atomicCAS) instead of appending them to a list

// Largest number of candidates the finalize kernel sorts in LDS.
constexpr uint32_t kSortCap = 16384;

// K1 segment: k-mer positions one lane hashes from one 64-base window
// (k = 21: 44), a multiple of the tau-branch group g, capped to bound the
// unrolled code.  Segments never straddle runs (sketch_core).
inline constexpr int k1_seg_len(int k, int g) { return ((65 - k) / g) * g < 48 ? ((65 - k) / g) * g : 48; }
int sketch_segment_len(int k);  // k1_seg_len at K1's tau-branch group

struct SketchLaunch {
  const uint32_t* words;
  uint64_t n_words;
  const gg_run* runs;          // [n_runs] (genome - slot_genome0 = slot within the batch)
  const uint64_t* run_sstart;  // [n_runs + 1] first segment of each run (segments seg0 .. seg0 + n_segs)
  uint32_t slot_genome0;       // genome of batch slot 0
  uint32_t n_runs;
  uint64_t seg0;
  uint64_t n_segs;
  const uint64_t* tau;         // [slots]
  uint64_t* table;             // [slots << cap_log2]
  uint32_t cap_log2;
  uint32_t* flags;             // [slots]
  uint32_t* count;             // [slots] candidates appended (append mode; 0 between passes)
  uint32_t any_set_mode = 0;   // some slot of the launch collects in set mode (flags[slot] & kFlagSetMode)
  uint64_t seed;
  // (first pass queued before the host has seen the run index) the segment
  // count on the device, and the run-table check: K1 does nothing if set
  const uint64_t* n_segs_dev = nullptr;
  const uint64_t* bad_dev = nullptr;
};

// runindex.hip: the run table's index on the device (all device pointers)
struct RunIndexDev {
  const gg_run* runs;  // [n_runs], uploaded
  uint64_t n_runs;
  uint32_t n_genomes;
  uint64_t n_words;
  int k;
  uint32_t seg;        // K1 segment length
  uint64_t* bad;       // [1] first bad run (2^64-1: none)
  uint64_t* sc;        // [n_runs + 1] scratch: segments per run
  uint64_t* rs;        // [n_runs + 1] first segment of each run; rs[n_runs] = total
  uint64_t* gr;        // [n_genomes + 1] first run of each genome
  uint64_t* grs;       // [n_genomes + 1] rs[gr[g]]
  uint64_t* nk;        // [n_genomes] k-mers per genome
  void* tmp;
  size_t tmp_bytes;
};
size_t run_index_tmp_bytes(uint64_t n_runs);
hipError_t launch_run_index(const RunIndexDev& x, hipStream_t st);
// tau[g] from nk[g] (want = oversampling * s) and identity slot maps for
// genomes [0, n_genomes)
hipError_t launch_first_pass(const uint64_t* nk, uint32_t n_genomes, double want, uint64_t* tau,
                             uint32_t* slot_genome, uint32_t* slot_list, hipStream_t st);

// First bottom-s threshold of a genome with nk k-mers: tau = want / nk * 2^64
// (want = over * s expected candidates), or 2^64 - 1 when the genome has at
// most `want` k-mers (every distinct hash is a candidate).  One formula for
// the device's first pass (runindex.hip) and the host's multi-batch path.
__host__ __device__ inline uint64_t first_tau(uint64_t nk, double want) {
  uint64_t t = ~0ull;
  if (nk != 0 && want < (double)nk) {
    const double x = want / (double)nk * 18446744073709551616.0;
    if (x < 18446744073709549568.0) t = (uint64_t)x;  // (the largest double below 2^64)
  }
  return t;
}

// sketch.hip
hipError_t launch_sketch_candidates(int k, const SketchLaunch& a, int grid,
                                    hipStream_t st);
hipError_t launch_sketch_finalize(const uint32_t* slot_list, uint32_t n_slots,
                                  const uint32_t* slot_genome,
                                  const uint64_t* tau, uint64_t* table,
                                  uint32_t cap_log2,
                                  uint32_t* flags, uint32_t s,
                                  uint32_t sort_pow2, const uint32_t* row_of, uint64_t* out,
                                  uint32_t* lens, uint32_t* status, uint32_t* count,
                                  hipStream_t st, const uint64_t* bad = nullptr);

// pairs.hip
struct PairsLaunch {
  const uint64_t* sketches;
  const uint32_t* lens;
  uint32_t n;
  uint32_t stride;      // u64 per sketch row (= sketch size)
  uint32_t n_row_tiles; // ceil(n / GG_PAIR_TILE)
  uint64_t tile_begin;
  uint64_t tile_end;
  const uint32_t* cmin; // [tmax + 1]; pass iff common >= cmin[total]
  uint32_t tmax;
  gg_pair* out;
  uint64_t out_cap;
  unsigned long long* count;
};
hipError_t launch_pairs(const PairsLaunch& a, hipStream_t st);

// Table kernel work unit: tile row I, column tiles [J0, J1) (same row).
struct PairSeg {
  uint32_t I, J0, J1, pad;
};
constexpr uint32_t kSegTiles = 16;
struct PairsTableLaunch {
  const uint64_t* sketches;
  const uint32_t* lens;
  uint32_t n;
  uint32_t stride;
  const PairSeg* segs;
  uint32_t n_segs;
  const uint32_t* cmin;
  uint32_t tmax;
  gg_pair* out;
  uint64_t out_cap;
  unsigned long long* count;
};
// rows per LDS table for sketch size s (0: table kernel not applicable)
uint32_t pairs_table_rows(uint32_t s);
hipError_t launch_pairs_table(const PairsTableLaunch& a, hipStream_t st);

// pairs_gate.hip: the gated-table pair kernel (default K2).
constexpr uint32_t kGateCap = 32768;    // keys per row block (R * s)
// Largest sketch size gg_create accepts, and the gate kernel bounds that
// depend on it: its per-lane 8-bit row counters hold at most ceil(s / 64)
// hits per lane, bucket starts / counts and queued column positions are
// 16-bit (R * s <= 65535).  gate_params() re-checks R * s at run time.
constexpr uint32_t kMaxSketch = 12000;
static_assert((kMaxSketch + 63) / 64 <= 255, "gate kernel: 8-bit per-lane row counters");
static_assert(kMaxSketch <= 65535, "gate kernel: 16-bit column positions and bucket starts");
constexpr uint32_t kGateRowsMax = 32;   // rows per row block (bits of a row mask)
constexpr uint32_t kGateSegTiles = 8;   // column tiles per work item
struct GateParams {
  uint32_t R;         // rows per row block
  uint32_t G;         // row blocks per tile row (ceil(GG_PAIR_TILE / R))
  uint32_t cap;       // R * s
  uint32_t nb;        // buckets (power of two, ~8 keys each)
  uint32_t bm_words;  // gate bitmap words (power of two)
  uint32_t nb_log2;
  uint32_t bm_log2;   // log2 of the gate's bits
  uint32_t wide;      // two-bit gate + directory in LDS (large sketches)
  uint64_t block_bytes;
};
GateParams gate_params(uint32_t s);  // requires s <= kMaxSketch (cap = R * s <= 65535)
struct GateBuildLaunch {
  const uint64_t* sketches;
  const uint32_t* lens;
  uint32_t n;
  uint32_t stride;
  uint32_t tile_row0;  // first tile row with a table
  uint32_t n_blocks;   // tables to build
  GateParams p;
  uint8_t* tables;
  uint32_t* lo32;      // [n * stride]: low words of rows >= tile_row0 * GG_PAIR_TILE
};
struct GateLaunch {
  const uint64_t* sketches;
  const uint32_t* lens;
  uint32_t n;
  uint32_t stride;
  const PairSeg* items;  // per blockIdx: {tile row, J0, J1, row block}; I = ~0: idle
  uint32_t n_items;
  uint32_t tile_row0;
  GateParams p;
  const uint8_t* tables;
  const uint32_t* lo32;
  const uint32_t* cmin;    // [tmax + 1]
  const uint32_t* sufmin;  // [tmax + 1] min(cmin[t..tmax])
  uint32_t tmax;
  uint32_t zero_passes;    // cmin[t] == 0 for some t (then every pair passes)
  gg_pair* out;
  uint64_t out_cap;
  unsigned long long* count;
};
hipError_t launch_gate_build(const GateBuildLaunch& a, hipStream_t st);
hipError_t launch_pairs_gate(const GateLaunch& a, hipStream_t st);

// pairs_index.hip: the inverted-index pair kernel (default K2 when
// eligible; see the file header).
// parse.hip: one batch of raw FASTA text (files concatenated) -> 2-bit codes
// and run starts; the host drives the passes and the per-block scans
// (multi.cpp: parse_raw_batch).
struct ParseLaunch {
  const uint8_t* raw;
  uint64_t n_bytes;
  uint32_t n_blocks;
  const uint32_t* blk_file;
  const uint64_t* blk_start;
  const uint64_t* blk_end;
  const uint64_t* file_start;
  uint64_t* blk_nl;      // pass 1 out
  const uint64_t* pre_nl;
  uint64_t* blk_bases;   // pass 2 out
  uint64_t* blk_last;    // pass 2 out
  const uint64_t* pre_last;
  uint64_t* blk_runs;    // pass 2 out: run starts as if no base came before the block
  uint64_t* blk_first;   // pass 2 out: 1 when the block's first non-dropped byte is a base
  const uint64_t* base_off;
  const uint64_t* run_off;
  uint64_t* starts;      // pass 3 out (run start positions)
  uint64_t n_words;
  uint32_t* words;       // pass 3 out (cleared before)
};
hipError_t parse_batch_pass(int pass, const ParseLaunch& p, hipStream_t st);
uint32_t parse_block_bytes();

// inflate.hip: gzip members inflated on the device (inflate_core.hpp).  All
// pointers are device memory.  The batch holds each file's deflate data
// from word file_word[f] (file_bits[f] bits), followed by >= 3 words of
// padding.
struct InflateSearch {
  const uint32_t* in;
  const uint64_t* file_word;
  const uint64_t* file_bits;
  const uint32_t* chunk_file;  // [n_chunks]
  const uint64_t* chunk_bit0;  // [n_chunks] first bit searched
  uint32_t chunk_bits;         // bits searched per chunk
  uint32_t n_chunks;
  uint64_t* start;             // [n_chunks] first block header found (~0: none)
  uint64_t* prof = nullptr;    // (GALAHGPU_INFLATE_DEBUG) cycles scanning, cycles checking, steps, check rounds, candidates checked
};
struct InflateDecode {
  const uint32_t* in;
  const uint64_t* file_word;
  const uint64_t* file_bits;
  const uint32_t* lane_file;   // [n_lanes]
  const uint64_t* lane_start;  // [n_lanes] a block start
  const uint64_t* lane_end;    // [n_lanes] the next lane's start (~0: the file's last lane)
  uint32_t n_lanes;
  uint32_t* tok;               // tokens of lane l at tok_off[l] (a multiple of 4), at most tok_cap[l]
  const uint64_t* tok_off;
  const uint64_t* tok_cap;
  uint32_t* scr;               // speculative sub-span tokens of lane l at scr_off[l] (inflate::decode_scratch)
  const uint64_t* scr_off;
  uint64_t* prof = nullptr;    // (debug) cycles in header / first decode / resync rounds / copy, blocks, tokens
  uint32_t* status;            // [n_lanes] inflate::DecodeStatus
  uint64_t* n_tok;             // [n_lanes]
  uint64_t* out_len;           // [n_lanes] bytes the lane's tokens stand for
  uint64_t* last_end;          // [n_lanes] bit after the lane's last block
  uint32_t* bfinal;            // [n_lanes] the lane decoded the stream's last block
  // lanes [0, n_staged) take the staged kernel (the compressed words copied
  // into LDS window by window; every stream read of the decode is an LDS
  // read), the rest read global memory
  uint32_t n_staged = 0;
  uint32_t stage_words = 0;  // LDS stage of the staged kernel (0: its default; GALAHGPU_TEST_STAGE_KB)
  uint32_t tight = 0;        // sub-span token areas sized for 1/4 token per bit (inflate::span_cap)
};
// The staged decode's default LDS stage, in words (inflate.hip).
uint32_t inflate_stage_words();
// The words from start_bit to end_bit touch, + the readers' look-ahead.
__host__ __device__ inline uint64_t inflate_segment_words(uint64_t start_bit, uint64_t end_bit) { return (end_bit + 31) / 32 - start_bit / 32 + 8; }
struct InflatePlace {
  const uint32_t* tok;
  const uint64_t* tok_off;
  const uint64_t* n_tok;
  const uint32_t* lane_file;
  const uint64_t* lane_out;    // [n_lanes] text position of the lane's first byte
  const uint64_t* lane_len;    // [n_lanes] the bytes the decode counted for it (its tokens must make as many)
  const uint64_t* file_text;   // [n_units] text position of the unit's first byte
  const uint64_t* unit_len;    // [n_units] its bytes
  const uint64_t* unit_pad;    // [n_units] a file's last unit: end of the '\n' padding after it (else 0)
  const uint32_t* unit_lane;   // [n_units + 1] the unit's lanes: unit_lane[u] .. unit_lane[u + 1] - 1
  uint32_t n_lanes, n_units;
  uint8_t* text;               // [text_len] the bytes (written by the resolve)
  uint16_t* sym;               // [text_len] a literal byte (< 0x100), or kSymPtr | (position copied & 0x7FFF):
                               // a byte of the 32 KB before the lane's first byte
  uint32_t* flags;             // bit 0: a distance before its file's start,
                               // bit 2: a lane's tokens make other than lane_len bytes
  uint64_t* prof = nullptr;    // (debug) expand cycles: fill, pointer rounds, write-out; steps, rounds
};
constexpr uint16_t kSymPtr = 0x8000u;
// one file of an inflate batch (inflate_host.cpp): its bytes at
// [data_off, data_off + data_len) of the batch (data_off 4-byte aligned):
// the deflate data of a gzip member with its trailer's isize and crc, or
// plain text (gz false)
// One gzip member of a file: its deflate data at [off, off + len) of the
// batch and its trailer's CRC-32 and ISIZE.
struct GzMember {
  uint64_t off = 0, len = 0;
  uint32_t isize = 0, crc = 0;
};
// A file of several gzip members (needletail's reader, behind
// src/finch.rs:47, reads them one after the other): `members` in file
// order, data_off the first one's deflate data (4-byte aligned).  Empty for
// one member (data_off / data_len / isize / crc) or plain text.
struct InflateFile {
  uint64_t data_off = 0, data_len = 0;
  uint32_t isize = 0, crc = 0;
  bool gz = false;
  std::vector<GzMember> members;
};
// The members of a BGZF file (bgzip: every member's header carries the 'BC'
// extra subfield with the member's size) at buf[0, n), whose first byte is
// at batch offset base; false (out untouched) when a member header lacks
// the subfield or a size runs past n -- the members are then found on the
// device as they end (inflate_batch).
bool bgzf_members(const uint8_t* buf, uint64_t n, uint64_t base, std::vector<GzMember>& out);
// A BGZF member's total size from the header at b[0, n) ('BC' subfield), 0 without one.
uint64_t bgzf_member_size(const uint8_t* b, uint64_t n);
bool gzip_member(const uint8_t* buf, size_t n, size_t* data_off, size_t* data_len, uint32_t* isize, uint32_t* crc);
// The gzip header at the start of buf[0, n) (of a file of file_size bytes):
// its length (*data_off); false when it is not gzip (CM 8), has reserved
// flags, or does not end within buf and before the trailer.
bool gzip_header(const uint8_t* buf, size_t n, uint64_t file_size, size_t* data_off);
hipError_t launch_inflate_search(const InflateSearch& a, hipStream_t st);
// bytes from mapped pinned host memory (its device address) to dst by a
// kernel on st (inflate.hip); both buffers hold a multiple of 16 bytes
hipError_t launch_slot_upload(uint8_t* dst, const uint8_t* src_mapped, uint64_t bytes, hipStream_t st);
hipError_t launch_inflate_decode(const InflateDecode& a, hipStream_t st);
// the text of a batch: expand (every lane's tokens into sym), then resolve
// (each unit's lanes in order into text, the padding after a file's last
// unit; sym is read only in the units' ranges, where the expand wrote it)
hipError_t launch_inflate_expand(const InflatePlace& a, hipStream_t st);
hipError_t launch_inflate_resolve(const InflatePlace& a, hipStream_t st);
// CRC-32 per file (file f's 4 KB segments are seg_first[f] .. seg_first[f +
// 1] - 1; crc receives n_files CRCs, then each file's first byte)
constexpr uint32_t kInflateCrcSeg = 4096;
hipError_t launch_inflate_crc(const uint8_t* text, uint32_t n_files, const uint64_t* file_text, const uint64_t* file_len,
                              const uint32_t* seg_first, uint32_t n_segs, uint32_t* seg_crc, uint32_t* crc,
                              hipStream_t st);

struct IndexBuild {
  const uint64_t* sketches;
  const uint32_t* lens;
  uint32_t n;
  uint32_t stride;
  uint32_t kbits;      // bits of a position k < stride in a packed value
  uint32_t max_run;    // longer runs: overflow (gate kernel instead)
  uint64_t* offs;      // [n] first entry of each row
  uint64_t* info;      // [2] entries, largest hash
  uint32_t* keys_in;   // [n * stride]
  uint32_t* keys_out;
  uint64_t* vals_in;
  uint64_t* vals_out;
  uint64_t* runinfo;   // [n * stride]
  uint32_t* mixed;     // [ceil(n * stride / 32)] bitset: runs of equal keys holding several hashes
  void* sort_tmp;
  size_t sort_tmp_bytes;
  uint32_t* flags;     // [4]: overflow
  // [1] after flags: the member reads the pairs kernel would make, summed
  // by the run passes (per entry of a run of g >= 2: the members after it
  // when the run is in row order, else g) -- the index's cost, which
  // pairs_index weighs against the gate kernel's before the pairs kernel
  unsigned long long* cost;
  // Row-range index (a device that evaluates only rows [r0, r1) of a
  // multi-device call): bloom != null keeps just the entries whose hash may
  // occur in those rows (a Bloom filter of the rows' hashes: no false
  // negatives, so every run of such a hash is complete), compacted by
  // index_fill, their count in flags[1].
  uint32_t* bloom = nullptr;  // [1 << (bloom_log2 - 5)] words
  uint32_t bloom_log2 = 0;
  uint32_t r0 = 0, r1 = 0;
  // Bucketed build (bucket): index_fill also histograms every entry by the
  // top 12 bits of its top-aligned key (hist [4096]) and splits each coarse
  // bin into sub-ranges of ~equal counts (bbase [4097], bbase[4096] = the
  // number of buckets, at most 2^16); the fill keys entries by bucket
  // (vals hold the 32-bit entries), the sort orders the bucket ids, bstart
  // [buckets + 1] bounds every bucket, and one workgroup per bucket groups
  // equal hashes in LDS.  A bucket too large for that sets flags[3].
  bool bucket = false;
  uint32_t* hist = nullptr;
  uint32_t* bbase = nullptr;
  uint32_t* bstart = nullptr;
  // Split build (split_cnt != null; bucketed, every row): instead of the
  // fill and the 16-bit sort, the entries are dealt to 256 super-bins (bucket
  // >> 8) row by row -- a row is sorted, so its entries of one super-bin are
  // contiguous -- at offsets from a scan of the per-row counts (split_cnt,
  // split_off: [256 * n + 1], super-bin major), and each super-bin's
  // entries are ordered by the low 8 bits of their bucket.
  uint32_t* split_cnt = nullptr;
  uint32_t* split_off = nullptr;
  uint32_t* split_hist = nullptr;  // [256 * 16 * 256]: per super-bin slice, its counts per bucket
};
struct IndexLaunch {
  const uint64_t* sketches;
  const uint32_t* lens;
  uint32_t n;
  uint32_t stride;
  uint32_t kbits;
  uint32_t row0;         // first row processed
  uint32_t n_rows;       // rows processed (set by launch_index_pairs)
  uint64_t nb;           // tile rows
  uint64_t tile_begin;
  uint64_t tile_end;
  const uint64_t* runinfo;
  const uint32_t* vals;  // entries (row << kbits | k) in hash order (those in runs of g >= 2)
  const uint32_t* cmin;
  const uint32_t* sufmin;
  uint32_t tmax;
  gg_pair* out;
  uint64_t out_cap;
  unsigned long long* count;
  uint32_t max_split_log2;  // a row's partners split into at most 2^this classes (16)
  uint32_t* overflow;       // set when a row's partners overflow the LDS map at the last split
  const uint32_t* build_flags = nullptr;  // the build's flags: [0] or [3] set -> emit nothing
  bool ents16 = false;                     // vals holds 16-bit rows (bucketed build, index_ents16)
  // the build's member-read count (IndexBuild::cost) and the count past
  // which the gate kernel is cheaper: with build_flags, more -> emit nothing
  const unsigned long long* cost = nullptr;
  unsigned long long cost_limit = ~0ull;
  bool big_map = false;  // the 2^13-slot partner map (rows that read thousands of members)
};
// Row offsets, the entry count and the largest hash (info[0], info[1]);
// then, with the key shift and the sort's bit range, the keys, the sort and
// the run pass (overflow: flags[0]).
// (row-range index: then the Bloom filter over rows [r0, r1) and the kept
// entries, already keyed: index_build sorts them)
hipError_t index_fill(const IndexBuild& b, hipStream_t st);
hipError_t index_build(const IndexBuild& b, uint64_t total, uint32_t sh, uint32_t end_bit, hipStream_t st);
// (bucketed build: total = sort items, n * stride unless the row-range fill
// compacted its kept entries; nb_bound >= the buckets the device computed,
// index_bucket_bound(entries))
hipError_t index_build_buckets(const IndexBuild& b, uint64_t total, uint32_t nb_bound, hipStream_t st);
uint32_t index_bucket_bound(uint64_t entries);
// bytes of the build's member-read counters (IndexBuild::cost: the total in
// word 0, the partial sums after it), cleared by index_fill with the flags
size_t index_cost_bytes();
// temporary storage of the full build's sort over bits [0, end_bit), and of
// the bucketed build's
size_t index_sort_tmp_bytes(uint64_t total, uint32_t end_bit);
size_t index_bucket_sort_tmp_bytes(uint64_t total);
// temporary bytes of the split build's scan over 256 * n + 1 counts
size_t index_split_tmp_bytes(uint32_t n);
constexpr uint32_t kIndexCoarse = 4096;  // coarse bins of the bucketed build
hipError_t launch_index_pairs(const IndexLaunch& a, uint32_t n_rows, hipStream_t st);
bool index_ents16(uint32_t n);
// Passing pairs sorted by (i, j) on the device into sorted[cnt] (keys,
// keys_out: [cnt] u64; idx, idx_out: [cnt] u32; cnt < 2^31)
uint32_t pair_key_bits(uint32_t n);
size_t pair_sort_tmp_bytes(uint64_t cnt, uint32_t n);
hipError_t sort_pairs_device(const gg_pair* d_pairs, uint64_t cnt, uint32_t n, uint64_t* keys, uint64_t* keys_out,
                             uint32_t* idx, uint32_t* idx_out, gg_pair* sorted, void* tmp, size_t tmp_bytes,
                             hipStream_t st);

// synth.hip
hipError_t launch_synth(uint32_t first_genome, uint32_t n_genomes, uint32_t genome_len,
                        uint32_t cluster_size, float max_sub_rate,
                        uint64_t seed, uint32_t* words, hipStream_t st);

hipError_t launch_synth_mixed(uint32_t first_genome, uint32_t n_genomes, const uint64_t* d_woff,
                              uint64_t max_words, uint32_t cluster_size, float max_sub_rate, uint64_t seed,
                              uint32_t* words, hipStream_t st);

// Size and mtime of a genome file, taken before it is read: a cache entry
// is stored only if the file still has them afterwards.
struct FileStamp {
  uint64_t size = 0;
  int64_t mtime_ns = 0;
  bool ok = false;
};
bool file_stamp(const char* path, FileStamp* out);

// pack.cpp: streaming ingest for gg_precluster_files / gg_sketch_files.
// Files are read, gunzipped and packed on n_threads workers (<= 0: the
// default of gg_pack_files) in index order; consumers take genome i with
// get(i) (blocks until it is packed) and give its memory back with
// release(i).  Workers stop taking new files while the packed, unreleased
// genomes hold more than budget_bytes (the genome at the release frontier
// is always taken), so host memory stays bounded whatever the file count.
int ingest_threads(int n_threads);
class PackStream {
 public:
  // raw: the workers only read (and decompress) each file and keep its
  // FASTA text for the device parser (parse.hip); FASTQ files are rewritten
  // as FASTA records on the way.  Otherwise they pack on the host.  (Gzip
  // lists for the device inflate are read by ingest_gz.cpp's stagers.)
  PackStream(const char* const* paths, uint32_t n, int k, int n_threads, uint64_t budget_bytes,
             bool stamp_files = false, bool raw = false);
  ~PackStream();
  PackStream(const PackStream&) = delete;
  PackStream& operator=(const PackStream&) = delete;
  // words: 2-bit packed bases of genome i from word 0; runs: its ACGT runs
  // (base relative to word 0, genome field unused).  Valid until release(i).
  gg_status get(uint32_t i, const std::vector<uint32_t>** words, const std::vector<gg_run>** runs,
                std::string* err);
  // raw streams: genome i's FASTA text.  Valid until release(i).
  gg_status get_raw(uint32_t i, const std::vector<uint8_t>** text, std::string* err);
  // The file's size and mtime as stat'ed just before it was read (valid
  // after get(i) succeeded; the streams are built with stamp_files).
  FileStamp stamp(uint32_t i);
  void release(uint32_t i);
  void abort();
  // After an abort: joins the workers and returns the error of the lowest
  // failing file index among the files read (every index below a failing
  // one has been read), GG_OK if none failed.
  gg_status first_error(std::string* err);

 private:
  struct Impl;
  std::unique_ptr<Impl> p_;
};

// The FASTA text of a file's bytes as the raw streams give it (gzip, bzip2
// or xz decoded on the host by their magic, FASTQ records rewritten): the
// host fallback of the device inflate.  bytes may be consumed.
gg_status host_text_from_bytes(std::vector<uint8_t>& bytes, const char* name, std::vector<uint8_t>& text,
                               std::string& err);

// api.cpp helpers used by pack.cpp
void set_thread_error(const std::string& msg);

// sketch_cache.cpp
void cache_load_many(const char* dir, const char* const* paths, uint32_t n, int k, uint32_t s,
                     uint64_t seed, uint64_t* rows, uint32_t* lens, uint8_t* hit);
gg_status cache_store(const char* dir, const char* path, int k, uint32_t s, uint64_t seed,
                      const uint64_t* hashes, uint32_t len, const FileStamp* before);

// host arithmetic (api.cpp)
double ani_f64(uint32_t common, uint32_t total, int k);
std::vector<uint32_t> build_cmin(uint32_t s, int k, float min_ani);

}  // namespace gg
