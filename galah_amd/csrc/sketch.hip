// Kernel K1: canonical k-mer hashing and per-genome bottom-s selection.
//
// Restates, bit for bit, what finch's MashSketcher computes for galah
// (src/finch.rs:33-47: SketchParams::Mash{kmers_to_sketch: s, final_size: s,
// no_strict: true, kmer_length: k, hash_seed: 0}, no filtering):
//   for every k-mer window of A/C/G/T inside a record:
//     canonical = lexicographically smaller of fwd and reverse complement
//     h = murmurhash3_x64_128(canonical ASCII bytes, seed).0
//   sketch = the min(s, #distinct) smallest distinct h, ascending.
//
// MI355X design
//   * Input is 2-bit packed (0.25 B/base).  Each lane owns a segment of 44
//     consecutive k-mer positions of one run (k = 21), loads the 64-base
//     window at its start and that window's reverse complement once, and
//     takes every k-mer's forward and reverse-complement codes as static
//     64-bit slices of the two (the canonical code is a 64-bit min).  Each
//     workgroup sweeps a contiguous chunk of segments.
//   * The first multiply of each murmur3 input word, the rotates and the
//     second multiply of the k1 and k2 words, and the whole tail word are
//     folded into LDS tables indexed by 8-bit groups of 4 bases (see
//     hash_parts).
//   * Bottom-s selection is a threshold prefilter: a k-mer survives iff
//     h <= tau[g] where tau[g] ~ C*s/nk_g * 2^64, so only ~C*s of the
//     ~nk_g hashes per genome reach a per-genome open-addressing set in HBM
//     (atomicCAS, duplicates collapse).  The test runs on the high words of
//     the two finalisers first; the k-mers that pass go to a per-wave LDS
//     queue whose drain finishes the exact hash and inserts.  The finalize
//     kernel sorts the set in LDS, keeps the first s and leaves the set
//     empty.  When the set holds fewer than s distinct values below tau
//     (tau < 2^64-1) or overflows, the host moves tau and re-runs the
//     affected genomes only; the result is exact in both cases because every
//     distinct hash <= tau is in the set.
#include "device_util.hpp"
#include "gg_internal.hpp"

namespace gg {
namespace {

constexpr int kGroup = 4;  // k-mers per tau-check branch (1 or 2: within noise, profiles/r02_k1_group_defer_ab/)
// K1 workgroup size.  The LDS holds the murmur tables (19 KB at k = 21) once
// per workgroup and one candidate queue per wave; at 256 threads that is
// 24.5 KB, six workgroups per CU, six waves per SIMD.  512 threads (seven
// waves per SIMD, VGPR-bound), also with 128-entry queues, measured the same
// (C3 K1 47.02 / 46.89 vs 47.14 ms, C5 65.02 / 64.04 vs 65.19 / 64.38 ms:
// profiles/r03_b/k1_block512*).
constexpr int kBlock = 256;
// min waves per SIMD forced on the register allocator: 7 (72 VGPRs, 4 dwords
// spilled at k = 21) beats the unconstrained 76 VGPRs / 6 waves with the
// candidate queue (C3 K1 49.3 -> 49.1 ms, C5 78.7 -> 77.9 ms)
#ifndef GG_K1_MIN_WAVES
#define GG_K1_MIN_WAVES 7
#endif

// 64-bit rotate left by a compile-time amount as two v_alignbit_b32
// (hipcc otherwise emits a 64-bit shift + shift + or).
template <int R>
__device__ __forceinline__ uint64_t rotl64(uint64_t x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (R >= 32) {
    const uint32_t t = lo;
    lo = hi;
    hi = t;
  }
  constexpr int r = R & 31;
  if (r == 0) return ((uint64_t)hi << 32) | lo;
  const uint32_t nh = __builtin_amdgcn_alignbit(hi, lo, 32 - r);
  const uint32_t nl = __builtin_amdgcn_alignbit(lo, hi, 32 - r);
  return ((uint64_t)nh << 32) | nl;
}

// rotl(x, 31) + y: two v_alignbit_b32 and one v_lshl_add_u64 (a 64-bit
// add in one instruction, ~5 cycles per wave against 2 x 4.2 for an
// add_co / addc pair: profiles/r02_ubench_dual_8wps.txt).
__device__ __forceinline__ uint64_t add_rotl31(uint64_t x, uint64_t y) {
  const uint64_t r = rotl64<31>(x);
  uint64_t out;
  asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(out) : "v"(r), "v"(y));
  return out;
}

__device__ __forceinline__ uint64_t fmix_last(uint64_t k) { return k ^ (k >> 33); }

// fmix64 up to its second multiply: fmix64_pre(k) = fmix64_mid(k) * kFmixC2
constexpr uint64_t kFmixC2 = 0xc4ceb9fe1a85ec53ull;
__device__ __forceinline__ uint64_t fmix64_mid(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  return k ^ (k >> 33);
}
// high word of y * kFmixC2 (mod 2^64) without the low word: one v_mul_hi_u32
// and two v_mul_lo_u32 instead of a v_mad_u64_u32 and two v_mul_lo_u32
__device__ __forceinline__ uint32_t hi_times_c2(uint64_t y) {
  const uint32_t lo = (uint32_t)y, hi = (uint32_t)(y >> 32);
  return __umulhi(lo, (uint32_t)kFmixC2) + lo * (uint32_t)(kFmixC2 >> 32) + hi * (uint32_t)kFmixC2;
}

// h * 5 + c with one v_lshl_add_u64 (hipcc otherwise lowers the multiply by
// 5 to v_mad_u64_u32 sequences).
__device__ __forceinline__ uint64_t times5_plus(uint64_t h, uint64_t c) {
  uint64_t r;
  asm("v_lshl_add_u64 %0, %1, 2, %1" : "=v"(r) : "v"(h));
  return r + c;
}

// Tail words of at most kTailMaxBases bases get a whole-word table.
constexpr int kTailMaxBases = 5;

template <int K>
struct HashShape {
  static constexpr int NW = (K + 3) / 4;          // 4-base groups
  static constexpr int NBLK = K / 16;             // full 16-byte blocks
  static constexpr int TAIL = K % 16;             // tail bytes
  static constexpr bool TAIL_TAB = TAIL >= 1 && TAIL <= kTailMaxBases;
  // per full block (u64 units): k1 group tables of 16-byte {T * (c2 << 31),
  // hi(T)} and 8-byte {hi(T * (c2 << 31)), hi(T)} entries (the second group's
  // T has a zero low word, so has its product), k2 group tables of 16-byte
  // {P(T), hi(T), 0} (see hash_parts) and 4-byte hi(T) entries
  static constexpr int K1A = 0, K1B = 512, K2A = 768, K2B = 1280;
  static constexpr int BLK_U64 = 512 + 256 + 512 + 128;
  // tail: a whole-word table, or one 8-byte group table per tail group
  static constexpr int TAIL_GROUPS = TAIL_TAB ? 0 : NW - 4 * NBLK;
  static constexpr int TAIL_ENTRIES = TAIL_TAB ? (1 << (2 * TAIL)) : 0;
  static constexpr int TAIL_BASE = NBLK * BLK_U64;
  static constexpr int TAB_U64 = TAIL_BASE + TAIL_GROUPS * 256 + TAIL_ENTRIES;
};

// 8-bit code of bases 4q..4q+3 of a top-aligned MSB-first k-mer code
// (base 0 in bits 63..62): byte 3 - q%4 of word q/4.
__device__ __forceinline__ uint32_t group_byte(uint32_t hi, uint32_t lo, int q) {
  const uint32_t w = (q < 4) ? hi : lo;
  return (w >> (8 * (3 - (q & 3)))) & 0xFFu;
}

// murmurhash3_x64_128(bytes, seed).0 = fmix_last(f1) + fmix_last(f2) with
// (f1, f2) from hash_parts, where byte p = ASCII of base p of the
// k-mer whose MSB-first 2-bit code is top-aligned in `code` (base 0 in bits
// 63..62; bits below 64-2K are ignored, K <= 32).
//
// Every 8-byte word w of the input enters murmur3 as w * c (c = c1 for the
// k1 words, c2 for the k2 words).  Multiplication mod 2^64 distributes over
// the word's bytes, and the bytes are ASCII images of 2-bit codes, so
//   w * c = T[2i][g_2i] + T[2i+1][g_2i+1]      (mod 2^64)
// with g_q the 8-bit code of bases 4q..4q+3 and
//   T[q][g] = ascii4(g) * (c << 32*(q & 1))  (bytes past K masked out).
// T[odd q] has a zero low word, so hi(w * c) = hi(T[2i]) + hi(T[2i+1]).
//
// A block's k1 word continues as rotl(x, 31) * c2 with x = k1 * c1.  The
// rotate's halves x << 31 and x >> 33 have disjoint bits, so
//   rotl(x, 31) * c2 = x * (c2 << 31) + (hi(x) >> 1) * c2     (mod 2^64)
// and x * (c2 << 31) is again a sum of two table entries: the k1 group
// tables hold {T[q][g] * (c2 << 31), hi(T[q][g])}, and the rotate + full
// multiply become one 32 x 64-bit multiply-add.  Entries of odd groups have
// zero low words and are stored as their high words only (4 bytes less LDS
// traffic each; the LDS pipe runs at ~40% in this kernel).
//
// A tail k1 word of <= 5 bases (k = 21: bases 16..20) is a function of at
// most 10 bits, so its whole contribution rotl(w * c1, 31) * c2, and the
// final h1 ^= len, is one table entry.  Tables live in LDS
// (HashShape<K>::TAB_U64 entries).
template <int K>
__device__ __forceinline__ void hash_parts(uint64_t code, const uint64_t* __restrict__ tab,
                                           uint64_t seed, uint64_t& f1, uint64_t& f2) {
  using S = HashShape<K>;
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  const uint32_t hi = (uint32_t)(code >> 32), lo = (uint32_t)code;
  uint64_t h1 = seed, h2 = seed;
#pragma unroll
  for (int b = 0; b < S::NBLK; ++b) {
    const uint64_t* bt = tab + b * S::BLK_U64;
    const ulonglong2 e0 = *(const ulonglong2*)(bt + S::K1A + 2 * group_byte(hi, lo, 4 * b));
    const uint2 e1 = *(const uint2*)(bt + S::K1B + group_byte(hi, lo, 4 * b + 1));
    const ulonglong2 e2q = *(const ulonglong2*)(bt + S::K2A + 2 * group_byte(hi, lo, 4 * b + 2));
    const uint4 e2 = make_uint4((uint32_t)e2q.x, (uint32_t)(e2q.x >> 32), (uint32_t)e2q.y, (uint32_t)(e2q.y >> 32));
    const uint32_t t3 = ((const uint32_t*)(bt + S::K2B))[group_byte(hi, lo, 4 * b + 3)];
    // rotl(k1 * c1, 31) * c2
    const uint32_t v = ((uint32_t)e0.y + e1.y) >> 1;
    uint64_t k1 = (uint64_t)v * (uint32_t)c2 + (e0.x + ((uint64_t)e1.x << 32));
    k1 += (uint64_t)(v * (uint32_t)(c2 >> 32)) << 32;
    // rotl(k2 * c2, 33) * c1 = P + hx * (2 c1): x = k2 * c2 = T2 + (hi(T3) << 32);
    // rotl(x, 33) = (x << 33) + (x >> 31) (disjoint bits) and x >> 31 =
    // 2 hi(x) + bit 31 of lo(x) = 2 hi(x) + bit 31 of lo(T2), so
    // rotl(x, 33) * c1 = [T2 * (c1 << 33) + (lo(T2) >> 31) * c1] + hi(x) * 2 c1,
    // the bracket a table entry P of group 4b+2, hi(x) = hi(T2) + hi(T3)
    asm volatile("" ::"v"(e2.w));
    const uint32_t hx = e2.z + t3;
    uint64_t k2 = (uint64_t)hx * (uint32_t)(c1 << 1) + (((uint64_t)e2.y << 32) | e2.x);
    k2 += (uint64_t)(hx * (uint32_t)((c1 << 1) >> 32)) << 32;
    h1 ^= k1;
    h1 = rotl64<27>(h1); h1 += h2; h1 = times5_plus(h1, 0x52dce729);
    h2 ^= k2;
    h2 = add_rotl31(h2, h1); h2 = times5_plus(h2, 0x38495ab5);
  }
  const uint64_t* tt = tab + S::TAIL_BASE;
  if constexpr (S::TAIL_TAB) {
    const uint32_t w = S::NBLK ? lo : hi;
    h1 ^= tt[w >> (32 - 2 * S::TAIL)];  // includes ^= len
  } else {
    constexpr int q0 = 4 * S::NBLK;  // first group of the tail
    if (S::TAIL > 8) {
      uint64_t k2 = tt[2 * 256 + group_byte(hi, lo, q0 + 2)];
      if (q0 + 3 < S::NW) k2 += tt[3 * 256 + group_byte(hi, lo, q0 + 3)];
      k2 = rotl64<33>(k2); k2 *= c1; h2 ^= k2;
    }
    if (S::TAIL > 0) {
      uint64_t k1 = tt[group_byte(hi, lo, q0)];
      if (q0 + 1 < S::NW) k1 += tt[256 + group_byte(hi, lo, q0 + 1)];
      k1 = rotl64<31>(k1); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint64_t)K;
  }
  h2 ^= (uint64_t)K;
  h1 += h2;
  h2 += h1;
  f1 = fmix64_mid(h1);  // the caller finishes with kFmixC2 (hi_times_c2 / full)
  f2 = fmix64_mid(h2);
}

// ASCII bytes of `nbases` bases of an MSB-first code of `width` bases
// (base j of the code -> byte j).
__device__ __forceinline__ uint64_t ascii_msb(uint32_t codes, int width, int nbases) {
  uint64_t v = 0;
  for (int j = 0; j < nbases; ++j) {
    const uint32_t c = (codes >> (2 * (width - 1 - j))) & 3u;
    v |= (uint64_t)((0x54474341u >> (8 * c)) & 0xFFu) << (8 * j);  // 'A','C','G','T'
  }
  return v;
}

// T[q][g] of hash_parts: group q (bases 4q..4q+3, those past K masked out)
// as its word's bytes times the word's first multiplier
template <int K>
__device__ __forceinline__ uint64_t group_term(int q, uint32_t g) {
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  const int nb = min(4, K - 4 * q);                  // valid bases of the group
  const uint64_t cw = ((q >> 1) & 1) ? c2 : c1;      // k1 words: c1, k2 words: c2
  return (ascii_msb(g, 4, nb) << (32 * (q & 1))) * cw;
}

template <int K>
__device__ __forceinline__ void build_tables(uint64_t* tab) {
  using S = HashShape<K>;
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  const uint64_t c2r = c2 << 31;
  for (uint32_t i = threadIdx.x; i < (uint32_t)S::TAB_U64; i += blockDim.x) {
    if (i < (uint32_t)S::TAIL_BASE) {
      const uint32_t b = i / S::BLK_U64, r = i % S::BLK_U64;
      if (r < 512) {  // k1 group 4b: {T * (c2 << 31), hi(T)}
        const uint64_t t = group_term<K>((int)(4 * b), r >> 1);
        tab[i] = (r & 1u) ? (t >> 32) : t * c2r;
      } else if (r < 768) {  // k1 group 4b+1: {hi(T * (c2 << 31)), hi(T)}
        const uint64_t t = group_term<K>((int)(4 * b + 1), r - 512);
        tab[i] = ((t * c2r) >> 32) | (t & 0xFFFFFFFF00000000ull);
      } else if (r < 1280) {  // k2 group 4b+2: {P = T * (c1 << 33) + (lo(T) >> 31) * c1, hi(T)}
        const uint64_t t = group_term<K>((int)(4 * b + 2), (r - 768) >> 1);
        tab[i] = (r & 1u) ? (t >> 32) : t * (c1 << 33) + ((t & 0xFFFFFFFFull) >> 31) * c1;
      } else {  // k2 group 4b+3: hi(T), two entries per u64
        const uint32_t g = 2 * (r - 1280);
        tab[i] = (group_term<K>((int)(4 * b + 3), g) >> 32) |
                 (group_term<K>((int)(4 * b + 3), g + 1) & 0xFFFFFFFF00000000ull);
      }
    } else if (!S::TAIL_TAB) {
      const uint32_t r = i - (uint32_t)S::TAIL_BASE;
      tab[i] = group_term<K>(4 * S::NBLK + (int)(r >> 8), r & 255u);
    } else {
      // whole tail k1 word: bases 16*NBLK .. +TAIL-1 -> rotl(w * c1, 31) * c2 ^ len
      const uint32_t x = i - (uint32_t)S::TAIL_BASE;
      const uint64_t w = ascii_msb(x, S::TAIL, S::TAIL);
      tab[i] = (rotl64<31>(w * c1) * c2) ^ (uint64_t)K;
    }
  }
}

// Insert h into genome slot's open-addressing set (linear probing; one
// atomicCAS per probe, no per-genome counter: the finalize kernel counts the
// set when it gathers it).
__device__ __forceinline__ void insert_candidate(uint64_t* __restrict__ tab,
                                                 uint32_t mask,
                                                 uint32_t* __restrict__ flags,
                                                 uint64_t h) {
  if (h == kEmpty) {  // only reachable when tau == 2^64-1
    atomicOr(flags, kFlagSawMax);
    return;
  }
  uint32_t i = (uint32_t)h & mask;
  for (uint32_t probe = 0; probe <= mask; ++probe) {
    const unsigned long long old =
        atomicCAS((unsigned long long*)&tab[i], (unsigned long long)kEmpty,
                  (unsigned long long)h);
    if (old == kEmpty || old == h) return;
    i = (i + 1) & mask;
  }
  atomicOr(flags, kFlagOverflow);  // table full
}

// The candidates hv <= tau of the active lanes with `pass`, each of genome
// slot sl.  Append mode (a slot's first pass): the slot's candidates are a
// list [0, count) of its table region, one position per candidate from ONE
// atomicAdd per group of lanes holding the same slot (a wave's drain is
// almost always one genome: one atomic per ~32 candidates, and stores into
// consecutive positions), duplicates included (the finalize collapses them).
// Set mode (kFlagSetMode, after a list outgrew the finalize's sort): the
// open-addressing set of insert_candidate, one atomicCAS per probe.  Both
// are exact: every distinct hash <= tau is kept.  At s = 10000 (C5) the
// candidates were ~1.3e8 memory-side atomicCAS per step in set mode.
__device__ __forceinline__ void emit_candidates(bool pass, uint64_t hv, uint32_t sl, bool setm,
                                                uint64_t* __restrict__ table, uint32_t cap_log2,
                                                uint32_t* __restrict__ flags, uint32_t* __restrict__ count) {
  bool app = false;
  if (pass) {
    if (setm || hv == kEmpty)
      insert_candidate(table + ((uint64_t)sl << cap_log2), (1u << cap_log2) - 1u, flags + sl, hv);
    else
      app = true;
  }
  uint64_t pending = __ballot(app);
  const uint32_t lane = __lane_id();
  while (pending) {  // (uniform: a ballot of the active lanes)
    const uint32_t lead = (uint32_t)__ffsll((unsigned long long)pending) - 1u;
    const uint32_t lsl = __shfl(sl, lead);
    const uint64_t grp = __ballot(app && sl == lsl);
    uint32_t base = 0;
    if (lane == lead) base = atomicAdd(&count[lsl], (uint32_t)__popcll(grp));
    base = __shfl(base, lead);
    if (app && sl == lsl) {
      const uint32_t pos = base + (uint32_t)__popcll(grp & ((1ull << lane) - 1ull));
      if (pos < (1u << cap_log2)) table[((uint64_t)sl << cap_log2) + pos] = hv;
      else atomicOr(flags + sl, kFlagOverflow);  // (the finalize re-runs the slot in set mode)
      app = false;
    }
    pending &= ~grp;
  }
}

// Per-wave LDS queue of exact candidates (hash, genome slot).  Candidates
// are rare (0.05% of k-mers at s = 1000, 0.4% at s = 10000) and arise in
// scattered lanes; inserting each where it arises runs the atomicCAS probe
// loop with one or two lanes active and exposes its latency once per
// candidate.  Queued, they are inserted at segment ends, 32 or more at a
// time, one per lane.  Everything is LDS atomics (no ballot: the hash loop
// must stay fully unrolled, and the lanes of a wave diverge at run
// boundaries): a push takes a position with ds_add; a push that finds the
// ring full inserts directly; a drain hands out entries with ds_add too.
// An entry carries everything its drain needs (the k-mer's tau and its
// slot's collection mode), so a drain reads no global memory before its
// emit: with the tau and mode loads there, each drain waited on two
// dependent global round trips before its append atomic (C5: ~4e6 drains).
constexpr uint32_t kQueue = 64;
constexpr uint32_t kQueueDrain = kQueue / 2;
constexpr uint32_t kSlotSetMode = 1u << 31;  // slot field: the slot collects in set mode
struct CandQueue {
  uint64_t f1[kQueue], f2[kQueue];  // fmix64_mid of h1 / h2: the exact test runs at the drain
  uint64_t tau[kQueue];
  uint32_t slot[kQueue];            // | kSlotSetMode
  uint32_t head, tail, claim;
};

__device__ __forceinline__ uint64_t exact_hash(uint64_t f1, uint64_t f2) {
  return fmix_last(f1 * kFmixC2) + fmix_last(f2 * kFmixC2);
}

// A k-mer whose high-word sum passed the prefilter: queued with its two
// finaliser states; the drain finishes the hash and inserts it if <= tau.
__device__ __forceinline__ void queue_push_mid(CandQueue& q, uint64_t f1, uint64_t f2, uint32_t slot_mode,
                                               uint64_t tau, uint64_t* __restrict__ table,
                                               uint32_t cap_log2, uint32_t* __restrict__ flags,
                                               uint32_t* __restrict__ count) {
  const uint32_t pos = atomicAdd(&q.tail, 1u);
  const bool queued = pos - __atomic_load_n(&q.head, __ATOMIC_RELAXED) < kQueue;
  if (queued) {
    q.f1[pos & (kQueue - 1)] = f1;
    q.f2[pos & (kQueue - 1)] = f2;
    q.tau[pos & (kQueue - 1)] = tau;
    q.slot[pos & (kQueue - 1)] = slot_mode;
  }
  if (!queued) {  // ring full (rare): finish and emit this one now, on its own
    const uint64_t hv = exact_hash(f1, f2);
    const uint32_t slot = slot_mode & ~kSlotSetMode;
    if (hv <= tau) {
      if ((slot_mode & kSlotSetMode) || hv == kEmpty) {
        insert_candidate(table + ((uint64_t)slot << cap_log2), (1u << cap_log2) - 1u, flags + slot, hv);
      } else {
        const uint32_t at = atomicAdd(&count[slot], 1u);
        if (at < (1u << cap_log2)) table[((uint64_t)slot << cap_log2) + at] = hv;
        else atomicOr(flags + slot, kFlagOverflow);
      }
    }
  }
}

// Finish the queued candidates with the lanes that are active (all of them
// at the end of the kernel), entry x of the ring by fn(x).  Positions past
// head + kQueue were finished by their pushes.
template <class F>
__device__ __forceinline__ void queue_drain(CandQueue& q, uint32_t min_pending, F&& fn) {
  const uint32_t head = __atomic_load_n(&q.head, __ATOMIC_RELAXED);
  const uint32_t tail = __atomic_load_n(&q.tail, __ATOMIC_RELAXED);
  if (tail - head < min_pending || tail == head) return;
  const uint32_t end = tail - head < kQueue ? tail : head + kQueue;
  for (;;) {
    const uint32_t e = atomicAdd(&q.claim, 1u);
    if (e >= end) break;
    fn(e & (kQueue - 1));
  }
  // every active lane is past its last claim here (lockstep): reopen the ring
  __atomic_store_n(&q.head, tail, __ATOMIC_RELAXED);
  __atomic_store_n(&q.claim, tail, __ATOMIC_RELAXED);
}

// Largest r with ks[r] <= p, searching forward from `from` (the segments
// of one lane increase monotonically).
__device__ __forceinline__ uint32_t find_run(const uint64_t* __restrict__ ks,
                                             uint32_t n_runs, uint64_t p,
                                             uint32_t from) {
  if (ks[from + 1] > p) return from;
  // gallop
  uint32_t lo = from + 1, step = 1;
  uint32_t hi = lo;
  while (true) {
    hi = lo + step;
    if (hi >= n_runs || ks[hi] > p) break;
    lo = hi;
    step <<= 1;
  }
  if (hi > n_runs) hi = n_runs;
  // invariant: ks[lo] <= p, ks[hi] > p (ks[n_runs] = total > p)
  while (hi - lo > 1) {
    const uint32_t mid = lo + (hi - lo) / 2;
    if (ks[mid] <= p) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Reverse complement of 16 MSB-first 2-bit bases: reverse the base order
// (bit reverse, then swap the two bits of each base) and complement.
__device__ __forceinline__ uint32_t revcomp16(uint32_t x) {
  const uint32_t y = __builtin_bitreverse32(x);
  return ~(((y >> 1) & 0x55555555u) | ((y << 1) & 0xAAAAAAAAu));
}

// 32 bits of the base stream held in w[0..3] (MSB-first, 16 bases per word)
// starting at base t; bases past the window read as 0.  t is a compile-time
// constant after unrolling, so this is a register pick or one v_alignbit_b32.
__device__ __forceinline__ uint32_t window32(const uint32_t (&w)[4], int t) {
  const int a = t >> 4, sh = t & 15;
  const uint32_t x = a < 4 ? w[a] : 0u;
  if (sh == 0) return x;
  const uint32_t y = a + 1 < 4 ? w[a + 1] : 0u;
  return __builtin_amdgcn_alignbit(x, y, 32 - 2 * sh);
}

// 64 bits of the base stream starting at base t, top-aligned, of which the
// top 2K bits are exact (the k-mer starting at t).  pair[a] = w[a]:w[a+1].
// When the k-mer lies inside one pair (2 * (t % 16) + 2K <= 64) that is one
// full-rate v_lshlrev_b64 (or nothing); otherwise two v_alignbit_b32.
template <int K>
__device__ __forceinline__ uint64_t window64(const uint32_t (&w)[4], const uint64_t (&pair)[4], int t) {
  const int a = t >> 4, sh = t & 15;
  if (sh == 0) return pair[a];
  if (sh <= 32 - K) {
    uint64_t r;
    asm("v_lshlrev_b64 %0, %1, %2" : "=v"(r) : "i"(2 * sh), "v"(pair[a]));
    return r;
  }
  return ((uint64_t)window32(w, t) << 32) | window32(w, t + 16);
}

// Each lane owns one segment: kSeg consecutive k-mer positions of one run
// (the last segment of a run is shorter).  It loads the 64-base window
// starting at the segment's first base (5 words, funnel-shifted to the base
// offset) and its reverse complement.  The forward and reverse-complement
// codes of k-mer i of the window are then static 64-bit slices of the two
// windows, top-aligned (bits below the k-mer hold the following bases and
// are ignored): no rolling state, and the canonical code is a 64-bit min.
// K-mers past the segment (i >= cnt) are hashed but never inserted.
template <int K, bool SEED0>
__global__ __launch_bounds__(kBlock, GG_K1_MIN_WAVES) void sketch_candidates_kernel(SketchLaunch a) {
  constexpr int kSeg = k1_seg_len(K, kGroup);
  static_assert(K >= 1 && K <= 32 && kSeg + K - 1 <= 64 && kSeg % kGroup == 0, "window");
  if (a.bad_dev && *a.bad_dev != ~0ull) return;  // (uniform) a bad run table: the host reports it
  __shared__ __attribute__((aligned(16))) uint64_t mtab[HashShape<K>::TAB_U64];  // murmur word tables (hash_parts)
  __shared__ CandQueue queues[kBlock / 64];
  CandQueue& q = queues[threadIdx.x >> 6];
  // Workgroup b sweeps its own contiguous chunk of segments, kBlock at a
  // time (a wave's 64 lanes read consecutive windows).  A lane's next
  // segment is then kBlock segments on, in the same run or a few runs later,
  // so find_run's forward search is one or two loads; with a grid stride
  // it was ~50 genomes on (C3: ~14 dependent loads per segment, C5's 3.6M
  // runs ~30).
  const uint64_t n_segs = a.n_segs_dev ? *a.n_segs_dev : a.n_segs;
  const uint64_t per_wg = (n_segs + (uint64_t)gridDim.x * kBlock - 1) / ((uint64_t)gridDim.x * kBlock) * kBlock;
  const uint64_t c0 = a.seg0 + (uint64_t)blockIdx.x * per_wg;
  const uint64_t send = min(a.seg0 + n_segs, c0 + per_wg);
  if (c0 >= send) return;  // (uniform) no segment for this workgroup
  if ((threadIdx.x & 63) == 0) q.head = q.tail = q.claim = 0;
  build_tables<K>(mtab);
  __syncthreads();

  const uint64_t seed = SEED0 ? 0ull : a.seed;
  uint32_t r = 0;
  auto drain = [&](uint32_t min_pending) {
    queue_drain(q, min_pending, [&](uint32_t x) {
      const uint32_t sm = q.slot[x];
      const uint64_t hv = exact_hash(q.f1[x], q.f2[x]);
      emit_candidates(hv <= q.tau[x], hv, sm & ~kSlotSetMode, (sm & kSlotSetMode) != 0, a.table, a.cap_log2,
                      a.flags, a.count);
    });
  };

  for (uint64_t sg = c0 + threadIdx.x; sg < send; sg += kBlock) {
    r = find_run(a.run_sstart, a.n_runs, sg, r);
    const gg_run run = a.runs[r];
    const uint32_t k0 = (uint32_t)(sg - a.run_sstart[r]) * (uint32_t)kSeg;  // first k-mer of the segment in the run
    const uint32_t cnt = min((uint32_t)kSeg, run.len - (uint32_t)K + 1u - k0);
    const uint32_t slot = run.genome - a.slot_genome0;
    const uint64_t tau = a.tau[slot];
    // prefilter on the high words: h = fmix_last(f1) + fmix_last(f2)
    // has high word S or S + 1 (carry), S = hi(f1) + hi(f2), so h <= tau
    // needs S <= hi(tau) or S = 2^32 - 1, i.e. S + 1 <= hi(tau) + 1 (mod
    // 2^32; every S passes when hi(tau) = 2^32 - 1)
    const uint32_t tau_hi = (uint32_t)(tau >> 32);
    const uint32_t thr = tau_hi == 0xFFFFFFFFu ? 0xFFFFFFFFu : tau_hi + 1u;
    const uint64_t b = run.base + k0;  // first base of the segment's first k-mer

    const uint64_t wi = b >> 4;
    const uint32_t off = (uint32_t)b & 15u;
    uint32_t w[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) w[j] = (wi + j < a.n_words) ? a.words[wi + j] : 0u;
    uint32_t F[4], R[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      F[j] = off ? __builtin_amdgcn_alignbit(w[j], w[j + 1], 32 - 2 * off) : w[j];
#pragma unroll
    for (int m = 0; m < 4; ++m) R[m] = revcomp16(F[3 - m]);
    uint64_t FP[4], RP[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      FP[m] = ((uint64_t)F[m] << 32) | (m + 1 < 4 ? F[m + 1] : 0u);
      RP[m] = ((uint64_t)R[m] << 32) | (m + 1 < 4 ? R[m + 1] : 0u);
    }

#pragma unroll
    for (int g = 0; g < kSeg / kGroup; ++g) {
      uint64_t f1[kGroup], f2[kGroup];
#pragma unroll
      for (int j = 0; j < kGroup; ++j) {
        const int i = g * kGroup + j;
        const uint64_t fwd = window64<K>(F, FP, i);
        const int t0 = 64 - K - i;  // reverse complement of k-mer i starts here
        const uint64_t rev = window64<K>(R, RP, t0);
        hash_parts<K>(fwd < rev ? fwd : rev, mtab, seed, f1[j], f2[j]);
      }
      uint32_t hs[kGroup];  // S + 1 per k-mer
#pragma unroll
      for (int j = 0; j < kGroup; ++j) hs[j] = hi_times_c2(f1[j]) + hi_times_c2(f2[j]) + 1u;
      bool any = false;
#pragma unroll
      for (int j = 0; j < kGroup; ++j) any |= hs[j] <= thr;
      if (any) {
        // (a lane of the wave has a k-mer whose high-word sum can reach
        // tau): finish the exact test for the group's k-mers and queue
        // the candidates
#pragma unroll
        for (int j = 0; j < kGroup; ++j) {
          if (hs[j] <= thr && (uint32_t)(g * kGroup + j) < cnt)
            queue_push_mid(q, f1[j], f2[j], slot | ((a.any_set_mode && (a.flags[slot] & kFlagSetMode)) ? kSlotSetMode : 0u),
                           tau, a.table, a.cap_log2, a.flags, a.count);
        }
      }
    }
    drain(kQueueDrain);
  }
  drain(1);  // every lane of the wave is back
}

// One workgroup per genome slot: gather the slot's candidates into LDS,
// sort them, keep the first s distinct.  Writes status[] for the host retry
// loop.  The candidates are values spread uniformly over [0, tau], so they
// are sorted by buckets of the top bits below tau (a counting sort: LDS
// histogram, scan, scatter into the genome's own table region in HBM, and
// back into LDS in bucket order), then every value's place is the number of
// distinct values below it: the distinct values of the buckets before its
// own (a scan of per-bucket distinct counts) plus those below it in its
// bucket (~4 values: a few LDS reads and compares).  A set-mode slot holds
// distinct values; an append-mode list may repeat one (a k-mer that occurs
// twice): only the first copy of a value in its bucket counts.
//   append mode: the list is [0, count[slot]) of the table region; nothing
//     to clear afterwards but the count; a list longer than the sort (or
//     past the region) re-runs the slot at the same tau in set mode
//     (kSketchRetrySet), its region cleared here for the set
//   set mode: the set is the whole region (EMPTY = free), cleared afterwards
// (C5: the list is ~1.3 s entries where the set was 2 x 16384 slots, read
// and cleared: 2.6 GB each way per step.)  Any block size up to
// kFinalizeMaxBlock.
constexpr int kFinalizeMaxBlock = 1024;
__global__ __launch_bounds__(kFinalizeMaxBlock) void sketch_finalize_kernel(
    const uint32_t* __restrict__ slot_list, const uint32_t* __restrict__ slot_genome,
    const uint64_t* __restrict__ tau, uint64_t* __restrict__ table,
    uint32_t cap_log2,
    uint32_t* __restrict__ flags, uint32_t s, uint32_t sort_pow2, uint32_t nb_log2,
    const uint32_t* __restrict__ row_of, uint64_t* __restrict__ out, uint32_t* __restrict__ lens,
    uint32_t* __restrict__ status, uint32_t* __restrict__ count, const uint64_t* __restrict__ bad) {
  extern __shared__ uint64_t buf[];  // [sort_pow2] values, then [1 << nb_log2] u32 bucket counters
  uint32_t* cnt = reinterpret_cast<uint32_t*>(buf + sort_pow2);
  __shared__ uint32_t fill;
  __shared__ uint32_t wsum[kFinalizeMaxBlock / 64];
  const uint32_t slot = slot_list[blockIdx.x];
  // output row of the genome: the caller's row map when given (batches of a
  // streamed file list land on their global rows)
  const uint32_t g = row_of ? row_of[slot_genome[slot]] : slot_genome[slot];
  const uint32_t f = flags[slot];
  const bool setm = (f & kFlagSetMode) != 0;
  const uint32_t listed = count[slot];
  const uint32_t T = blockDim.x, tid = threadIdx.x, lane = tid & 63;
  uint64_t* tab = table + ((uint64_t)slot << cap_log2);
  const uint32_t cap = 1u << cap_log2;
  __syncthreads();  // (every thread has read flags[slot] and count[slot])
  auto clear_set = [&]() {
    for (uint32_t i = tid; i < cap; i += T) tab[i] = kEmpty;
  };
  // every path leaves the slot ready for the next K1 pass: count 0, flags 0
  // or kFlagSetMode (set mode next: the set cleared)
  auto finish = [&](uint32_t st, bool set_next) {
    if (set_next) clear_set();
    if (tid == 0) {
      flags[slot] = set_next ? kFlagSetMode : 0u;
      count[slot] = 0u;
      if (st != ~0u) {
        status[slot] = st;
        if (st != kSketchOk) lens[g] = 0;
      }
    }
  };
  if (bad && *bad != ~0ull) {  // (uniform) a bad run table: K1 did nothing, the caller's rows stay untouched
    finish(~0u, setm);
    return;
  }
  if (f & kFlagOverflow) {  // set: more distinct candidates than slots; list: past its region
    finish(setm ? kSketchRetrySmaller : kSketchRetrySet, true);
    return;
  }
  const uint32_t NB = 1u << nb_log2;
  const uint64_t t = tau[slot];
  // bucket = the nb_log2 bits below tau's top bit (monotone in the value)
  const uint32_t tbits = 64 - __builtin_clzll(t | 1ull);
  const uint32_t shift = tbits > nb_log2 ? tbits - nb_log2 : 0u;
  // exclusive scan of cnt's low halves (or high halves: hi) over the buckets:
  // each thread a contiguous range, the ranges' totals scanned across waves;
  // returns the total
  auto scan = [&](bool hi) -> uint32_t {
    const uint32_t per = (NB + T - 1) / T;
    const uint32_t b0 = min(tid * per, NB), b1 = min(b0 + per, NB);
    uint32_t sum = 0;
    for (uint32_t b = b0; b < b1; ++b) sum += hi ? cnt[b] >> 16 : cnt[b] & 0xFFFFu;
    uint32_t inc = sum;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if ((tid & 63) >= (uint32_t)o) inc += y;
    }
    if ((tid & 63) == 63) wsum[tid >> 6] = inc;
    __syncthreads();
    uint32_t run = inc - sum;
    for (uint32_t w = 0; w < (tid >> 6); ++w) run += wsum[w];
    uint32_t total = 0;
    for (uint32_t w = 0; w < (T + 63) / 64; ++w) total += wsum[w];
    for (uint32_t b = b0; b < b1; ++b) {
      const uint32_t c = cnt[b];
      if (hi) {
        cnt[b] = (c & 0xFFFFu) | (run << 16);
        run += c >> 16;
      } else {
        cnt[b] = run;
        run += c;
      }
    }
    __syncthreads();
    return total;
  };
  // (n <= sort_pow2 <= 16384: positions and counts fit 16 bits)
  uint32_t n;
  for (uint32_t i = tid; i < NB; i += T) cnt[i] = 0;
  if (!setm) {
    // The list is read from HBM twice: for the bucket histogram, then to
    // scatter each value straight to its bucket's place in LDS (a copy in
    // LDS scattered through the table region and read back cost a write and
    // a dependent read of the whole list).  8 values per thread per step,
    // all loads in flight at once (one load after another waited on HBM
    // latency each).
    n = listed;
    if (n > sort_pow2) {
      finish(kSketchRetrySet, true);
      return;
    }
    constexpr uint32_t kListV = 8;
    auto list_pass = [&](auto&& fn) {
      for (uint32_t i0 = tid * kListV; i0 < n; i0 += T * kListV) {
        uint64_t v[kListV];
#pragma unroll
        for (uint32_t j = 0; j < kListV; j += 2) {
          if (i0 + j + 1 < n) {
            const ulonglong2 p = *(const ulonglong2*)(tab + i0 + j);
            v[j] = p.x;
            v[j + 1] = p.y;
          } else if (i0 + j < n) {
            v[j] = tab[i0 + j];
          }
        }
#pragma unroll
        for (uint32_t j = 0; j < kListV; ++j)
          if (i0 + j < n) fn(v[j]);
      }
    };
    __syncthreads();
    list_pass([&](uint64_t v) { atomicAdd(&cnt[(uint32_t)(v >> shift)], 1u); });
    __syncthreads();
    scan(false);
    list_pass([&](uint64_t v) { buf[atomicAdd(&cnt[(uint32_t)(v >> shift)], 1u)] = v; });
    __syncthreads();  // (cnt[b] = end of bucket b)
  } else {
    if (tid == 0) fill = 0;
    __syncthreads();
    // gather: each thread 8 consecutive slots per step, all loads in flight
    // at once (one workgroup per CU at s = 10000: with one load per thread per
    // step the gather waited on HBM latency step after step), a wave prefix
    // sum of the values found and one LDS atomic per wave
    constexpr uint32_t kGatherV = 8;
    const uint32_t steps = (cap + T * kGatherV - 1) / (T * kGatherV);
    for (uint32_t it = 0; it < steps; ++it) {
      const uint32_t i0 = (it * T + tid) * kGatherV;
      uint64_t v[kGatherV];
#pragma unroll
      for (uint32_t j = 0; j < kGatherV; j += 2) {
        if (i0 + j < cap) {
          const ulonglong2 p = *(const ulonglong2*)(tab + i0 + j);
          v[j] = p.x;
          v[j + 1] = p.y;
        } else {
          v[j] = v[j + 1] = kEmpty;
        }
      }
      uint32_t c = 0;
#pragma unroll
      for (uint32_t j = 0; j < kGatherV; ++j) c += v[j] != kEmpty ? 1u : 0u;
      uint32_t inc = c;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= (uint32_t)o) inc += y;
      }
      uint32_t base = 0;
      if (lane == 63 && inc) base = atomicAdd(&fill, inc);
      uint32_t at = __shfl(base, 63) + inc - c;
#pragma unroll
      for (uint32_t j = 0; j < kGatherV; ++j) {
        if (v[j] != kEmpty) {
          if (at < sort_pow2) buf[at] = v[j];
          ++at;
        }
      }
    }
    __syncthreads();
    n = fill;  // distinct candidates <= tau
    if (n > sort_pow2) {  // cannot sort in LDS
      finish(kSketchRetrySmaller, true);
      return;
    }
    for (uint32_t e = tid; e < n; e += T) atomicAdd(&cnt[(uint32_t)(buf[e] >> shift)], 1u);
    __syncthreads();
    scan(false);
    // scatter into the table (afterwards cnt[b] = end of bucket b), then back
    // into LDS in bucket order
    for (uint32_t e = tid; e < n; e += T) {
      const uint64_t v = buf[e];
      tab[atomicAdd(&cnt[(uint32_t)(v >> shift)], 1u)] = v;
    }
    __syncthreads();
    for (uint32_t e0 = tid; e0 < n; e0 += 4 * T) {
      uint64_t v[4];
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) v[j] = e0 + j * T < n ? tab[e0 + j * T] : 0ull;
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j)
        if (e0 + j * T < n) buf[e0 + j * T] = v[j];
    }
    __syncthreads();
  }
  // the first copy of a value in its bucket: no equal value before it there
  auto first_copy = [&](uint32_t b0, uint32_t e, uint64_t v) {
    for (uint32_t q = b0; q < e; ++q)
      if (buf[q] == v) return false;
    return true;
  };
  // a list may repeat a value (a set never does): when it does, the
  // distinct values per bucket go to cnt's high halves and are scanned,
  // cnt[b] = end of bucket b | (distinct values before bucket b) << 16
  if (tid == 0) fill = 0;  // (any repeat)
  __syncthreads();
  if (!setm) {
    for (uint32_t e = tid; e < n; e += T) {
      const uint64_t v = buf[e];
      const uint32_t b = (uint32_t)(v >> shift);
      if (!first_copy(b ? cnt[b - 1] : 0u, e, v)) fill = 1u;
    }
  }
  __syncthreads();
  const bool dups = fill != 0;
  uint32_t distinct = n;
  if (dups) {
    for (uint32_t e = tid; e < n; e += T) {
      const uint64_t v = buf[e];
      const uint32_t b = (uint32_t)(v >> shift);
      const uint32_t b0 = b ? cnt[b - 1] & 0xFFFFu : 0u;
      if (first_copy(b0, e, v)) atomicAdd(&cnt[b], 1u << 16);
    }
    __syncthreads();
    distinct = scan(true);
  }
  uint32_t st = kSketchOk;
  if (distinct < s && t != kEmpty) st = kSketchRetryLarger;
  if (st != kSketchOk) {
    // (the table region held only the scatter's copies: a list needs no
    // clearing, a set is cleared for its next pass)
    finish(st, setm);
    return;
  }
  if (setm) clear_set();  // (the table's values are all in LDS now)
  // every first copy of a bucket whose distinct values start below s: its
  // rank among the distinct values
  uint64_t* o = out + (uint64_t)g * s;
  const uint32_t m = min(s, distinct);
  if (!dups) {  // every value distinct: its rank is its bucket's start plus the smaller values there
    for (uint32_t e = tid; e < n; e += T) {
      const uint64_t v = buf[e];
      const uint32_t b = (uint32_t)(v >> shift);
      const uint32_t b0 = b ? cnt[b - 1] : 0u, b1 = cnt[b];
      if (b0 >= m) continue;
      uint32_t r = b0;
      for (uint32_t q = b0; q < b1; ++q) r += buf[q] < v ? 1u : 0u;
      if (r < m) o[r] = v;
    }
  } else {  // the first copies only, ranked among the first copies
    for (uint32_t e = tid; e < n; e += T) {
      const uint64_t v = buf[e];
      const uint32_t b = (uint32_t)(v >> shift);
      const uint32_t b0 = b ? cnt[b - 1] & 0xFFFFu : 0u, b1 = cnt[b] & 0xFFFFu;
      const uint32_t d0 = cnt[b] >> 16;
      if (d0 >= m || !first_copy(b0, e, v)) continue;
      uint32_t r = d0;
      for (uint32_t q = b0; q < b1; ++q) {
        const uint64_t x = buf[q];
        if (x < v && first_copy(b0, q, x)) ++r;
      }
      if (r < m) o[r] = v;
    }
  }
  uint32_t mm = m;
  if ((f & kFlagSawMax) && mm < s) {
    if (tid == 0) o[mm] = kEmpty;  // 2^64-1 is the largest hash
    ++mm;
  }
  if (tid == 0) {
    lens[g] = mm;
    status[slot] = kSketchOk;
    flags[slot] = 0u;
    count[slot] = 0u;
  }
}

template <int K>
hipError_t launch_k(const SketchLaunch& a, int grid, hipStream_t st) {
  // finch always hashes with seed 0 (src/finch.rs:41); that variant drops the
  // seed terms from the murmur3 block at compile time.
  if (a.seed == 0)
    hipLaunchKernelGGL((sketch_candidates_kernel<K, true>), dim3(grid), dim3(kBlock), 0, st, a);
  else
    hipLaunchKernelGGL((sketch_candidates_kernel<K, false>), dim3(grid), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

}  // namespace

int sketch_segment_len(int k) { return k1_seg_len(k, kGroup); }


hipError_t launch_sketch_candidates(int k, const SketchLaunch& a, int grid,
                                    hipStream_t st) {
  if (a.n_segs == 0 && !a.n_segs_dev) return hipSuccess;
  switch (k) {
#define GG_K(N) case N: return launch_k<N>(a, grid, st);
    GG_K(1) GG_K(2) GG_K(3) GG_K(4) GG_K(5) GG_K(6) GG_K(7) GG_K(8)
    GG_K(9) GG_K(10) GG_K(11) GG_K(12) GG_K(13) GG_K(14) GG_K(15) GG_K(16)
    GG_K(17) GG_K(18) GG_K(19) GG_K(20) GG_K(21) GG_K(22) GG_K(23) GG_K(24)
    GG_K(25) GG_K(26) GG_K(27) GG_K(28) GG_K(29) GG_K(30) GG_K(31) GG_K(32)
#undef GG_K
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_sketch_finalize(const uint32_t* slot_list, uint32_t n_slots,
                                  const uint32_t* slot_genome,
                                  const uint64_t* tau, uint64_t* table,
                                  uint32_t cap_log2,
                                  uint32_t* flags, uint32_t s,
                                  uint32_t sort_pow2, const uint32_t* row_of, uint64_t* out,
                                  uint32_t* lens, uint32_t* status, uint32_t* count,
                                  hipStream_t st, const uint64_t* bad) {
  if (n_slots == 0) return hipSuccess;
  // ~4 candidates per bucket
  uint32_t nb_log2 = 6;
  while (nb_log2 < 12 && (1u << (nb_log2 + 2)) < sort_pow2) ++nb_log2;
  const size_t lds = (size_t)sort_pow2 * sizeof(uint64_t) + ((size_t)4 << nb_log2);
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute((const void*)sketch_finalize_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  // sorts of >= 4096 entries (>= 32 KiB of LDS: few workgroups per CU) get
  // 1024 threads; at s = 10000 (16384 entries) this cuts the finalize ~3x
  const int threads = sort_pow2 >= 4096 ? kFinalizeMaxBlock : 256;
  hipLaunchKernelGGL(sketch_finalize_kernel, dim3(n_slots), dim3(threads), lds, st,
                     slot_list, slot_genome, tau, table, cap_log2, flags, s,
                     sort_pow2, nb_log2, row_of, out, lens, status, count, bad);
  return hipGetLastError();
}

}  // namespace gg
