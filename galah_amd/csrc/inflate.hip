// Device gzip inflate: gzip FASTA files go to the GPU compressed (PCIe and
// host memory carry ~1/3 of the text bytes, and the host threads only read
// files) and come out as the FASTA text parse.hip reads.  finch's
// sketch_files (src/finch.rs:47) reads .fna.gz through needletail / flate2;
// the host path (pack.cpp) decodes with libdeflate on the host threads.
//
// DEFLATE is serial within a stream, so the parallel units are the stream's
// blocks (zlib level 6: ~16k symbols, ~100 KB of FASTA each; a 3 Mbp genome
// has ~30 of them).  Kernels (inflate_core.hpp has the bit-level decoding):
//   inflate_search_kernel   one wave per ~4 KB chunk of compressed data: the
//                           first bit position where a dynamic block header
//                           parses (64 positions per step, one per lane)
//   inflate_decode_kernel   one lane per found start: Huffman-decode into
//                           tokens until landing on the next start (its own
//                           tables in LDS, 4 tokens per 16-byte store)
//   inflate_place_kernel    one workgroup per lane: token output offsets by
//                           a block scan, every output byte written as a
//                           literal or a pointer to the earlier byte it
//                           copies (the 32 KB window is never needed)
//   inflate_resolve_kernel  pointers followed to their literals, 16 bytes per
//                           thread, each resolved byte written back (later
//                           chains through it stop there)
//   inflate_crc_kernel      one workgroup per file: CRC-32 of the text
//                           (segments, folded with x^(8n) mod P), checked with
//                           ISIZE against the gzip trailer by the host
#include "device_util.hpp"
#include "gg_internal.hpp"
#include "inflate_core.hpp"

namespace gg {
namespace {

using namespace inflate;

constexpr int kSearchWaves = 4;  // chunks per search workgroup (one wave each)

__global__ __launch_bounds__(64 * kSearchWaves) void inflate_search_kernel(InflateSearch a) {
  const uint32_t c = blockIdx.x * kSearchWaves + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  if (c >= a.n_chunks) return;
  const uint32_t f = a.chunk_file[c];
  const Bits in{a.in + a.file_word[f]};
  const uint64_t b0 = a.chunk_bit0[c];
  const uint64_t b1 = min(b0 + (uint64_t)a.chunk_bits, a.file_bits[f]);
  uint64_t found = ~0ull;
  for (uint64_t p0 = b0; p0 < b1; p0 += 64) {  // (uniform per wave)
    const uint64_t p = p0 + lane;
    bool ok = false;
    if (p < b1) {
      uint64_t q = p;
      ok = block_header_ok(in, q);
    }
    const uint64_t m = __ballot(ok);
    if (m) {
      found = p0 + (uint64_t)(__ffsll((unsigned long long)m) - 1);
      break;
    }
  }
  if (lane == 0) a.start[c] = found;
}

struct LdsStore {
  int32_t* lb;
  int32_t* db;
  uint16_t* ls;
  uint8_t* ds;
  __device__ int32_t& lbase(int l) { return lb[l]; }
  __device__ int32_t& dbase(int l) { return db[l]; }
  __device__ uint16_t& lsym(int i) { return ls[i]; }
  __device__ uint8_t& dsym(int i) { return ds[i]; }
};

constexpr int kDecodeLanes = 64;  // one wave per workgroup: its lanes' tables fill ~47 KB of LDS

__global__ __launch_bounds__(kDecodeLanes) void inflate_decode_kernel(InflateDecode a) {
  __shared__ int32_t lb[kDecodeLanes][kMaxBits + 1], db[kDecodeLanes][kMaxBits + 1];
  __shared__ uint16_t ls[kDecodeLanes][kLitSyms];
  __shared__ uint8_t ds[kDecodeLanes][kDistSyms];
  const uint32_t t = threadIdx.x;
  const uint32_t lane = blockIdx.x * kDecodeLanes + t;
  if (lane >= a.n_lanes) return;
  LaneTables<LdsStore> tab;
  tab.s = LdsStore{lb[t], db[t], ls[t], ds[t]};
  const uint32_t f = a.lane_file[lane];
  const Bits in{a.in + a.file_word[f]};
  uint32_t* out = a.tok + a.tok_off[lane];
  const uint64_t cap = a.tok_cap[lane];
  uint64_t n = 0;
  uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;  // the last 4 tokens (a 16-byte store every 4)
  auto emit = [&](uint32_t tk) -> bool {
    if (n >= cap) return false;
    w0 = w1;
    w1 = w2;
    w2 = w3;
    w3 = tk;
    ++n;
    if ((n & 3u) == 0) *(uint4*)(out + n - 4) = make_uint4(w0, w1, w2, w3);
    return true;
  };
  uint64_t out_len = 0, last_end = 0;
  uint32_t fin = 0;
  uint32_t st = decode_blocks(in, a.lane_start[lane], a.lane_end[lane], a.file_bits[f], tab, emit, out_len, last_end,
                              fin);
  if (st == kDecOk && n >= cap && cap) st = kDecOk;  // (exactly full is fine)
  const uint32_t r = (uint32_t)(n & 3u);  // tokens not yet stored: the last r
  if (r >= 1) out[n - 1] = w3;
  if (r >= 2) out[n - 2] = w2;
  if (r >= 3) out[n - 3] = w1;
  a.status[lane] = st;
  a.n_tok[lane] = n;
  a.out_len[lane] = out_len;
  a.last_end[lane] = last_end;
  a.bfinal[lane] = fin;
}

// One workgroup per decode lane: tiles of 256 tokens, each token's output
// offset by a block scan of the token lengths, literals written as
// 0x80000000 | byte and match bytes as the batch position they copy.
constexpr int kPlaceThreads = 256;
__global__ __launch_bounds__(kPlaceThreads) void inflate_place_kernel(InflatePlace a) {
  __shared__ uint32_t wsum[kPlaceThreads / 64];
  __shared__ uint32_t tile_base;
  const uint32_t lane = blockIdx.x;
  const uint32_t tid = threadIdx.x, ln = tid & 63u, wave = tid >> 6;
  const uint32_t* tok = a.tok + a.tok_off[lane];
  const uint64_t n = a.n_tok[lane];
  const uint64_t text0 = a.file_text[a.lane_file[lane]];  // the file's first text position
  uint64_t base = a.lane_out[lane];
  bool bad = false;
  for (uint64_t t0 = 0; t0 < n; t0 += kPlaceThreads) {
    const uint64_t ti = t0 + tid;
    const uint32_t tk = ti < n ? tok[ti] : 0u;
    const uint32_t len = ti < n ? tok_len(tk) : 0u;
    uint32_t inc = len;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if (ln >= (uint32_t)o) inc += y;
    }
    if (ln == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t before = inc - len;
    for (uint32_t w = 0; w < wave; ++w) before += wsum[w];
    if (tid == kPlaceThreads - 1) tile_base = before + len;
    const uint64_t pos = base + before;
    if (ti < n) {
      if (!tok_is_match(tk)) {
        a.val[pos] = 0x80000000u | tk;
      } else {
        const uint32_t dist = tok_dist(tk);
        if (pos < text0 + dist) {
          bad = true;  // a distance before the file's first byte
        } else {
          for (uint32_t j = 0; j < len; ++j) a.val[pos + j] = (uint32_t)(pos + j - dist);
        }
      }
    }
    __syncthreads();
    base += tile_base;
    __syncthreads();
  }
  if (bad) atomicOr(a.flags, 1u);
}

// Pointers followed to their literals; 16 output bytes per thread, written
// as one store; every resolved byte is written back as a literal.
__global__ __launch_bounds__(256) void inflate_resolve_kernel(uint32_t* __restrict__ val, uint8_t* __restrict__ text,
                                                              uint64_t n, uint32_t* __restrict__ flags) {
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g * 16 < n; g += (uint64_t)gridDim.x * 256) {
    uint32_t out[4] = {0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const uint64_t i = g * 16 + b;
      uint32_t byte = '\n';  // (positions between files: the parser's padding)
      if (i < n) {
        uint32_t v = val[i];
        uint32_t hops = 0;
        while (!(v >> 31)) {
          v = __atomic_load_n(&val[v], __ATOMIC_RELAXED);
          if (++hops > (1u << 22)) {  // (cannot happen: every pointer goes back)
            atomicOr(flags, 2u);
            break;
          }
        }
        if (hops) __atomic_store_n(&val[i], v, __ATOMIC_RELAXED);
        byte = v & 0xFFu;
      }
      out[b >> 2] |= byte << (8 * (b & 3));
    }
    if (g * 16 + 16 <= n) *(uint4*)(text + g * 16) = make_uint4(out[0], out[1], out[2], out[3]);
    else
      for (int b = 0; b < 16 && g * 16 + b < n; ++b) text[g * 16 + b] = (uint8_t)(out[b >> 2] >> (8 * (b & 3)));
  }
}

// CRC-32 (gzip, reflected 0xEDB88320), table in LDS.
constexpr uint32_t kCrcPoly = 0xEDB88320u;
__device__ uint32_t crc_mul(uint32_t a, uint32_t b) {  // a * b mod P (reflected)
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = b & 1 ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}
__device__ uint32_t crc_x8n(uint64_t n, const uint32_t* __restrict__ x2k) {  // x^(8n) mod P
  uint32_t p = 1u << 31;  // x^0
  uint32_t k = 3;
  while (n) {
    if (n & 1) p = crc_mul(x2k[k & 63], p);
    n >>= 1;
    ++k;
  }
  return p;
}

constexpr int kCrcThreads = 256;
constexpr uint64_t kCrcSeg = 16384;  // bytes per thread per round
__global__ __launch_bounds__(kCrcThreads) void inflate_crc_kernel(const uint8_t* __restrict__ text,
                                                                  const uint64_t* __restrict__ file_text,
                                                                  const uint64_t* __restrict__ file_len,
                                                                  uint32_t* __restrict__ crc_out) {
  __shared__ uint32_t table[256];
  __shared__ uint32_t x2k[64];
  __shared__ uint32_t seg[kCrcThreads];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 256; i += kCrcThreads) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = c & 1 ? (c >> 1) ^ kCrcPoly : c >> 1;
    table[i] = c;
  }
  if (tid == 0) {  // x^(2^k) mod P
    uint32_t p = 1u << 30;  // x^1
    for (int k = 0; k < 64; ++k) {
      x2k[k] = p;
      p = crc_mul(p, p);
    }
  }
  __syncthreads();
  const uint32_t f = blockIdx.x;
  const uint8_t* t = text + file_text[f];
  const uint64_t len = file_len[f];
  uint32_t crc = 0;  // of the bytes so far (standard CRC-32; 0 for none)
  for (uint64_t r0 = 0; r0 < len; r0 += kCrcSeg * kCrcThreads) {
    const uint64_t s0 = r0 + tid * kCrcSeg;
    const uint64_t s1 = min(s0 + kCrcSeg, len);
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = s0; i < s1; ++i) c = table[(c ^ t[i]) & 0xFFu] ^ (c >> 8);
    seg[tid] = s0 < s1 ? ~c : 0u;
    __syncthreads();
    if (tid == 0) {  // crc(A || B) = x^(8|B|) crc(A) ^ crc(B)
      for (uint32_t k = 0; k < kCrcThreads; ++k) {
        const uint64_t a0 = r0 + k * kCrcSeg;
        if (a0 >= len) break;
        const uint64_t bl = min(kCrcSeg, len - a0);
        crc = crc_mul(crc_x8n(bl, x2k), crc) ^ seg[k];
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    crc_out[f] = crc;
    crc_out[gridDim.x + f] = len ? t[0] : 0u;  // (the caller checks the format: FASTA starts with '>')
  }
}

}  // namespace

hipError_t launch_inflate_search(const InflateSearch& a, hipStream_t st) {
  if (a.n_chunks == 0) return hipSuccess;
  hipLaunchKernelGGL(inflate_search_kernel, dim3((a.n_chunks + kSearchWaves - 1) / kSearchWaves),
                     dim3(64 * kSearchWaves), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_inflate_decode(const InflateDecode& a, hipStream_t st) {
  if (a.n_lanes == 0) return hipSuccess;
  hipLaunchKernelGGL(inflate_decode_kernel, dim3((a.n_lanes + kDecodeLanes - 1) / kDecodeLanes), dim3(kDecodeLanes),
                     0, st, a);
  return hipGetLastError();
}

hipError_t launch_inflate_place(const InflatePlace& a, uint64_t text_len, uint8_t* text, uint32_t n_files,
                                const uint64_t* file_text, const uint64_t* file_len, uint32_t* crc,
                                hipStream_t st) {
  if (a.n_lanes) hipLaunchKernelGGL(inflate_place_kernel, dim3(a.n_lanes), dim3(kPlaceThreads), 0, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint64_t groups = (text_len + 15) / 16;
  if (groups)
    hipLaunchKernelGGL(inflate_resolve_kernel, dim3((uint32_t)std::min<uint64_t>(65536, (groups + 255) / 256)),
                       dim3(256), 0, st, a.val, text, text_len, a.flags);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (n_files) hipLaunchKernelGGL(inflate_crc_kernel, dim3(n_files), dim3(kCrcThreads), 0, st, text, file_text,
                                  file_len, crc);
  return hipGetLastError();
}

}  // namespace gg
