// Which VALU instructions dual-issue on gfx950?  (round-2 K1 roofline)
//
// scripts/ubench_valu2.hip found most integer and f32 VALU instructions at
// ~4.2 cycles per wave64 instruction (effective clock, 8 waves/SIMD, 16
// independent chains) but v_lshrrev_b32 with an inline-constant shift at
// ~2.3, and rocprofv3 lists SQ_ACTIVE_INST_VALU2 ("quad-cycles in which two
// VALU instructions are issued").  This probe times operand-form variants
// (inline constant / SGPR / one or two VGPRs, 32- and 64-bit) and pairs of
// opcodes interleaved, to find the forms that co-issue.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/ubench_dual.hip -o scripts/ubench_dual
#include <hip/hip_runtime.h>

#include <cstdio>
#include <utility>

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

constexpr int kIters = 8192;
constexpr int kChains = 16;

#define VARIANTS(X)                                                                      \
  X(0, "add_u32 v,inl", A32("v_add_u32 %0, 3, %0"))                                     \
  X(1, "add_u32 v,s", A32("v_add_u32 %0, %1, %0"))                                      \
  X(2, "add_u32 v,v", A32("v_add_u32 %0, %2, %0"))                                      \
  X(3, "xor_b32 v,inl", A32("v_xor_b32 %0, 5, %0"))                                     \
  X(4, "xor_b32 v,v", A32("v_xor_b32 %0, %2, %0"))                                      \
  X(5, "lshrrev_b32 inl,v", A32("v_lshrrev_b32 %0, 3, %0"))                             \
  X(6, "lshrrev_b32 s,v", A32("v_lshrrev_b32 %0, %1, %0"))                              \
  X(7, "lshrrev_b32 v,v", A32("v_lshrrev_b32 %0, %2, %0"))                              \
  X(8, "lshlrev_b32 inl,v", A32("v_lshlrev_b32 %0, 3, %0"))                             \
  X(9, "and_b32 inl,v", A32("v_and_b32 %0, 63, %0"))                                    \
  X(10, "mul_lo_u32 v,v", A32("v_mul_lo_u32 %0, %0, %2"))                               \
  X(11, "mul_lo_u32 v,inl", A32("v_mul_lo_u32 %0, %0, 7"))                              \
  X(12, "mul_hi_u32 v,v", A32("v_mul_hi_u32 %0, %0, %2"))                               \
  X(13, "mov_b32 v", A32("v_mov_b32 %0, %2"))                                           \
  X(14, "alignbit v,v,inl", A32("v_alignbit_b32 %0, %0, %2, 7"))                        \
  X(15, "alignbit v,v(same),inl", A32("v_alignbit_b32 %0, %0, %0, 7"))                  \
  X(16, "add3_u32 v,v,v", A32("v_add3_u32 %0, %0, %2, %2"))                             \
  X(17, "add_f32 inl,v", A32("v_add_f32 %0, 1.0, %0"))                                  \
  X(18, "add_f32 v,v", A32("v_add_f32 %0, %2, %0"))                                     \
  X(19, "fma_f32 v,v,v", A32("v_fma_f32 %0, %0, %2, %2"))                               \
  X(20, "mad_u64_u32 v,v,v64", A64("v_mad_u64_u32 %0, vcc, %3, %3, %0"))                \
  X(21, "lshl_add_u64 v64,inl,v64", A64("v_lshl_add_u64 %0, %0, 2, %0"))                \
  X(22, "lshrrev_b64 inl,v64", A64("v_lshrrev_b64 %0, 33, %0"))                         \
  X(23, "lshlrev_b64 inl,v64", A64("v_lshlrev_b64 %0, 3, %0"))                          \
  X(24, "add_co/addc pair", A64P("v_add_co_u32 %0, vcc, %0, %3\n v_addc_co_u32 %1, vcc, %1, %3, vcc")) \
  X(25, "pk_add_f32", A64("v_pk_add_f32 %0, %0, %0"))                                   \
  X(26, "mix add_u32 v,s + lshr inl", MIX("v_add_u32 %0, %2, %0", "v_lshrrev_b32 %0, 3, %0")) \
  X(27, "mix mul_lo v,v + lshr inl", MIX("v_mul_lo_u32 %0, %0, %2", "v_lshrrev_b32 %0, 3, %0")) \
  X(28, "mix xor v,v + add v,v", MIX("v_xor_b32 %0, %2, %0", "v_add_u32 %0, %2, %0"))    \
  X(29, "mix mad_u64 + xor v,v", MIXW("v_mad_u64_u32 %1, vcc, %3, %3, %1", "v_xor_b32 %0, %2, %0")) \
  X(30, "cndmask_e32 vcc", A32("v_cndmask_b32_e32 %0, %2, %0, vcc"))                    \
  X(31, "bfe_u32 v,inl,inl", A32("v_bfe_u32 %0, %0, 8, 8"))                             \
  X(32, "lshlrev_b32 sdwa", A32("v_lshlrev_b32_sdwa %0, 3, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1")) \
  X(33, "cmp_lt_u32 + cndmask_e32 (2)", A64P("v_cmp_lt_u32_e32 vcc, %0, %3\n v_cndmask_b32_e32 %0, %3, %0, vcc")) \
  X(34, "cndmask_e64 sgpr-pair mask", A32M("v_cndmask_b32_e64 %0, %0, %2, %3"))            \
  X(35, "add_u32 literal,v", A32("v_add_u32_e32 %0, 0x12345, %0"))                        \
  X(36, "xor_b32 literal,v", A32("v_xor_b32_e32 %0, 0x12345678, %0"))                     \
  X(37, "or3_b32 v,v,v", A32("v_or3_b32 %0, %0, %2, %2"))                                  \
  X(38, "and_or_b32 v,inl,v", A32("v_and_or_b32 %0, %0, 63, %2"))                          \
  X(39, "lshl_or_b32 v,inl,v", A32("v_lshl_or_b32 %0, %0, 3, %2"))                         \
  X(40, "perm_b32 v,v,v", A32("v_perm_b32 %0, %0, %2, %2"))                                \
  X(41, "mov_b32 from sgpr", A32("v_mov_b32 %0, %1"))                                      \
  X(42, "lshlrev_b32 v,v", A32("v_lshlrev_b32 %0, %2, %0"))                                \
  X(43, "lshl_add_u32 v,inl,v", A32("v_lshl_add_u32 %0, %0, 3, %2"))                       \
  X(44, "sub_u32 v,v", A32("v_sub_u32 %0, %0, %2"))                                        \
  X(45, "ffbl_b32 v", A32("v_ffbl_b32 %0, %0"))                                            \
  X(46, "add_co_u32_e32 v,v (carry out)", A32("v_add_co_u32_e32 %0, vcc, %2, %0"))         \
  X(47, "mad_u32_u24 v,v,v", A32("v_mad_u32_u24 %0, %0, %2, %2"))                          \
  X(48, "mul_u32_u24 v,v", A32("v_mul_u32_u24 %0, %0, %2"))                                \
  X(49, "mul_hi_u32_u24 v,v", A32("v_mul_hi_u32_u24 %0, %0, %2"))                          \
  X(50, "xad_u32 v,v,v", A32("v_xad_u32 %0, %0, %2, %2"))                                  \
  X(51, "bitop3_b32 v,v,v", A32("v_bitop3_b32 %0, %0, %2, %2 bitop3:0x96"))                \
  X(52, "alignbit v,v,v", A32("v_alignbit_b32 %0, %0, %2, %2"))                            \
  X(53, "lshrrev+xor pair (xorshift)", A64P("v_lshrrev_b32 %1, 1, %0\n v_xor_b32 %0, %0, %1")) \
  X(54, "add_u32 v,v dep chain x1", A1("v_add_u32 %0, %0, %2"))                            \
  X(55, "cmp_lt_u64 + 2 cndmask (3)", A64Q("v_cmp_lt_u64_e32 vcc, %0, %3\n v_cndmask_b32_e32 %1, %1, %4, vcc\n v_cndmask_b32_e32 %2, %2, %5, vcc")) \
  X(56, "pk_mul_lo_u16 v,v", A32("v_pk_mul_lo_u16 %0, %0, %2"))                            \
  X(57, "lshlrev_b32 inl,v e64", A32("v_lshlrev_b32_e64 %0, 3, %0"))                       \
  X(58, "lshlrev_b16 inl,v", A32("v_lshlrev_b16 %0, 3, %0"))                               \
  X(59, "add_lshl_u32 v,v,inl", A32("v_add_lshl_u32 %0, %0, %2, 3"))                     \
  X(60, "mul_lo_u32 v,s", A32("v_mul_lo_u32 %0, %0, %1"))                                  \
  X(61, "mul_hi_u32 v,s", A32("v_mul_hi_u32 %0, %0, %1"))                                  \
  X(62, "mad_u64_u32 v,s,v64", A64("v_mad_u64_u32 %0, vcc, %3, %1, %0"))                   \
  X(63, "lshl_add_u64 v64,0,s64", A64S("v_lshl_add_u64 %0, %0, 0, %1"))                    \
  X(64, "lshl_add_u64 v64,0,v64", A64V("v_lshl_add_u64 %0, %0, 0, %1"))                    \
  X(65, "mad_u64_u32 v,v,0", A64("v_mad_u64_u32 %0, vcc, %3, %3, 0"))                      \
  X(66, "min_u32 v,v", A32("v_min_u32 %0, %2, %0"))                                        \
  X(67, "cmp_lt_u64_e64 + 2 cndmask_e64 (3)", A64C("v_cmp_lt_u64_e64 %3, %0, %4\n v_cndmask_b32_e64 %1, %1, %5, %3\n v_cndmask_b32_e64 %2, %2, %6, %3")) \
  X(68, "min_f64 v64,v64", A64V("v_min_f64 %0, %0, %1"))                                   \
  X(69, "mad_u64_u32 v,v,s64", A64SY("v_mad_u64_u32 %0, vcc, %2, %2, %1"))                  \
  X(70, "mul_hi_u32 v,v,+mul_lo v,v (2)", A64P("v_mul_hi_u32 %0, %0, %3\n v_mul_lo_u32 %1, %1, %3")) \
  X(71, "mad_u64_u32 v,v(vgpr c),v64", A64("v_mad_u64_u32 %0, vcc, %3, %2, %0"))

// 32-bit chains r[q]; 64-bit chains w[q]; y: a VGPR, c: an SGPR
#define A32(S) asm volatile(S : "+v"(r[q]) : "s"(c), "v"(y));
#define A64(S) asm volatile(S : "+v"(w[q]) : "s"(c), "v"(y), "v"(y) : "vcc");
#define A64P(S) asm volatile(S : "+v"(lo[q]), "+v"(hi[q]) : "s"(c), "v"(y) : "vcc");
#define A32M(S) asm volatile(S : "+v"(r[q]) : "s"(c), "v"(y), "s"(mask));
#define A64S(S) asm volatile(S : "+v"(w[q]) : "s"(mask) : "vcc");
#define A64SY(S) asm volatile(S : "+v"(w[q]) : "s"(mask), "v"(y) : "vcc");
#define A64V(S) asm volatile(S : "+v"(w[q]) : "v"(wy) : "vcc");
#define A64C(S) { uint64_t sm_; asm volatile(S : "+v"(w[q]), "+v"(lo[q]), "+v"(hi[q]), "=&s"(sm_) : "v"(wy), "v"(y), "v"(y)); }
#define A1(S) { if (q == 0) asm volatile(S : "+v"(r[q]) : "s"(c), "v"(y)); }
#define A64Q(S) asm volatile(S : "+v"(w[q]), "+v"(lo[q]), "+v"(hi[q]) : "v"(wy), "v"(y), "v"(y) : "vcc");
#define MIX(S1, S2)                                            \
  {                                                            \
    if (q & 1) asm volatile(S1 : "+v"(r[q]) : "s"(c), "v"(y)); \
    else asm volatile(S2 : "+v"(r[q]) : "s"(c), "v"(y));       \
  }
#define MIXW(S1, S2)                                                                  \
  {                                                                                   \
    if (q & 1) asm volatile(S1 : "+v"(r[q]), "+v"(w[q]) : "s"(c), "v"(y) : "vcc");   \
    else asm volatile(S2 : "+v"(r[q]) : "s"(c), "v"(y));                              \
  }

#define KCASE(ID, NAME, BODY) if (V == ID) BODY
#define NAMES(ID, NAME, BODY) NAME,
static const char* kNames[] = {VARIANTS(NAMES)};
constexpr int kVariants = sizeof(kNames) / sizeof(kNames[0]);

template <int V>
__global__ __launch_bounds__(256) void ubench(uint32_t* out, uint32_t seed) {
  uint32_t r[kChains], lo[kChains], hi[kChains];
  uint64_t w[kChains];
  const uint32_t y = threadIdx.x * 0x9E3779B9u + seed;
  const uint32_t c = 0x85EBCA6Bu ^ seed;
  const uint64_t mask = 0xF0F0F0F0F0F0F0F0ull ^ seed;
  const uint64_t wy = ((uint64_t)y << 32) | (y * 5u);
#pragma unroll
  for (int q = 0; q < kChains; ++q) {
    r[q] = threadIdx.x + q * 7919u + seed;
    lo[q] = r[q] * 3u;
    hi[q] = r[q] ^ 0x1234u;
    w[q] = ((uint64_t)r[q] << 32) | (r[q] * 3u);
  }
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int q = 0; q < kChains; ++q) {
      VARIANTS(KCASE)
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int q = 0; q < kChains; ++q) x ^= r[q] ^ lo[q] ^ hi[q] ^ (uint32_t)w[q] ^ (uint32_t)(w[q] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int V>
int run(uint32_t* d_out, int n_cu, int wps) {
  const int blocks = n_cu * wps;
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(ubench<V>, dim3(blocks), dim3(256), 0, 0, d_out, 1u);
  CHK(hipDeviceSynchronize());
  const int reps = 3;
  CHK(hipEventRecord(a));
  for (int rr = 0; rr < reps; ++rr) hipLaunchKernelGGL(ubench<V>, dim3(blocks), dim3(256), 0, 0, d_out, (uint32_t)rr);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double per = (V == 24 || V == 33 || V == 53 || V == 70) ? 2.0 : (V == 55 || V == 67) ? 3.0 : V == 54 ? 1.0 / kChains : 1.0;
  const double instr = per * kIters * kChains * wps;  // wave-instructions per SIMD
  std::printf("{\"variant\": %d, \"name\": \"%s\", \"waves_per_simd\": %d, \"ms_per_launch\": %.4f, "
              "\"cycles_per_instr_at_2.4GHz\": %.3f}\n",
              V, kNames[V], wps, ms / reps, (ms / reps) * 1e-3 * 2.4e9 / instr);
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(b));
  return 0;
}

template <int... V>
int run_all(uint32_t* d_out, int n_cu, int wps, std::integer_sequence<int, V...>) {
  int rc = 0;
  ((rc |= run<V>(d_out, n_cu, wps)), ...);
  return rc;
}

int main(int argc, char** argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 8;
  int n_cu = 0;
  CHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t* d_out;
  CHK(hipMalloc(&d_out, (size_t)n_cu * 8 * 256 * 4));
  const int rc = run_all(d_out, n_cu, wps, std::make_integer_sequence<int, kVariants>{});
  CHK(hipFree(d_out));
  return rc;
}
