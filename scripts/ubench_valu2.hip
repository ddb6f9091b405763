// VALU issue-rate calibration for the K1 roofline (round 2).
//
// Cycles per wave64 instruction, per opcode, with 16 independent chains per
// wave (dependency distance 16) and 8 waves per SIMD (8 x 256-thread
// workgroups per CU: 2048 threads per CU), so neither latency nor occupancy
// limits issue.  Each opcode is its own kernel; run it under
//   rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES
// to read the effective clock of every dispatch (GRBM_GUI_ACTIVE / 8 is the
// per-XCD busy cycle count; MI355X_MICROARCH.md "DVFS give-back").  The
// program itself prints cycles at the nominal 2.4 GHz and the dispatch time.
//   hipcc -O3 --offload-arch=gfx950 scripts/ubench_valu2.hip -o scripts/ubench_valu2
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

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

enum Op {
  ADD_U32, XOR_B32, ADD3_U32, MUL_LO_U32, MUL_HI_U32, MAD_U64_U32, ALIGNBIT, LSHL_ADD_U64,
  LSHLREV_B64, CNDMASK, FMA_F32, ADD_F32, PK_FMA_F32, BITOP3, XAD_U32, LSHRREV_B32, OP_COUNT
};
static const char* kNames[OP_COUNT] = {
    "v_add_u32", "v_xor_b32", "v_add3_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32",
    "v_alignbit_b32", "v_lshl_add_u64", "v_lshlrev_b64", "v_cndmask_b32", "v_fma_f32", "v_add_f32",
    "v_pk_fma_f32", "v_bitop3_b32", "v_xad_u32", "v_lshrrev_b32"};

// one instruction on chain register x (32-bit chains)
#define C32(OPSTR) asm volatile(OPSTR : "+v"(r[q]) : "s"(c), "v"(y));
#define C64(OPSTR) asm volatile(OPSTR : "+v"(w[q]) : "s"(c), "v"(y) : "vcc");

template <int OP>
__global__ __launch_bounds__(256) void ubench(uint32_t* out, uint32_t seed) {
  uint32_t r[kChains];
  uint64_t w[kChains];
  const uint32_t y = threadIdx.x * 0x9E3779B9u + seed;
  const uint32_t c = 0x85EBCA6Bu ^ seed;
#pragma unroll
  for (int q = 0; q < kChains; ++q) {
    r[q] = threadIdx.x + q * 7919u + seed;
    w[q] = ((uint64_t)r[q] << 32) | (r[q] * 3u);
  }
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int q = 0; q < kChains; ++q) {
      if (OP == ADD_U32) C32("v_add_u32 %0, %0, %1")
      if (OP == XOR_B32) C32("v_xor_b32 %0, %1, %0")
      if (OP == ADD3_U32) C32("v_add3_u32 %0, %0, %1, %2")
      if (OP == MUL_LO_U32) C32("v_mul_lo_u32 %0, %0, %1")
      if (OP == MUL_HI_U32) C32("v_mul_hi_u32 %0, %0, %1")
      if (OP == MAD_U64_U32) C64("v_mad_u64_u32 %0, vcc, %2, %1, %0")
      if (OP == ALIGNBIT) C32("v_alignbit_b32 %0, %0, %2, 31")
      if (OP == LSHL_ADD_U64) C64("v_lshl_add_u64 %0, %0, 2, %0")
      if (OP == LSHLREV_B64) C64("v_lshlrev_b64 %0, 3, %0")
      if (OP == CNDMASK) C32("v_cndmask_b32 %0, %0, %2, vcc")
      if (OP == FMA_F32) C32("v_fma_f32 %0, %0, %1, %2")
      if (OP == ADD_F32) C32("v_add_f32 %0, %1, %0")
      if (OP == PK_FMA_F32) C64("v_pk_fma_f32 %0, %0, %0, %0")
      if (OP == BITOP3) C32("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
      if (OP == XAD_U32) C32("v_xad_u32 %0, %0, %1, %2")
      if (OP == LSHRREV_B32) C32("v_lshrrev_b32 %0, 3, %0")
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int q = 0; q < kChains; ++q) x ^= r[q] ^ (uint32_t)w[q] ^ (uint32_t)(w[q] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int OP>
int run(uint32_t* d_out, int n_cu, int waves_per_simd) {
  const int blocks = n_cu * waves_per_simd;  // 256-thread blocks: one wave per SIMD each
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(ubench<OP>, dim3(blocks), dim3(256), 0, 0, d_out, 1u);
  CHK(hipDeviceSynchronize());
  const int reps = 3;
  CHK(hipEventRecord(a));
  for (int rr = 0; rr < reps; ++rr) hipLaunchKernelGGL(ubench<OP>, dim3(blocks), dim3(256), 0, 0, d_out, (uint32_t)rr);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double per_simd = (double)kIters * kChains * waves_per_simd;  // wave-instructions per SIMD per launch
  const double cyc = (ms / reps) * 1e-3 * 2.4e9 / per_simd;
  std::printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms_per_launch\": %.4f, "
              "\"wave_instr_per_simd\": %.0f, \"cycles_per_instr_at_2.4GHz\": %.3f}\n",
              kNames[OP], waves_per_simd, ms / reps, per_simd, cyc);
  CHK(hipEventDestroy(a));
  CHK(hipEventDestroy(b));
  return 0;
}

template <int... OPS>
int run_all(uint32_t* d_out, int n_cu, int wps, std::integer_sequence<int, OPS...>) {
  int rc = 0;
  ((rc |= run<OPS>(d_out, n_cu, wps)), ...);
  return rc;
}

int main(int argc, char** argv) {
  int wps = argc > 1 ? atoi(argv[1]) : 8;
  int n_cu = 0;
  CHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t* d_out;
  CHK(hipMalloc(&d_out, (size_t)n_cu * 8 * 256 * 4));
  int rc = run_all(d_out, n_cu, wps, std::make_integer_sequence<int, OP_COUNT>{});
  CHK(hipFree(d_out));
  return rc;
}
