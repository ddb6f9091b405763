// VALU issue-rate calibration for the K1 roofline: cycles per wave64
// instruction for the integer ops the murmur3 mix uses, measured with 8
// waves per SIMD and independent chains (inline asm so nothing folds).
//   hipcc -O3 --offload-arch=gfx950 scripts/ubench_valu.hip -o scripts/ubench_valu
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHK(x)                                                           \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                          \
    }                                                                    \
  } while (0)

constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void ubench(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  uint32_t a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint64_t w0 = a0, w1 = a1, w2 = a2, w3 = a3;
  const uint32_t c = 0x9E3779B9u;
  for (int i = 0; i < kIters; ++i) {
    if (OP == 0) {  // v_add_u32 x8
      asm volatile(
          "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
          "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "s"(c));
    } else if (OP == 1) {  // v_mul_lo_u32 x8
      asm volatile(
          "v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n"
          "v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "s"(c));
    } else if (OP == 2) {  // v_mad_u64_u32 x8 (4 chains, 2 each)
      asm volatile(
          "v_mad_u64_u32 %0, vcc, %4, %5, %0\n v_mad_u64_u32 %1, vcc, %4, %5, %1\n"
          "v_mad_u64_u32 %2, vcc, %4, %5, %2\n v_mad_u64_u32 %3, vcc, %4, %5, %3\n"
          "v_mad_u64_u32 %0, vcc, %4, %5, %0\n v_mad_u64_u32 %1, vcc, %4, %5, %1\n"
          "v_mad_u64_u32 %2, vcc, %4, %5, %2\n v_mad_u64_u32 %3, vcc, %4, %5, %3\n"
          : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3)
          : "v"(a0), "s"(c)
          : "vcc");
    } else if (OP == 3) {  // v_lshl_add_u64 x8
      asm volatile(
          "v_lshl_add_u64 %0, %0, 2, %0\n v_lshl_add_u64 %1, %1, 2, %1\n"
          "v_lshl_add_u64 %2, %2, 2, %2\n v_lshl_add_u64 %3, %3, 2, %3\n"
          "v_lshl_add_u64 %0, %0, 2, %0\n v_lshl_add_u64 %1, %1, 2, %1\n"
          "v_lshl_add_u64 %2, %2, 2, %2\n v_lshl_add_u64 %3, %3, 2, %3\n"
          : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3));
    } else if (OP == 4) {  // v_alignbit_b32 x8
      asm volatile(
          "v_alignbit_b32 %0, %0, %1, 31\n v_alignbit_b32 %1, %1, %2, 31\n v_alignbit_b32 %2, %2, %3, 31\n"
          "v_alignbit_b32 %3, %3, %4, 31\n v_alignbit_b32 %4, %4, %5, 31\n v_alignbit_b32 %5, %5, %6, 31\n"
          "v_alignbit_b32 %6, %6, %7, 31\n v_alignbit_b32 %7, %7, %0, 31\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if (OP == 6 || OP == 7) {  // 16 independent chains
      uint32_t b[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) b[q] = a0 + q;
#pragma unroll
      for (int rep = 0; rep < 4; ++rep) {
        if (OP == 6)
          asm volatile(
              "v_add_u32 %0, %0, %16\n v_add_u32 %1, %1, %16\n v_add_u32 %2, %2, %16\n v_add_u32 %3, %3, %16\n"
              "v_add_u32 %4, %4, %16\n v_add_u32 %5, %5, %16\n v_add_u32 %6, %6, %16\n v_add_u32 %7, %7, %16\n"
              "v_add_u32 %8, %8, %16\n v_add_u32 %9, %9, %16\n v_add_u32 %10, %10, %16\n v_add_u32 %11, %11, %16\n"
              "v_add_u32 %12, %12, %16\n v_add_u32 %13, %13, %16\n v_add_u32 %14, %14, %16\n v_add_u32 %15, %15, %16\n"
              : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]),
                "+v"(b[8]), "+v"(b[9]), "+v"(b[10]), "+v"(b[11]), "+v"(b[12]), "+v"(b[13]), "+v"(b[14]), "+v"(b[15])
              : "s"(c));
        else
          asm volatile(
              "v_mul_lo_u32 %0, %0, %16\n v_mul_lo_u32 %1, %1, %16\n v_mul_lo_u32 %2, %2, %16\n v_mul_lo_u32 %3, %3, %16\n"
              "v_mul_lo_u32 %4, %4, %16\n v_mul_lo_u32 %5, %5, %16\n v_mul_lo_u32 %6, %6, %16\n v_mul_lo_u32 %7, %7, %16\n"
              "v_mul_lo_u32 %8, %8, %16\n v_mul_lo_u32 %9, %9, %16\n v_mul_lo_u32 %10, %10, %16\n v_mul_lo_u32 %11, %11, %16\n"
              "v_mul_lo_u32 %12, %12, %16\n v_mul_lo_u32 %13, %13, %16\n v_mul_lo_u32 %14, %14, %16\n v_mul_lo_u32 %15, %15, %16\n"
              : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]),
                "+v"(b[8]), "+v"(b[9]), "+v"(b[10]), "+v"(b[11]), "+v"(b[12]), "+v"(b[13]), "+v"(b[14]), "+v"(b[15])
              : "s"(c));
      }
      uint32_t x = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) x ^= b[q];
      a1 ^= x;
    } else if (OP == 8) {  // v_lshlrev_b64 x8
      asm volatile(
          "v_lshlrev_b64 %0, 3, %0\n v_lshlrev_b64 %1, 3, %1\n v_lshlrev_b64 %2, 3, %2\n v_lshlrev_b64 %3, 3, %3\n"
          "v_lshlrev_b64 %0, 5, %0\n v_lshlrev_b64 %1, 5, %1\n v_lshlrev_b64 %2, 5, %2\n v_lshlrev_b64 %3, 5, %3\n"
          : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3));
    } else if (OP == 9) {  // v_cndmask_b32 x8 (vcc mask)
      asm volatile(
          "v_cndmask_b32 %0, %0, %1, vcc\n v_cndmask_b32 %1, %1, %2, vcc\n v_cndmask_b32 %2, %2, %3, vcc\n"
          "v_cndmask_b32 %3, %3, %4, vcc\n v_cndmask_b32 %4, %4, %5, vcc\n v_cndmask_b32 %5, %5, %6, vcc\n"
          "v_cndmask_b32 %6, %6, %7, vcc\n v_cndmask_b32 %7, %7, %0, vcc\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if (OP == 5) {  // v_mul_hi_u32 x8
      asm volatile(
          "v_mul_hi_u32 %0, %0, %8\n v_mul_hi_u32 %1, %1, %8\n v_mul_hi_u32 %2, %2, %8\n v_mul_hi_u32 %3, %3, %8\n"
          "v_mul_hi_u32 %4, %4, %8\n v_mul_hi_u32 %5, %5, %8\n v_mul_hi_u32 %6, %6, %8\n v_mul_hi_u32 %7, %7, %8\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "s"(c));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] =
      a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)(w0 ^ w1 ^ w2 ^ w3) ^ (uint32_t)((w0 ^ w1 ^ w2 ^ w3) >> 32);
}

template <int OP>
int run(const char* name, uint32_t* d_out, int n_cu, int waves_per_simd = 8) {
  const int blocks = n_cu * waves_per_simd;  // 256-thread blocks: 1 wave per SIMD each
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  hipLaunchKernelGGL(ubench<OP>, dim3(blocks), dim3(256), 0, 0, d_out, 1u);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(a));
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(ubench<OP>, dim3(blocks), dim3(256), 0, 0, d_out, (uint32_t)r);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  const double per_iter = (OP == 6 || OP == 7) ? 64.0 : 8.0;
  const double wave_instr_per_simd = 5.0 * kIters * per_iter * (blocks * 4.0) / (n_cu * 4.0);
  const double cyc = ms * 1e-3 * 2.4e9 / wave_instr_per_simd;
  std::printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"cycles_per_wave64_instr_at_2.4GHz\": %.3f}\n",
              name, waves_per_simd, ms / 5, cyc);
  return 0;
}

int main() {
  int n_cu = 0;
  CHK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));
  uint32_t* d_out;
  CHK(hipMalloc(&d_out, (size_t)n_cu * 8 * 256 * 4));
  run<0>("v_add_u32", d_out, n_cu);
  run<1>("v_mul_lo_u32", d_out, n_cu);
  run<5>("v_mul_hi_u32", d_out, n_cu);
  run<2>("v_mad_u64_u32", d_out, n_cu);
  run<3>("v_lshl_add_u64", d_out, n_cu);
  run<4>("v_alignbit_b32", d_out, n_cu);
  run<8>("v_lshlrev_b64", d_out, n_cu);
  run<9>("v_cndmask_b32", d_out, n_cu);
  run<6>("v_add_u32 x16 chains", d_out, n_cu);
  run<7>("v_mul_lo_u32 x16 chains", d_out, n_cu);
  run<6>("v_add_u32 x16 chains", d_out, n_cu, 1);
  run<7>("v_mul_lo_u32 x16 chains", d_out, n_cu, 1);
  run<6>("v_add_u32 x16 chains", d_out, n_cu, 2);
  run<7>("v_mul_lo_u32 x16 chains", d_out, n_cu, 2);
  run<0>("v_add_u32", d_out, n_cu, 1);
  run<1>("v_mul_lo_u32", d_out, n_cu, 1);
  CHK(hipFree(d_out));
  return 0;
}
