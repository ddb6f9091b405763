// VALU issue cost per wave64 instruction on gfx950, with the operands'
// VGPR banks under control (round 3: reconciles the round-2 measurement of
// v_fma_f32 at 3.8 cycles with MI355X_MICROARCH.md's "2 cycles per wave64
// VALU").  Every variant is ONE instruction with fixed registers repeated
// 64 times per loop iteration, no dependence between repeats (the
// destination is never a source), so the loop measures issue throughput,
// not latency.  VGPR bank = register number mod 4.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 scripts/ubench_vop3.hip -o scripts/ubench_vop3
//   scripts/ubench_vop3 [waves_per_simd]
// Output: one JSON line per variant, cycles per wave64 instruction per SIMD
// at 2.4 GHz and at the clock the reference variant implies.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                             \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

constexpr int kIters = 4096;
constexpr int kRep = 64;

#define R8(x) x x x x x x x x
#define R64(x) R8(R8(x))
#define CLOB "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "s20", "s21", "vcc"

// name, instruction text (one line, ends in \n)
#define VARIANTS(X)                                                                             \
  X(0, "v_xor_b32 v,v,v (VOP2, banks 2/3/0)", "v_xor_b32 v10, v11, v12\n")                     \
  X(1, "v_add_u32 v,v,v (VOP2)", "v_add_u32 v10, v11, v12\n")                                   \
  X(2, "v_add_f32 v,v,v (VOP2)", "v_add_f32 v10, v11, v12\n")                                   \
  X(3, "v_add_f32_e64 v,v,v (VOP3 encoding)", "v_add_f32_e64 v10, v11, v12\n")                  \
  X(4, "v_fma_f32 banks 3/0/1", "v_fma_f32 v10, v11, v12, v13\n")                               \
  X(5, "v_fma_f32 banks 3/3/3", "v_fma_f32 v10, v11, v15, v19\n")                               \
  X(6, "v_fma_f32 same src x3", "v_fma_f32 v10, v11, v11, v11\n")                               \
  X(7, "v_fmac_f32 (VOP2, dst is src2)", "v_fmac_f32 v10, v11, v12\n")                          \
  X(8, "v_pk_fma_f32 banks distinct", "v_pk_fma_f32 v[10:11], v[12:13], v[14:15], v[16:17]\n")  \
  X(9, "v_mul_f32 v,v,v (VOP2)", "v_mul_f32 v10, v11, v12\n")                                   \
  X(10, "v_mul_lo_u32 banks 3/0", "v_mul_lo_u32 v10, v11, v12\n")                               \
  X(11, "v_mul_hi_u32 banks 3/0", "v_mul_hi_u32 v10, v11, v12\n")                               \
  X(12, "v_alignbit_b32 v,v,inl", "v_alignbit_b32 v10, v11, v12, 5\n")                          \
  X(13, "v_add3_u32 banks 3/0/1", "v_add3_u32 v10, v11, v12, v13\n")                            \
  X(14, "v_lshlrev_b32 inl,v (VOP2)", "v_lshlrev_b32 v10, 3, v11\n")                            \
  X(15, "v_lshrrev_b32 inl,v (VOP2)", "v_lshrrev_b32 v10, 3, v11\n")                            \
  X(16, "v_mad_u64_u32", "v_mad_u64_u32 v[10:11], s[20:21], v12, v13, v[14:15]\n")              \
  X(17, "v_lshl_add_u64", "v_lshl_add_u64 v[10:11], v[12:13], 2, v[14:15]\n")                  \
  X(18, "v_cndmask_b32_e64 sgpr mask", "v_cndmask_b32_e64 v10, v11, v12, s[20:21]\n")           \
  X(19, "v_mov_b32 v (VOP1)", "v_mov_b32 v10, v11\n")                                           \
  X(20, "v_add_u32 v,s (SGPR source)", "v_add_u32 v10, s20, v12\n")                             \
  X(21, "v_add_u32_e64 v,v (VOP3 encoding)", "v_add_u32_e64 v10, v11, v12\n")                   \
  X(22, "v_xor_b32_e64 v,v (VOP3 encoding)", "v_xor_b32_e64 v10, v11, v12\n")                   \
  X(23, "v_bitop3_b32 banks 3/0/1", "v_bitop3_b32 v10, v11, v12, v13 bitop3:0x96\n")           \
  X(24, "v_pk_add_f32 banks distinct", "v_pk_add_f32 v[10:11], v[12:13], v[14:15]\n")           \
  X(25, "v_pk_mul_f32 banks distinct", "v_pk_mul_f32 v[10:11], v[12:13], v[14:15]\n")           \
  X(26, "v_lshlrev_b32_sdwa byte3 (K1 table address)",                                          \
    "v_lshlrev_b32_sdwa v10, v11, v12 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3\n") \
  X(27, "v_bfe_u32 v,v,inl,inl", "v_bfe_u32 v10, v11, 8, 8\n")                                  \
  X(28, "v_perm_b32 banks 3/0/1", "v_perm_b32 v10, v11, v12, v13\n")                            \
  X(29, "v_and_b32 literal,v", "v_and_b32 v10, 0xff0, v11\n")                                   \
  X(30, "v_lshrrev_b32 20,v", "v_lshrrev_b32 v10, 20, v11\n")                                   \
  X(31, "v_mul_u32_u24 v,v", "v_mul_u32_u24 v10, v11, v12\n")                                   \
  X(32, "v_lshl_or_b32 v,inl,v", "v_lshl_or_b32 v10, v11, 4, v12\n")                            \
  X(33, "v_and_or_b32 banks 3/0/1", "v_and_or_b32 v10, v11, v12, v13\n")                        \
  X(34, "v_cndmask_b32_e32 vcc", "v_cndmask_b32_e32 v10, v11, v12, vcc\n")                       \
  X(35, "v_cmp_lt_u64_e64 -> sgpr", "v_cmp_lt_u64_e64 s[20:21], v[12:13], v[14:15]\n")          \
  X(36, "v_mad_u32_u24 banks 3/0/1", "v_mad_u32_u24 v10, v11, v12, v13\n")                      \
  X(37, "v_lshlrev_b64 inl", "v_lshlrev_b64 v[10:11], 4, v[12:13]\n")                           \
  X(38, "v_lshl_add_u32 v,inl,v", "v_lshl_add_u32 v10, v11, 4, v12\n")                          \
  X(39, "v_add_co_u32 vcc", "v_add_co_u32 v10, vcc, v11, v12\n")                                \
  X(40, "v_lshrrev_b32_sdwa byte1", "v_lshrrev_b32_sdwa v10, v11, v12 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n") \
  X(41, "v_and_b32_sdwa byte2 (src0 sel)", "v_and_b32_sdwa v10, v11, v12 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD\n")

#define KERNEL(id, name, text)                                        \
  __global__ __launch_bounds__(256) void k##id(int* sink) {           \
    asm volatile("v_mov_b32 v11, 1.0\n v_mov_b32 v12, 2.0\n v_mov_b32 v13, 3.0\n" \
                 "v_mov_b32 v14, 1\n v_mov_b32 v15, 2\n v_mov_b32 v16, 3\n"       \
                 "v_mov_b32 v17, 4\n v_mov_b32 v19, 5\n s_mov_b64 s[20:21], -1\n" ::: CLOB); \
    for (int i = 0; i < kIters; ++i) asm volatile(R64(text) ::: CLOB); \
    int out;                                                          \
    asm volatile("v_mov_b32 %0, v10" : "=v"(out) :: CLOB);            \
    if (out == 0x7fffffff) sink[0] = out;                             \
  }
VARIANTS(KERNEL)

using KFn = void (*)(int*);
struct V {
  int id;
  const char* name;
  KFn fn;
};
#define ENTRY(id, name, text) {id, name, k##id},
static const V kVariants[] = {VARIANTS(ENTRY)};

int main(int argc, char** argv) {
  const int wps = argc > 1 ? atoi(argv[1]) : 8;
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  int* sink;
  CHK(hipMalloc(&sink, 4));
  const int blocks = cus * wps;  // 256 threads = 4 waves per block, one per SIMD
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  double ref = 0.0;
  for (const V& v : kVariants) {
    hipLaunchKernelGGL(v.fn, dim3(blocks), dim3(256), 0, 0, sink);  // warm-up
    CHK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      CHK(hipEventRecord(a));
      hipLaunchKernelGGL(v.fn, dim3(blocks), dim3(256), 0, 0, sink);
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms;
      CHK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    // instructions per SIMD: wps waves x kIters x kRep
    const double instr = (double)wps * kIters * kRep;
    const double cyc = best * 1e-3 * 2.4e9 / instr;
    if (v.id == 0) ref = cyc;
    std::printf("{\"variant\": %d, \"name\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, "
                "\"cycles_at_2.4GHz\": %.3f, \"ratio_to_xor\": %.3f}\n",
                v.id, v.name, wps, best, cyc, cyc / ref);
  }
  return 0;
}
