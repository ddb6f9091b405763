// The run table's index for K1, built on the device (sketch_core).
//
// K1 needs, for the caller's run table (one gg_run per ACGT stretch >= k of
// a genome, grouped by non-decreasing genome):
//   * the table checked (genome < n_genomes and non-decreasing, len >= k,
//     base + len inside the packed words) before any kernel reads through it;
//   * the first K1 segment of every run: rs = exclusive prefix sum of
//     ceil((len - k + 1) / seg) (segments never straddle runs, sketch.hip);
//   * per genome: its first run gr[g] and its k-mer count nk[g] (the host
//     derives the genome's initial tau from it) and grs[g] = rs[gr[g]].
// C5's 3.6M runs took 2.2 ms in two host passes plus 0.5 ms to upload rs;
// here one upload of the runs and four short kernels.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "device_util.hpp"
#include "gg_internal.hpp"

namespace gg {
namespace {

// per run: its segment count (rs before the scan; entry n_runs = 0) and the
// first bad run (atomicMin)
__global__ __launch_bounds__(256) void run_check_kernel(const gg_run* __restrict__ runs, uint64_t n_runs,
                                                        uint32_t n_genomes, uint64_t n_bases, uint32_t k,
                                                        uint32_t seg, uint64_t* __restrict__ sc,
                                                        unsigned long long* __restrict__ bad) {
  for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r <= n_runs; r += (uint64_t)gridDim.x * 256) {
    if (r == n_runs) {
      sc[r] = 0;
      continue;
    }
    const gg_run x = runs[r];
    const uint32_t prev = r ? runs[r - 1].genome : 0u;
    const uint64_t end = x.base + x.len;
    const bool ok = x.genome < n_genomes && x.genome >= prev && x.len >= k && end <= n_bases && end >= x.base;
    sc[r] = ok ? (x.len - k + 1 + seg - 1) / seg : 0ull;
    if (!ok) atomicMin(bad, (unsigned long long)r);
  }
}

// gr[g] = first run of genome g (lower bound on the genome field; g =
// n_genomes -> n_runs), for g in [0, n_genomes]
__global__ __launch_bounds__(256) void run_genome_start_kernel(const gg_run* __restrict__ runs, uint64_t n_runs,
                                                               uint32_t n_genomes, uint64_t* __restrict__ gr) {
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g <= n_genomes; g += (uint64_t)gridDim.x * 256) {
    uint64_t lo = 0, hi = n_runs;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (runs[mid].genome < g) lo = mid + 1;
      else hi = mid;
    }
    gr[g] = lo;
  }
}

// one workgroup per genome: nk[g] = sum of (len - k + 1) over its runs;
// grs[g] = rs[gr[g]] (g = n_genomes: the total)
__global__ __launch_bounds__(256) void run_genome_kmers_kernel(const gg_run* __restrict__ runs,
                                                               const uint64_t* __restrict__ gr,
                                                               const uint64_t* __restrict__ rs, uint32_t n_genomes,
                                                               uint32_t k, uint64_t* __restrict__ nk,
                                                               uint64_t* __restrict__ grs) {
  __shared__ unsigned long long part[4];
  for (uint32_t g = blockIdx.x; g <= n_genomes; g += gridDim.x) {
    const uint64_t r0 = gr[g];
    if (threadIdx.x == 0) grs[g] = rs[r0];
    if (g == n_genomes) break;
    const uint64_t r1 = gr[g + 1];
    unsigned long long acc = 0;
    for (uint64_t r = r0 + threadIdx.x; r < r1; r += 256) acc += runs[r].len - k + 1;
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) nk[g] = part[0] + part[1] + part[2] + part[3];
    __syncthreads();
  }
}

// First K1 pass of a single-batch call, set up on the device: each genome's
// initial threshold tau = over * s / nk * 2^64 (2^64 - 1 when the genome has
// at most over * s k-mers: every distinct hash is a candidate) and the
// identity slot maps.  The host reads tau back for its threshold search.
__global__ __launch_bounds__(256) void first_pass_kernel(const uint64_t* __restrict__ nk, uint32_t n_genomes,
                                                         double want, uint64_t* __restrict__ tau,
                                                         uint32_t* __restrict__ slot_genome,
                                                         uint32_t* __restrict__ slot_list) {
  for (uint32_t g = blockIdx.x * 256 + threadIdx.x; g < n_genomes; g += gridDim.x * 256) {
    tau[g] = first_tau(nk[g], want);
    slot_genome[g] = g;
    slot_list[g] = g;
  }
}

}  // namespace

hipError_t launch_first_pass(const uint64_t* nk, uint32_t n_genomes, double want, uint64_t* tau,
                             uint32_t* slot_genome, uint32_t* slot_list, hipStream_t st) {
  hipLaunchKernelGGL(first_pass_kernel, dim3(std::min<uint32_t>(4096, (n_genomes + 255) / 256)), dim3(256), 0, st, nk,
                     n_genomes, want, tau, slot_genome, slot_list);
  return hipGetLastError();
}

size_t run_index_tmp_bytes(uint64_t n_runs) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                         (int)(n_runs + 1));
  return bytes;
}

hipError_t launch_run_index(const RunIndexDev& x, hipStream_t st) {
  hipError_t e = hipMemsetAsync(x.bad, 0xFF, sizeof(uint64_t), st);
  if (e != hipSuccess) return e;
  const uint32_t g1 = (uint32_t)std::min<uint64_t>(8192, (x.n_runs + 1 + 255) / 256);
  hipLaunchKernelGGL(run_check_kernel, dim3(g1), dim3(256), 0, st, x.runs, x.n_runs, x.n_genomes, x.n_words * 16ull,
                     (uint32_t)x.k, x.seg, x.sc, (unsigned long long*)x.bad);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  size_t bytes = x.tmp_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(x.tmp, bytes, x.sc, x.rs, (int)(x.n_runs + 1), st);
  if (e != hipSuccess) return e;
  const uint32_t g2 = (uint32_t)std::min<uint64_t>(4096, ((uint64_t)x.n_genomes + 1 + 255) / 256);
  hipLaunchKernelGGL(run_genome_start_kernel, dim3(g2), dim3(256), 0, st, x.runs, x.n_runs, x.n_genomes, x.gr);
  hipLaunchKernelGGL(run_genome_kmers_kernel, dim3(std::min<uint32_t>(x.n_genomes + 1, 16384)), dim3(256), 0, st,
                     x.runs, x.gr, x.rs, x.n_genomes, (uint32_t)x.k, x.nk, x.grs);
  return hipGetLastError();
}

}  // namespace gg
