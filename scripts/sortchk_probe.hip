// Checks hipcub::DeviceRadixSort::SortPairs over a bit range [begin, 32) on
// keys read from a file: output ordered by the key bits >= begin and a
// permutation of the input (pairs).
#include <hipcub/hipcub.hpp>
#include <cstdio>
#include <vector>
#include <algorithm>
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  std::vector<uint32_t> k; uint32_t x;
  while (fread(&x, 4, 1, f) == 1) k.push_back(x);
  fclose(f);
  const int n = (int)k.size();
  std::vector<uint64_t> v(n);
  for (int i = 0; i < n; ++i) v[i] = ((uint64_t)k[i] << 32) | (uint32_t)i;
  uint32_t *dk, *dko; uint64_t *dv, *dvo;
  hipMalloc(&dk, 4 * n); hipMalloc(&dko, 4 * n); hipMalloc(&dv, 8 * n); hipMalloc(&dvo, 8 * n);
  for (int begin : {0, 16, 28, 30}) {
    hipMemcpy(dk, k.data(), 4 * n, hipMemcpyHostToDevice);
    hipMemcpy(dv, v.data(), 8 * n, hipMemcpyHostToDevice);
    hipMemset(dko, 0xAB, 4 * n); hipMemset(dvo, 0xAB, 8 * n);
    size_t bytes = 0;
    hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, dk, dko, dv, dvo, n, begin, 32);
    void* tmp; hipMalloc(&tmp, bytes ? bytes : 1);
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(tmp, bytes, dk, dko, dv, dvo, n, begin, 32);
    hipError_t e2 = hipDeviceSynchronize();
    std::vector<uint32_t> ko(n); std::vector<uint64_t> vo(n);
    hipMemcpy(ko.data(), dko, 4 * n, hipMemcpyDeviceToHost);
    hipMemcpy(vo.data(), dvo, 8 * n, hipMemcpyDeviceToHost);
    int unsorted = 0, badpair = 0;
    std::vector<int> seen(n, 0);
    for (int i = 0; i < n; ++i) {
      if (i && (ko[i - 1] >> begin) > (ko[i] >> begin)) ++unsorted;
      uint32_t idx = (uint32_t)vo[i];
      if (idx >= (uint32_t)n || (uint32_t)(vo[i] >> 32) != ko[i] || k[idx] != ko[i]) ++badpair; else seen[idx]++;
    }
    int missing = (int)std::count(seen.begin(), seen.end(), 0);
    printf("n %d begin %d tmp %zu err %d/%d unsorted %d badpair %d missing %d\n", n, begin, bytes, (int)e, (int)e2,
           unsorted, badpair, missing);
    hipFree(tmp);
  }
}
