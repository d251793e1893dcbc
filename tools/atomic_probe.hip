// atomic_probe.hip -- rate of the HBM-table path's counter atomics: 10 M spans
// x 2 no-return u64 atomic adds to random rows of a 1 M-row table.
//   split     count and sum cells in different 64-B segments (the current
//             [cap][18] u64 layout, sum last), one lane does both
//   seg       both cells in one 64-B segment (sum first, 192-B rows), one lane
//             does both (two instructions)
//   pair      both cells in one segment and issued by ONE instruction from two
//             adjacent lanes (even lane: count of span A, odd lane: sum of A)
// Build: hipcc -O3 --offload-arch=gfx950 tools/atomic_probe.hip -o tools/atomic_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned long long *t, uint64_t n, uint32_t rows) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t h = mix(i);
    const uint32_t row = (uint32_t)(h % rows), b = (uint32_t)(h >> 40) % 7;
    if (MODE == 0) {  // split: 144-B rows, count at 8b, sum at 136
      atomicAdd(t + (uint64_t)row * 18 + b, 1ULL);
      atomicAdd(t + (uint64_t)row * 18 + 17, 5ULL);
    } else if (MODE == 1) {  // seg: 192-B rows, sum at 0, count at 8(b+1)
      atomicAdd(t + (uint64_t)row * 24 + 1 + b, 1ULL);
      atomicAdd(t + (uint64_t)row * 24, 5ULL);
    } else {  // pair: lane 2j and 2j+1 share span A then span B
      const uint32_t lane = threadIdx.x & 63u;
      const uint32_t prow = __shfl_xor((int)row, 1), pb = __shfl_xor((int)b, 1);
      // instruction 1: even lane -> its count, odd lane -> the even lane's sum
      const bool even = (lane & 1u) == 0;
      atomicAdd(t + (uint64_t)(even ? row : prow) * 24 + (even ? 1 + b : 0), even ? 1ULL : 5ULL);
      // instruction 2: odd lane -> its count, even lane -> the odd lane's sum
      atomicAdd(t + (uint64_t)(even ? prow : row) * 24 + (even ? 0 : 1 + b), even ? 5ULL : 1ULL);
      (void)pb;
    }
  }
}

int main() {
  const uint64_t n = 10000000;
  const uint32_t rows = 1 << 20;
  unsigned long long *t;
  hipMalloc(&t, (size_t)rows * 24 * 8);
  hipMemset(t, 0, (size_t)rows * 24 * 8);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char *names[] = {"split", "seg", "pair"};
  for (int mode = 0; mode < 3; ++mode) {
    std::vector<float> ts;
    for (int r = 0; r < 8; ++r) {
      hipEventRecord(a, 0);
      if (mode == 0) k<0><<<cus * 8, 256>>>(t, n, rows);
      if (mode == 1) k<1><<<cus * 8, 256>>>(t, n, rows);
      if (mode == 2) k<2><<<cus * 8, 256>>>(t, n, rows);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (r) ts.push_back(ms * 1000);
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"mode\": \"%s\", \"us_med\": %.1f, \"atomics_per_s\": %.3g}\n", names[mode], ts[ts.size() / 2],
           2.0 * n / (ts[ts.size() / 2] * 1e-6));
  }
  return 0;
}
