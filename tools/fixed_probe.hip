// Fixed per-launch cost of the small-table ingest kernel's shape, piece by
// piece: 256 workgroups x 1,024 threads with ~155 KB of dynamic LDS.
//   k_empty      launch only (LDS reserved, no work)
//   k_zero       + zero 105 KB of LDS
//   k_table      + load a 16 KB key table from HBM into LDS (+ zero)
//   k_tiles      + two 2,048-span SoA tiles per workgroup (44 B/span)
//   k_flush      + sparse 90 KB slab read-modify-write at the end
// Build: hipcc -O3 --offload-arch=gfx950 tools/fixed_probe.hip -o /tmp/fixed_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

constexpr int kBlock = 1024, kG = 256;
constexpr size_t kLds = 155 * 1024;
constexpr uint32_t kCap = 2048, kNw = 9;

__global__ __launch_bounds__(kBlock) void k_empty(int *sink) {
  extern __shared__ uint32_t sm[];
  if (threadIdx.x == 0 && sink == nullptr) sm[0] = 1;
}

template <bool ZERO, bool TABLE, bool TILES, bool FLUSH>
__global__ __launch_bounds__(kBlock) void k_piece(const uint64_t *keys, const uint64_t *cols,
                                                  uint32_t *slab, uint64_t *sink) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t *lkeys = reinterpret_cast<uint64_t *>(smem);
  uint32_t *lcnt = reinterpret_cast<uint32_t *>(lkeys + 2 * kCap);
  uint64_t acc = 0;
  ulonglong2 t[2][5];
  if (TILES) {
    // 5 u64 columns of 2 spans per lane per tile: same bytes as the kernel's tiles
    for (int b = 0; b < 2; ++b)
      for (int c = 0; c < 5; ++c) {
        const size_t off = (size_t)c * kG * 4096 + (size_t)blockIdx.x * 4096 + b * 2048 + threadIdx.x * 2;
        t[b][c] = *reinterpret_cast<const ulonglong2 *>(cols + off);
      }
  }
  if (TABLE) {
    const ulonglong2 v = reinterpret_cast<const ulonglong2 *>(keys)[threadIdx.x];
    reinterpret_cast<ulonglong2 *>(lkeys)[threadIdx.x] = v;
  }
  if (ZERO)
    for (uint32_t i = threadIdx.x * 4; i < kCap * kNw + 2 * kCap * 2; i += kBlock * 4)
      *reinterpret_cast<uint4 *>(lcnt + i - (i >= kCap * kNw ? 0 : 0)) = make_uint4(0, 0, 0, 0);
  __syncthreads();
  if (TILES)
    for (int b = 0; b < 2; ++b)
      for (int c = 0; c < 5; ++c) acc += t[b][c].x ^ t[b][c].y;
  if (TABLE) acc += lkeys[(threadIdx.x * 7) & (2 * kCap - 1)];
  if (FLUSH) {
    // each workgroup: cap * nw / 2 16-B cells, ~60% touched
    uint4 *s = reinterpret_cast<uint4 *>(slab + (size_t)blockIdx.x * kCap * 2 * kNw);
    for (uint32_t k = threadIdx.x; k < kCap * kNw / 2; k += kBlock) {
      if ((k * 2654435761u) % 10 < 6) {
        uint4 g = s[k];
        g.x += 1;
        s[k] = g;
      }
    }
  }
  if (acc == 0x123456789ULL) sink[0] = acc;
}

int main() {
  uint64_t *keys, *cols, *sink;
  uint32_t *slab;
  hipMalloc(&keys, kCap * 8);
  hipMalloc(&cols, (size_t)5 * kG * 4096 * 8);
  hipMalloc(&slab, (size_t)kG * kCap * 2 * kNw * 4);
  hipMalloc(&sink, 64);
  hipMemset(keys, 0, kCap * 8);
  hipMemset(cols, 1, (size_t)5 * kG * 4096 * 8);
  hipMemset(slab, 0, (size_t)kG * kCap * 2 * kNw * 4);
  struct K {
    const char *name;
    const void *fn;
  } ks[] = {
      {"empty", (const void *)&k_empty},
      {"zero", (const void *)&k_piece<true, false, false, false>},
      {"table+zero", (const void *)&k_piece<true, true, false, false>},
      {"tiles", (const void *)&k_piece<false, false, true, false>},
      {"table+zero+tiles", (const void *)&k_piece<true, true, true, false>},
      {"flush", (const void *)&k_piece<false, false, false, true>},
      {"all", (const void *)&k_piece<true, true, true, true>},
  };
  for (auto &k : ks) hipFuncSetAttribute(k.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLds);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (auto &k : ks) {
    std::vector<float> ts;
    for (int r = 0; r < 30; ++r) {
      void *args4[] = {&keys, &cols, &slab, &sink};
      void *args1[] = {&sink};
      void **args = k.fn == (const void *)&k_empty ? args1 : args4;
      hipEventRecord(a, 0);
      hipLaunchKernel(k.fn, dim3(kG), dim3(kBlock), args, kLds, 0);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (r >= 5) ts.push_back(ms * 1000);
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"case\": \"%s\", \"us_med\": %.2f, \"us_min\": %.2f}\n", k.name, ts[ts.size() / 2], ts[0]);
  }
  // reference: the same launch with no dynamic LDS
  {
    std::vector<float> ts;
    for (int r = 0; r < 30; ++r) {
      void *args1[] = {&sink};
      hipEventRecord(a, 0);
      hipLaunchKernel((const void *)&k_empty, dim3(kG), dim3(kBlock), args1, 0, 0);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (r >= 5) ts.push_back(ms * 1000);
    }
    std::sort(ts.begin(), ts.end());
    printf("{\"case\": \"empty_no_lds\", \"us_med\": %.2f, \"us_min\": %.2f}\n", ts[ts.size() / 2], ts[0]);
  }
  return 0;
}
