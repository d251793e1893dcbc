// valu_probe.hip -- how much per-span VALU work hides under the 44 B/span
// stream at 1 workgroup of 1024 threads per CU (the ingest kernel's shape).
// K rounds of 3 dependent-free 32-bit VALU ops per span (+ optional xxh64).
// Build: hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o build/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)
constexpr unsigned long long XP1 = 0x9E3779B185EBCA87ULL, XP2 = 0xC2B2AE3D27D4EB4FULL, XP3 = 0x165667B19E3779F9ULL, XP4 = 0x85EBCA77C2B2AE63ULL, XP5 = 0x27D4EB2F165667C5ULL;
__device__ __forceinline__ unsigned long long rotl(unsigned long long x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ unsigned long long xxh(unsigned long long a, unsigned long long b) {
  unsigned long long h = XP5 + 16;
  h ^= rotl(a * XP2, 31) * XP1; h = rotl(h, 27) * XP1 + XP4;
  h ^= rotl(b * XP2, 31) * XP1; h = rotl(h, 27) * XP1 + XP4;
  h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; h ^= h >> 32; return h;
}
struct Cols { const unsigned long long *k, *s, *e, *a, *b; const unsigned *m; };
template <int K, bool HASH, int GATHER_LOG2 = 0>
__global__ __launch_bounds__(1024) void probe(Cols c, unsigned long long n, unsigned long long *out,
                                              const unsigned *gtab = nullptr) {
  unsigned long long chunk = (n + gridDim.x - 1) / gridDim.x; chunk = (chunk + 3) / 4 * 4;
  const unsigned long long lo = blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
  unsigned acc = threadIdx.x;
  for (unsigned long long i = lo + threadIdx.x * 4; i < hi; i += 4096) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const ulonglong2 k = *reinterpret_cast<const ulonglong2 *>(c.k + i + 2 * h);
      const ulonglong2 s = *reinterpret_cast<const ulonglong2 *>(c.s + i + 2 * h);
      const ulonglong2 e = *reinterpret_cast<const ulonglong2 *>(c.e + i + 2 * h);
      const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(c.a + i + 2 * h);
      const ulonglong2 b = *reinterpret_cast<const ulonglong2 *>(c.b + i + 2 * h);
      unsigned x0 = (unsigned)(k.x ^ s.x ^ e.x), x1 = (unsigned)(k.y ^ s.y ^ e.y);
#pragma unroll
      for (int r = 0; r < K; ++r) {
        x0 = (x0 ^ (x0 >> 7)) + (x0 << 3) + r;
        x1 = (x1 ^ (x1 >> 7)) + (x1 << 3) + r;
      }
      if (HASH) { x0 ^= (unsigned)(xxh(a.x, b.x) >> 40); x1 ^= (unsigned)(xxh(a.y, b.y) >> 40); }
      else { x0 ^= (unsigned)(a.x ^ b.x); x1 ^= (unsigned)(a.y ^ b.y); }
      if (GATHER_LOG2) {  // one random 4-B gather per span (HLL-register read pattern)
        const unsigned m = (1u << GATHER_LOG2) - 1;
        acc += gtab[((unsigned)(a.x >> 20) * 0x9E3779B1u >> 2) & m];
        acc += gtab[((unsigned)(a.y >> 20) * 0x9E3779B1u >> 2) & m];
      }
      acc += x0 ^ x1;
    }
    const uint4 m = *reinterpret_cast<const uint4 *>(c.m + i);
    acc ^= m.x ^ m.y ^ m.z ^ m.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
template <typename F> float time_it(F f, int reps) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize()); CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}
int main() {
  const unsigned long long n = 10000000ULL;
  int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  void *buf; const size_t bytes = n * 44; CK(hipMalloc(&buf, bytes + 4096)); CK(hipMemset(buf, 1, bytes));
  unsigned long long *out; CK(hipMalloc(&out, 64));
  Cols c; c.k = (const unsigned long long *)buf; c.s = c.k + n; c.e = c.s + n; c.a = c.e + n; c.b = c.a + n; c.m = (const unsigned *)(c.b + n);
#define RUN(K, H) std::printf("{\"K\": %d, \"hash\": %d, \"valu_per_span\": %d, \"us\": %.2f}\n", K, H, 3 * K, time_it([&] { probe<K, H><<<cus, 1024>>>(c, n, out); }, 20));
  RUN(0, false) RUN(8, false) RUN(16, false) RUN(32, false) RUN(48, false) RUN(64, false) RUN(96, false)
  RUN(0, true) RUN(16, true) RUN(32, true) RUN(64, true)
  unsigned *gtab; CK(hipMalloc(&gtab, 64 << 20)); CK(hipMemset(gtab, 0, 64 << 20));
#define RUNG(G) std::printf("{\"gather_table_bytes\": %d, \"us\": %.2f}\n", 4 << G, time_it([&] { probe<16, true, G><<<cus, 1024>>>(c, n, out, gtab); }, 20));
  RUNG(13) RUNG(16) RUNG(19) RUNG(21) RUNG(24)
  return 0;
}
