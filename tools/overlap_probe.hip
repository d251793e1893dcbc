// overlap_probe.hip -- can a 44 B/span HBM stream and one random 1-B gather
// per span (the HLL register read) overlap, if the gather is consumed one or
// two steps after it is issued and the stream is prefetched two tiles ahead?
// Build: hipcc --offload-arch=gfx950 -O3 tools/overlap_probe.hip -o build/overlap_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)
using u64 = unsigned long long;
struct Cols { const u64 *k, *s, *e, *a, *b; const unsigned *m; };
struct Tile { ulonglong2 k, s, e, a, b; uint2 m; };
__device__ __forceinline__ void ld(const Cols &c, u64 i, u64 hi, Tile &t) {
  if (i + 2 > hi) i = hi - 2;  // clamp (timing only)
  t.k = *reinterpret_cast<const ulonglong2 *>(c.k + i); t.s = *reinterpret_cast<const ulonglong2 *>(c.s + i);
  t.e = *reinterpret_cast<const ulonglong2 *>(c.e + i); t.a = *reinterpret_cast<const ulonglong2 *>(c.a + i);
  t.b = *reinterpret_cast<const ulonglong2 *>(c.b + i); t.m = *reinterpret_cast<const uint2 *>(c.m + i);
}
__device__ __forceinline__ unsigned use(const Tile &t) {
  return (unsigned)(t.k.x ^ t.k.y ^ t.s.x ^ t.s.y ^ t.e.x ^ t.e.y ^ t.a.x ^ t.a.y ^ t.b.x ^ t.b.y) ^ t.m.x ^ t.m.y;
}
// NG gathers per step (2 spans per lane per step => NG=2 is one per span), deferred D steps
template <int NG, int D, int TABLE_LOG2>
__global__ __launch_bounds__(1024) void kern(Cols c, u64 n, const unsigned char *tab, unsigned *out) {
  u64 chunk = (n + gridDim.x - 1) / gridDim.x; chunk = (chunk + 3) / 4 * 4;
  const u64 lo = blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
  const u64 lane = threadIdx.x * 2, tile = 2048;
  Tile A, B;
  ld(c, lo + lane, hi, A); ld(c, lo + tile + lane, hi, B);
  unsigned acc = 0, g0[NG > 0 ? NG : 1] = {}, g1[NG > 0 ? NG : 1] = {};
  const unsigned mask = (1u << TABLE_LOG2) - 1;
  for (u64 t = lo; t < hi; t += 2 * tile) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      Tile &T = half ? B : A;
      const u64 tt = t + half * tile;
      acc += use(T);
      unsigned g[NG > 0 ? NG : 1];
#pragma unroll
      for (int q = 0; q < NG; ++q) {
        const unsigned h = ((unsigned)(tt + lane + q) * 0x9E3779B1u) ^ ((unsigned)(tt >> 11) * 0x85EBCA6Bu);
        g[q] = tab[(h >> 5) & mask];
      }
      ld(c, tt + 2 * tile + lane, hi, T);
      if (D == 0) { for (int q = 0; q < NG; ++q) acc += g[q]; }
      if (D == 1) { for (int q = 0; q < NG; ++q) { acc += g0[q]; g0[q] = g[q]; } }
      if (D == 2) { for (int q = 0; q < NG; ++q) { acc += g1[q]; g1[q] = g0[q]; g0[q] = g[q]; } }
    }
  }
  for (int q = 0; q < NG; ++q) acc += g0[q] + g1[q];
  if (acc == 0x12345678u) out[0] = acc;
}
// The same, but the gathers go through the scalar unit: each lane's address is
// read out with v_readlane, loaded with s_load_dword (constant address space,
// so the address path of the vector memory pipeline is not used), and written
// back with a per-lane select.  16 loads are in flight per batch.
using cu32 = const __attribute__((address_space(4))) unsigned;
template <int NG, int D, int TABLE_LOG2>
__global__ __launch_bounds__(1024) void kern_s(Cols c, u64 n, const unsigned char *tab, unsigned *out) {
  u64 chunk = (n + gridDim.x - 1) / gridDim.x; chunk = (chunk + 3) / 4 * 4;
  const u64 lo = blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
  const u64 lane = threadIdx.x * 2, tile = 2048;
  Tile A, B;
  ld(c, lo + lane, hi, A); ld(c, lo + tile + lane, hi, B);
  unsigned acc = 0, g0[NG] = {}, g1[NG] = {};
  const unsigned mask = (1u << TABLE_LOG2) - 1;
  cu32 *ctab = (cu32 *)tab;
  const unsigned lid = __lane_id();
  for (u64 t = lo; t < hi; t += 2 * tile) {
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      Tile &T = half ? B : A;
      const u64 tt = t + half * tile;
      acc += use(T);
      unsigned g[NG];
#pragma unroll
      for (int q = 0; q < NG; ++q) {
        const unsigned h = ((unsigned)(tt + lane + q) * 0x9E3779B1u) ^ ((unsigned)(tt >> 11) * 0x85EBCA6Bu);
        const unsigned w = ((h >> 5) & mask) >> 2;  // u32 word index
        unsigned v = 0;
#pragma unroll
        for (int L0 = 0; L0 < 64; L0 += 16) {
          unsigned sv[16];
#pragma unroll
          for (int L = 0; L < 16; ++L) sv[L] = ctab[__builtin_amdgcn_readlane((int)w, L0 + L)];
#pragma unroll
          for (int L = 0; L < 16; ++L) v = (lid == (unsigned)(L0 + L)) ? sv[L] : v;
        }
        g[q] = v;
      }
      ld(c, tt + 2 * tile + lane, hi, T);
      if (D == 0) { for (int q = 0; q < NG; ++q) acc += g[q]; }
      if (D == 1) { for (int q = 0; q < NG; ++q) { acc += g0[q]; g0[q] = g[q]; } }
    }
  }
  for (int q = 0; q < NG; ++q) acc += g0[q] + g1[q];
  if (acc == 0x12345678u) out[0] = acc;
}
// stream-only shapes: S4 simple loop (11 x 16-B loads per lane per iteration),
// and the S2 ring with meta loaded 8 B/lane vs 16 B/lane on even lanes + DPP.
template <int MODE>
__global__ __launch_bounds__(1024) void shape(Cols c, u64 n, unsigned *out) {
  u64 chunk = (n + gridDim.x - 1) / gridDim.x; chunk = (chunk + 3) / 4 * 4;
  const u64 lo = blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
  unsigned acc = 0;
  if (MODE == 0) {
    for (u64 i = lo + threadIdx.x * 4; i < hi; i += 4096) {
      Tile a, b; ld(c, i, hi, a); ld(c, i + 2, hi, b);
      a.m = make_uint2(0, 0); b.m = make_uint2(0, 0);
      const uint4 m = *reinterpret_cast<const uint4 *>(c.m + i);
      acc += use(a) ^ use(b) ^ m.x ^ m.w;
    }
  } else {
    const u64 lane = threadIdx.x * 2, tile = 2048;
    Tile A, B;
    ld(c, lo + lane, hi, A); ld(c, lo + tile + lane, hi, B);
    for (u64 t = lo; t < hi; t += 2 * tile) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        Tile &T = half ? B : A;
        const u64 tt = t + half * tile;
        acc += use(T);
        ld(c, tt + 2 * tile + lane, hi, T);
      }
    }
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
  const u64 n = 10000000ULL;
  int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  void *buf; CK(hipMalloc(&buf, n * 44 + 4096)); CK(hipMemset(buf, 1, n * 44));
  Cols c; c.k = (const u64 *)buf; c.s = c.k + n; c.e = c.s + n; c.a = c.e + n; c.b = c.a + n; c.m = (const unsigned *)(c.b + n);
  unsigned char *tab; CK(hipMalloc(&tab, 64 << 20)); CK(hipMemset(tab, 0, 64 << 20));
  unsigned *out; CK(hipMalloc(&out, 64));
#define R(NG, D, TL) std::printf("{\"gathers_per_step\": %d, \"defer\": %d, \"table_bytes\": %d, \"us\": %.2f}\n", NG, D, 1 << TL, time_it([&] { kern<NG, D, TL><<<cus, 1024>>>(c, n, tab, out); }, 20));
  std::printf("{\"shape\": \"S4 simple loop\", \"us\": %.2f}\n", time_it([&] { shape<0><<<cus, 1024>>>(c, n, out); }, 20));
  std::printf("{\"shape\": \"S2 ring\", \"us\": %.2f}\n", time_it([&] { shape<1><<<cus, 1024>>>(c, n, out); }, 20));
  R(0, 0, 21) R(2, 0, 21) R(2, 1, 21) R(2, 2, 21) R(2, 1, 15) R(2, 1, 18) R(2, 1, 23) R(1, 1, 21) R(4, 1, 21)
#define RS(NG, D, TL) std::printf("{\"scalar_gathers_per_step\": %d, \"defer\": %d, \"table_bytes\": %d, \"us\": %.2f}\n", NG, D, 1 << TL, time_it([&] { kern_s<NG, D, TL><<<cus, 1024>>>(c, n, tab, out); }, 20));
  RS(2, 0, 21) RS(2, 1, 21) RS(1, 1, 21) RS(2, 1, 15)
  return 0;
}
