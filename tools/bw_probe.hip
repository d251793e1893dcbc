// bw_probe.hip -- calibrate the HBM read ceiling for the SoA v1 access pattern
// (5 u64 columns + 1 u32 column, 44 B/span) under different launch shapes.
// Build: hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o build/bw_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);     \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

struct Cols {
  const unsigned long long *k, *s, *e, *a, *b;
  const unsigned *m;
};

// contiguous per-workgroup ranges, S spans per lane, 16-B loads
template <int S, int BLOCK>
__global__ __launch_bounds__(BLOCK) void read_contig(Cols c, unsigned long long n,
                                                     unsigned long long *out) {
  unsigned long long chunk = (n + gridDim.x - 1) / gridDim.x;
  chunk = (chunk + 3) / 4 * 4;
  const unsigned long long lo = blockIdx.x * chunk;
  const unsigned long long hi = lo + chunk < n ? lo + chunk : n;
  unsigned long long acc = 0;
  for (unsigned long long i = lo + threadIdx.x * S; i < hi; i += (unsigned long long)BLOCK * S) {
#pragma unroll
    for (int h = 0; h < S / 2; ++h) {
      const ulonglong2 k = *reinterpret_cast<const ulonglong2 *>(c.k + i + 2 * h);
      const ulonglong2 s = *reinterpret_cast<const ulonglong2 *>(c.s + i + 2 * h);
      const ulonglong2 e = *reinterpret_cast<const ulonglong2 *>(c.e + i + 2 * h);
      const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(c.a + i + 2 * h);
      const ulonglong2 b = *reinterpret_cast<const ulonglong2 *>(c.b + i + 2 * h);
      acc ^= k.x ^ k.y ^ s.x ^ s.y ^ e.x ^ e.y ^ a.x ^ a.y ^ b.x ^ b.y;
    }
    if (S == 4) {
      const uint4 m = *reinterpret_cast<const uint4 *>(c.m + i);
      acc ^= m.x ^ m.y ^ m.z ^ m.w;
    } else {
      const uint2 m = *reinterpret_cast<const uint2 *>(c.m + i);
      acc ^= m.x ^ m.y;
    }
  }
  if (acc == 0x123456789ULL) out[0] = acc;
}

// contiguous ranges through buffer loads with cache-policy bits AUX
// (gfx950: 1 = sc0, 2 = nt, 16 = sc1)
template <int AUX>
__global__ __launch_bounds__(1024) void read_buf(Cols c, unsigned long long n, unsigned long long *out) {
  unsigned long long chunk = (n + gridDim.x - 1) / gridDim.x;
  chunk = (chunk + 3) / 4 * 4;
  unsigned long long lo = blockIdx.x * chunk;
  if (lo > n) lo = n;
  const unsigned long long hi = lo + chunk < n ? lo + chunk : n;
  const unsigned len = (unsigned)(hi - lo);
  auto mk = [&](const void *p, unsigned b) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)b, 0x00020000);
  };
  const auto rk = mk(c.k + lo, len * 8), rs = mk(c.s + lo, len * 8), re = mk(c.e + lo, len * 8),
             ra = mk(c.a + lo, len * 8), rb = mk(c.b + lo, len * 8), rm = mk(c.m + lo, len * 4);
  unsigned acc = 0;
  for (unsigned i = threadIdx.x * 4; i < len; i += 1024 * 4) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int o = (int)(i * 8 + 16 * h);
      const auto k = __builtin_amdgcn_raw_buffer_load_b128(rk, o, 0, AUX);
      const auto s = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, AUX);
      const auto e = __builtin_amdgcn_raw_buffer_load_b128(re, o, 0, AUX);
      const auto a = __builtin_amdgcn_raw_buffer_load_b128(ra, o, 0, AUX);
      const auto b = __builtin_amdgcn_raw_buffer_load_b128(rb, o, 0, AUX);
      acc ^= k[0] ^ k[3] ^ s[1] ^ s[2] ^ e[0] ^ e[3] ^ a[1] ^ a[2] ^ b[0] ^ b[3];
    }
    const auto m = __builtin_amdgcn_raw_buffer_load_b128(rm, (int)(i * 4), 0, AUX);
    acc ^= m[0] ^ m[1] ^ m[2] ^ m[3];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// grid-stride (interleaved) tiles
template <int S, int BLOCK>
__global__ __launch_bounds__(BLOCK) void read_stride(Cols c, unsigned long long n,
                                                     unsigned long long *out) {
  unsigned long long acc = 0;
  const unsigned long long step = (unsigned long long)gridDim.x * BLOCK * S;
  for (unsigned long long i = ((unsigned long long)blockIdx.x * BLOCK + threadIdx.x) * S; i + S <= n;
       i += step) {
#pragma unroll
    for (int h = 0; h < S / 2; ++h) {
      const ulonglong2 k = *reinterpret_cast<const ulonglong2 *>(c.k + i + 2 * h);
      const ulonglong2 s = *reinterpret_cast<const ulonglong2 *>(c.s + i + 2 * h);
      const ulonglong2 e = *reinterpret_cast<const ulonglong2 *>(c.e + i + 2 * h);
      const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(c.a + i + 2 * h);
      const ulonglong2 b = *reinterpret_cast<const ulonglong2 *>(c.b + i + 2 * h);
      acc ^= k.x ^ k.y ^ s.x ^ s.y ^ e.x ^ e.y ^ a.x ^ a.y ^ b.x ^ b.y;
    }
    const uint2 m = *reinterpret_cast<const uint2 *>(c.m + i);
    acc ^= m.x ^ m.y;
  }
  if (acc == 0x123456789ULL) out[0] = acc;
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;  // us
}

int main(int argc, char **argv) {
  const unsigned long long n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 10000000ULL;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  void *buf;
  const size_t bytes = n * 44;
  CK(hipMalloc(&buf, bytes + 4096));
  CK(hipMemset(buf, 1, bytes));
  unsigned long long *out;
  CK(hipMalloc(&out, 64));
  Cols c;
  c.k = (const unsigned long long *)buf;
  c.s = c.k + n;
  c.e = c.s + n;
  c.a = c.e + n;
  c.b = c.a + n;
  c.m = (const unsigned *)(c.b + n);
  const int reps = 20;
  auto report = [&](const char *name, float us) {
    std::printf("{\"probe\": \"%s\", \"us\": %.2f, \"GBps\": %.1f}\n", name, us, bytes / (us * 1e-6) / 1e9);
  };
  report("buf aux0 b1024 x1/CU", time_it([&] { read_buf<0><<<cus, 1024>>>(c, n, out); }, reps));
  report("buf nt b1024 x1/CU", time_it([&] { read_buf<2><<<cus, 1024>>>(c, n, out); }, reps));
  report("buf sc0 b1024 x1/CU", time_it([&] { read_buf<1><<<cus, 1024>>>(c, n, out); }, reps));
  report("buf aux0 b1024 x1/CU", time_it([&] { read_buf<0><<<cus, 1024>>>(c, n, out); }, reps));
  for (int per_cu : {1, 2, 4}) {
    const int g = cus * per_cu;
    char nm[96];
    std::snprintf(nm, sizeof nm, "contig S4 b1024 x%d/CU", per_cu);
    if (per_cu <= 2)
      report(nm, time_it([&] { read_contig<4, 1024><<<g, 1024>>>(c, n, out); }, reps));
    std::snprintf(nm, sizeof nm, "contig S4 b256 x%d/CU", per_cu * 4);
    report(nm, time_it([&] { read_contig<4, 256><<<g * 4, 256>>>(c, n, out); }, reps));
    std::snprintf(nm, sizeof nm, "contig S2 b1024 x%d/CU", per_cu);
    if (per_cu <= 2)
      report(nm, time_it([&] { read_contig<2, 1024><<<g, 1024>>>(c, n, out); }, reps));
    std::snprintf(nm, sizeof nm, "stride S2 b256 x%d/CU", per_cu * 4);
    report(nm, time_it([&] { read_stride<2, 256><<<g * 4, 256>>>(c, n, out); }, reps));
  }
  CK(hipFree(buf));
  return 0;
}
