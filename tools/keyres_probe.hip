// keyres_probe.hip -- prices key resolution in the C4 scatter: the span
// stream of SoA v1 (44 B/span, 10 M spans, one 1,024-thread workgroup per CU,
// two tiles in flight as bt_scatter2_kernel) plus one random read per span of
// the key table bucket its series id hashes to.
//   MODE 0  loads only
//   MODE 1  + one 8-B read at a random slot of a T-byte table
//   MODE 2  + one 32-B bucket read (two 16-B loads) of a T-byte table
//   MODE 3  + one 16-B read of a T-byte table
// The bucket reads of step t are issued one step before they are used (the
// shape a resolving scatter would take).  Table sizes: 16 MB (2^21 u64 keys:
// C4's key table) and 64 MB.
// Build: hipcc --offload-arch=gfx950 -O3 tools/keyres_probe.hip -o build/keyres_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

typedef unsigned long long u64;
constexpr int kBlock = 1024;

struct Args {
  const u64 *k, *s, *e, *a, *b;
  const unsigned *m;
  u64 n, chunk;
  const u64 *table;
  unsigned tmask;  // slots - 1 (power of two)
  u64 *out;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rs(const void *p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void ld2(__amdgpu_buffer_rsrc_t r, int off, u64 &x, u64 &y) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
  x = (u64)v[0] | ((u64)v[1] << 32);
  y = (u64)v[2] | ((u64)v[3] << 32);
}

struct Tile {
  u64 k[2], s[2], e[2], a[2], b[2];
  unsigned m[2];
};

__device__ __forceinline__ void load_tile(const Args &A, u64 lo, unsigned len, unsigned off, Tile &t) {
  const unsigned r8 = (unsigned)__builtin_amdgcn_readfirstlane((int)(len > (off & ~127u) ? (len - (off & ~127u)) * 8 : 0));
  const u64 tb = lo + (off & ~127u);
  const unsigned lane_off = (off & 127u);
  ld2(rs(A.k + tb, r8), lane_off * 8, t.k[0], t.k[1]);
  ld2(rs(A.s + tb, r8), lane_off * 8, t.s[0], t.s[1]);
  ld2(rs(A.e + tb, r8), lane_off * 8, t.e[0], t.e[1]);
  ld2(rs(A.a + tb, r8), lane_off * 8, t.a[0], t.a[1]);
  ld2(rs(A.b + tb, r8), lane_off * 8, t.b[0], t.b[1]);
  const auto mm = __builtin_amdgcn_raw_buffer_load_b64(rs(A.m + tb, r8 / 2), lane_off * 4, 0, 2);
  t.m[0] = mm[0];
  t.m[1] = mm[1];
}

__device__ __forceinline__ unsigned slot_of(u64 key, unsigned mask) {
  return (unsigned)((key * 0x9E3779B97F4A7C15ULL) >> 40) & mask;
}

struct Bk {
  u64 x[4];
};

template <int MODE>
__device__ __forceinline__ void issue(const Args &A, u64 key, Bk &r) {
  const unsigned s = slot_of(key, A.tmask);
  if (MODE == 1) r.x[0] = A.table[s];
  if (MODE == 2) {
    const ulonglong2 *p = reinterpret_cast<const ulonglong2 *>(A.table + (s & ~3u));
    const ulonglong2 v0 = p[0], v1 = p[1];
    r.x[0] = v0.x; r.x[1] = v0.y; r.x[2] = v1.x; r.x[3] = v1.y;
  }
  if (MODE == 3) {
    const ulonglong2 v0 = *reinterpret_cast<const ulonglong2 *>(A.table + (s & ~1u));
    r.x[0] = v0.x; r.x[1] = v0.y;
  }
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void p_keyres(Args A) {
  const u64 lo = min((u64)blockIdx.x * A.chunk, A.n), hi = min(lo + A.chunk, A.n);
  const unsigned len = (unsigned)(hi - lo);
  const unsigned wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u64 acc = 0;
  Tile t[2];
  const unsigned off0 = wave * 128 + lane * 2;
  load_tile(A, lo, len, off0, t[0]);
  load_tile(A, lo, len, off0 + 2048, t[1]);
  Bk pend[2] = {};
  // the bucket reads of the tile about to be processed are issued one step early
  if (MODE) {
#pragma unroll
    for (int j = 0; j < 2; ++j) issue<MODE>(A, t[0].k[j], pend[j]);
  }
  for (unsigned off = off0; off < len; off += 4096) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const unsigned o = off + h * 2048;
      Tile c = t[h];
      Bk cur[2] = {pend[0], pend[1]};
      if (MODE) {
#pragma unroll
        for (int j = 0; j < 2; ++j) issue<MODE>(A, t[h ^ 1].k[j], pend[j]);
      }
      load_tile(A, lo, len, o + 4096, t[h]);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (o + j >= len) continue;
        const u64 d = c.e[j] > c.s[j] ? c.e[j] - c.s[j] : 0;
        acc ^= d ^ c.a[j] ^ c.b[j] ^ c.m[j] ^ c.k[j];
        if (MODE) acc += cur[j].x[0] ^ cur[j].x[1] ^ cur[j].x[2] ^ cur[j].x[3];
      }
    }
  }
  if (acc == 0x1234567ULL) A.out[0] = acc;
}

__global__ void evict(const uint4 *p, u64 n, u64 *out) {
  unsigned acc = 0;
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) acc ^= p[i].x;
  if (acc == 0x12345u) out[0] = acc;
}

int main(int argc, char **argv) {
  const u64 n = argc > 1 ? strtoull(argv[1], 0, 10) : 10000000ULL;
  const int reps = 9;
  const unsigned G = 256;
  std::vector<u64> h(n);
  u64 x = 88172645463325252ULL;
  auto rnd = [&]() {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
  };
  // keys: 1 M distinct series ids, uniform
  std::vector<u64> ids(1 << 20);
  for (auto &v : ids) v = rnd();
  u64 *col[5];
  for (int c = 0; c < 5; ++c) {
    for (u64 i = 0; i < n; ++i) h[i] = c == 0 ? ids[rnd() & ((1 << 20) - 1)] : rnd();
    CK(hipMalloc(&col[c], n * 8));
    CK(hipMemcpy(col[c], h.data(), n * 8, hipMemcpyHostToDevice));
  }
  unsigned *meta;
  CK(hipMalloc(&meta, n * 4));
  CK(hipMemset(meta, 0, n * 4));
  u64 *table;
  const u64 tmax = 64ULL << 20;
  CK(hipMalloc(&table, tmax));
  CK(hipMemset(table, 7, tmax));
  Args A{};
  A.k = col[0];
  A.s = col[1];
  A.e = col[2];
  A.a = col[3];
  A.b = col[4];
  A.m = meta;
  A.n = n;
  A.chunk = ((n + G - 1) / G + 127) / 128 * 128;
  A.table = table;
  CK(hipMalloc(&A.out, 64));
  const u64 ev_n = (1ULL << 30) / 16;
  uint4 *evb;
  CK(hipMalloc(&evb, ev_n * 16));
  CK(hipMemset(evb, 1, ev_n * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, unsigned tbytes, auto kern) {
    A.tmask = tbytes / 8 - 1;
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
      hipLaunchKernelGGL(evict, dim3(2048), dim3(256), 0, 0, evb, ev_n, A.out);
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(kern, dim3(G), dim3(kBlock), 0, 0, A);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms * 1000);
    }
    std::sort(t.begin(), t.end());
    std::printf("{\"probe\": \"%s\", \"table_mb\": %u, \"median_us\": %.1f, \"min_us\": %.1f}\n", name,
                tbytes >> 20, t[t.size() / 2], t[0]);
    std::fflush(stdout);
  };
  for (int pass = 0; pass < 2; ++pass) {
    timeit("loads", 16u << 20, p_keyres<0>);
    for (unsigned tb : {16u << 20, 64u << 20}) {
      timeit("read8", tb, p_keyres<1>);
      timeit("read16", tb, p_keyres<3>);
      timeit("read32", tb, p_keyres<2>);
    }
  }
  return 0;
}
