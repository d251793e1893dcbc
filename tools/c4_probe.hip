// c4_probe.hip -- price the pieces of the high-cardinality (C4) scatter /
// aggregate design on the real access pattern: 10 M spans of SoA v1, random
// 64-bit keys, 2,048 bins by the top 11 key bits, one 1,024-thread workgroup
// per CU.  Each probe is timed with HIP events (median of reps).
// Build: hipcc --offload-arch=gfx950 -O3 tools/c4_probe.hip -o build/c4_probe
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
constexpr int kBlock = 1024, kBinBits = 11, kBins = 1 << kBinBits;
constexpr int kShift = 64 - kBinBits;

struct Args {
  const u64 *k, *s, *e, *a, *b;
  const unsigned *m;
  u64 n, chunk;
  ulonglong2 *rec;   // [bin][G][region]
  unsigned *cnt;     // [bin][G]
  unsigned region, G;
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
  const unsigned rem = off < len ? len - off : 0;
  const u64 base = lo + off;
  const unsigned r8 = (unsigned)__builtin_amdgcn_readfirstlane((int)(len > (off & ~127u) ? (len - (off & ~127u)) * 8 : 0));
  (void)rem;
  (void)base;
  const u64 tb = lo + (off & ~127u);  // wave tile base (128 spans)
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

// MODE 0: loads only; 1: + LDS cursor atomic; 2: + direct 16-B store into the
// (bin, workgroup) region; 3: + store to the span's own position (coalesced)
template <int MODE>
__global__ __launch_bounds__(kBlock) void p_direct(Args A) {
  __shared__ unsigned cur[kBins];
  const u64 lo = min((u64)blockIdx.x * A.chunk, A.n), hi = min(lo + A.chunk, A.n);
  const unsigned len = (unsigned)(hi - lo);
  for (unsigned b = threadIdx.x; b < kBins; b += kBlock) cur[b] = 0;
  __syncthreads();
  const unsigned wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u64 acc = 0;
  Tile t[2];
  unsigned off0 = wave * 128 + lane * 2;
  load_tile(A, lo, len, off0, t[0]);
  load_tile(A, lo, len, off0 + 2048, t[1]);
  for (unsigned off = off0; off < len; off += 4096) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const unsigned o = off + h * 2048;
      Tile c = t[h];
      load_tile(A, lo, len, o + 4096, t[h]);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (o + j >= len) continue;
        const u64 d = c.e[j] > c.s[j] ? c.e[j] - c.s[j] : 0;
        const u64 key = c.k[j];
        acc ^= d ^ c.a[j] ^ c.b[j] ^ c.m[j] ^ key;
        if (MODE >= 1) {
          const unsigned bin = (unsigned)(key >> kShift);
          const unsigned r = atomicAdd(&cur[bin], 1u);
          if (MODE == 1) acc += r;
          if (MODE == 2 && r < A.region)
            A.rec[((u64)bin * A.G + blockIdx.x) * A.region + r] = make_ulonglong2(key, d);
          if (MODE == 3) A.rec[lo + o + j] = make_ulonglong2(key, d);
        }
      }
    }
  }
  __syncthreads();
  if (MODE == 2)
    for (unsigned b = threadIdx.x; b < kBins; b += kBlock) A.cnt[(u64)b * A.G + blockIdx.x] = min(cur[b], A.region);
  if (acc == 0x1234567ULL) A.out[0] = acc;
}

// Tile sort: each iteration the workgroup takes T = 1024 * 2 * H spans,
// ranks them per bin in LDS, writes them bin-sorted into an LDS tile, and
// stores the tile's runs into the (bin, workgroup) regions with consecutive
// lanes on consecutive records.
template <int H>
__global__ __launch_bounds__(kBlock) void p_tilesort(Args A) {
  constexpr unsigned T = kBlock * 2 * H;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned *cur = reinterpret_cast<unsigned *>(smem);  // region fill per bin
  unsigned *hist = cur + kBins;                        // this tile's count per bin
  unsigned *start = hist + kBins;                      // exclusive prefix
  unsigned *wsum = start + kBins;                      // [16] wave totals
  ulonglong2 *srt = reinterpret_cast<ulonglong2 *>(wsum + 16);
  const u64 lo = min((u64)blockIdx.x * A.chunk, A.n), hi = min(lo + A.chunk, A.n);
  const unsigned len = (unsigned)(hi - lo);
  for (unsigned b = threadIdx.x; b < kBins; b += kBlock) cur[b] = hist[b] = 0;
  __syncthreads();
  const unsigned wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Tile t[H];
  // tile h of iteration it: spans [it*T + h*2048 + wave*128 + lane*2, +2)
  const unsigned base_off = wave * 128 + lane * 2;
#pragma unroll
  for (int h = 0; h < H; ++h) load_tile(A, lo, len, base_off + h * 2048, t[h]);
  u64 acc = 0;
  for (unsigned it0 = 0; it0 < len; it0 += T) {
    u64 rk[H][2], rd[H][2];
    unsigned rank[H][2], bin[H][2];
#pragma unroll
    for (int h = 0; h < H; ++h) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const unsigned o = it0 + h * 2048 + base_off + j;
        const bool v = o < len;
        rk[h][j] = t[h].k[j];
        rd[h][j] = t[h].e[j] > t[h].s[j] ? t[h].e[j] - t[h].s[j] : 0;
        acc ^= t[h].a[j] ^ t[h].b[j] ^ t[h].m[j];
        bin[h][j] = v ? (unsigned)(rk[h][j] >> kShift) : 0xFFFFFFFFu;
      }
      load_tile(A, lo, len, it0 + T + h * 2048 + base_off, t[h]);
    }
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j) rank[h][j] = bin[h][j] != 0xFFFFFFFFu ? atomicAdd(&hist[bin[h][j]], 1u) : 0u;
    __syncthreads();
    // exclusive scan of hist (2 bins per thread)
    const unsigned v0 = hist[2 * threadIdx.x], v1 = hist[2 * threadIdx.x + 1];
    unsigned incl = v0 + v1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned x = (unsigned)__shfl_up((int)incl, o, 64);
      if ((int)lane >= o) incl += x;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    unsigned wpre = 0;
    for (unsigned w = 0; w < wave; ++w) wpre += wsum[w];
    const unsigned ex = wpre + incl - v0 - v1;
    start[2 * threadIdx.x] = ex;
    start[2 * threadIdx.x + 1] = ex + v0;
    __syncthreads();
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (bin[h][j] != 0xFFFFFFFFu) srt[start[bin[h][j]] + rank[h][j]] = make_ulonglong2(rk[h][j], rd[h][j]);
    __syncthreads();
    const unsigned tn = min(T, len - it0);
    for (unsigned i = threadIdx.x; i < tn; i += kBlock) {
      const ulonglong2 r = srt[i];
      const unsigned b = (unsigned)(r.x >> kShift);
      const unsigned pos = cur[b] + (i - start[b]);
      if (pos < A.region) A.rec[((u64)b * A.G + blockIdx.x) * A.region + pos] = r;
    }
    __syncthreads();
    for (unsigned b = threadIdx.x; b < kBins; b += kBlock) {
      cur[b] += hist[b];
      hist[b] = 0;
    }
    __syncthreads();
  }
  for (unsigned b = threadIdx.x; b < kBins; b += kBlock) A.cnt[(u64)b * A.G + blockIdx.x] = min(cur[b], A.region);
  if (acc == 0x1234567ULL) A.out[0] = acc;
}

// Aggregate-side read: one workgroup per bin reads its records (one wave per
// region) and folds them into a checksum
__global__ __launch_bounds__(512) void a_read(Args A) {
  const unsigned bin = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u64 acc = 0;
  for (unsigned g = wave; g < A.G; g += 8) {
    const unsigned c = A.cnt[(u64)bin * A.G + g];
    const ulonglong2 *r = A.rec + ((u64)bin * A.G + g) * A.region;
    for (unsigned i = lane; i < c; i += 64) {
      const ulonglong2 x = r[i];
      acc += x.x ^ x.y;
    }
  }
  if (acc == 0x1234567ULL) A.out[0] = acc;
}


// Chunked scatter: the span loads of p_direct plus, per record, a 16-B store
// into a random chunk of C bytes: lanes c*(C/16) .. +C/16 of a wave write one
// chunk together (the write shape of a C-byte LDS stage flush)
template <int C>
__global__ __launch_bounds__(kBlock) void p_chunked(Args A) {
  constexpr unsigned L = C / 16;  // lanes per chunk
  const u64 lo = min((u64)blockIdx.x * A.chunk, A.n), hi = min(lo + A.chunk, A.n);
  const unsigned len = (unsigned)(hi - lo);
  const unsigned wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u64 nchunks = A.n * 16 / C * 4;  // 4x sparse target
  u64 acc = 0, st = 0x9E3779B97F4A7C15ULL * (blockIdx.x * 64 + wave + 1);
  Tile t[2];
  unsigned off0 = wave * 128 + lane * 2;
  load_tile(A, lo, len, off0, t[0]);
  load_tile(A, lo, len, off0 + 2048, t[1]);
  for (unsigned off = off0; off < len; off += 4096) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const unsigned o = off + h * 2048;
      Tile c = t[h];
      load_tile(A, lo, len, o + 4096, t[h]);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const u64 d = c.e[j] > c.s[j] ? c.e[j] - c.s[j] : 0;
        acc ^= d ^ c.a[j] ^ c.b[j] ^ c.m[j];
        st = st * 6364136223846793005ULL + 1442695040888963407ULL;
        const u64 ch = ((st >> 20) + (lane / L) * 0x9E3779B1ULL) % nchunks;
        if (o + j < len) A.rec[ch * L + (lane % L)] = make_ulonglong2(c.k[j], d);
      }
    }
  }
  if (acc == 0x1234567ULL) A.out[0] = acc;
}

// The same with 8-B records (C-byte chunks of C / 8 lanes): the store side of
// a scatter whose records carry a resolved key slot instead of the key
template <int C>
__global__ __launch_bounds__(kBlock) void p_chunked8(Args A) {
  constexpr unsigned L = C / 8;  // lanes per chunk
  const u64 lo = min((u64)blockIdx.x * A.chunk, A.n), hi = min(lo + A.chunk, A.n);
  const unsigned len = (unsigned)(hi - lo);
  const unsigned wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u64 nchunks = A.n * 8 / C * 4;  // 4x sparse target
  u64 acc = 0, st = 0x9E3779B97F4A7C15ULL * (blockIdx.x * 64 + wave + 1);
  u64 *rec = reinterpret_cast<u64 *>(A.rec);
  Tile t[2];
  unsigned off0 = wave * 128 + lane * 2;
  load_tile(A, lo, len, off0, t[0]);
  load_tile(A, lo, len, off0 + 2048, t[1]);
  for (unsigned off = off0; off < len; off += 4096) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const unsigned o = off + h * 2048;
      Tile c = t[h];
      load_tile(A, lo, len, o + 4096, t[h]);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const u64 d = c.e[j] > c.s[j] ? c.e[j] - c.s[j] : 0;
        acc ^= c.a[j] ^ c.b[j] ^ c.m[j];
        st = st * 6364136223846793005ULL + 1442695040888963407ULL;
        const u64 ch = ((st >> 20) + (lane / L) * 0x9E3779B1ULL) % nchunks;
        if (o + j < len) rec[ch * L + (lane % L)] = c.k[j] ^ d;
      }
    }
  }
  if (acc == 0x1234567ULL) A.out[0] = acc;
}

// Chunked read: 160 MB read as random C-byte chunks (lanes as above)
template <int C>
__global__ __launch_bounds__(512) void a_chunked(Args A) {
  constexpr unsigned L = C / 16;
  const unsigned lane = threadIdx.x & 63;
  const u64 nchunks = A.n * 16 / C * 4;
  const u64 per = A.n / (gridDim.x * (512 / 64)) / (64 / L);
  u64 acc = 0, st = 0x9E3779B97F4A7C15ULL * (blockIdx.x * 8 + (threadIdx.x >> 6) + 1);
  for (u64 i = 0; i < per; ++i) {
    st = st * 6364136223846793005ULL + 1442695040888963407ULL;
    const u64 ch = ((st >> 20) + (lane / L) * 0x9E3779B1ULL) % nchunks;
    const ulonglong2 x = A.rec[ch * L + (lane % L)];
    acc += x.x ^ x.y;
  }
  if (acc == 0x1234567ULL) A.out[0] = acc;
}

// streaming read of a big buffer (evicts the caches between probes)
__global__ void evict(const uint4 *p, u64 n, u64 *out) {
  unsigned acc = 0;
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) acc ^= p[i].x;
  if (acc == 0x12345u) out[0] = acc;
}

int main(int argc, char **argv) {
  const u64 n = argc > 1 ? strtoull(argv[1], 0, 10) : 10000000ULL;
  const int reps = 7;
  const unsigned G = 256;
  std::vector<u64> h(n);
  u64 x = 88172645463325252ULL;
  auto rnd = [&]() {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    return x;
  };
  u64 *col[5];
  for (int c = 0; c < 5; ++c) {
    for (u64 i = 0; i < n; ++i) h[i] = c == 2 ? (h[i] + (rnd() & 0xFFFFFF)) : rnd();
    if (c == 1) {
      for (u64 i = 0; i < n; ++i) h[i] = rnd() >> 8;
    }
    CK(hipMalloc(&col[c], n * 8));
    CK(hipMemcpy(col[c], h.data(), n * 8, hipMemcpyHostToDevice));
  }
  unsigned *meta;
  CK(hipMalloc(&meta, n * 4));
  CK(hipMemset(meta, 0, n * 4));
  Args A{};
  A.k = col[0];
  A.s = col[1];
  A.e = col[2];
  A.a = col[3];
  A.b = col[4];
  A.m = meta;
  A.n = n;
  A.chunk = ((n + G - 1) / G + 127) / 128 * 128;
  A.G = G;
  A.region = (unsigned)(A.chunk / kBins * 5 / 4 + 64);
  CK(hipMalloc(&A.rec, std::max((u64)kBins * G * A.region * 16, n * 16 * 4 + 4096)));
  CK(hipMalloc(&A.cnt, (u64)kBins * G * 4));
  CK(hipMalloc(&A.out, 64));
  const u64 ev_n = (1ULL << 30) / 16;
  uint4 *evb;
  CK(hipMalloc(&evb, ev_n * 16));
  CK(hipMemset(evb, 1, ev_n * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, auto launch, bool evict_first) {
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
      if (evict_first) hipLaunchKernelGGL(evict, dim3(2048), dim3(256), 0, 0, evb, ev_n, A.out);
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms * 1000);
    }
    std::sort(t.begin(), t.end());
    std::printf("{\"probe\": \"%s\", \"median_us\": %.1f, \"min_us\": %.1f}\n", name, t[t.size() / 2], t[0]);
  };
  auto L = [&](auto kern, size_t lds) {
    return [=]() { hipLaunchKernelGGL(kern, dim3(G), dim3(kBlock), lds, 0, A); };
  };
  const size_t ts2 = kBins * 12 + 64 + (size_t)kBlock * 2 * 2 * 16;
  const size_t ts4 = kBins * 12 + 64 + (size_t)kBlock * 2 * 4 * 16;
  CK(hipFuncSetAttribute((const void *)&p_tilesort<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ts2));
  CK(hipFuncSetAttribute((const void *)&p_tilesort<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ts4));
  if (argc > 2) {
    timeit("loads", L(p_direct<0>, 0), true);
    timeit("chunk_32", L(p_chunked<32>, 0), true);
    timeit("chunk_64", L(p_chunked<64>, 0), true);
    timeit("chunk_128", L(p_chunked<128>, 0), true);
    timeit("chunk_256", L(p_chunked<256>, 0), true);
    timeit("chunk_512", L(p_chunked<512>, 0), true);
    timeit("chunk_1024", L(p_chunked<1024>, 0), true);
    timeit("chunk8_32", L(p_chunked8<32>, 0), true);
    timeit("chunk8_64", L(p_chunked8<64>, 0), true);
    timeit("chunk8_128", L(p_chunked8<128>, 0), true);
    auto R = [&](auto kern) { return [=]() { hipLaunchKernelGGL(kern, dim3(2048), dim3(512), 0, 0, A); }; };
    timeit("read_chunk_16", R(a_chunked<16>), true);
    timeit("read_chunk_64", R(a_chunked<64>), true);
    timeit("read_chunk_128", R(a_chunked<128>), true);
    timeit("read_chunk_256", R(a_chunked<256>), true);
    timeit("read_chunk_512", R(a_chunked<512>), true);
    timeit("read_chunk_1024", R(a_chunked<1024>), true);
    return 0;
  }
  for (int pass = 0; pass < 2; ++pass) {
    timeit("loads", L(p_direct<0>, 0), true);
    timeit("lds_cursor", L(p_direct<1>, 0), true);
    timeit("direct_store", L(p_direct<2>, 0), true);
    timeit("a_read_after_direct", [&]() { hipLaunchKernelGGL(a_read, dim3(kBins), dim3(512), 0, 0, A); }, false);
    timeit("a_read_evicted", [&]() { hipLaunchKernelGGL(a_read, dim3(kBins), dim3(512), 0, 0, A); }, true);
    timeit("coalesced_store", L(p_direct<3>, 0), true);
    timeit("tilesort_4096", L(p_tilesort<2>, ts2), true);
    timeit("a_read_after_ts4096", [&]() { hipLaunchKernelGGL(a_read, dim3(kBins), dim3(512), 0, 0, A); }, false);
    timeit("tilesort_8192", L(p_tilesort<4>, ts4), true);
  }
  // check: every record of the tile sort landed in its bin's region
  std::vector<unsigned> cnt((size_t)kBins * G);
  CK(hipMemcpy(cnt.data(), A.cnt, cnt.size() * 4, hipMemcpyDeviceToHost));
  u64 tot = 0;
  for (unsigned c : cnt) tot += c;
  std::printf("{\"records\": %llu, \"n\": %llu, \"region\": %u}\n", tot, n, A.region);
  return 0;
}
