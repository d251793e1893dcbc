// spanagg_kernels.hip -- CDNA4 (gfx950) kernels of libspanagg.
//
// One fused streaming pass per span batch replaces the connector's per-span
// body ([UPSTREAM] spanmetricsconnector connector.go `aggregateMetrics`:
// duration, buildKey -> map lookup, Sum.Add(1), explicitHistogram.Observe;
// SURVEY.md 3A step 5) and adds the per-service HLL / error count-min updates
// (SURVEY.md Appendix C).  Memory- and atomic-bound, no MFMA:
//   * coalesced SoA reads, 2 spans per lane (16-B loads per column);
//   * duration -> bucket by u64 compares against host-derived integer
//     thresholds (exactly SearchFloat64s(bounds, float64(d)/1e6));
//   * small-table path: the HBM key table is mirrored in LDS (same slots), and
//     per-workgroup LDS u16 counters + u64 ns sums are flushed, every epoch of
//     <= 65535 spans, into a workgroup-private HBM slab with plain
//     read-modify-write (no global atomics on the hot path); the slabs are
//     summed only at flush time (reduce kernel);
//   * HBM-table path (high cardinality): lock-free CAS insert + u64 atomics;
//   * HLL: u8 registers in HBM, read-filtered, CAS-max only when rho grows;
//   * count-min: u64 cells, atomic add per ERROR span per row.
#include "sa_internal.h"

namespace sa {
namespace {

constexpr uint64_t XP1 = 0x9E3779B185EBCA87ULL;
constexpr uint64_t XP2 = 0xC2B2AE3D27D4EB4FULL;
constexpr uint64_t XP3 = 0x165667B19E3779F9ULL;
constexpr uint64_t XP4 = 0x85EBCA77C2B2AE63ULL;
constexpr uint64_t XP5 = 0x27D4EB2F165667C5ULL;

__device__ __forceinline__ uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// xxh64 of the 16 trace-id bytes, seed 0 (lanes = the two LE words).
__device__ __forceinline__ uint64_t xxh64_16(uint64_t a, uint64_t b) {
  uint64_t h = XP5 + 16;
  h ^= rotl(a * XP2, 31) * XP1;
  h = rotl(h, 27) * XP1 + XP4;
  h ^= rotl(b * XP2, 31) * XP1;
  h = rotl(h, 27) * XP1 + XP4;
  h ^= h >> 33;
  h *= XP2;
  h ^= h >> 29;
  h *= XP3;
  h ^= h >> 32;
  return h;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// floor(n / d) with magic = floor((2^64-1)/d): estimate is low by at most 2.
__device__ __forceinline__ uint64_t fast_div(uint64_t n, uint64_t d, uint64_t magic) {
  uint64_t q = __umul64hi(n, magic);
  uint64_t r = n - q * d;
  while (r >= d) {
    ++q;
    r -= d;
  }
  return q;
}

template <int NB>
__device__ __forceinline__ uint32_t bucket_of(uint64_t d, const IngestParams &P) {
  if constexpr (NB >= 0) {
    uint32_t b = 0;
#pragma unroll
    for (int i = 0; i < NB; ++i) b += d > P.thr[i] ? 1u : 0u;
    return b;
  } else {
    uint32_t b = P.nneg;
    for (uint32_t i = 0; i < P.npos; ++i) b += d > P.thr[i] ? 1u : 0u;
    return b;
  }
}

__device__ __forceinline__ uint32_t g_find_insert(unsigned long long *keys, uint64_t key,
                                                  uint32_t log2cap, uint32_t max_probe) {
  const uint64_t mask = (1ULL << log2cap) - 1;
  uint64_t s = slot_of(key, log2cap);
  for (uint32_t i = 0; i < max_probe; ++i) {
    unsigned long long k = __hip_atomic_load(&keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == key) return (uint32_t)s;
    if (k == 0) {
      unsigned long long prev = atomicCAS(&keys[s], 0ULL, (unsigned long long)key);
      if (prev == 0 || prev == key) return (uint32_t)s;
    }
    s = (s + 1) & mask;
  }
  return kNotFound;
}

__device__ __forceinline__ uint32_t g_find(const unsigned long long *keys, uint64_t key,
                                           uint32_t log2cap, uint32_t max_probe) {
  const uint64_t mask = (1ULL << log2cap) - 1;
  uint64_t s = slot_of(key, log2cap);
  for (uint32_t i = 0; i < max_probe; ++i) {
    unsigned long long k = keys[s];
    if (k == key) return (uint32_t)s;
    if (k == 0) return kNotFound;
    s = (s + 1) & mask;
  }
  return kNotFound;
}

// Raise one u8 HLL register to rho (CAS on the containing aligned u32).
__device__ __forceinline__ void hll_raise(uint8_t *reg, uint32_t rho) {
  uint32_t *word = reinterpret_cast<uint32_t *>(reinterpret_cast<uintptr_t>(reg) & ~uintptr_t(3));
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(reg) & 3) * 8;
  uint32_t old = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (((old >> sh) & 0xFFu) < rho) {
    const uint32_t nw = (old & ~(0xFFu << sh)) | (rho << sh);
    const uint32_t prev = atomicCAS(word, old, nw);
    if (prev == old) break;
    old = prev;
  }
}

// Per-lane event counters, updated arithmetically (no addressable struct, so
// the compiler keeps them in VGPRs instead of scratch).
struct LaneStats {
  uint32_t zero_key, bad_svc, oor, dropped;
};

// Per-span sketch work: HLL of distinct trace ids per (window, service);
// count-min of ERROR spans per window keyed by the series hash.
// Returns 0 when applied, 1 for an invalid service id, 2 for a window outside
// the resident ring.
__device__ __forceinline__ uint32_t sketch_span(const IngestParams &P, uint64_t key, uint64_t end,
                                                uint64_t w0, uint64_t w1, uint32_t meta) {
  const uint32_t svc = meta & 0xFFFFu;
  if (svc >= P.n_services) return 1;
  const uint64_t win = fast_div(end, P.window_ns, P.win_magic);
  if (win - P.win_base >= (uint64_t)P.n_windows) return 2;
  const uint64_t ws = win & P.win_mask;
  const uint64_t x = xxh64_16(w0, w1);
  const uint64_t idx = x >> (64 - P.p);
  const uint32_t rho = (uint32_t)__clzll((long long)((x << P.p) | (1ULL << (P.p - 1)))) + 1;
  uint8_t *reg = P.hll + (((ws * P.n_services + svc) << P.p) + idx);
  if (*reg < rho) hll_raise(reg, rho);
  if (((meta >> 19) & 3u) == 2u) {
    unsigned long long *row = P.cms + ws * P.cms_d * P.cms_w;
    for (uint32_t j = 0; j < P.cms_d; ++j) {
      const uint64_t col = splitmix64(key ^ P.cms_seed[j]) >> P.cms_shift;
      atomicAdd(row + (uint64_t)j * P.cms_w + col, 1ULL);
    }
  }
  return 0;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ void flush_stats(const IngestParams &P, LaneStats &st) {
  const uint32_t a = wave_sum(st.zero_key), b = wave_sum(st.bad_svc), c = wave_sum(st.oor),
                 d = wave_sum(st.dropped);
  if ((threadIdx.x & 63) == 0) {
    if (a) atomicAdd(&P.stats[kStatZeroKey], (unsigned long long)a);
    if (b) atomicAdd(&P.stats[kStatInvalidService], (unsigned long long)b);
    if (c) atomicAdd(&P.stats[kStatWindowOOR], (unsigned long long)c);
    if (d) atomicAdd(&P.stats[kStatDropped], (unsigned long long)d);
  }
}

// Loads 2 consecutive spans (16-B per column) or one at the tail.
struct Span2 {
  uint64_t key[2], s[2], e[2], a[2], b[2];
  uint32_t meta[2];
  int cnt;
};

__device__ __forceinline__ void load_span2(const IngestParams &P, uint64_t i0, Span2 &v) {
  if (i0 + 1 < P.n) {
    const ulonglong2 k = *reinterpret_cast<const ulonglong2 *>(P.key + i0);
    const ulonglong2 s = *reinterpret_cast<const ulonglong2 *>(P.start + i0);
    const ulonglong2 e = *reinterpret_cast<const ulonglong2 *>(P.end + i0);
    const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(P.w0 + i0);
    const ulonglong2 b = *reinterpret_cast<const ulonglong2 *>(P.w1 + i0);
    const uint2 m = *reinterpret_cast<const uint2 *>(P.meta + i0);
    v.key[0] = k.x; v.key[1] = k.y;
    v.s[0] = s.x; v.s[1] = s.y;
    v.e[0] = e.x; v.e[1] = e.y;
    v.a[0] = a.x; v.a[1] = a.y;
    v.b[0] = b.x; v.b[1] = b.y;
    v.meta[0] = m.x; v.meta[1] = m.y;
    v.cnt = 2;
  } else if (i0 < P.n) {
    v.key[0] = P.key[i0];
    v.s[0] = P.start[i0];
    v.e[0] = P.end[i0];
    v.a[0] = P.w0[i0];
    v.b[0] = P.w1[i0];
    v.meta[0] = P.meta[i0];
    v.cnt = 1;
  } else {
    v.cnt = 0;
  }
}

// ---------------------------------------------------------------------------
// Small-table path.  LDS layout (dynamic, 16-B aligned):
//   lkeys [cap] u64   mirror of the HBM key table (same slot positions)
//   lsum  [cap] u64   per-slot ns sum of this epoch
//   lcnt  [cap][nw] u32, nw = ceil(nbk/2): two u16 bucket counters per word
template <int NB>
__device__ __forceinline__ void flush_lds(const IngestParams &P, uint32_t cap, uint32_t nbk,
                                          uint32_t nw, unsigned long long *lsum, uint32_t *lcnt) {
  uint32_t *scnt = P.slab_cnt + (uint64_t)blockIdx.x * cap * nbk;
  unsigned long long *ssum = P.slab_sum + (uint64_t)blockIdx.x * cap;
  const uint32_t cells = cap * nw;
  for (uint32_t c = threadIdx.x; c < cells; c += blockDim.x) {
    const uint32_t v = lcnt[c];
    if (v) {
      const uint32_t slot = c / nw, w = c - slot * nw;
      uint32_t *dst = scnt + (uint64_t)slot * nbk + 2 * w;
      if (v & 0xFFFFu) dst[0] += v & 0xFFFFu;
      if (v >> 16) dst[1] += v >> 16;
      lcnt[c] = 0;
    }
  }
  for (uint32_t s = threadIdx.x; s < cap; s += blockDim.x) {
    const unsigned long long v = lsum[s];
    if (v) {
      ssum[s] += v;
      lsum[s] = 0;
    }
  }
}

template <int NB>
__global__ __launch_bounds__(1024) void ingest_small_kernel(IngestParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t cap = 1u << P.log2cap;
  const uint64_t mask = cap - 1;
  const uint32_t nbk = NB >= 0 ? (uint32_t)NB + 1 : P.nbk;
  const uint32_t nw = (nbk + 1) >> 1;
  unsigned long long *lkeys = reinterpret_cast<unsigned long long *>(smem);
  unsigned long long *lsum = lkeys + cap;
  uint32_t *lcnt = reinterpret_cast<uint32_t *>(lsum + cap);

  for (uint32_t i = threadIdx.x; i < cap; i += blockDim.x) {
    lkeys[i] = __hip_atomic_load(&P.gkeys[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lsum[i] = 0;
  }
  for (uint32_t i = threadIdx.x; i < cap * nw; i += blockDim.x) lcnt[i] = 0;
  __syncthreads();

  LaneStats st{0, 0, 0, 0};
  const uint64_t tile = (uint64_t)blockDim.x * 2;
  const uint64_t ntiles = (P.n + tile - 1) / tile;
  uint32_t in_epoch = 0;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    Span2 v;
    load_span2(P, t * tile + (uint64_t)threadIdx.x * 2, v);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j < v.cnt) {
        const uint64_t key = v.key[j];
        const uint64_t d = v.e[j] > v.s[j] ? v.e[j] - v.s[j] : 0;
        st.zero_key += key == 0 ? 1u : 0u;
        if (key != 0) {
          const uint32_t b = bucket_of<NB>(d, P);
          uint64_t s = slot_of(key, P.log2cap);
          uint32_t found = kNotFound;
          for (uint32_t q = 0; q < P.max_probe; ++q) {
            const unsigned long long k = lkeys[s];
            if (k == key) {
              found = (uint32_t)s;
              break;
            }
            if (k == 0) break;
            s = (s + 1) & mask;
          }
          if (found == kNotFound) {
            found = g_find_insert(P.gkeys, key, P.log2cap, P.max_probe);
            if (found != kNotFound) lkeys[found] = key;
          }
          if (found != kNotFound) {
            atomicAdd(&lcnt[found * nw + (b >> 1)], 1u << ((b & 1) * 16));
            atomicAdd(&lsum[found], (unsigned long long)d);
          }
          st.dropped += found == kNotFound ? 1u : 0u;
        }
        const uint32_t sk = sketch_span(P, key, v.e[j], v.a[j], v.b[j], v.meta[j]);
        st.bad_svc += sk == 1 ? 1u : 0u;
        st.oor += sk == 2 ? 1u : 0u;
      }
    }
    if (++in_epoch == P.epoch_tiles) {
      __syncthreads();
      flush_lds<NB>(P, cap, nbk, nw, lsum, lcnt);
      __syncthreads();
      in_epoch = 0;
    }
  }
  __syncthreads();
  flush_lds<NB>(P, cap, nbk, nw, lsum, lcnt);
  flush_stats(P, st);
}

// ---------------------------------------------------------------------------
// HBM-table path (table larger than LDS): CAS insert + u64 atomics per span.
template <int NB>
__global__ __launch_bounds__(256) void ingest_hbm_kernel(IngestParams P) {
  LaneStats st{0, 0, 0, 0};
  const uint32_t nbk = NB >= 0 ? (uint32_t)NB + 1 : P.nbk;
  const uint32_t stride = nbk + 1;
  const uint64_t tile = (uint64_t)blockDim.x * 2;
  const uint64_t ntiles = (P.n + tile - 1) / tile;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    Span2 v;
    load_span2(P, t * tile + (uint64_t)threadIdx.x * 2, v);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (j < v.cnt) {
        const uint64_t key = v.key[j];
        const uint64_t d = v.e[j] > v.s[j] ? v.e[j] - v.s[j] : 0;
        st.zero_key += key == 0 ? 1u : 0u;
        if (key != 0) {
          const uint32_t b = bucket_of<NB>(d, P);
          const uint32_t found = g_find_insert(P.gkeys, key, P.log2cap, P.max_probe);
          if (found != kNotFound) {
            unsigned long long *row = P.gcounts + (uint64_t)found * stride;
            atomicAdd(row + b, 1ULL);
            atomicAdd(row + nbk, (unsigned long long)d);
          }
          st.dropped += found == kNotFound ? 1u : 0u;
        }
        const uint32_t sk = sketch_span(P, key, v.e[j], v.a[j], v.b[j], v.meta[j]);
        st.bad_svc += sk == 1 ? 1u : 0u;
        st.oor += sk == 2 ? 1u : 0u;
      }
    }
  }
  flush_stats(P, st);
}

// ---------------------------------------------------------------------------
// Flush-time kernels.
__global__ void reduce_slabs_kernel(uint32_t *slab_cnt, unsigned long long *slab_sum,
                                    unsigned long long *gcounts, uint32_t G, uint64_t cap,
                                    uint32_t nbk) {
  const uint64_t cells = cap * nbk;
  const uint32_t stride = nbk + 1;
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < cells + cap;
       c += (uint64_t)gridDim.x * blockDim.x) {
    if (c < cells) {
      unsigned long long acc = 0;
      for (uint32_t g = 0; g < G; ++g) {
        uint32_t *p = slab_cnt + (uint64_t)g * cells + c;
        const uint32_t v = *p;
        if (v) {
          acc += v;
          *p = 0;
        }
      }
      if (acc) {
        const uint64_t slot = c / nbk, b = c - slot * nbk;
        gcounts[slot * stride + b] += acc;
      }
    } else {
      const uint64_t slot = c - cells;
      unsigned long long acc = 0;
      for (uint32_t g = 0; g < G; ++g) {
        unsigned long long *p = slab_sum + (uint64_t)g * cap + slot;
        const unsigned long long v = *p;
        if (v) {
          acc += v;
          *p = 0;
        }
      }
      if (acc) gcounts[slot * stride + nbk] += acc;
    }
  }
}

// Compacts occupied slots with a non-zero row into (out_keys, out_rows); order
// is arrival order of the atomic ticket (the host sorts by key).
__global__ void compact_kernel(const unsigned long long *gkeys, unsigned long long *gcounts,
                               uint64_t cap, uint32_t stride, unsigned long long *out_keys,
                               unsigned long long *out_rows, unsigned long long *out_n,
                               uint64_t out_cap, int reset) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap;
       s += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long k = gkeys[s];
    if (!k) continue;
    unsigned long long *row = gcounts + s * stride;
    bool any = false;
    for (uint32_t b = 0; b < stride; ++b) any |= row[b] != 0;
    if (!any) continue;
    const unsigned long long pos = atomicAdd(out_n, 1ULL);
    if (pos < out_cap) {
      if (out_keys) out_keys[pos] = k;
      if (out_rows)
        for (uint32_t b = 0; b < stride; ++b) out_rows[pos * stride + b] = row[b];
    }
    if (reset)
      for (uint32_t b = 0; b < stride; ++b) row[b] = 0;
  }
}

__global__ void gather_dense_kernel(const unsigned long long *gkeys,
                                    const unsigned long long *gcounts, uint32_t log2cap,
                                    uint32_t max_probe, uint32_t stride, const uint64_t *keys,
                                    uint64_t n, uint64_t *rows) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    const uint32_t s = k ? g_find(gkeys, k, log2cap, max_probe) : kNotFound;
    for (uint32_t b = 0; b < stride; ++b)
      rows[i * stride + b] = s == kNotFound ? 0 : gcounts[(uint64_t)s * stride + b];
  }
}

__global__ void count_keys_kernel(const unsigned long long *gkeys, uint64_t cap,
                                  unsigned long long *out) {
  uint32_t c = 0;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap;
       s += (uint64_t)gridDim.x * blockDim.x)
    c += gkeys[s] != 0;
  c = wave_sum(c);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, (unsigned long long)c);
}

uint32_t grid_for(uint64_t work, uint32_t block, uint32_t cap_blocks) {
  uint64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap_blocks) g = cap_blocks;
  return (uint32_t)g;
}

}  // namespace

hipError_t prepare_ingest_small(size_t lds_bytes) {
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&ingest_small_kernel<16>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute(reinterpret_cast<const void *>(&ingest_small_kernel<-1>),
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
}

hipError_t launch_ingest_small(const IngestParams &P, uint32_t grid, uint32_t block,
                               size_t lds_bytes, hipStream_t s) {
  if (P.nneg == 0 && P.npos == 16)
    hipLaunchKernelGGL(ingest_small_kernel<16>, dim3(grid), dim3(block), lds_bytes, s, P);
  else
    hipLaunchKernelGGL(ingest_small_kernel<-1>, dim3(grid), dim3(block), lds_bytes, s, P);
  return hipGetLastError();
}

hipError_t launch_ingest_hbm(const IngestParams &P, uint32_t grid, uint32_t block,
                             hipStream_t s) {
  if (P.nneg == 0 && P.npos == 16)
    hipLaunchKernelGGL(ingest_hbm_kernel<16>, dim3(grid), dim3(block), 0, s, P);
  else
    hipLaunchKernelGGL(ingest_hbm_kernel<-1>, dim3(grid), dim3(block), 0, s, P);
  return hipGetLastError();
}

hipError_t launch_reduce_slabs(uint32_t *slab_cnt, unsigned long long *slab_sum,
                               unsigned long long *gcounts, uint32_t G, uint64_t cap,
                               uint32_t nbk, hipStream_t s) {
  const uint32_t block = 256;
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3(grid_for(cap * (nbk + 1), block, 4096)),
                     dim3(block), 0, s, slab_cnt, slab_sum, gcounts, G, cap, nbk);
  return hipGetLastError();
}

hipError_t launch_compact(const unsigned long long *gkeys, unsigned long long *gcounts,
                          uint64_t cap, uint32_t stride, unsigned long long *out_keys,
                          unsigned long long *out_rows, unsigned long long *out_n,
                          uint64_t out_cap, int reset, hipStream_t s) {
  const uint32_t block = 256;
  hipLaunchKernelGGL(compact_kernel, dim3(grid_for(cap, block, 4096)), dim3(block), 0, s, gkeys,
                     gcounts, cap, stride, out_keys, out_rows, out_n, out_cap, reset);
  return hipGetLastError();
}

hipError_t launch_gather_dense(const unsigned long long *gkeys, const unsigned long long *gcounts,
                               uint32_t log2cap, uint32_t max_probe, uint32_t stride,
                               const uint64_t *keys, uint64_t n, uint64_t *rows, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t block = 256;
  hipLaunchKernelGGL(gather_dense_kernel, dim3(grid_for(n, block, 4096)), dim3(block), 0, s,
                     gkeys, gcounts, log2cap, max_probe, stride, keys, n, rows);
  return hipGetLastError();
}

hipError_t launch_count_keys(const unsigned long long *gkeys, uint64_t cap,
                             unsigned long long *out, hipStream_t s) {
  const uint32_t block = 256;
  hipLaunchKernelGGL(count_keys_kernel, dim3(grid_for(cap, block, 2048)), dim3(block), 0, s,
                     gkeys, cap, out);
  return hipGetLastError();
}

}  // namespace sa
