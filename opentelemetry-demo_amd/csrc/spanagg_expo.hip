// spanagg_expo.hip -- exponential histograms on the GPU (gfx950): the
// spanmetrics connector's `histogram.exponential` option ([UPSTREAM]
// spanmetricsconnector internal/metrics exponentialHistogram.Observe ->
// github.com/lightstep/go-expohisto structure.Histogram[float64].Update).
//
// go-expohisto updates one value at a time and downscales (merges bucket
// pairs) whenever a value would widen the positive index range to max_size or
// more.  Bucket i at scale s-1 is exactly buckets 2i and 2i+1 at scale s (the
// index mapping is consistent across scales: Log(v) * Ldexp(Log2E, s) scales
// by exact powers of two), so the final histogram depends only on the set of
// values: its scale is the largest s <= 20 at which the indices of the
// smallest and largest positive value are less than max_size apart.  The
// kernels use that:
//   expo_pass1_kernel  per span: key slot (HBM table), count, ns sum, min/max
//                      of all durations and of the positive ones (atomics),
//                      zero count; the slot is kept for pass 3
//   expo_rescale_kernel per series: the scale its values so far need; buckets
//                      kept at a higher scale are merged down pairwise
//   expo_count_kernel  per span: bucket index at the series' scale (Go's
//                      math.Log, restated operation for operation with no
//                      contraction), one u32 atomic into a circular array of
//                      max_size buckets (index mod max_size; the live range is
//                      shorter than max_size)
// The sketches of these spans run through the HBM-table ingest kernel.
#include <algorithm>

#include "sa_device.h"

// No fused multiply-adds anywhere in this file: Go computes every operation of
// math.Log and of the index mapping with its own rounding (amd64, no FMA).
#pragma clang fp contract(off)

namespace sa {
namespace {

// Go's math.Log (src/math/log.go), the same operations in the same order.
__device__ __forceinline__ double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  // Frexp of a positive normal value: x = f1 * 2^ki, f1 in [0.5, 1)
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  int ki = (int)((b >> 52) & 0x7FF) - 1022;
  double f1 = __longlong_as_double((long long)((b & 0x800FFFFFFFFFFFFFULL) | (1022ULL << 52)));
  if (f1 < 1.4142135623730951 / 2) {
    f1 *= 2;
    ki--;
  }
  const double f = f1 - 1, k = (double)ki;
  const double s = f / (2 + f), s2 = s * s, s4 = s2 * s2;
  const double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  const double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  const double R = t1 + t2, hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

// go-expohisto MapToIndex of a positive normal value (durations >= 1 ns are
// normal doubles in ms and in s)
__device__ __forceinline__ int32_t expo_index(double v, int32_t scale) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const int32_t exp = (int32_t)((b >> 52) & 0x7FF) - 1023;
  const bool pow2 = (b & ((1ULL << 52) - 1)) == 0;
  if (scale > 0) {
    if (pow2) return (exp << scale) - 1;
    const double x = floor(go_log(v) * ldexp(1.4426950408889634, scale));
    const double max_index = (double)((1024 << scale) - 1);
    return x >= max_index ? (int32_t)max_index : (int32_t)x;
  }
  return (exp + (pow2 ? -1 : 0)) >> (-scale);
}

__device__ __forceinline__ double expo_value(uint64_t d_ns, double div) {
  return (double)d_ns / div;
}

constexpr int32_t kExpoMaxScale = 20, kExpoMinScale = -10;
constexpr int32_t kExpoEmpty = 0x7FFFFFFF;  // ExpoHdr.lo when no positive value is kept

__device__ __forceinline__ uint32_t expo_mod(int32_t i, uint32_t m) {
  const int32_t r = i % (int32_t)m;
  return (uint32_t)(r < 0 ? r + (int32_t)m : r);
}

// pass 1: slot, count, sum, min/max, zero count (one span per thread)
__global__ __launch_bounds__(256) void expo_pass1_kernel(ExpoParams E) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < E.n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t key = E.key[i];
    uint32_t slot = kNotFound;
    if (key != 0) {
      slot = g_find_insert(E.gkeys, key, E.log2cap, E.max_probe);
      if (slot == kNotFound) {
        atomicAdd(E.dropped, 1ULL);
      } else {
        const uint64_t d = E.end[i] > E.start[i] ? E.end[i] - E.start[i] : 0;
        ExpoHdr &h = E.hdr[slot];
        atomicAdd(&h.count, 1ULL);
        atomicAdd(&h.sum_ns, (unsigned long long)d);
        atomicMin(&h.min_ns, (unsigned long long)d);
        atomicMax(&h.max_ns, (unsigned long long)d);
        if (d == 0) {
          atomicAdd(&h.zero, 1ULL);
        } else {
          atomicMin(&h.minpos_ns, (unsigned long long)d);
          atomicMax(&h.maxpos_ns, (unsigned long long)d);
        }
      }
    }
    E.slot_of[i] = slot;
  }
}

// per series: fix the scale for every positive value seen so far; merge the
// kept buckets down when it drops
__device__ __forceinline__ void rescale_slot(const ExpoParams &E, uint64_t s) {
  {
    ExpoHdr &h = E.hdr[s];
    if (h.maxpos_ns == 0) return;  // no positive value
    const double vlo = expo_value(h.minpos_ns, E.div), vhi = expo_value(h.maxpos_ns, E.div);
    int32_t lo = expo_index(vlo, kExpoMaxScale), hi = expo_index(vhi, kExpoMaxScale), change = 0;
    while (hi - lo >= (int32_t)E.max_size) {  // changeScale
      hi >>= 1;
      lo >>= 1;
      ++change;
    }
    int32_t target = kExpoMaxScale - change;
    if (target < kExpoMinScale) target = kExpoMinScale;
    if (h.lo != kExpoEmpty && h.scale < target) target = h.scale;  // scales only go down
    if (h.lo != kExpoEmpty && target < h.scale) {
      const uint32_t diff = (uint32_t)(h.scale - target), M = E.max_size;
      uint32_t *src = E.buckets + ((uint64_t)h.cur * E.cap + s) * M;
      uint32_t *dst = E.buckets + ((uint64_t)(h.cur ^ 1u) * E.cap + s) * M;
      for (int32_t i = h.lo; i <= h.hi; ++i) {
        const uint32_t c = src[expo_mod(i, M)];
        if (c) dst[expo_mod(i >> diff, M)] += c;
        src[expo_mod(i, M)] = 0;
      }
      h.cur ^= 1u;
    }
    h.scale = target;
    h.lo = expo_index(vlo, target);
    h.hi = expo_index(vhi, target);
  }
}

// (one thread per slot)
__global__ __launch_bounds__(256) void expo_rescale_kernel(ExpoParams E) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < E.cap; s += (uint64_t)gridDim.x * blockDim.x)
    rescale_slot(E, s);
}

// Small-table engines: the ingest kernel (EXPO mode) leaves per-workgroup
// header partials in slabs [xG][cap].  One block per 64 slots: 16 groups of
// 64 threads sum every 16th workgroup's partials (coalesced 32-B rows,
// zeroing what they consumed), LDS combines the groups, then one thread per
// slot folds the sum into the series header and rescales it.
__global__ __launch_bounds__(1024) void expo_reduce_rescale_kernel(ExpoParams E) {
  __shared__ XHdr part[16][64];
  const uint32_t sl = threadIdx.x & 63u, gg = threadIdx.x >> 6;
  const uint64_t s = blockIdx.x * 64ull + sl;
  XHdr acc{0, 0, 0, 0, 0};
  if (s < E.cap) {
    for (uint32_t g = gg; g < E.xG; g += 16) {
      XHdr *p = E.xslab + (uint64_t)g * E.cap + s;
      const XHdr x = *p;
      if (x.cnt) {
        acc.cnt += x.cnt;
        acc.zero += x.zero;
        acc.sum += x.sum;
        acc.minx = x.minx > acc.minx ? x.minx : acc.minx;
        acc.max = x.max > acc.max ? x.max : acc.max;
        *p = XHdr{0, 0, 0, 0, 0};
      }
    }
  }
  part[gg][sl] = acc;
  __syncthreads();
  if (gg != 0 || s >= E.cap) return;
#pragma unroll
  for (uint32_t k = 1; k < 16; ++k) {
    const XHdr x = part[k][sl];
    acc.cnt += x.cnt;
    acc.zero += x.zero;
    acc.sum += x.sum;
    acc.minx = x.minx > acc.minx ? x.minx : acc.minx;
    acc.max = x.max > acc.max ? x.max : acc.max;
  }
  if (acc.cnt) {
    ExpoHdr &h = E.hdr[s];
    const unsigned long long minpos = ~acc.minx;  // UINT64_MAX when no positive duration
    const unsigned long long mn = acc.zero ? 0ULL : minpos;
    h.count += acc.cnt;
    h.zero += acc.zero;
    h.sum_ns += acc.sum;
    h.min_ns = mn < h.min_ns ? mn : h.min_ns;
    h.max_ns = acc.max > h.max_ns ? acc.max : h.max_ns;
    h.minpos_ns = minpos < h.minpos_ns ? minpos : h.minpos_ns;
    h.maxpos_ns = acc.max > h.maxpos_ns ? acc.max : h.maxpos_ns;
  }
  rescale_slot(E, s);
}

// Bucket counting with per-workgroup LDS privatisation: the slots' (scale,
// buffer) in LDS, and a cache of kXcEntries series (claimed first come, four
// probes from the slot's home, so a mix's frequent series hold them) whose
// max_size bucket counts are added in LDS and leave once per workgroup; spans
// of other series add to the HBM buckets directly.
constexpr uint32_t kXcBlock = 1024;
// u16 cache counts (a workgroup takes at most 2^16 - 1 spans): 64 KiB, so two
// workgroups share a CU with the slot table
constexpr uint32_t kXcLdsBudget = 64 * 1024;
constexpr uint64_t kXcMaxSpans = 65535;
__host__ __device__ inline uint32_t xc_entries(uint32_t max_size) {
  uint32_t e = 256;
  while (e > 4 && (uint64_t)e * max_size * 2 > kXcLdsBudget) e >>= 1;
  return e;
}
__global__ __launch_bounds__(kXcBlock) void expo_count_cached_kernel(ExpoParams E, uint64_t per_wg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t M = E.max_size, NE = xc_entries(M), cap = (uint32_t)E.cap;
  int2 *meta = reinterpret_cast<int2 *>(smem);                     // [cap] {scale, cur}
  uint32_t *tag = reinterpret_cast<uint32_t *>(meta + cap);         // [NE] slot + 1 (0: free)
  uint32_t *cnt = tag + NE;                                          // [NE][M] u16, packed in pairs
  for (uint32_t i = threadIdx.x; i < cap; i += kXcBlock) {
    const ExpoHdr &h = E.hdr[i];
    meta[i] = make_int2(h.scale, (int)h.cur);
  }
  for (uint32_t i = threadIdx.x; i < NE; i += kXcBlock) tag[i] = 0;
  for (uint32_t i = threadIdx.x; i < (NE * M + 1) / 2; i += kXcBlock) cnt[i] = 0;
  __syncthreads();
  const uint64_t lo = blockIdx.x * per_wg, hi = lo + per_wg < E.n ? lo + per_wg : E.n;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += kXcBlock) {
    const uint32_t slot = E.slot_of[i];
    const uint64_t st = E.start[i], en = E.end[i];
    if (slot == kNotFound) continue;
    const uint64_t d = en > st ? en - st : 0;
    if (d == 0) continue;
    const int2 m = meta[slot];
    const uint32_t at = expo_mod(expo_index(expo_value(d, E.div), m.x), M);
    uint32_t e = (((slot * 0x9E3779B1u) >> 16) & (NE / 4 - 1)) * 4, hit = kNotFound;  // home group of 4
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      uint32_t t = tag[e + k];
      if (t == 0) t = atomicCAS(&tag[e + k], 0u, slot + 1);
      if (t == 0 || t == slot + 1) {
        hit = e + k;
        break;
      }
    }
    if (hit != kNotFound) atomicAdd(&cnt[(hit * M + at) >> 1], 1u << (((hit * M + at) & 1u) * 16));
    else atomicAdd(E.buckets + ((uint64_t)m.y * E.cap + slot) * M + at, 1u);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < NE * M; i += kXcBlock) {
    const uint32_t c = (cnt[i >> 1] >> ((i & 1u) * 16)) & 0xFFFFu, t = tag[i / M];
    if (c && t) atomicAdd(E.buckets + ((uint64_t)meta[t - 1].y * E.cap + (t - 1)) * M + i % M, c);
  }
}

// pass 3: one bucket increment per positive duration
__global__ __launch_bounds__(256) void expo_count_kernel(ExpoParams E) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < E.n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t slot = E.slot_of[i];
    if (slot == kNotFound) continue;
    const uint64_t d = E.end[i] > E.start[i] ? E.end[i] - E.start[i] : 0;
    if (d == 0) continue;
    const ExpoHdr &h = E.hdr[slot];
    const int32_t idx = expo_index(expo_value(d, E.div), h.scale);
    atomicAdd(E.buckets + ((uint64_t)h.cur * E.cap + slot) * E.max_size + expo_mod(idx, E.max_size), 1u);
  }
}

// flush: non-empty series -> rows {key, count, zero, sum_ns, min_ns, max_ns,
// scale, offset, n} plus their buckets in index order; then the state resets
__global__ __launch_bounds__(256) void expo_compact_kernel(ExpoParams E, unsigned long long *out_keys,
                                                           ExpoRow *out_rows, uint32_t *out_buckets,
                                                           unsigned long long *out_n) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < E.cap; s += (uint64_t)gridDim.x * blockDim.x) {
    ExpoHdr &h = E.hdr[s];
    if (h.count == 0) continue;
    const unsigned long long r = atomicAdd(out_n, 1ULL);
    out_keys[r] = E.gkeys[s];
    ExpoRow row;
    row.count = h.count;
    row.zero = h.zero;
    row.sum_ns = h.sum_ns;
    row.min_ns = h.min_ns;
    row.max_ns = h.max_ns;
    row.scale = h.lo == kExpoEmpty ? kExpoMaxScale : h.scale;
    row.offset = h.lo == kExpoEmpty ? 0 : h.lo;
    row.n = h.lo == kExpoEmpty ? 0u : (uint32_t)(h.hi - h.lo + 1);
    row.pad = 0;
    out_rows[r] = row;
    const uint32_t M = E.max_size;
    uint32_t *src = E.buckets + ((uint64_t)h.cur * E.cap + s) * M;
    for (uint32_t j = 0; j < row.n; ++j) {
      const uint32_t at = expo_mod(h.lo + (int32_t)j, M);
      out_buckets[r * M + j] = src[at];
      src[at] = 0;
    }
    h = expo_hdr_empty();
  }
}

__global__ void expo_init_kernel(ExpoHdr *hdr, uint64_t cap) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x)
    hdr[s] = expo_hdr_empty();
}

uint32_t grid_of(uint64_t n) { return (uint32_t)std::min<uint64_t>((n + 255) / 256, 8192); }

}  // namespace

__host__ __device__ ExpoHdr expo_hdr_empty() {
  ExpoHdr h{};
  h.min_ns = ~0ULL;
  h.minpos_ns = ~0ULL;
  h.scale = kExpoMaxScale;
  h.lo = kExpoEmpty;
  h.hi = kExpoEmpty;
  return h;
}

size_t expo_count_lds_bytes(uint64_t cap, uint32_t max_size) {
  const uint32_t ne = xc_entries(max_size);
  return (size_t)cap * 8 + (size_t)ne * 4 + ((size_t)ne * max_size + 1) / 2 * 4;
}

hipError_t prepare_expo_count(size_t lds_bytes) {
  return hipFuncSetAttribute((const void *)&expo_count_cached_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds_bytes);
}

hipError_t launch_expo_ingest(const ExpoParams &E, hipStream_t s) {
  if (E.n == 0) return hipSuccess;
  if (E.xslab) {  // small table: the ingest kernel left header partials and slots
    hipLaunchKernelGGL(expo_reduce_rescale_kernel, dim3((uint32_t)((E.cap + 63) / 64)), dim3(1024), 0, s, E);
    // u16 LDS counts: at most kXcMaxSpans spans per workgroup; ~512 workgroups (two per CU)
    const uint64_t per_wg = std::min<uint64_t>(kXcMaxSpans, std::max<uint64_t>(4096, (E.n + 511) / 512));
    const uint32_t grid = (uint32_t)((E.n + per_wg - 1) / per_wg);
    hipLaunchKernelGGL(expo_count_cached_kernel, dim3(grid), dim3(kXcBlock), expo_count_lds_bytes(E.cap, E.max_size),
                       s, E, per_wg);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(expo_pass1_kernel, dim3(grid_of(E.n)), dim3(256), 0, s, E);
  hipLaunchKernelGGL(expo_rescale_kernel, dim3(grid_of(E.cap)), dim3(256), 0, s, E);
  hipLaunchKernelGGL(expo_count_kernel, dim3(grid_of(E.n)), dim3(256), 0, s, E);
  return hipGetLastError();
}

hipError_t launch_expo_compact(const ExpoParams &E, unsigned long long *out_keys, ExpoRow *out_rows,
                               uint32_t *out_buckets, unsigned long long *out_n, hipStream_t s) {
  hipLaunchKernelGGL(expo_compact_kernel, dim3(grid_of(E.cap)), dim3(256), 0, s, E, out_keys, out_rows,
                     out_buckets, out_n);
  return hipGetLastError();
}

hipError_t launch_expo_init(ExpoHdr *hdr, uint64_t cap, hipStream_t s) {
  hipLaunchKernelGGL(expo_init_kernel, dim3(grid_of(cap)), dim3(256), 0, s, hdr, cap);
  return hipGetLastError();
}

// (host) go-expohisto index of a positive value, for tests of the mapping
__global__ void expo_index_probe_kernel(const double *v, const int32_t *scale, int32_t *out, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = expo_index(v[i], scale[i]);
}

__global__ void go_log_probe_kernel(const double *v, double *out, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = go_log(v[i]);
}

hipError_t launch_expo_probe(const double *v, const int32_t *scale, int32_t *idx_out, double *log_out, uint64_t n,
                             hipStream_t s) {
  hipLaunchKernelGGL(expo_index_probe_kernel, dim3(grid_of(n)), dim3(256), 0, s, v, scale, idx_out, n);
  hipLaunchKernelGGL(go_log_probe_kernel, dim3(grid_of(n)), dim3(256), 0, s, v, log_out, n);
  return hipGetLastError();
}

}  // namespace sa
