// spanagg_union.hip -- the sorted union of series ids on the device (gfx950),
// for the engine group's flush (spanagg_group.cpp sa_group_flush): the
// members' non-zero series ids, gathered onto one device (or onto every
// member by ncclAllGather), become the sorted dense index every member
// densifies its counters against.  Replaces the host
// std::sort / unique of round 3.
//
// Bucket sort by the ids' top bits, then a bitonic sort of each bucket in LDS:
//   1. union_hist_kernel: ids per bucket (LDS histogram per workgroup, one
//      global add per touched bucket), and the largest bucket;
//   2. union_scan_kernel (one workgroup): bucket offsets;
//   3. union_scatter_kernel: each workgroup reserves one run per touched
//      bucket with one global atomic, then places its ids in it (LDS cursors);
//   4. union_sort_kernel: one workgroup per bucket sorts it in LDS (bitonic,
//      padded with ~0 to a power of two), drops repeats (the padding id 0
//      never reaches a bucket: steps 1 and 3 skip it),
//      and writes the bucket's distinct ids at its offset (bucket counts);
//   5. union_scan_kernel again over the distinct counts, then
//      union_compact_kernel packs the buckets' runs into the output.
// Series ids are xxh64 outputs (uniform), and the bucket count is chosen so a
// bucket holds ~1,024 ids on average; a bucket above the LDS sort's 8,192
// ids (never seen on hash ids; a member contributes each id at most once) is
// sorted by the same network in a global scratch buffer instead.
#include <algorithm>
#include <vector>

#include "sa_device.h"

namespace sa {
namespace {

constexpr uint32_t kUnionBlock = 1024;
constexpr uint32_t kUnionLdsKeys = 8192;  // ids one workgroup sorts in LDS (64 KiB)
constexpr uint32_t kUnionMaxBuckets = 1u << 14;

__device__ __forceinline__ uint32_t ubucket(uint64_t k, uint32_t bits) {
  return bits ? (uint32_t)(k >> (64 - bits)) : 0u;
}

__global__ __launch_bounds__(kUnionBlock) void union_hist_kernel(const uint64_t *in, uint64_t n, uint32_t bits,
                                                                 uint32_t *hist) {
  __shared__ uint32_t h[kUnionMaxBuckets];
  const uint32_t nb = 1u << bits;
  for (uint32_t b = threadIdx.x; b < nb; b += kUnionBlock) h[b] = 0;
  __syncthreads();
  // (the padding id 0 is neither counted nor placed: an RCCL group pads every
  // member's list to the longest, and those zeros would all land in bucket 0)
  for (uint64_t i = blockIdx.x * (uint64_t)kUnionBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kUnionBlock) {
    const uint64_t k = in[i];
    if (k != 0) atomicAdd(&h[ubucket(k, bits)], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += kUnionBlock)
    if (h[b]) atomicAdd(&hist[b], h[b]);
}

// Exclusive scan of cnt[0..nb) into off[] (and cur[] when given); out[0] =
// the total, out[1] = the largest entry.  One workgroup: each thread scans a
// contiguous chunk, the chunk totals are scanned in LDS.
__global__ __launch_bounds__(kUnionBlock) void union_scan_kernel(const uint32_t *cnt, uint32_t nb, uint32_t *off,
                                                                 uint32_t *cur, uint32_t *out) {
  __shared__ uint32_t part[kUnionBlock], mx[kUnionBlock];
  const uint32_t t = threadIdx.x, per = (nb + kUnionBlock - 1) / kUnionBlock, b0 = t * per;
  uint32_t sum = 0, m = 0;
  for (uint32_t b = b0; b < b0 + per && b < nb; ++b) {
    sum += cnt[b];
    m = max(m, cnt[b]);
  }
  part[t] = sum;
  mx[t] = m;
  __syncthreads();
  for (uint32_t o = 1; o < kUnionBlock; o <<= 1) {
    const uint32_t x = t >= o ? part[t - o] : 0u;
    const uint32_t y = t >= o ? mx[t - o] : 0u;
    __syncthreads();
    part[t] += x;
    mx[t] = max(mx[t], y);
    __syncthreads();
  }
  uint32_t acc = part[t] - sum;
  for (uint32_t b = b0; b < b0 + per && b < nb; ++b) {
    off[b] = acc;
    if (cur) cur[b] = acc;
    acc += cnt[b];
  }
  if (t == kUnionBlock - 1) {
    out[0] = part[t];
    out[1] = mx[t];
  }
}

// Each workgroup takes a tile of 8 ids per thread, reserves one run per
// touched bucket (a global atomic each), then places its ids with LDS cursors.
constexpr uint32_t kScatterTile = kUnionBlock * 8;
__global__ __launch_bounds__(kUnionBlock) void union_scatter_kernel(const uint64_t *in, uint64_t n, uint32_t bits,
                                                                    uint32_t *cur, uint64_t *bucketed) {
  __shared__ uint32_t h[kUnionMaxBuckets];
  const uint32_t nb = 1u << bits;
  for (uint64_t t0 = (uint64_t)blockIdx.x * kScatterTile; t0 < n; t0 += (uint64_t)gridDim.x * kScatterTile) {
    for (uint32_t b = threadIdx.x; b < nb; b += kUnionBlock) h[b] = 0;
    __syncthreads();
    uint64_t k[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t i = t0 + threadIdx.x + (uint64_t)u * kUnionBlock;
      k[u] = i < n ? in[i] : 0;
      if (k[u] != 0) atomicAdd(&h[ubucket(k[u], bits)], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += kUnionBlock)
      if (h[b]) h[b] = atomicAdd(&cur[b], h[b]);  // this tile's run of bucket b
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (k[u] != 0) bucketed[atomicAdd(&h[ubucket(k[u], bits)], 1u)] = k[u];  // (0 past n)
    __syncthreads();
  }
}

// Bitonic sort of a[0..p) (p a power of two) by one workgroup.
template <typename T>
__device__ void bitonic(T *a, uint32_t p) {
  for (uint32_t k = 2; k <= p; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < p; i += kUnionBlock) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const uint64_t x = a[i], y = a[l];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[l] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

// Keeps a[i] (i < size) when it is not the padding id 0 and differs from
// a[i - 1]: writes the kept ids, in order, to dst; returns their count.
__device__ uint32_t keep_distinct(const uint64_t *a, uint32_t size, uint64_t *dst, uint32_t *wtot) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  constexpr uint32_t kWaves = kUnionBlock / 64;
  uint32_t base = 0;
  for (uint32_t i0 = 0; i0 < size; i0 += kUnionBlock) {
    const uint32_t i = i0 + threadIdx.x;
    const uint64_t x = i < size ? a[i] : 0;
    const bool keep = i < size && x != 0 && (i == 0 || a[i - 1] != x);
    const uint64_t m = __ballot(keep);
    if (lane == 0) wtot[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t w = 0; w < kWaves; ++w) {
      before += w < wave ? wtot[w] : 0u;
      all += wtot[w];
    }
    if (keep) dst[base + before + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = x;
    base += all;
    __syncthreads();
  }
  return base;
}

__global__ __launch_bounds__(kUnionBlock) void union_sort_kernel(const uint64_t *bucketed, const uint32_t *off,
                                                                 const uint32_t *cnt, uint64_t *distinct,
                                                                 uint32_t *dcnt, uint64_t *scratch) {
  __shared__ uint64_t a[kUnionLdsKeys];
  __shared__ uint32_t wtot[kUnionBlock / 64];
  const uint32_t b = blockIdx.x, size = cnt[b], o = off[b];
  if (size == 0) {
    if (threadIdx.x == 0) dcnt[b] = 0;
    return;
  }
  uint32_t p = 1;
  while (p < size) p <<= 1;
  // ~0 pads to a power of two and sorts last (the first `size` sorted ids are
  // the bucket's, whatever their values)
  uint64_t *buf = p <= kUnionLdsKeys ? a : scratch;
  for (uint32_t i = threadIdx.x; i < p; i += kUnionBlock) buf[i] = i < size ? bucketed[o + i] : ~0ULL;
  __syncthreads();
  bitonic(buf, p);
  const uint32_t kept = keep_distinct(buf, size, distinct + o, wtot);
  if (threadIdx.x == 0) dcnt[b] = kept;
}

__global__ __launch_bounds__(256) void union_compact_kernel(const uint64_t *distinct, const uint32_t *off,
                                                            const uint32_t *dcnt, const uint32_t *doff,
                                                            uint64_t *out) {
  const uint32_t b = blockIdx.x, c = dcnt[b];
  for (uint32_t i = threadIdx.x; i < c; i += 256) out[doff[b] + i] = distinct[off[b] + i];
}

}  // namespace

size_t key_union_scratch_bytes(uint64_t n) {
  // bucketed ids + distinct ids (n each), 4 u32 arrays of buckets, 4 counters
  return n * 16 + (size_t)kUnionMaxBuckets * 16 + 64;
}

hipError_t key_union(const uint64_t *in, uint64_t n, uint64_t *out, uint32_t *d_total, void *scratch,
                     uint64_t **big_scratch, size_t *big_bytes, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(d_total, 0, 4, s);
  if (n > 0xFFFFFFFFull) return hipErrorInvalidValue;  // u32 offsets
  uint32_t bits = 0;
  while (bits < 14 && ((n >> bits) > 1024)) ++bits;
  const uint32_t nb = 1u << bits;
  auto *bucketed = static_cast<uint64_t *>(scratch);
  uint64_t *distinct = bucketed + n;
  auto *cnt = reinterpret_cast<uint32_t *>(distinct + n);
  uint32_t *off = cnt + kUnionMaxBuckets, *cur = off + kUnionMaxBuckets, *doff = cur + kUnionMaxBuckets;
  uint32_t *tot = doff + kUnionMaxBuckets;  // [0] ids, [1] largest bucket, [2] distinct, [3] largest count
  if (hipError_t e = hipMemsetAsync(cnt, 0, (size_t)nb * 4, s); e != hipSuccess) return e;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(512, (n + kScatterTile - 1) / kScatterTile);
  hipLaunchKernelGGL(union_hist_kernel, dim3(grid), dim3(kUnionBlock), 0, s, in, n, bits, cnt);
  hipLaunchKernelGGL(union_scan_kernel, dim3(1), dim3(kUnionBlock), 0, s, cnt, nb, off, cur, tot);
  hipLaunchKernelGGL(union_scatter_kernel, dim3(grid), dim3(kUnionBlock), 0, s, in, n, bits, cur, bucketed);
  // the largest bucket decides whether the LDS sort holds every bucket
  uint32_t host_tot[2] = {0, 0};
  if (hipError_t e = hipMemcpyAsync(host_tot, tot, 8, hipMemcpyDeviceToHost, s); e != hipSuccess) return e;
  if (hipError_t e = hipStreamSynchronize(s); e != hipSuccess) return e;
  uint64_t *big = nullptr;
  if (host_tot[1] > kUnionLdsKeys) {  // global scratch for the oversized buckets' network
    size_t p = 1;
    while (p < host_tot[1]) p <<= 1;
    if (*big_bytes < p * 8) {
      if (*big_scratch) (void)hipFree(*big_scratch);
      *big_scratch = nullptr;
      *big_bytes = 0;
      if (hipError_t e = hipMalloc(reinterpret_cast<void **>(big_scratch), p * 8); e != hipSuccess) return e;
      *big_bytes = p * 8;
    }
    big = *big_scratch;
    // one oversized bucket at a time shares the scratch: launch them one by one
  }
  if (!big) {
    hipLaunchKernelGGL(union_sort_kernel, dim3(nb), dim3(kUnionBlock), 0, s, bucketed, off, cnt, distinct, cur,
                       nullptr);
  } else {
    std::vector<uint32_t> hc(nb);
    if (hipError_t e = hipMemcpyAsync(hc.data(), cnt, (size_t)nb * 4, hipMemcpyDeviceToHost, s); e != hipSuccess)
      return e;
    if (hipError_t e = hipStreamSynchronize(s); e != hipSuccess) return e;
    for (uint32_t b = 0; b < nb; ++b)  // bucket b alone (grid offset through the pointers)
      hipLaunchKernelGGL(union_sort_kernel, dim3(1), dim3(kUnionBlock), 0, s, bucketed, off + b, cnt + b, distinct,
                         cur + b, big);
  }
  // cur[] now holds the distinct counts per bucket
  hipLaunchKernelGGL(union_scan_kernel, dim3(1), dim3(kUnionBlock), 0, s, cur, nb, doff, nullptr, tot + 2);
  hipLaunchKernelGGL(union_compact_kernel, dim3(nb), dim3(256), 0, s, distinct, off, cur, doff, out);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  return hipMemcpyAsync(d_total, tot + 2, 4, hipMemcpyDeviceToDevice, s);
}

}  // namespace sa
