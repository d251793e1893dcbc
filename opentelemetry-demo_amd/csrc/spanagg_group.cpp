// spanagg_group.cpp -- engine groups (include/spanagg.h, sa_group_*): the
// spanmetrics connector's ConsumeTraces / exportMetrics over several GPUs of
// one node behind one handle.  Spans shard by trace id,
// so each member aggregates whole traces; at flush and window read the group
// merges the members' partials:
//   - key union: the members' non-zero series ids (sa_export_keys), gathered
//     with ncclAllGather (or device copies) and made a sorted dense index;
//   - RED rows densified against it (sa_gather_dense), summed (ncclAllReduce
//     sum u64, or copies onto member 0's device + a reduce kernel);
//   - HLL registers max-merged (ncclAllReduce max u8), count-min cells summed.
// Every merge is integer sums and maxima, so both transports give the same
// bits as one engine fed the whole stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <map>
#include <memory>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "sa_group_hooks.h"
#include "sa_internal.h"
#include "sa_results.h"
#include "spanagg.h"

namespace {

__global__ void sum_slices_u64(unsigned long long *dst, const unsigned long long *src, uint32_t n, uint64_t len) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < len; i += (uint64_t)gridDim.x * blockDim.x) {
    unsigned long long acc = 0;
    for (uint32_t k = 0; k < n; ++k) acc += src[k * len + i];
    dst[i] = acc;
  }
}

__global__ void max_slices_u8(uint8_t *dst, const uint8_t *src, uint32_t n, uint64_t len) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < len; i += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t m = 0;
    for (uint32_t k = 0; k < n; ++k) m = src[k * len + i] > m ? src[k * len + i] : m;
    dst[i] = m;
  }
}

uint32_t grid_for(uint64_t len) { return (uint32_t)std::min<uint64_t>((len + 255) / 256, 4096); }

constexpr uint32_t kMaxMembers = 64;

// Sum of members' dense rows that live on one device: dst[i] = sum_k src[k][i]
// straight from each member's buffer (no stacking copy).
struct SrcPtrs {
  const unsigned long long *p[kMaxMembers];
};
__global__ void sum_ptrs_u64(unsigned long long *dst, SrcPtrs src, uint32_t n, uint64_t len) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < len; i += (uint64_t)gridDim.x * blockDim.x) {
    unsigned long long acc = 0;
    for (uint32_t k = 0; k < n; ++k) acc += src.p[k][i];
    dst[i] = acc;
  }
}

// The merged dense rows [nu][nbk + 1] (bucket counts, ns sum) -> the result's
// columns on the device: counts [nu][nbk], calls = sum of counts (A8),
// sum_ns, and sum = sum_ns / div (IEEE division, as the host's).
// One 32-lane half wave per row: lane b moves bucket b (b, b + 32, ...), the
// calls are a half-wave sum (coalesced rows in and out).
__global__ void finalize_rows_kernel(const unsigned long long *rows, uint64_t nu, uint32_t nbk,
                                     unsigned long long *counts, unsigned long long *calls,
                                     unsigned long long *sum_ns, double *sum, double div) {
  const uint32_t b0 = threadIdx.x & 31u;
  for (uint64_t r = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 5; r < nu;
       r += ((uint64_t)gridDim.x * blockDim.x) >> 5) {
    const unsigned long long *row = rows + r * (nbk + 1);
    unsigned long long c = 0;
    for (uint32_t b = b0; b < nbk; b += 32) {
      const unsigned long long v = row[b];
      counts[r * nbk + b] = v;
      c += v;
    }
#pragma unroll
    for (int o = 16; o > 0; o >>= 1)  // (xor offsets < 32 stay inside the half wave)
      c += (unsigned long long)(uint32_t)__shfl_xor((int)(uint32_t)c, o, 64) |
           ((unsigned long long)(uint32_t)__shfl_xor((int)(uint32_t)(c >> 32), o, 64) << 32);
    if (b0 == 0) {
      calls[r] = c;
      sum_ns[r] = row[nbk];
      sum[r] = (double)row[nbk] / div;
    }
  }
}

// ---- trace-id sharding (engine = trace_w1 % n) ------------------------------
// trace_w1 % n from 32-bit remainders: w1 = hi * 2^32 + lo, so
// w1 % n = ((hi % n) * (2^32 % n) + lo % n) % n (< n^2 <= 4096 before the
// last remainder); no 64-bit division per span.
__host__ __device__ inline uint32_t shard_of(uint64_t w1, uint32_t n, uint32_t r32) {
  return (((uint32_t)(w1 >> 32) % n) * r32 + (uint32_t)w1 % n) % n;
}

// ---- device partition (sa_group_ingest_device) -------------------------------
// Workgroup b of the partition owns the contiguous span range [b * per,
// (b + 1) * per) and walks it in chunks of kPartChunk spans.
constexpr uint32_t kShardBlock = 256;
constexpr uint32_t kPartChunk = 1024;  // spans staged in LDS per round (44 KiB)

// Spans per shard and workgroup: per-wave LDS counters, written to
// blk[shard][workgroup]; the totals (one global add per shard and workgroup)
// are what the host reads to size the shards.
__global__ __launch_bounds__(kShardBlock) void shard_count_kernel(const uint64_t *w1, uint64_t n, uint64_t per,
                                                                   uint32_t nm, uint32_t r32,
                                                                   unsigned long long *cnt, uint32_t *blk) {
  __shared__ uint32_t c[kShardBlock / 64][kMaxMembers];
  const uint32_t wave = threadIdx.x >> 6;
  for (uint32_t i = threadIdx.x; i < (kShardBlock / 64) * kMaxMembers; i += kShardBlock) (&c[0][0])[i] = 0;
  __syncthreads();
  const uint64_t lo = blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  // two spans per lane per step (16-B loads: lo and per are even and the
  // columns 16-B aligned; a last odd span is read on its own)
  for (uint64_t i = lo + 2 * threadIdx.x; i < hi; i += 2 * kShardBlock) {
    if (i + 1 < hi) {
      const ulonglong2 v = *reinterpret_cast<const ulonglong2 *>(w1 + i);
      atomicAdd(&c[wave][shard_of(v.x, nm, r32)], 1u);
      atomicAdd(&c[wave][shard_of(v.y, nm, r32)], 1u);
    } else {
      atomicAdd(&c[wave][shard_of(w1[i], nm, r32)], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < nm) {
    uint32_t t = 0;
    for (uint32_t w = 0; w < kShardBlock / 64; ++w) t += c[w][threadIdx.x];
    blk[(uint64_t)threadIdx.x * gridDim.x + blockIdx.x] = t;
    if (t) atomicAdd(&cnt[threadIdx.x], (unsigned long long)t);
  }
}

// Exclusive scan of one shard's counts over the workgroups (one block per
// shard, grid <= 4096: four workgroups per thread): blk[j][b] becomes
// workgroup b's first position in shard j.
__global__ __launch_bounds__(1024) void shard_scan_kernel(uint32_t *blk, uint32_t grid) {
  __shared__ uint32_t part[1024];
  uint32_t *row = blk + (uint64_t)blockIdx.x * grid;
  const uint32_t t = threadIdx.x, b0 = 4 * t;
  uint32_t v[4], sum = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = b0 + k < grid ? row[b0 + k] : 0u;
    sum += v[k];
  }
  part[t] = sum;
  __syncthreads();
  for (uint32_t o = 1; o < 1024; o <<= 1) {  // inclusive scan of the thread sums
    const uint32_t x = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t acc = part[t] - sum;  // exclusive
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (b0 + k < grid) row[b0 + k] = acc;
    acc += v[k];
  }
}

// One member's packed shard (SoA v1 columns) in the partition staging buffer.
struct ShardCols {
  uint64_t *k, *s, *e, *a, *b;
  uint32_t *m;
};
struct ShardArgs {  // by value (kernel argument segment): nm <= kMaxMembers
  ShardCols c[kMaxMembers];
};

// Scatter, LDS-staged: per chunk of 1,024 spans, every span takes a position
// in its shard's run of the chunk (a ballot per shard present in the wave,
// one LDS add per shard and wave), the chunk is written into LDS in shard
// order (SoA), and then each column leaves as the shards' contiguous runs
// (~128 spans = 1 KiB per u64 column at 8 members), so the stores coalesce.
// (Round 3 wrote every wave's 64 spans straight to their shards: runs of ~8
// spans, 2.2 TB/s.)  Order inside a shard is not kept: every aggregate is
// order-independent (integer sums and maxima).
__global__ __launch_bounds__(kShardBlock) void shard_scatter_kernel(sa_span_batch in, uint64_t per, uint32_t nm,
                                                                     uint32_t r32, ShardArgs out,
                                                                     const uint32_t *first) {
  __shared__ uint64_t sk[kPartChunk], ss[kPartChunk], se[kPartChunk], sa_[kPartChunk], sb[kPartChunk];
  __shared__ uint32_t sm[kPartChunk];
  __shared__ uint8_t sid[kPartChunk];
  __shared__ uint32_t ccnt[kMaxMembers], coff[kMaxMembers], cur[kMaxMembers];
  __shared__ ShardCols cols[kMaxMembers];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  if (tid < nm) {
    cur[tid] = first[(uint64_t)tid * gridDim.x + blockIdx.x];
    ccnt[tid] = 0;
    cols[tid] = out.c[tid];
  }
  __syncthreads();
  const uint64_t lo = blockIdx.x * per, hi = lo + per < in.n ? lo + per : in.n;
  constexpr uint32_t kPer = kPartChunk / kShardBlock;  // spans per thread per chunk
  for (uint64_t c0 = lo; c0 < hi; c0 += kPartChunk) {
    // 1. loads (spans c0 + 2 tid + {0, 1} + 512 h: 16-B loads of two spans per
    //    u64 column, 8 B of meta) and positions within the shards' runs
    uint64_t k[kPer], s[kPer], e[kPer], a[kPer], b[kPer];
    uint32_t m[kPer], sh[kPer], rk[kPer];
#pragma unroll
    for (uint32_t h = 0; h < kPer / 2; ++h) {
      const uint64_t i = c0 + 2 * tid + h * 2 * kShardBlock;
      const uint32_t u = 2 * h;
      if (i + 1 < hi) {
        const ulonglong2 kk = *reinterpret_cast<const ulonglong2 *>(in.key_hash + i);
        const ulonglong2 ss = *reinterpret_cast<const ulonglong2 *>(in.start_ns + i);
        const ulonglong2 ee = *reinterpret_cast<const ulonglong2 *>(in.end_ns + i);
        const ulonglong2 aa = *reinterpret_cast<const ulonglong2 *>(in.trace_w0 + i);
        const ulonglong2 bb = *reinterpret_cast<const ulonglong2 *>(in.trace_w1 + i);
        const uint2 mm = *reinterpret_cast<const uint2 *>(in.meta + i);
        k[u] = kk.x, k[u + 1] = kk.y, s[u] = ss.x, s[u + 1] = ss.y, e[u] = ee.x, e[u + 1] = ee.y;
        a[u] = aa.x, a[u + 1] = aa.y, b[u] = bb.x, b[u + 1] = bb.y, m[u] = mm.x, m[u + 1] = mm.y;
      } else {  // the range's last odd span, or nothing
        const bool ok = i < hi;
        k[u] = ok ? in.key_hash[i] : 0, s[u] = ok ? in.start_ns[i] : 0, e[u] = ok ? in.end_ns[i] : 0;
        a[u] = ok ? in.trace_w0[i] : 0, b[u] = ok ? in.trace_w1[i] : 0, m[u] = ok ? in.meta[i] : 0;
        k[u + 1] = s[u + 1] = e[u + 1] = a[u + 1] = b[u + 1] = 0, m[u + 1] = 0;
      }
      sh[u] = i < hi ? shard_of(b[u], nm, r32) : 0xFFFFFFFFu;
      sh[u + 1] = i + 1 < hi ? shard_of(b[u + 1], nm, r32) : 0xFFFFFFFFu;
    }
#pragma unroll
    for (uint32_t u = 0; u < kPer; ++u) {
      uint64_t pending = __ballot(sh[u] != 0xFFFFFFFFu);
      rk[u] = 0;
      while (pending) {  // wave-uniform: one round per shard present among the wave's spans
        const uint32_t j = (uint32_t)__builtin_amdgcn_readlane((int)sh[u], __builtin_ctzll(pending));
        const uint64_t mj = __ballot(sh[u] == j);
        pending &= ~mj;
        const int leader = __builtin_ctzll(mj);
        uint32_t base = 0;
        if ((int)lane == leader) base = atomicAdd(&ccnt[j], (uint32_t)__popcll(mj));
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
        if (sh[u] == j)
          rk[u] = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(mj >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mj, 0u));
      }
    }
    __syncthreads();
    if (tid < 64) {  // the shards' runs within the chunk (nm <= 64: one wave scan)
      const uint32_t v = tid < nm ? ccnt[tid] : 0u;
      uint32_t x = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if ((int)lane >= o) x += y;
      }
      if (tid < nm) coff[tid] = x - v;
    }
    __syncthreads();
    // 2. the chunk into LDS in shard order
#pragma unroll
    for (uint32_t u = 0; u < kPer; ++u) {
      if (sh[u] == 0xFFFFFFFFu) continue;
      const uint32_t p = coff[sh[u]] + rk[u];
      sk[p] = k[u];
      ss[p] = s[u];
      se[p] = e[u];
      sa_[p] = a[u];
      sb[p] = b[u];
      sm[p] = m[u];
      sid[p] = (uint8_t)sh[u];
    }
    __syncthreads();
    // 3. out as runs: position p of shard j goes to cur[j] + p - coff[j]
    const uint32_t nchunk = (uint32_t)(hi - c0 < kPartChunk ? hi - c0 : kPartChunk);
#pragma unroll
    for (uint32_t u = 0; u < kPer; ++u) {
      const uint32_t p = tid + u * kShardBlock;
      if (p >= nchunk) continue;
      const uint32_t j = sid[p];
      const uint64_t g = (uint64_t)cur[j] + p - coff[j];
      const ShardCols &c = cols[j];
      c.k[g] = sk[p];
      c.s[g] = ss[p];
      c.e[g] = se[p];
      c.a[g] = sa_[p];
      c.b[g] = sb[p];
      c.m[g] = sm[p];
    }
    __syncthreads();
    if (tid < nm) {
      cur[tid] += ccnt[tid];
      ccnt[tid] = 0;
    }
    __syncthreads();
  }
}

// Device buffer on one member's device, grown on demand.
struct Buf {
  void *p = nullptr;
  size_t bytes = 0;
};

}  // namespace

struct sa_group {
  sa_config cfg{};
  std::vector<double> bounds;
  std::vector<sa_engine *> eng;
  std::vector<int> dev;
  std::vector<hipStream_t> st;  // one merge stream per member, on its device
  bool rccl = false;
  std::vector<ncclComm_t> comm;
  std::vector<Buf> keys, gath, uni, rows, hll, cms;
  std::vector<Buf> srt, ucnt;  // device key union (sa::key_union): its scratch and the distinct count
  std::vector<uint64_t *> big;  // key_union's scratch for oversized buckets (per member)
  std::vector<size_t> big_bytes;
  Buf fin;                               // member 0's device: the result's columns (finalize_rows_kernel)
  Buf stack;  // member 0's device: every member's slice for the copy-path reduce
  // sa_group_ingest_device: two staging sets (a call waits only for the
  // members' use of the set two calls back).  part[k][i]: set k's packed
  // shards on member i's device when that device partitions (the source),
  // peer[k][i]: member i's shard copied to its own device; ev_scat[k][i]
  // (device i) marks the partition of set k, ev_done[k][i] member i's ingest
  // of it.
  int pset = 0;
  Buf part[2][kMaxMembers], peer[2][kMaxMembers];
  hipEvent_t ev_scat[2][kMaxMembers] = {}, ev_done[2][kMaxMembers] = {};
  bool done_used[2][kMaxMembers] = {};
  // [2][n] shard counters + per-workgroup cursors, per staging set and source
  // device: a call's count/scan may overlap the scatter of the call before it
  // (when the caller alternates streams), never the one of the same set
  std::vector<Buf> pcnt;
  unsigned long long *hcnt = nullptr;    // pinned host copy of the counts
  uint64_t *hflush = nullptr;            // pinned [3][kMaxMembers]: flush key counts, drop counters, resident keys
  // page-locked blocks the flush results' columns are copied into (sa_results.h)
  std::shared_ptr<PinPool> pins = std::make_shared<PinPool>();
  // sa_group_ingest: per-member packed host shards, reused across calls
  std::vector<std::vector<uint64_t>> hcol;
  std::vector<std::vector<uint32_t>> hmeta;
  std::vector<uint64_t> dropped_seen;
  uint32_t nbk = 0;
  size_t hll_bytes = 0, cms_elems = 0;
  std::string err;
};

namespace {

int gfail(sa_group *g, int code, const std::string &msg) {
  if (g) g->err = msg;
  return code;
}

#define SG_HIP(g, call)                                                                  \
  do {                                                                                   \
    hipError_t _s = (call);                                                              \
    if (_s != hipSuccess)                                                                \
      return gfail((g), SA_EDEVICE, std::string(#call) + ": " + hipGetErrorString(_s)); \
  } while (0)

#define SG_NCCL(g, call)                                                                   \
  do {                                                                                     \
    ncclResult_t _r = (call);                                                              \
    if (_r != ncclSuccess)                                                                 \
      return gfail((g), SA_EDEVICE, std::string(#call) + ": " + ncclGetErrorString(_r)); \
  } while (0)

int ensure(sa_group *g, int dev, Buf &b, size_t bytes) {
  if (b.bytes >= bytes) return SA_OK;
  SG_HIP(g, hipSetDevice(dev));
  if (b.p) SG_HIP(g, hipFree(b.p));
  b.p = nullptr;
  b.bytes = 0;
  if (hipMalloc(&b.p, bytes) != hipSuccess) return gfail(g, SA_ENOMEM, "group buffer hipMalloc failed");
  b.bytes = bytes;
  return SA_OK;
}

int member_error(sa_group *g, uint32_t i, int rc, const char *what) {
  return gfail(g, rc, std::string(what) + " (member " + std::to_string(i) + "): " + sa_last_error(g->eng[i]));
}

// Copy-path reduction: every member's `len` elements of `bufs` onto member 0's
// device (stacked), then one kernel writes the sum (u64) or max (u8) into
// bufs[0].  Member streams are drained first; the result is ordered on st[0].
int copy_reduce(sa_group *g, std::vector<Buf> &bufs, uint64_t len, bool max_u8) {
  const uint32_t n = (uint32_t)g->eng.size();
  const size_t esz = max_u8 ? 1 : 8, bytes = len * esz;
  if (n == 1 || len == 0) return SA_OK;
  if (int rc = ensure(g, g->dev[0], g->stack, bytes * n)) return rc;
  for (uint32_t i = 0; i < n; ++i) {
    SG_HIP(g, hipSetDevice(g->dev[i]));
    SG_HIP(g, hipStreamSynchronize(g->st[i]));
  }
  SG_HIP(g, hipSetDevice(g->dev[0]));
  char *dst = static_cast<char *>(g->stack.p);
  for (uint32_t i = 0; i < n; ++i) {
    if (g->dev[i] == g->dev[0])
      SG_HIP(g, hipMemcpyAsync(dst + i * bytes, bufs[i].p, bytes, hipMemcpyDeviceToDevice, g->st[0]));
    else
      SG_HIP(g, hipMemcpyPeerAsync(dst + i * bytes, g->dev[0], bufs[i].p, g->dev[i], bytes, g->st[0]));
  }
  if (max_u8)
    hipLaunchKernelGGL(max_slices_u8, dim3(grid_for(len)), dim3(256), 0, g->st[0], static_cast<uint8_t *>(bufs[0].p),
                       static_cast<const uint8_t *>(g->stack.p), n, len);
  else
    hipLaunchKernelGGL(sum_slices_u64, dim3(grid_for(len)), dim3(256), 0, g->st[0],
                       static_cast<unsigned long long *>(bufs[0].p),
                       static_cast<const unsigned long long *>(g->stack.p), n, len);
  SG_HIP(g, hipGetLastError());
  return SA_OK;
}

// The sorted union of `n_in` series ids in `in` (member i's device, stream
// st[i]; ids may repeat, 0 = padding) into uni[i]: sa::key_union (bucket
// sort by the top bits, bitonic per bucket in LDS, repeats and 0 dropped).
// Its distinct count lands in ucnt[i] (device u32), read by union_count.
int device_union(sa_group *g, uint32_t i, const uint64_t *in, uint64_t n_in) {
  const int dev = g->dev[i];
  if (int rc = ensure(g, dev, g->srt[i], sa::key_union_scratch_bytes(n_in))) return rc;
  if (int rc = ensure(g, dev, g->uni[i], std::max<uint64_t>(1, n_in) * 8)) return rc;
  if (int rc = ensure(g, dev, g->ucnt[i], 64)) return rc;
  SG_HIP(g, hipSetDevice(dev));
  SG_HIP(g, sa::key_union(in, n_in, static_cast<uint64_t *>(g->uni[i].p), static_cast<uint32_t *>(g->ucnt[i].p),
                          g->srt[i].p, &g->big[i], &g->big_bytes[i], g->st[i]));
  return SA_OK;
}

// Reads member i's union size (waits for its stream).
int union_count(sa_group *g, uint32_t i, uint64_t *nu) {
  uint32_t h = 0;
  SG_HIP(g, hipSetDevice(g->dev[i]));
  SG_HIP(g, hipMemcpyAsync(&h, g->ucnt[i].p, 4, hipMemcpyDeviceToHost, g->st[i]));
  SG_HIP(g, hipStreamSynchronize(g->st[i]));
  *nu = h;
  return SA_OK;
}

// One series' exponential histogram while members' deltas are folded in.
struct ExpoAcc {
  uint64_t count = 0, zero = 0, sum_ns = 0;
  double min = 0, max = 0;
  int32_t scale = 20, offset = 0;  // go-expohisto's initial scale
  std::vector<uint64_t> c;         // positive buckets offset .. offset + size - 1
};

inline int64_t shr_floor(int64_t v, int k) { return v >= 0 ? v >> k : -((-v - 1) >> k) - 1; }

// Folds one member's histogram into a: go-expohisto's state depends only on
// the values, and index(v) at scale s is index(v) at scale s + k shifted
// right by k, so both go to the smaller scale, the index ranges unite and
// the least further downscale that fits max_size applies (changeScale) --
// exactly the histogram one engine fed both members' spans would hold.
void expo_fold(ExpoAcc &a, const sa_exp_result &r, uint64_t j, uint32_t max_size) {
  if (r.count[j] == 0) return;
  if (a.count == 0) {
    a.min = r.min[j];
    a.max = r.max[j];
  } else {
    a.min = std::min(a.min, r.min[j]);
    a.max = std::max(a.max, r.max[j]);
  }
  a.count += r.count[j];
  a.zero += r.zero_count[j];
  a.sum_ns += r.sum_ns[j];
  const uint32_t nb = r.n_buckets[j];
  const uint64_t *cnt = r.bucket_counts + j * r.max_size;
  if (nb == 0) return;
  if (a.c.empty()) {
    a.scale = r.scale[j];
    a.offset = r.offset[j];
    a.c.assign(cnt, cnt + nb);
    return;
  }
  int s = std::min(a.scale, r.scale[j]);
  const int ka = a.scale - s, kd = r.scale[j] - s;
  int64_t lo = std::min(shr_floor(a.offset, ka), shr_floor(r.offset[j], kd));
  int64_t hi = std::max(shr_floor((int64_t)a.offset + (int64_t)a.c.size() - 1, ka),
                        shr_floor((int64_t)r.offset[j] + nb - 1, kd));
  int c = 0;
  while (hi - lo >= (int64_t)max_size) lo = shr_floor(lo, 1), hi = shr_floor(hi, 1), ++c;
  std::vector<uint64_t> out((size_t)(hi - lo + 1), 0);
  for (size_t i = 0; i < a.c.size(); ++i) out[(size_t)(shr_floor((int64_t)a.offset + (int64_t)i, ka + c) - lo)] += a.c[i];
  for (uint32_t i = 0; i < nb; ++i) out[(size_t)(shr_floor((int64_t)r.offset[j] + i, kd + c) - lo)] += cnt[i];
  a.scale = s - c;
  a.offset = (int32_t)lo;
  a.c.swap(out);
}

}  // namespace

extern "C" {

int sa_group_create(const sa_config *cfg, const int32_t *devices, uint32_t n, sa_group **out) {
  if (!out) return SA_EINVAL;
  *out = nullptr;
  if (!cfg || !devices || n == 0 || n > kMaxMembers) return SA_EINVAL;
  auto *g = new sa_group();
  g->cfg = *cfg;
  g->bounds.assign(cfg->bounds, cfg->bounds + cfg->n_bounds);
  g->cfg.bounds = g->bounds.data();
  g->nbk = cfg->n_bounds + 1;
  g->hll_bytes = (size_t)cfg->n_services << cfg->hll_p;
  g->cms_elems = (size_t)cfg->cms_d * cfg->cms_w;
  for (uint32_t i = 0; i < n; ++i) {
    sa_config c = g->cfg;
    c.device = devices[i];
    sa_engine *e = nullptr;
    const int rc = sa_create(&c, &e);
    if (rc != SA_OK || !e) {
      sa_group_destroy(g);
      return rc ? rc : SA_EDEVICE;
    }
    g->eng.push_back(e);
    g->dev.push_back(devices[i]);
    hipStream_t s = nullptr;
    if (hipSetDevice(devices[i]) != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
      sa_group_destroy(g);
      return SA_EDEVICE;
    }
    g->st.push_back(s);
  }
  g->keys.resize(n);
  g->srt.resize(n);
  g->ucnt.resize(n);
  g->big.assign(n, nullptr);
  g->big_bytes.assign(n, 0);
  g->gath.resize(n);
  g->uni.resize(n);
  g->rows.resize(n);
  g->hll.resize(n);
  g->cms.resize(n);
  g->dropped_seen.assign(n, 0);
  g->pcnt.resize(2 * n);
  g->hcol.resize(n);
  g->hmeta.resize(n);
  for (uint32_t i = 0; i < n; ++i) {
    if (hipSetDevice(devices[i]) != hipSuccess) {
      sa_group_destroy(g);
      return SA_EDEVICE;
    }
    for (int k = 0; k < 2; ++k)
      if (hipEventCreateWithFlags(&g->ev_scat[k][i], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&g->ev_done[k][i], hipEventDisableTiming) != hipSuccess) {
        sa_group_destroy(g);
        return SA_EDEVICE;
      }
  }
  if (hipHostMalloc((void **)&g->hcnt, kMaxMembers * 8, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void **)&g->hflush, 3 * kMaxMembers * 8, hipHostMallocDefault) != hipSuccess) {
    sa_group_destroy(g);
    return SA_ENOMEM;
  }
  // RCCL over distinct devices (a communicator cannot hold two ranks of one
  // device); SA_OPT_GROUP_COPY keeps the copy transport, and a group of one
  // uses RCCL only when SA_OPT_GROUP_RCCL asks
  std::vector<int> sorted(g->dev);
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  const bool want = !(cfg->options & SA_OPT_GROUP_COPY) && (n > 1 || (cfg->options & SA_OPT_GROUP_RCCL));
  if (distinct && want) {
    g->comm.resize(n);
    if (ncclCommInitAll(g->comm.data(), (int)n, g->dev.data()) == ncclSuccess) {
      g->rccl = true;
    } else {
      g->comm.clear();
      g->err = "ncclCommInitAll failed: merging through device copies";
    }
  }
  *out = g;
  return SA_OK;
}

void sa_group_destroy(sa_group *g) {
  if (!g) return;
  for (ncclComm_t c : g->comm)
    if (c) (void)ncclCommDestroy(c);
  for (size_t i = 0; i < g->eng.size(); ++i) {
    (void)hipSetDevice(g->dev[i]);
    if (i < g->st.size() && g->st[i]) {
      (void)hipStreamSynchronize(g->st[i]);
      (void)hipStreamDestroy(g->st[i]);
    }
    for (std::vector<Buf> *v : {&g->keys, &g->gath, &g->uni, &g->rows, &g->hll, &g->cms, &g->srt, &g->ucnt})
      if (i < v->size() && (*v)[i].p) (void)hipFree((*v)[i].p);
    if (i < g->big.size() && g->big[i]) (void)hipFree(g->big[i]);
    for (size_t k = 0; k < 2; ++k)
      if (k * g->eng.size() + i < g->pcnt.size() && g->pcnt[k * g->eng.size() + i].p)
        (void)hipFree(g->pcnt[k * g->eng.size() + i].p);
    for (int k = 0; k < 2; ++k) {
      if (i < kMaxMembers && g->part[k][i].p) (void)hipFree(g->part[k][i].p);
      if (i < kMaxMembers && g->peer[k][i].p) (void)hipFree(g->peer[k][i].p);
      if (g->ev_scat[k][i]) (void)hipEventDestroy(g->ev_scat[k][i]);
      if (g->ev_done[k][i]) (void)hipEventDestroy(g->ev_done[k][i]);
    }
    if (i == 0 && g->stack.p) (void)hipFree(g->stack.p);
    if (i == 0 && g->fin.p) (void)hipFree(g->fin.p);
    sa_destroy(g->eng[i]);
  }
  if (g->hcnt) (void)hipHostFree(g->hcnt);
  if (g->hflush) (void)hipHostFree(g->hflush);
  delete g;
}

const char *sa_group_last_error(const sa_group *g) { return g ? g->err.c_str() : "null group"; }
uint32_t sa_group_size(const sa_group *g) { return g ? (uint32_t)g->eng.size() : 0; }
int sa_group_uses_rccl(const sa_group *g) { return g && g->rccl ? 1 : 0; }
sa_engine *sa_group_member(sa_group *g, uint32_t i) { return g && i < g->eng.size() ? g->eng[i] : nullptr; }

// Host batch.  One pass computes every span's shard (worker threads over
// contiguous chunks, per-chunk shard counts); the prefix over chunks gives
// each chunk's write position in every member's packed shard; a second pass
// gathers the spans there (the same threads); then each member ingests its
// shard (sa_ingest copies it out before returning, so the shard buffers are
// reused by the next call).
int sa_group_ingest(sa_group *g, const sa_span_batch *b) {
  if (!g || !b) return SA_EINVAL;
  const uint32_t n = (uint32_t)g->eng.size();
  if (n == 1 || b->n == 0) {
    const int rc = sa_ingest(g->eng[0], b);
    return rc ? member_error(g, 0, rc, "sa_ingest") : SA_OK;
  }
  if (!b->key_hash || !b->start_ns || !b->end_ns || !b->trace_w0 || !b->trace_w1 || !b->meta)
    return gfail(g, SA_EINVAL, "null batch column");
  const uint64_t N = b->n;
  const uint32_t r32 = (uint32_t)((1ULL << 32) % n);
  const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
  const uint32_t T = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)std::min(hw, 16u), N / 65536 + 1}));
  const uint64_t per = (N + T - 1) / T;
  std::vector<uint8_t> sid(N);
  std::vector<uint64_t> cnt((size_t)T * n, 0);
  auto run = [&](auto &&fn) {
    std::vector<std::thread> th;
    for (uint32_t t = 1; t < T; ++t) th.emplace_back(fn, t);
    fn(0u);
    for (auto &x : th) x.join();
  };
  run([&](uint32_t t) {  // 1. shard ids and per-chunk counts
    const uint64_t a = std::min(N, t * per), z = std::min(N, a + per);
    uint64_t *c = cnt.data() + (size_t)t * n;
    for (uint64_t j = a; j < z; ++j) {
      const uint32_t sh = shard_of(b->trace_w1[j], n, r32);
      sid[j] = (uint8_t)sh;
      ++c[sh];
    }
  });
  std::vector<uint64_t> total(n, 0), off((size_t)T * n);
  for (uint32_t i = 0; i < n; ++i)
    for (uint32_t t = 0; t < T; ++t) {
      off[(size_t)t * n + i] = total[i];
      total[i] += cnt[(size_t)t * n + i];
    }
  for (uint32_t i = 0; i < n; ++i) {
    if (g->hcol[i].size() < total[i] * 5) g->hcol[i].resize(total[i] * 5);
    if (g->hmeta[i].size() < total[i]) g->hmeta[i].resize(total[i]);
  }
  run([&](uint32_t t) {  // 2. gather into the packed shards
    const uint64_t a = std::min(N, t * per), z = std::min(N, a + per);
    std::vector<uint64_t> o(off.begin() + (size_t)t * n, off.begin() + (size_t)(t + 1) * n);
    for (uint64_t j = a; j < z; ++j) {
      const uint32_t i = sid[j];
      const uint64_t p = o[i]++, cap = total[i];
      uint64_t *c = g->hcol[i].data();
      c[p] = b->key_hash[j];
      c[cap + p] = b->start_ns[j];
      c[2 * cap + p] = b->end_ns[j];
      c[3 * cap + p] = b->trace_w0[j];
      c[4 * cap + p] = b->trace_w1[j];
      g->hmeta[i][p] = b->meta[j];
    }
  });
  std::vector<int> rcs(n, SA_OK);
  std::vector<std::thread> th;
  for (uint32_t i = 0; i < n; ++i) {  // 3. members ingest their shards
    if (!total[i]) continue;
    th.emplace_back([&, i]() {
      const uint64_t cap = total[i];
      const uint64_t *c = g->hcol[i].data();
      const sa_span_batch sh{c, c + cap, c + 2 * cap, c + 3 * cap, c + 4 * cap, g->hmeta[i].data(), cap};
      rcs[i] = sa_ingest(g->eng[i], &sh);
    });
  }
  for (auto &x : th) x.join();
  for (uint32_t i = 0; i < n; ++i)
    if (rcs[i] != SA_OK) return member_error(g, i, rcs[i], "sa_ingest");
  return SA_OK;
}

int sa_group_ingest_device(sa_group *g, const sa_span_batch *b, uint32_t src, void *stream) {
  if (!g || !b) return SA_EINVAL;
  const uint32_t n = (uint32_t)g->eng.size();
  if (src >= n) return gfail(g, SA_EINVAL, "source member out of range");
  if (b->n == 0) return SA_OK;
  if (!b->key_hash || !b->start_ns || !b->end_ns || !b->trace_w0 || !b->trace_w1 || !b->meta)
    return gfail(g, SA_EINVAL, "null batch column");
  for (const void *c : {(const void *)b->key_hash, (const void *)b->start_ns, (const void *)b->end_ns,
                        (const void *)b->trace_w0, (const void *)b->trace_w1})
    if (reinterpret_cast<uintptr_t>(c) & 15) return gfail(g, SA_EINVAL, "device batch u64 columns must be 16-byte aligned");
  if (reinterpret_cast<uintptr_t>(b->meta) & 7) return gfail(g, SA_EINVAL, "device batch meta column must be 8-byte aligned");
  const int sdev = g->dev[src];
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : g->st[src];
  if (n == 1) {
    const int rc = sa_ingest_device(g->eng[0], b, s);
    return rc ? member_error(g, 0, rc, "sa_ingest_device") : SA_OK;
  }
  const uint32_t r32 = (uint32_t)((1ULL << 32) % n);
  const int k = g->pset;
  g->pset ^= 1;
  SG_HIP(g, hipSetDevice(sdev));
  // the staging set's previous users (each member's ingest of it) are done
  for (uint32_t i = 0; i < n; ++i)
    if (g->done_used[k][i]) SG_HIP(g, hipStreamWaitEvent(s, g->ev_done[k][i], 0));
  // 1. shard sizes (workgroup b of the partition owns spans [b * per, (b + 1) * per))
  const uint64_t per = std::max<uint64_t>(kPartChunk, (b->n + 2047) / 2048 + kPartChunk - 1) / kPartChunk * kPartChunk;
  const uint32_t pgrid = (uint32_t)((b->n + per - 1) / per);  // <= 2048
  Buf &pc = g->pcnt[(size_t)k * n + src];  // this set's: the previous call's scatter may still read the other
  if (int rc = ensure(g, sdev, pc, kMaxMembers * 8 + (size_t)4096 * kMaxMembers * 4)) return rc;
  unsigned long long *dcnt = static_cast<unsigned long long *>(pc.p);
  uint32_t *dblk = reinterpret_cast<uint32_t *>(dcnt + kMaxMembers);  // [n][pgrid] counts -> first positions
  if (b->n > 0xFFFFFFFFull) return gfail(g, SA_EINVAL, "device batch above 2^32 spans (u32 shard positions)");
  SG_HIP(g, hipMemsetAsync(dcnt, 0, kMaxMembers * 8, s));
  hipLaunchKernelGGL(shard_count_kernel, dim3(pgrid), dim3(kShardBlock), 0, s, b->trace_w1, b->n, per, n, r32, dcnt,
                     dblk);
  SG_HIP(g, hipGetLastError());
  SG_HIP(g, hipMemcpyAsync(g->hcnt, dcnt, n * 8, hipMemcpyDeviceToHost, s));
  hipLaunchKernelGGL(shard_scan_kernel, dim3(n), dim3(1024), 0, s, dblk, pgrid);  // (while the host reads the counts)
  SG_HIP(g, hipGetLastError());
  SG_HIP(g, hipStreamSynchronize(s));
  std::vector<uint64_t> cnt(g->hcnt, g->hcnt + n), cap(n);
  size_t bytes = 0;
  std::vector<size_t> at(n);
  for (uint32_t i = 0; i < n; ++i) {
    cap[i] = (cnt[i] + 1) & ~1ULL;  // even: every u64 column stays 16-B aligned
    at[i] = bytes;
    bytes += cap[i] * 44 + 64;
    bytes = (bytes + 255) & ~(size_t)255;
  }
  // 2. scatter into the packed shards (set k on the source device)
  if (int rc = ensure(g, sdev, g->part[k][src], bytes)) return rc;
  char *base = static_cast<char *>(g->part[k][src].p);
  ShardArgs args{};
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t *c = reinterpret_cast<uint64_t *>(base + at[i]);
    args.c[i] = ShardCols{c, c + cap[i], c + 2 * cap[i], c + 3 * cap[i], c + 4 * cap[i],
                          reinterpret_cast<uint32_t *>(c + 5 * cap[i])};
  }
  hipLaunchKernelGGL(shard_scatter_kernel, dim3(pgrid), dim3(kShardBlock), 0, s, *b, per, n, r32, args, dblk);
  SG_HIP(g, hipGetLastError());
  SG_HIP(g, hipEventRecord(g->ev_scat[k][src], s));
  // 3. every member ingests its shard on its own stream (peer copy first when
  //    it lives on another device)
  for (uint32_t i = 0; i < n; ++i) {
    if (!cnt[i]) continue;
    const int d = g->dev[i];
    SG_HIP(g, hipSetDevice(d));
    hipStream_t ms = g->st[i];
    SG_HIP(g, hipStreamWaitEvent(ms, g->ev_scat[k][src], 0));
    const ShardCols &c0 = args.c[i];
    ShardCols c = c0;
    if (d != sdev) {
      const size_t sb = cap[i] * 44;
      if (int rc = ensure(g, d, g->peer[k][i], sb)) return rc;
      SG_HIP(g, hipMemcpyPeerAsync(g->peer[k][i].p, d, c0.k, sdev, sb, ms));
      uint64_t *p = static_cast<uint64_t *>(g->peer[k][i].p);
      c = ShardCols{p, p + cap[i], p + 2 * cap[i], p + 3 * cap[i], p + 4 * cap[i],
                    reinterpret_cast<uint32_t *>(p + 5 * cap[i])};
    }
    const sa_span_batch sh{c.k, c.s, c.e, c.a, c.b, c.m, cnt[i]};
    if (int rc = sa_ingest_device(g->eng[i], &sh, ms)) return member_error(g, i, rc, "sa_ingest_device");
    SG_HIP(g, hipSetDevice(d));
    SG_HIP(g, hipEventRecord(g->ev_done[k][i], ms));
    g->done_used[k][i] = true;
  }
  return SA_OK;
}

int sa_group_sync(sa_group *g) {
  if (!g) return SA_EINVAL;
  for (uint32_t i = 0; i < g->eng.size(); ++i)
    if (int rc = sa_sync(g->eng[i])) return member_error(g, i, rc, "sa_sync");
  return SA_OK;
}

int sa_group_flush(sa_group *g, sa_red_result **out) {
  if (!g || !out) return SA_EINVAL;
  *out = nullptr;
  if (g->cfg.exp_max_size) return gfail(g, SA_ESTATE, "exponential-histogram group: use sa_group_flush_exp");
  const uint32_t n = (uint32_t)g->eng.size(), stride = g->nbk + 1;
  // 1. each member's non-zero series ids and its drop counter: every
  //    member's export is enqueued first, then one wait per member stream
  uint64_t *hn = g->hflush, *hdrop = g->hflush + kMaxMembers, *hkeys = g->hflush + 2 * kMaxMembers;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t tc = sa_grp::table_capacity(g->eng[i]);
    if (int rc = ensure(g, g->dev[i], g->keys[i], tc * 8)) return rc;
    if (int rc = sa_grp::export_keys_async(g->eng[i], static_cast<uint64_t *>(g->keys[i].p), tc, &hn[i], &hdrop[i],
                                           g->st[i]))
      return member_error(g, i, rc, "sa_export_keys");
  }
  for (uint32_t i = 0; i < n; ++i) {
    SG_HIP(g, hipSetDevice(g->dev[i]));
    SG_HIP(g, hipStreamSynchronize(g->st[i]));
  }
  std::vector<uint64_t> cnt(hn, hn + n), dropped(hdrop, hdrop + n);
  // 2. the sorted key union (the dense index every member densifies against),
  //    built on the devices: RCCL gathers every member's list onto every
  //    member, and each sorts / uniques its copy (identical bits everywhere,
  //    no broadcast); the copy transport gathers the lists onto member 0's
  //    device, builds the union there and copies it to the others.
  const uint64_t nmax = *std::max_element(cnt.begin(), cnt.end());
  uint64_t nu = 0;
  if (nmax) {
    if (g->rccl) {
      for (uint32_t i = 0; i < n; ++i) {
        SG_HIP(g, hipSetDevice(g->dev[i]));
        if (cnt[i] < nmax)  // pad with 0, the reserved id
          SG_HIP(g, hipMemsetAsync(static_cast<uint64_t *>(g->keys[i].p) + cnt[i], 0, (nmax - cnt[i]) * 8, g->st[i]));
        if (int rc = ensure(g, g->dev[i], g->gath[i], nmax * n * 8)) return rc;
      }
      SG_NCCL(g, ncclGroupStart());
      for (uint32_t i = 0; i < n; ++i)
        SG_NCCL(g, ncclAllGather(g->keys[i].p, g->gath[i].p, nmax, ncclUint64, g->comm[i], g->st[i]));
      SG_NCCL(g, ncclGroupEnd());
      for (uint32_t i = 0; i < n; ++i)
        if (int rc = device_union(g, i, static_cast<const uint64_t *>(g->gath[i].p), nmax * n)) return rc;
      if (int rc = union_count(g, 0, &nu)) return rc;
      for (uint32_t i = 1; i < n; ++i) {
        uint64_t nu_i = 0;
        if (int rc = union_count(g, i, &nu_i)) return rc;
        if (nu_i != nu) return gfail(g, SA_EDEVICE, "members disagree on the key union");
      }
    } else {
      uint64_t total = 0;
      for (uint32_t i = 0; i < n; ++i) total += cnt[i];
      if (int rc = ensure(g, g->dev[0], g->gath[0], total * 8)) return rc;
      for (uint32_t i = 1; i < n; ++i) {  // member 0's stream orders after every member's export
        SG_HIP(g, hipSetDevice(g->dev[i]));
        SG_HIP(g, hipStreamSynchronize(g->st[i]));
      }
      SG_HIP(g, hipSetDevice(g->dev[0]));
      uint64_t at = 0;
      for (uint32_t i = 0; i < n; ++i) {
        uint64_t *dst = static_cast<uint64_t *>(g->gath[0].p) + at;
        if (cnt[i] && g->dev[i] == g->dev[0])
          SG_HIP(g, hipMemcpyAsync(dst, g->keys[i].p, cnt[i] * 8, hipMemcpyDeviceToDevice, g->st[0]));
        else if (cnt[i])
          SG_HIP(g, hipMemcpyPeerAsync(dst, g->dev[0], g->keys[i].p, g->dev[i], cnt[i] * 8, g->st[0]));
        at += cnt[i];
      }
      if (int rc = device_union(g, 0, static_cast<const uint64_t *>(g->gath[0].p), total)) return rc;
      if (int rc = union_count(g, 0, &nu)) return rc;
      const uint64_t *u0 = static_cast<const uint64_t *>(g->uni[0].p);
      for (uint32_t i = 1; i < n && nu; ++i) {
        if (int rc = ensure(g, g->dev[i], g->uni[i], nu * 8)) return rc;
        SG_HIP(g, hipSetDevice(g->dev[i]));
        if (g->dev[i] == g->dev[0])
          SG_HIP(g, hipMemcpyAsync(g->uni[i].p, u0, nu * 8, hipMemcpyDeviceToDevice, g->st[0]));
        else
          SG_HIP(g, hipMemcpyPeerAsync(g->uni[i].p, g->dev[i], u0, g->dev[0], nu * 8, g->st[0]));
      }
      if (nu) {  // the members' streams wait for the union copies on st[0]
        SG_HIP(g, hipSetDevice(g->dev[0]));
        SG_HIP(g, hipStreamSynchronize(g->st[0]));
      }
    }
  }
  auto union_of = [&](uint32_t i) -> const uint64_t * { return static_cast<const uint64_t *>(g->uni[i].p); };
  const uint64_t len = nu * stride;
  // 3. dense rows per member (and its counters reset), 4. their sum, 5. the
  //    result's columns on member 0's device
  // The result's columns go to one page-locked block (keys, counts, calls,
  // ns sums, sums): DMA'd straight from the device, no zero fill, no staging.
  std::unique_ptr<red_holder> h(new red_holder());
  uint64_t *hk = nullptr, *hc = nullptr, *hcl = nullptr, *hns = nullptr;
  double *hs = nullptr;
  if (nu) {
    const size_t need = (size_t)nu * (g->nbk + 4) * 8;
    h->pool = g->pins;
    h->pin = g->pins->take(need, &h->pin_bytes);
    if (!h->pin) return gfail(g, SA_ENOMEM, "group flush: page-locked result block");
    hk = static_cast<uint64_t *>(h->pin);
    hc = hk + nu;
    hcl = hc + nu * g->nbk;
    hns = hcl + nu;
    hs = reinterpret_cast<double *>(hns + nu);
  }
  auto drop = [](int rc) { return rc; };
  if (nu) {
    for (uint32_t i = 0; i < n; ++i) {
      if (int rc = ensure(g, g->dev[i], g->rows[i], len * 8)) return drop(rc);
      if (int rc = sa_gather_dense(g->eng[i], union_of(i), nu, static_cast<uint64_t *>(g->rows[i].p), 1, g->st[i]))
        return drop(member_error(g, i, rc, "sa_gather_dense"));
    }
    bool one_device = true;
    for (uint32_t i = 1; i < n; ++i) one_device = one_device && g->dev[i] == g->dev[0];
    if (g->rccl) {
      SG_NCCL(g, ncclGroupStart());
      for (uint32_t i = 0; i < n; ++i)
        SG_NCCL(g, ncclAllReduce(g->rows[i].p, g->rows[i].p, len, ncclUint64, ncclSum, g->comm[i], g->st[i]));
      SG_NCCL(g, ncclGroupEnd());
    } else if (one_device && n > 1) {
      // every member's rows on one device: summed from their buffers into
      // member 0's (each element read from every member before its one write)
      for (uint32_t i = 1; i < n; ++i) {
        SG_HIP(g, hipSetDevice(g->dev[i]));
        SG_HIP(g, hipStreamSynchronize(g->st[i]));
      }
      SG_HIP(g, hipSetDevice(g->dev[0]));
      SrcPtrs src{};
      for (uint32_t i = 0; i < n; ++i) src.p[i] = static_cast<const unsigned long long *>(g->rows[i].p);
      hipLaunchKernelGGL(sum_ptrs_u64, dim3(grid_for(len)), dim3(256), 0, g->st[0],
                         static_cast<unsigned long long *>(g->rows[0].p), src, n, len);
      SG_HIP(g, hipGetLastError());
    } else if (int rc = copy_reduce(g, g->rows, len, false)) {
      return drop(rc);
    }
    const size_t fin_bytes = (size_t)nu * (g->nbk + 3) * 8;
    if (int rc = ensure(g, g->dev[0], g->fin, fin_bytes)) return drop(rc);
    SG_HIP(g, hipSetDevice(g->dev[0]));
    auto *fin = static_cast<unsigned long long *>(g->fin.p);
    unsigned long long *d_counts = fin, *d_calls = fin + nu * g->nbk, *d_sum_ns = d_calls + nu;
    double *d_sum = reinterpret_cast<double *>(d_sum_ns + nu);
    const double div = g->cfg.unit == SA_UNIT_S ? 1e9 : 1e6;
    hipLaunchKernelGGL(finalize_rows_kernel, dim3(grid_for(nu * 32)), dim3(256), 0, g->st[0],
                       static_cast<const unsigned long long *>(g->rows[0].p), nu, g->nbk, d_counts, d_calls,
                       d_sum_ns, d_sum, div);
    SG_HIP(g, hipGetLastError());
    // (counts, calls, ns sums and sums are contiguous in fin: one copy)
    SG_HIP(g, hipMemcpyAsync(hk, union_of(0), nu * 8, hipMemcpyDeviceToHost, g->st[0]));
    SG_HIP(g, hipMemcpyAsync(hc, d_counts, fin_bytes, hipMemcpyDeviceToHost, g->st[0]));
    (void)d_sum;
    // every member's counters are reset (gather_dense), so its key table can
    // be reclaimed now, while the result's copy is in flight: the resident-key
    // counts of all members first (one wait), then the reclamation of the
    // tables over the threshold (sa_flush's policy), waited for at the end
    for (uint32_t i = 0; i < n; ++i)
      if (int rc = sa_grp::count_keys_async(g->eng[i], &hkeys[i])) return drop(member_error(g, i, rc, "count keys"));
    for (uint32_t i = 0; i < n; ++i)
      if (int rc = sa_grp::sync_stream(g->eng[i])) return drop(member_error(g, i, rc, "count keys"));
    for (uint32_t i = 0; i < n; ++i)
      if (sa_grp::over_reclaim_threshold(g->eng[i], hkeys[i]))
        if (int rc = sa_grp::reclaim_async(g->eng[i])) return drop(member_error(g, i, rc, "sa_reclaim_keys"));
    for (uint32_t i = 0; i < n; ++i)
      if (int rc = sa_grp::sync_stream(g->eng[i])) return drop(member_error(g, i, rc, "sa_reclaim_keys"));
  }
  // (the members' key-table reclamation above is the flush-time policy
  // sa_flush applies)
  for (uint32_t i = 0; i < n; ++i) {
    SG_HIP(g, hipSetDevice(g->dev[i]));
    SG_HIP(g, hipStreamSynchronize(g->st[i]));
  }
  h->r.n_series = nu;
  h->r.n_buckets = g->nbk;
  h->r.key_hash = hk;
  h->r.bucket_counts = hc;
  h->r.calls = hcl;
  h->r.sum_ns = hns;
  h->r.sum = hs;
  *out = &h.release()->r;
  bool full = false;
  for (uint32_t i = 0; i < n; ++i) {
    full = full || dropped[i] != g->dropped_seen[i];
    g->dropped_seen[i] = dropped[i];
  }
  return full ? gfail(g, SA_EFULL, "key table full: spans were dropped since the previous flush") : SA_OK;
}

// exportMetrics of an exponential-histogram group: every member's delta
// histograms (sa_flush_exp, which also reclaims its key table), folded per
// series on the host (expo_fold).
int sa_group_flush_exp(sa_group *g, sa_exp_result **out) {
  if (!g || !out) return SA_EINVAL;
  *out = nullptr;
  if (!g->cfg.exp_max_size) return gfail(g, SA_ESTATE, "explicit-bucket group: use sa_group_flush");
  const uint32_t n = (uint32_t)g->eng.size(), M = g->cfg.exp_max_size;
  std::vector<sa_exp_result *> rs(n, nullptr);
  bool full = false;
  int bad = SA_OK;
  uint32_t bad_i = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const int rc = sa_flush_exp(g->eng[i], &rs[i]);
    if (rc == SA_EFULL) full = true;
    else if (rc != SA_OK && bad == SA_OK) bad = rc, bad_i = i;
  }
  std::map<uint64_t, ExpoAcc> acc;
  if (bad == SA_OK)
    for (uint32_t i = 0; i < n; ++i)
      for (uint64_t j = 0; rs[i] && j < rs[i]->n_series; ++j) expo_fold(acc[rs[i]->key_hash[j]], *rs[i], j, M);
  for (sa_exp_result *r : rs)
    if (r) sa_exp_result_free(r);
  if (bad != SA_OK) return member_error(g, bad_i, bad, "sa_flush_exp");
  const size_t ns = acc.size();
  auto *h = new exp_holder();
  h->keys.reserve(ns);
  h->count.reserve(ns), h->zero.reserve(ns), h->sum_ns.reserve(ns), h->sum.reserve(ns);
  h->min.reserve(ns), h->max.reserve(ns), h->scale.reserve(ns), h->offset.reserve(ns), h->nb.reserve(ns);
  h->buckets.assign(ns * M, 0);
  const double div = g->cfg.unit == SA_UNIT_S ? 1e9 : 1e6;
  size_t r = 0;
  for (const auto &kv : acc) {  // ascending keys
    const ExpoAcc &a = kv.second;
    h->keys.push_back(kv.first);
    h->count.push_back(a.count);
    h->zero.push_back(a.zero);
    h->sum_ns.push_back(a.sum_ns);
    h->sum.push_back((double)a.sum_ns / div);
    h->min.push_back(a.min);
    h->max.push_back(a.max);
    h->scale.push_back(a.scale);
    h->offset.push_back(a.offset);
    h->nb.push_back((uint32_t)a.c.size());
    std::copy(a.c.begin(), a.c.end(), h->buckets.begin() + r * M);
    ++r;
  }
  h->r.n_series = ns;
  h->r.max_size = M;
  h->r.unit = g->cfg.unit;
  h->r.key_hash = h->keys.data();
  h->r.count = h->count.data();
  h->r.zero_count = h->zero.data();
  h->r.sum_ns = h->sum_ns.data();
  h->r.sum = h->sum.data();
  h->r.min = h->min.data();
  h->r.max = h->max.data();
  h->r.scale = h->scale.data();
  h->r.offset = h->offset.data();
  h->r.n_buckets = h->nb.data();
  h->r.bucket_counts = h->buckets.data();
  *out = &h->r;
  return full ? gfail(g, SA_EFULL, "key table full: spans were dropped since the previous flush") : SA_OK;
}

int sa_group_window_read(sa_group *g, uint64_t window_id, sa_sketch_result **out) {
  if (!g || !out) return SA_EINVAL;
  *out = nullptr;
  const uint32_t n = (uint32_t)g->eng.size();
  for (uint32_t i = 0; i < n; ++i) {
    if (int rc = ensure(g, g->dev[i], g->hll[i], g->hll_bytes)) return rc;
    if (int rc = ensure(g, g->dev[i], g->cms[i], g->cms_elems * 8)) return rc;
    if (int rc = sa_window_export(g->eng[i], window_id, static_cast<uint8_t *>(g->hll[i].p),
                                  static_cast<uint64_t *>(g->cms[i].p), g->st[i]))
      return member_error(g, i, rc, "sa_window_export");
  }
  if (g->rccl) {
    SG_NCCL(g, ncclGroupStart());
    for (uint32_t i = 0; i < n; ++i) {
      SG_NCCL(g, ncclAllReduce(g->hll[i].p, g->hll[i].p, g->hll_bytes, ncclUint8, ncclMax, g->comm[i], g->st[i]));
      SG_NCCL(g, ncclAllReduce(g->cms[i].p, g->cms[i].p, g->cms_elems, ncclUint64, ncclSum, g->comm[i], g->st[i]));
    }
    SG_NCCL(g, ncclGroupEnd());
  } else {
    if (int rc = copy_reduce(g, g->hll, g->hll_bytes, true)) return rc;
    if (int rc = copy_reduce(g, g->cms, g->cms_elems, false)) return rc;
  }
  auto *h = new sketch_holder();
  h->hll.resize(g->hll_bytes);
  std::vector<uint64_t> c64(g->cms_elems);
  (void)hipSetDevice(g->dev[0]);
  hipError_t a = hipMemcpyAsync(h->hll.data(), g->hll[0].p, g->hll_bytes, hipMemcpyDeviceToHost, g->st[0]);
  hipError_t b = hipMemcpyAsync(c64.data(), g->cms[0].p, g->cms_elems * 8, hipMemcpyDeviceToHost, g->st[0]);
  hipError_t c = hipStreamSynchronize(g->st[0]);
  for (uint32_t i = 1; i < n && c == hipSuccess; ++i) {
    (void)hipSetDevice(g->dev[i]);
    c = hipStreamSynchronize(g->st[i]);
  }
  if (a != hipSuccess || b != hipSuccess || c != hipSuccess) {
    delete h;
    return gfail(g, SA_EDEVICE, "group window read failed");
  }
  h->cms.resize(g->cms_elems);
  for (size_t i = 0; i < c64.size(); ++i) h->cms[i] = c64[i] > UINT32_MAX ? UINT32_MAX : (uint32_t)c64[i];
  h->r.window_id = window_id;
  h->r.n_services = g->cfg.n_services;
  h->r.hll_p = g->cfg.hll_p;
  h->r.hll = h->hll.data();
  h->r.cms_d = g->cfg.cms_d;
  h->r.cms_w = g->cfg.cms_w;
  h->r.cms = h->cms.data();
  *out = &h->r;
  return SA_OK;
}

int sa_group_window_advance(sa_group *g, uint64_t new_base) {
  if (!g) return SA_EINVAL;
  for (uint32_t i = 0; i < g->eng.size(); ++i)
    if (int rc = sa_window_advance(g->eng[i], new_base)) return member_error(g, i, rc, "sa_window_advance");
  return SA_OK;
}

int sa_group_get_stats(sa_group *g, sa_stats *o) {
  if (!g || !o) return SA_EINVAL;
  std::memset(o, 0, sizeof *o);
  for (uint32_t i = 0; i < g->eng.size(); ++i) {
    sa_stats s;
    if (int rc = sa_get_stats(g->eng[i], &s)) return member_error(g, i, rc, "sa_get_stats");
    o->spans += s.spans;
    o->zero_key += s.zero_key;
    o->invalid_service += s.invalid_service;
    o->window_out_of_range += s.window_out_of_range;
    o->dropped_table_full += s.dropped_table_full;
    o->n_keys += s.n_keys;
    o->table_capacity += s.table_capacity;
    o->hll_filtered += s.hll_filtered;
    if (i == 0) {
      o->window_base = s.window_base;
      o->small_table = s.small_table;
    }
  }
  return SA_OK;
}

}  // extern "C"
