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
#include <climits>
#include <cstdlib>
#include <cmath>

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

// (the fast bucket index, expo_index_fast, is in sa_device.h: the ingest
// kernel computes it too)

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
// kept buckets down when it drops.  h is the series header in registers (the
// caller stores it back).  At a positive target scale the indices of the
// smallest and largest positive value are their scale-20 indices shifted
// right: Go's index is floor(Log(v) * Ldexp(Log2E, s)), and the product with
// an exact power of two rounds the same at every scale, so the scale-s value
// is the scale-20 value times 2^(s-20) exactly, and floor(y / 2^k) =
// floor(y) >> k (the max-index clamp and the power-of-two case shift the same
// way).  Scales <= 0 take Go's exponent formula instead.
__device__ __forceinline__ void rescale_hdr(const ExpoParams &E, uint64_t s, ExpoHdr &h) {
  if (h.maxpos_ns == 0) return;  // no positive value
  const double vlo = expo_value(h.minpos_ns, E.div), vhi = expo_value(h.maxpos_ns, E.div);
  const int32_t lo20 = expo_index(vlo, kExpoMaxScale), hi20 = expo_index(vhi, kExpoMaxScale);
  int32_t lo = lo20, hi = hi20, change = 0;
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
  if (target > 0) {
    h.lo = lo20 >> (kExpoMaxScale - target);
    h.hi = hi20 >> (kExpoMaxScale - target);
  } else {
    h.lo = expo_index(vlo, target);
    h.hi = expo_index(vhi, target);
  }
}

__device__ __forceinline__ void rescale_slot(const ExpoParams &E, uint64_t s) {
  ExpoHdr h = E.hdr[s];
  if (h.maxpos_ns == 0) return;
  rescale_hdr(E, s, h);
  E.hdr[s] = h;
  if (E.xscale) E.xscale[s] = (int8_t)h.scale;
}

// (one thread per slot)
__global__ __launch_bounds__(256) void expo_rescale_kernel(ExpoParams E) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < E.cap; s += (uint64_t)gridDim.x * blockDim.x)
    rescale_slot(E, s);
}

// Small-table engines: the ingest kernel (EXPO mode) leaves per-workgroup
// header partials in slabs [xG][cap] (every slot, each launch).  One block
// per kXrSlots slots (8 by default, 256 blocks at C2's 2,048 slots): the
// block's 1,024 / kXrSlots groups sum a strided share of the workgroups'
// partials (coalesced runs), the lanes of a wave holding the same slot
// combine by shuffles and the 16 waves through LDS, then one thread per slot
// folds the sum into the series header and rescales it.  A thread issues all
// its partial reads (kXrBatch at a time) and the owner its header read before
// any is used: a loop with the zeroing store in it kept one round trip per
// partial in a row, and a 64-block grid left three quarters of the CUs idle.
constexpr uint32_t kXrBatch = 8;
__device__ __forceinline__ void xhdr_add(XHdr &acc, const XHdr &x) {
  acc.cnt += x.cnt;
  acc.zero += x.zero;
  acc.sum += x.sum;
  acc.minx = x.minx > acc.minx ? x.minx : acc.minx;
  acc.max = x.max > acc.max ? x.max : acc.max;
}
__device__ __forceinline__ unsigned long long shfl_xor_u64(unsigned long long v, int o) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o, 64);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o, 64);
  return ((unsigned long long)hi << 32) | lo;
}
template <uint32_t kXrSlots>
__global__ __launch_bounds__(1024) void expo_reduce_rescale_kernel(ExpoParams E) {
  static_assert(kXrSlots >= 1 && kXrSlots <= 64 && (kXrSlots & (kXrSlots - 1)) == 0, "slots per block");
  constexpr uint32_t kXrGroups = 1024 / kXrSlots;
  __shared__ XHdr part[16][kXrSlots];
  const uint32_t sl = threadIdx.x % kXrSlots, gg = threadIdx.x / kXrSlots;
  const uint64_t s = blockIdx.x * (uint64_t)kXrSlots + sl;
  const bool owner = gg == 0 && s < E.cap;
  ExpoHdr h{};
  if (owner) h = E.hdr[s];
  // the counting kernel's word of the slot (its scale, bucket buffer and the
  // multiple of M below its kept range), so its 256 workgroups read 8 B a
  // slot instead of the 72-B header
  auto put_meta = [&](const ExpoHdr &x) {
    if (!E.xmeta) return;
    const int32_t l = x.lo == kExpoEmpty ? 0 : x.lo;
    E.xmeta[s] = make_int2((x.scale & 0xFF) | (int)(x.cur << 8), l - (int32_t)expo_mod(l, E.max_size));
  };
  XHdr acc{0, 0, 0, 0, 0};
  if (s < E.cap) {
    for (uint32_t g0 = gg; g0 < E.xG; g0 += kXrBatch * kXrGroups) {
      XHdr x[kXrBatch];
#pragma unroll
      for (uint32_t u = 0; u < kXrBatch; ++u) {
        const uint32_t g = g0 + u * kXrGroups;
        x[u] = g < E.xG ? E.xslab[(uint64_t)g * E.cap + s] : XHdr{0, 0, 0, 0, 0};
      }
#pragma unroll
      for (uint32_t u = 0; u < kXrBatch; ++u)
        if (x[u].cnt) xhdr_add(acc, x[u]);
    }
  }
  // lanes l, l ^ kXrSlots, ... of a wave hold the same slot
#pragma unroll
  for (int o = kXrSlots; o < 64; o <<= 1) {
    XHdr y;
    y.cnt = (uint32_t)__shfl_xor((int)acc.cnt, o, 64);
    y.zero = (uint32_t)__shfl_xor((int)acc.zero, o, 64);
    y.sum = shfl_xor_u64(acc.sum, o);
    y.minx = shfl_xor_u64(acc.minx, o);
    y.max = shfl_xor_u64(acc.max, o);
    xhdr_add(acc, y);
  }
  if ((threadIdx.x & 63u) < kXrSlots) part[threadIdx.x >> 6][sl] = acc;
  __syncthreads();
  if (!owner) return;
  acc = part[0][sl];
  // (two at a time: the 15 partials loaded at once held 120 registers and
  // pushed the rescale's into scratch)
#pragma unroll 2
  for (uint32_t k = 1; k < 16; ++k) xhdr_add(acc, part[k][sl]);
  if (E.lcount) E.lcount[s] = acc.cnt - acc.zero;  // this launch's positive durations (the entry selection)
  if (!acc.cnt) {  // no new values: the header (scale, range) stays as it is
    if (E.xscale) E.xscale[s] = (int8_t)h.scale;
    put_meta(h);
    return;
  }
  const unsigned long long minpos = ~acc.minx;  // UINT64_MAX when no positive duration
  const unsigned long long mn = acc.zero ? 0ULL : minpos;
  h.count += acc.cnt;
  h.zero += acc.zero;
  h.sum_ns += acc.sum;
  h.min_ns = mn < h.min_ns ? mn : h.min_ns;
  h.max_ns = acc.max > h.max_ns ? acc.max : h.max_ns;
  h.minpos_ns = minpos < h.minpos_ns ? minpos : h.minpos_ns;
  h.maxpos_ns = acc.max > h.maxpos_ns ? acc.max : h.maxpos_ns;
  rescale_hdr(E, s, h);
  E.hdr[s] = h;
  if (E.xscale) E.xscale[s] = (int8_t)h.scale;
  put_meta(h);
}

constexpr uint32_t kXcBlock = 1024;

// SA_OPT_STAMPS: a counting workgroup's phase stamp (thread 0, s_memrealtime)
__device__ __forceinline__ void xc_stamp(const ExpoParams &E, uint32_t slot) {
  if (threadIdx.x == 0) E.dbg[blockIdx.x * kDbgPerWg + slot] = __builtin_amdgcn_s_memrealtime();
}
// laboratory ablations of the counting and fold kernels (SPANAGG_XC_DIAG
// bits; counts wrong): 2 = the counting loop's loads only, 4 = no slab
// stores, 8 / 16 = no slab / tail fold.  (Bit 1, the tail's records off, is
// older and in both builds.)
#ifdef SPANAGG_AB
#define XC_ABL(bit) ((E.diag & (bit)) != 0u)
#else
#define XC_ABL(bit) false
#endif
constexpr uint64_t kXcMaxSpans = 65535;  // u16 LDS counts: spans per counting workgroup
constexpr uint32_t kXcDefer = 256;       // long-duration records a counting workgroup defers to after its loop

// Bucket counting of small tables, two kernels:
//   expo_count_slab_kernel every workgroup first selects the xc_ne series with
//                          the most positive durations this launch (lcount,
//                          left by the reduce pass) for its LDS entries: by bit
//                          length of the count, ties in slot order.  Every
//                          workgroup computes the same selection; workgroup 0
//                          also writes it out for the fold.  Then per span:
//                          bucket index at the series' scale; an entry's spans
//                          add to LDS u16 counts, which leave as plain
//                          coalesced stores into the workgroup's slab; other
//                          spans leave as (slot, bucket) tail records sorted
//                          by fold bin.  The spans come as the 8-B records
//                          the ingest kernel wrote (slot | duration,
//                          span_rec_of), not as slot + both times (20 B)
//   expo_fold_kernel       per (entry, bucket pair): the sum over the
//                          workgroups' slabs, added to the series' buckets;
//                          and per tail bin: every workgroup's records of the
//                          bin counted in LDS, then added to the buckets
//                          (one owner each, no atomics; one launch)
// A launch's C2 mix (10 M spans, ~1.4 k series, Zipf) put ~6 M atomics on
// HBM with per-workgroup caches flushed by atomics: ~200 us of the ~310 us
// the counting took.  The selection was a one-block kernel of its own, 6 us
// of block-wide scans plus a launch; in the counting kernel's prologue it is
// two wave-shuffle scans.  Which series hold entries changes where counts are
// added, never the counts.

// Exclusive scan of v over a 1,024-thread block (wave shuffles, then the 16
// wave totals through LDS wsum[16]); total = the block's sum.  Every thread
// calls it.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *wsum, uint32_t &total) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    const uint32_t t = wsum[k];
    base += k < w ? t : 0u;
    tot += t;
  }
  __syncthreads();  // wsum is free again
  total = tot;
  return base + x - v;
}

// The entry selection (cap <= 2,048: slots 2t and 2t + 1 of thread t) into
// en[2], the entries of thread t's two slots (-1: none), and soe_next, the
// slot of each entry (~0u past the selected ones; write_soe).  scratch: 64 LDS words.
// lc: lcount of slots 2t and 2t + 1 (0 past cap).
__device__ __forceinline__ void expo_select_lds(const ExpoParams &E, uint32_t *scratch, const uint32_t (&lc)[2],
                                                int32_t (&en)[2], bool write_soe) {
  const uint32_t t = threadIdx.x, K = E.xc_ne, lane = t & 63u;
  uint32_t *hist = scratch, *wsum = scratch + 48;  // hist[33], wsum[16]
  uint32_t bl[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) bl[k] = lc[k] ? 32u - (uint32_t)__clz(lc[k]) : 0u;
  if (t < 33) hist[t] = 0;
  // the wave's count of each bit length by ballots (lane b keeps length b's),
  // then one conflict-free LDS add per lane: per-slot adds into a few hot
  // bit lengths serialised on their words (~3 us)
  uint32_t mine = 0;
#pragma unroll
  for (uint32_t b = 1; b <= 32; ++b) {
    const uint32_t c = (uint32_t)__popcll(__ballot(bl[0] == b)) + (uint32_t)__popcll(__ballot(bl[1] == b));
    mine = lane == b ? c : mine;
  }
  __syncthreads();
  if (mine) atomicAdd(&hist[lane], mine);
  __syncthreads();
  // every wave: suffix sums S[b] = #slots of bit length >= b (lane b); the
  // boundary bit length tb is the largest b >= 1 with S[b] > K (0: every
  // series fits), and S[tb + 1] of the entries go above it
  uint32_t sfx = lane <= 32 ? hist[lane] : 0u;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_down((int)sfx, (unsigned)o, 64);
    if (lane + (uint32_t)o < 64) sfx += y;
  }
  const uint64_t over = __ballot(lane >= 1 && lane <= 32 && sfx > K);
  const uint32_t tb = over ? 63u - (uint32_t)__clzll((long long)over) : 0u;
  const uint32_t room = K - (uint32_t)__shfl((int)sfx, (int)(tb + 1), 64);
  // boundary-bin slots in slot order take the room left
  const uint32_t b0 = (tb && bl[0] == tb) ? 1u : 0u, b1 = (tb && bl[1] == tb) ? 1u : 0u;
  uint32_t tot;
  const uint32_t bx = block_excl_scan(b0 + b1, wsum, tot);
  const bool sel0 = bl[0] && (bl[0] > tb || (b0 && bx < room));
  const bool sel1 = bl[1] && (bl[1] > tb || (b1 && bx + b0 < room));
  const uint32_t n0 = sel0 ? 1u : 0u, n1 = sel1 ? 1u : 0u;
  uint32_t nsel;
  const uint32_t ex = block_excl_scan(n0 + n1, wsum, nsel);
  en[0] = sel0 ? (int32_t)ex : -1;
  en[1] = sel1 ? (int32_t)(ex + n0) : -1;
  if (!write_soe) return;
  if (sel0) E.soe_next[ex] = 2 * t;
  if (sel1) E.soe_next[ex + n0] = 2 * t + 1;
  for (uint32_t k = nsel + t; k < K; k += 1024) E.soe_next[k] = ~0u;
}

// IN: the spans as 0 = the key slot (E.slot_of) and both times (20 B per
// span), 1 = the ingest kernel's 8-B span records (E.span_rec), 2 = its index
// records (E.slot_of, ixrec: 4 B, the bucket index already computed)
template <int IN>
__global__ __launch_bounds__(1024) void expo_count_slab_kernel(ExpoParams E, uint64_t per_wg) {
  constexpr bool REC = IN == 1, IXR = IN == 2;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t M = E.max_size, NE = E.xc_ne, cap = (uint32_t)E.cap, wpe = (M + 1) / 2;
  int2 *meta = reinterpret_cast<int2 *>(smem);                   // [cap] (below)
  uint32_t *cnt = reinterpret_cast<uint32_t *>(meta + cap);       // [NE][wpe] u16 pairs
  uint32_t *scratch = cnt + NE * wpe;                             // [64] selection scratch
  // the tail: records of the spans without an entry, their count, and the
  // fold bins' histogram / cursors at the end
  uint32_t *trec = scratch + 64;                                  // [kXtCap]
  uint32_t *tmisc = trec + kXtCap;                                // [0] records, [1..] bin hist / cursors
  // (IXR) long-duration records deferred to after the loop: their spans, slots and count
  uint32_t *dl_i = tmisc + 1 + xt_bins(cap, M), *dl_s = dl_i + kXcDefer, *dl_n = dl_s + kXcDefer;
  const bool tail = E.xt_rec != nullptr;
  if (E.dbg) xc_stamp(E, kXcStamp);
  if (threadIdx.x == 0) tmisc[0] = tmisc[1] = *dl_n = 0;
  // meta of slot s: {scale (8 bits) | buffer << 8 | (entry + 1) << 9, base},
  // base = lo - (lo mod M), the multiple of M at or below the kept range's
  // first index lo: a bucket index ix with ix - base in [0, 2M) sits at
  // position (ix - base) wrapped once (this launch's positive values lie in
  // [lo, lo + M)).  The reduce pass left all but the entry (xmeta); the
  // entries are the selection the previous launch's workgroup 0 made (xent:
  // which series hold entries changes where counts are added, never the
  // counts, and a mix's frequent series change slowly); slots 2t and 2t + 1
  // are thread t's, as in the selection.
  // (an engine's first launch has no selection yet, E.xent null: every
  // workgroup makes this launch's, the same one, as workgroup 0 does)
  int4 xm = make_int4(0, 0, 0, 0);
  int2 ec = make_int2(-1, -1);
  if (2 * threadIdx.x < cap) {  // (cap even)
    xm = *reinterpret_cast<const int4 *>(E.xmeta + 2 * threadIdx.x);
    if (E.xent) ec = *reinterpret_cast<const int2 *>(E.xent + 2 * threadIdx.x);
  }
  for (uint32_t i = threadIdx.x; i < NE * wpe; i += kXcBlock) cnt[i] = 0;
  if (E.dbg) xc_stamp(E, kXcStampZeroed);
  if (blockIdx.x == 0 || !E.xent) {  // (workgroup-uniform) the next launch's entries, from this launch's counts
    uint32_t lc[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) lc[k] = 2 * threadIdx.x + k < cap ? E.lcount[2 * threadIdx.x + k] : 0u;
    int32_t en[2];
    expo_select_lds(E, scratch, lc, en, blockIdx.x == 0);
    if (blockIdx.x == 0 && 2 * threadIdx.x < cap)
      *reinterpret_cast<int2 *>(E.xent_next + 2 * threadIdx.x) = make_int2(en[0], en[1]);
    if (!E.xent) ec = make_int2(en[0], en[1]);
  }
  if (E.dbg) xc_stamp(E, kXcStampSelected);
  if (2 * threadIdx.x < cap)
    *reinterpret_cast<int4 *>(meta + 2 * threadIdx.x) =
        make_int4(xm.x | (ec.x + 1) << 9, xm.y, xm.z | (ec.y + 1) << 9, xm.w);
  __syncthreads();
  if (E.dbg) xc_stamp(E, kXcStamp + 1);
  const uint64_t lo = blockIdx.x * per_wg, hi = lo + per_wg < E.n ? lo + per_wg : E.n;
  const uint32_t len = hi > lo ? (uint32_t)(hi - lo) : 0u;
  // the span's bucket index ix at its series' scale -> its LDS entry or a tail record
  auto add = [&](uint32_t slot, int32_t ix, int2 m) {
    const uint32_t rel = (uint32_t)(ix - m.y);
    const uint32_t at = rel < 2 * M ? (rel >= M ? rel - M : rel) : expo_mod(ix, M);
    const int32_t en_ = (int32_t)((uint32_t)m.x >> 9) - 1;
    if (en_ >= 0) {
      atomicAdd(&cnt[(uint32_t)en_ * wpe + (at >> 1)], 1u << ((at & 1u) * 16));
    } else if (!(E.diag & 1u)) {
      // a series without an entry: a record for the tail fold, not a
      // scattered HBM atomic (past the record buffer: the atomic)
      const uint32_t r = tail ? atomicAdd(&tmisc[0], 1u) : kXtCap;
      if (r < kXtCap) trec[r] = slot << 12 | at;
      else atomicAdd(E.buckets + ((uint64_t)(((uint32_t)m.x >> 8) & 1u) * E.cap + slot) * M + at, 1u);
    }
  };
  auto count = [&](uint32_t slot, uint64_t d) {
    if (d == 0) return;
    const int2 m = meta[slot];
    const int32_t sc = (int32_t)(int8_t)(m.x & 0xFF);
    int32_t ix;
    if (!expo_index_fast(d, E.log2div_q24, sc, ix)) ix = expo_index(expo_value(d, E.div), sc);
    add(slot, ix, m);
  };
  // one index record (ixrec_of): the index at the scale the ingest kernel
  // read, shifted to the scale the reduce pass settled on (never higher: a
  // series' scale only falls within a flush interval)
  auto count_ix = [&](uint32_t w, uint64_t i) {
    const uint32_t slot = w >> kIxSlotShift;
    if (slot == kSpanRecNoSlot || w == (slot << kIxSlotShift | kIxZero)) return;
    if (w & 1u) {
      count(slot, E.span_long[i]);
      return;
    }
    const int2 m = meta[slot];
    const int32_t sn = (int32_t)(int8_t)(m.x & 0xFF);
    const int32_t su = (int32_t)((w >> kIxScaleShift) & 31u) - (int32_t)kIxScaleBias;
    // (su < sn would need a shift the other way: the series' scale rose since
    // the ingest kernel read it, which no reset path may allow -- compact and
    // init reset xscale with the header.  Should one ever break that, the
    // span is reported as dropped, never counted in a wrong bucket.)
    if (__builtin_expect(su < sn, 0)) {
      atomicAdd(E.dropped, 1ULL);
      return;
    }
    const int32_t ix = ((int32_t)(w << 17) >> 18) >> (su - sn);  // the 14-bit field, sign-extended
    add(slot, ix, m);
  };
  // one span record (span_rec_of; 0 past the range: no duration); a duration
  // past the record's field is read from span_long
  auto count_rec = [&](unsigned long long r, uint64_t i) {
    const uint32_t slot = (uint32_t)(r >> kSpanRecShift);
    if (slot == kSpanRecNoSlot) return;
    uint64_t d = r & kSpanRecDurMask;
    if (d == kSpanRecDurMask) d = E.span_long[i];
    count(slot, d);
  };
  // four consecutive spans per thread through 16-B buffer loads (0 past the
  // range), two rounds in flight: with the tail off HBM atomics the loop is
  // bound by its loads, and one span per thread per round kept only ~20 KB
  // per CU in flight
  const __amdgpu_buffer_rsrc_t rr = rsrc(REC ? (const void *)(E.span_rec + lo) : (const void *)(E.slot_of + lo),
                                         REC ? len * 8 : len * 4);
  constexpr bool kTimes = IN == 0;
  const __amdgpu_buffer_rsrc_t rst = rsrc(E.start + lo, kTimes ? len * 8 : 0u),
                               ren = rsrc(E.end + lo, kTimes ? len * 8 : 0u);
  struct Quad {
    unsigned long long r[4];  // REC: the records; else the slots
    uint64_t s[kTimes ? 4 : 1], e[kTimes ? 4 : 1];
  };
  auto load = [&](uint32_t base, Quad &q) {
    const int o = (int)(base + 4 * threadIdx.x);
    if constexpr (REC) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(rr, o * 8 + 16 * h, 0, 0);
        q.r[2 * h] = (unsigned long long)x[0] | ((unsigned long long)x[1] << 32);
        q.r[2 * h + 1] = (unsigned long long)x[2] | ((unsigned long long)x[3] << 32);
      }
    } else {
      const auto a = __builtin_amdgcn_raw_buffer_load_b128(rr, o * 4, 0, 0);
#pragma unroll
      for (int j = 0; j < 4; ++j) q.r[j] = a[j];
      if constexpr (kTimes) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const auto x = __builtin_amdgcn_raw_buffer_load_b128(rst, o * 8 + 16 * h, 0, 0);
          const auto y = __builtin_amdgcn_raw_buffer_load_b128(ren, o * 8 + 16 * h, 0, 0);
          q.s[2 * h] = (uint64_t)x[0] | ((uint64_t)x[1] << 32);
          q.s[2 * h + 1] = (uint64_t)x[2] | ((uint64_t)x[3] << 32);
          q.e[2 * h] = (uint64_t)y[0] | ((uint64_t)y[1] << 32);
          q.e[2 * h + 1] = (uint64_t)y[2] | ((uint64_t)y[3] << 32);
        }
      }
    }
  };
  auto run = [&](uint32_t base, const Quad &q) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (base + 4 * threadIdx.x + j >= len) continue;
      if constexpr (REC) {
        count_rec(q.r[j], lo + base + 4 * threadIdx.x + j);
      } else if constexpr (IXR) {
        count_ix((uint32_t)q.r[j], lo + base + 4 * threadIdx.x + j);
      } else {
        const uint32_t slot = (uint32_t)q.r[j];
        if (slot != kNotFound) count(slot, q.e[j] > q.s[j] ? q.e[j] - q.s[j] : 0);
      }
    }
  };
  // IXR: a thread's four index records with one LDS read each and no branch
  // on the common path (a per-record early exit, long-duration branch and
  // tail claim kept ~100 instructions a record under exec-mask branching;
  // the loop was issue-bound at ~4x its loads' time): an entry's record is
  // one LDS add; the tail's records of the quad claim their buffer slots with
  // one LDS add per wave; the rare cases -- a long duration, a scale that
  // rose, a bucket outside the kept range -- go through count_ix after a
  // wave-uniform test.
  auto count_quad = [&](uint32_t base, const Quad &q) {
    uint32_t w[4], slot[4], at[4], en1[4];
    bool tl[4], rare[4], add[4];
    int2 m[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      w[j] = (uint32_t)q.r[j];
      slot[j] = w[j] >> kIxSlotShift;
      m[j] = meta[slot[j] & (cap - 1u)];
    }
    // (bitwise, not short-circuit, conditions: no branches)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool pos = (base + 4 * threadIdx.x + (uint32_t)j < len) & (slot[j] != kSpanRecNoSlot) &
                       (w[j] != (slot[j] << kIxSlotShift | kIxZero));
      const int32_t sn = (int32_t)(int8_t)(m[j].x & 0xFF);
      const int32_t su = (int32_t)((w[j] >> kIxScaleShift) & 31u) - (int32_t)kIxScaleBias;
      const int32_t ix = ((int32_t)(w[j] << 17) >> 18) >> ((su - sn) & 31);  // the 14-bit field, sign-extended
      const uint32_t rel = (uint32_t)(ix - m[j].y);
      at[j] = rel >= M ? rel - M : rel;
      en1[j] = (uint32_t)m[j].x >> 9;
      const bool ok = pos & !(w[j] & 1u) & (su >= sn) & (rel < 2 * M);
      rare[j] = pos & !ok;
      tl[j] = ok & (en1[j] == 0);
      add[j] = ok & (en1[j] != 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (add[j]) atomicAdd(&cnt[__umul24(en1[j] - 1u, wpe) + (at[j] >> 1)], 1u << ((at[j] & 1u) * 16));
    if (!(E.diag & 1u)) {
      uint64_t tb[4];
      uint32_t pre[4], total = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        tb[j] = __ballot(tl[j]);
        pre[j] = total;
        total += (uint32_t)__popcll(tb[j]);
      }
      if (total) {  // wave-uniform; every lane is active here
        uint32_t t0 = kXtCap;
        if ((threadIdx.x & 63u) == 0 && tail) t0 = atomicAdd(&tmisc[0], total);
        t0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)t0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!tl[j]) continue;
          const uint32_t r = t0 + pre[j] +
                             __builtin_amdgcn_mbcnt_hi((uint32_t)(tb[j] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)tb[j], 0u));
          if (r < kXtCap) {
            trec[r] = slot[j] << 12 | at[j];
          } else {  // past the record buffer: the bucket's HBM atomic
            const uint32_t cur = ((uint32_t)meta[slot[j]].x >> 8) & 1u;
            atomicAdd(E.buckets + ((uint64_t)cur * E.cap + slot[j]) * M + at[j], 1u);
          }
        }
      }
    }
    if (__builtin_expect(__ballot(rare[0] || rare[1] || rare[2] || rare[3]) != 0, 0)) {
      if (E.dbg && (threadIdx.x & 63u) == 0) atomicAdd(&tmisc[1], 1u);  // (SA_OPT_STAMPS: waves on the rare path)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (!rare[j]) continue;
        const uint32_t i = (uint32_t)(lo + base + 4 * threadIdx.x + j);
        // a long duration (the fast index declined it in the ingest kernel: at
        // high scales ~1e-3 of spans, near a bucket boundary) waits for the
        // end of the loop, where every deferred record's side-array read goes
        // out at once -- here each one held its wave for a memory round trip
        uint32_t k = kXcDefer;
        if (w[j] & 1u) k = atomicAdd(dl_n, 1u);
        if (k < kXcDefer) {
          dl_i[k] = i;
          dl_s[k] = slot[j];
        } else {
          count_ix(w[j], i);
        }
      }
    }
  };
  constexpr uint32_t kStep = 4 * kXcBlock;
  // (an 8-round ring of loads in flight instead of two measured slower: 41.9
  // against 38.2 us per 10 M spans -- the loop is not waiting on its loads)
  Quad qa, qb;
  load(0, qa);
  if (XC_ABL(2u)) {  // laboratory ablation: the loads only (their words folded into one sink)
    uint32_t sink = 0;
    for (uint32_t base = 0; base < len; base += 2 * kStep) {
      load(base + kStep, qb);
      sink ^= (uint32_t)(qa.r[0] ^ qa.r[1] ^ qa.r[2] ^ qa.r[3]);
      load(base + 2 * kStep, qa);
      sink ^= (uint32_t)(qb.r[0] ^ qb.r[1] ^ qb.r[2] ^ qb.r[3]);
    }
    if (sink == 0x9E3779B9u) atomicAdd(E.dropped, 1ULL);
  } else {
    for (uint32_t base = 0; base < len; base += 2 * kStep) {
      load(base + kStep, qb);
      if constexpr (IXR) count_quad(base, qa);
      else run(base, qa);
      load(base + 2 * kStep, qa);
      if constexpr (IXR) count_quad(base + kStep, qb);
      else run(base + kStep, qb);
    }
  }
  __syncthreads();
  if (IXR) {  // the deferred long durations
    const uint32_t nd = min(*dl_n, kXcDefer);
    for (uint32_t k = threadIdx.x; k < nd; k += kXcBlock) count(dl_s[k], E.span_long[dl_i[k]]);
    __syncthreads();
  }
  if (E.dbg) xc_stamp(E, kXcStamp + 2);
  if (E.dbg && threadIdx.x == 0) {  // (counts: tail records claimed, rare-path wave steps)
    E.dbg[blockIdx.x * kDbgPerWg + kXcStampTail] = tmisc[0];
    E.dbg[blockIdx.x * kDbgPerWg + kXcStampTail - 8] = tmisc[1];
    E.dbg[blockIdx.x * kDbgPerWg + kXcStampTail - 16] = *dl_n;
  }
  uint32_t *slab = E.xcslab + (uint64_t)blockIdx.x * xc_slab_stride(NE, M);
  if (!XC_ABL(4u))
    for (uint32_t i = threadIdx.x; i < NE * wpe; i += kXcBlock) slab[i] = cnt[i];
  if (E.dbg) xc_stamp(E, kXcStampSlab);
  if (!tail) {
    if (E.dbg) xc_stamp(E, kXcStamp + 3);
    return;
  }
  // the tail records leave by fold bin (slot / xt_bin_slots), each bin's run
  // at a fixed place (kXtRun records; a record past a full run takes its
  // bucket's HBM atomic), with the runs' lengths: the fold reads a run and
  // its length in one round trip
  const uint32_t nt = min(tmisc[0], kXtCap), nb = xt_bins(cap, M), bs = xt_bin_slots(M);
  uint32_t *hist = tmisc + 1;  // [nb] the runs' cursors
  for (uint32_t b = threadIdx.x; b < nb; b += kXcBlock) hist[b] = 0;
  __syncthreads();
  uint32_t *rec = E.xt_rec + (uint64_t)blockIdx.x * nb * kXtRun;
  for (uint32_t i = threadIdx.x; i < nt; i += kXcBlock) {
    const uint32_t v = trec[i], sl = v >> 12, b = sl / bs;
    const uint32_t r = atomicAdd(&hist[b], 1u);
    if (r < kXtRun) {
      rec[b * kXtRun + r] = v;
    } else {
      const uint32_t cur = ((uint32_t)meta[sl].x >> 8) & 1u;
      atomicAdd(E.buckets + ((uint64_t)cur * E.cap + sl) * M + (v & 0xFFFu), 1u);
    }
  }
  __syncthreads();
  uint32_t *off = E.xt_off + (uint64_t)blockIdx.x * (nb + 1);
  for (uint32_t b = threadIdx.x; b < nb; b += kXcBlock) off[b] = min(hist[b], kXtRun);
  if (E.dbg) xc_stamp(E, kXcStamp + 3);
}

// The counting kernel's tail records, one workgroup per fold bin (xt_bin_slots
// slots): every counting workgroup's run of the bin's records added in LDS
// ([bin slots][M] u32), then each non-zero cell added to its bucket -- one
// owner per slot (a slot is an entry in every workgroup or in none, so the
// slab fold never touches these slots), no atomics on HBM.
__device__ __forceinline__ void expo_fold_tail(const ExpoParams &E, uint32_t grid, uint32_t b, uint32_t *acc,
                                               uint32_t *cur) {
  const uint32_t M = E.max_size, nb = xt_bins(E.cap, M), bs = xt_bin_slots(M);
  for (uint32_t i = threadIdx.x; i < bs * M; i += 1024) acc[i] = 0;
  if (threadIdx.x < bs) {
    const uint64_t sl = (uint64_t)b * bs + threadIdx.x;
    cur[threadIdx.x] = sl < E.cap ? E.hdr[sl].cur : 0u;
  }
  __syncthreads();
  // wave w takes the counting workgroups w, w + 16, ...: every run's length
  // and records (64 lanes a run, at most kXtRun records) in flight together,
  // one round trip.  (Runs at offsets from a sorted list took two, and one
  // run at a time one per run in a row.)
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  constexpr uint32_t kPer = 16;  // counting workgroups per wave and batch (grid <= 256 in one batch)
  constexpr uint32_t kNoRec = 0xFFFFFFFFu;  // (a record's slot is < 2^11)
  static_assert(kXtRun == 64, "a run is one record per lane");
  auto add_rec = [&](uint32_t v) { atomicAdd(&acc[((v >> 12) % bs) * M + (v & 0xFFFu)], 1u); };
  for (uint32_t g0 = wave; g0 < grid; g0 += 16 * kPer) {
    uint32_t n[kPer], v[kPer];
#pragma unroll
    for (uint32_t u = 0; u < kPer; ++u) {
      const uint32_t g = g0 + u * 16;
      n[u] = g < grid ? E.xt_off[(uint64_t)g * (nb + 1) + b] : 0u;
      v[u] = g < grid ? E.xt_rec[((uint64_t)g * nb + b) * kXtRun + lane] : kNoRec;  // (past the run: stale, masked below)
    }
#pragma unroll
    for (uint32_t u = 0; u < kPer; ++u)
      if (lane < n[u]) add_rec(v[u]);
  }
  __syncthreads();
  // the non-zero cells: every bucket word read before the first is written
  // (a cell per thread per round, up to four rounds at C2's 16 x 160 cells;
  // one round trip instead of one per round -- each cell has one owner)
  constexpr uint32_t kR = 4;
  for (uint32_t i0 = 0; i0 < bs * M; i0 += kR * 1024) {
    uint32_t c[kR], old[kR];
    uint32_t *p[kR];
#pragma unroll
    for (uint32_t r = 0; r < kR; ++r) {
      const uint32_t i = i0 + r * 1024 + threadIdx.x;
      c[r] = i < bs * M ? acc[i] : 0u;
      const uint32_t k = i / M, sl = b * bs + k;
      p[r] = c[r] ? E.buckets + ((uint64_t)cur[k] * E.cap + sl) * M + i % M : nullptr;
      old[r] = c[r] ? *p[r] : 0u;
    }
#pragma unroll
    for (uint32_t r = 0; r < kR; ++r)
      if (c[r]) *p[r] = old[r] + c[r];
  }
}

// (entry words x 16 workgroup groups) per block of 1024 threads: four words
// a lane, 256 a block, so the slab blocks and the tail bins fit one resident
// round (C2: 126 + 128 blocks; one word a lane took ~3 rounds).  part: the
// 16 groups' sums, [16][64][8] u32 (the dynamic LDS).
constexpr size_t kXfPartBytes = 16 * 64 * 8 * 4;
__device__ __forceinline__ void expo_fold_slab(const ExpoParams &E, uint32_t grid, uint32_t blk, uint32_t *part) {
  const uint32_t M = E.max_size, wpe = (M + 1) / 2, total = E.xc_ne * wpe, stride = xc_slab_stride(E.xc_ne, M);
  const uint32_t wl = threadIdx.x & 63u, gq = threadIdx.x >> 6;
  const uint32_t w4 = blk * 256u + 4u * wl;  // the lane's first word
  const bool live = w4 < total;
  // the owner's chains (entry -> slot -> buffer) are read while the slab
  // words are in flight; the bucket words after the barrier (no other thread
  // of the fold touches them: a slot is an entry everywhere or nowhere)
  const bool own = gq == 0 && live;
  uint32_t slot[4] = {~0u, ~0u, ~0u, ~0u}, cur[4] = {}, q[4] = {};
  if (own) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (w4 + c < total) {
        q[c] = (w4 + c) % wpe;
        slot[c] = E.slot_of_entry[(w4 + c) / wpe];
      }
  }
  // grid <= 256 counting workgroups: at most 16 slab rows per thread, all in flight
  // (buffer loads: one lane offset, the row step in the scalar offset; rows
  // past the grid and lanes past the words read 0 through the bounds check)
  constexpr uint32_t kG = 16;
  const uint32_t nrec = min(grid, 256u) * stride * 4u;
  const __amdgpu_buffer_rsrc_t rs = rsrc(E.xcslab, nrec);
  const int vo = live ? (int)((gq * stride + w4) * 4u) : (int)0x80000000u;
  uint4 v[kG];
#pragma unroll
  for (uint32_t k = 0; k < kG; ++k) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b128(rs, vo, (int)(k * 16u * stride * 4u), 0);
    v[k] = make_uint4(x[0], x[1], x[2], x[3]);
  }
  if (own) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (slot[c] != ~0u) cur[c] = E.hdr[slot[c]].cur;
  }
  uint32_t lo[4] = {}, hi[4] = {};
#pragma unroll
  for (uint32_t k = 0; k < kG; ++k) {
    const uint32_t x[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      lo[c] += x[c] & 0xFFFFu;
      hi[c] += x[c] >> 16;
    }
  }
  // (grid > 256: the rest; the engine's grids do not get here)
  for (uint32_t g = gq + 16 * kG; g < grid && live; g += 16) {
    const uint4 y = *reinterpret_cast<const uint4 *>(E.xcslab + (uint64_t)g * stride + w4);
    const uint32_t x[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      lo[c] += x[c] & 0xFFFFu;
      hi[c] += x[c] >> 16;
    }
  }
  uint4 *pp = reinterpret_cast<uint4 *>(part) + (gq * 64u + wl) * 2u;
  pp[0] = make_uint4(lo[0], lo[1], lo[2], lo[3]);
  pp[1] = make_uint4(hi[0], hi[1], hi[2], hi[3]);
  __syncthreads();
  if (!own) return;
#pragma unroll 3
  for (uint32_t k = 1; k < 16; ++k) {
    const uint4 *o = reinterpret_cast<const uint4 *>(part) + (k * 64u + wl) * 2u;
    const uint4 l = o[0], h = o[1];
    lo[0] += l.x, lo[1] += l.y, lo[2] += l.z, lo[3] += l.w;
    hi[0] += h.x, hi[1] += h.y, hi[2] += h.z, hi[3] += h.w;
  }
  uint32_t *bp[4], b0[4] = {}, b1[4] = {};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    bp[c] = E.buckets + ((uint64_t)cur[c] * E.cap + (slot[c] == ~0u ? 0u : slot[c])) * M + 2 * q[c];
    if (slot[c] != ~0u && lo[c]) b0[c] = bp[c][0];
    if (slot[c] != ~0u && hi[c] && 2 * q[c] + 1 < M) b1[c] = bp[c][1];
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (slot[c] == ~0u) continue;
    if (lo[c]) bp[c][0] = b0[c] + lo[c];
    if (hi[c] && 2 * q[c] + 1 < M) bp[c][1] = b1[c] + hi[c];
  }
}

// One launch for both folds of a counting pass: blocks [0, slab_blocks) fold
// the entries' slabs, the rest one tail bin each (the two touch disjoint
// slots: a slot is an entry in every workgroup or in none)
__global__ __launch_bounds__(1024) void expo_fold_kernel(ExpoParams E, uint32_t grid, uint32_t slab_blocks) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // slab blocks: part; tail blocks: acc
  __shared__ uint32_t cur[kXtBinSlotsMax];
  if (blockIdx.x < slab_blocks) {
    if (!XC_ABL(8u)) expo_fold_slab(E, grid, blockIdx.x, reinterpret_cast<uint32_t *>(smem));  // (laboratory ablations: 8 / 16 skip a kind)
  } else if (!XC_ABL(16u)) {
    expo_fold_tail(E, grid, blockIdx.x - slab_blocks, reinterpret_cast<uint32_t *>(smem), cur);
  }
}

// Bucket counting with per-workgroup LDS privatisation: the slots' (scale,
// buffer) in LDS, and a cache of kXcEntries series (claimed first come, four
// probes from the slot's home, so a mix's frequent series hold them) whose
// max_size bucket counts are added in LDS and leave once per workgroup; spans
// of other series add to the HBM buckets directly.
// u16 cache counts (a workgroup takes at most 2^16 - 1 spans): 64 KiB, so two
// workgroups share a CU with the slot table
constexpr uint32_t kXcLdsBudget = 64 * 1024;
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
    int32_t ix;
    if (E.diag & 8u) ix = (int32_t)(d & 127u);
    else if ((E.diag & 4u) || !expo_index_fast(d, E.log2div_q24, m.x, ix)) ix = expo_index(expo_value(d, E.div), m.x);
    const uint32_t at = expo_mod(ix, M);
    uint32_t e = (((slot * 0x9E3779B1u) >> 16) & (NE / 4 - 1)) * 4, hit = kNotFound;  // home group of 4
#pragma unroll
    for (uint32_t k = 0; k < 4 && !(E.diag & 2u); ++k) {
      uint32_t t = tag[e + k];
      if (t == 0) t = atomicCAS(&tag[e + k], 0u, slot + 1);
      if (t == 0 || t == slot + 1) {
        hit = e + k;
        break;
      }
    }
    if (hit != kNotFound) atomicAdd(&cnt[(hit * M + at) >> 1], 1u << (((hit * M + at) & 1u) * 16));
    else if (!(E.diag & 1u)) atomicAdd(E.buckets + ((uint64_t)m.y * E.cap + slot) * M + at, 1u);
    else if (at == 0xFFFFFFFFu) E.buckets[0] = 0;  // keeps the index live
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
    if (E.xscale) E.xscale[s] = (int8_t)kExpoMaxScale;
  }
}

__global__ void expo_init_kernel(ExpoHdr *hdr, int8_t *xscale, uint64_t cap) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
    hdr[s] = expo_hdr_empty();
    if (xscale) xscale[s] = (int8_t)kExpoMaxScale;
  }
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

// the counting kernel's LDS: slot table, entries' counts, selection scratch,
// the tail record buffer and its bin histogram
static size_t xc_fixed_lds(uint64_t cap, uint32_t max_size) {
  return (size_t)cap * 8 + 256 + (size_t)kXtCap * 4 + 4 + xt_bins(cap, max_size) * 4 + (size_t)kXcDefer * 8 + 4;
}

uint32_t expo_slab_entries(uint64_t cap, uint32_t max_size, size_t budget) {
  const size_t fixed = xc_fixed_lds(cap, max_size), per = (size_t)((max_size + 1) / 2) * 4;
  if (budget <= fixed + per) return 0;
  return (uint32_t)std::min<size_t>(cap, (budget - fixed) / per);
}

size_t expo_slab_lds_bytes(uint64_t cap, uint32_t max_size, uint32_t ne) {
  return xc_fixed_lds(cap, max_size) + (size_t)ne * ((max_size + 1) / 2) * 4;
}

hipError_t prepare_expo_slab(size_t lds_bytes) {
#ifdef SPANAGG_AB
  for (const void *f : {(const void *)&expo_count_slab_kernel<0>, (const void *)&expo_count_slab_kernel<1>})
    if (hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
        e != hipSuccess)
      return e;
#endif
  if (hipError_t e = hipFuncSetAttribute((const void *)&expo_count_slab_kernel<2>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
      e != hipSuccess)
    return e;
  return hipFuncSetAttribute((const void *)&expo_fold_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)std::max<size_t>(kXfPartBytes, 8 * kExpoMaxSize * 4));  // (the largest bin x max_size)
}

size_t expo_count_lds_bytes(uint64_t cap, uint32_t max_size) {
  const uint32_t ne = xc_entries(max_size);
  return (size_t)cap * 8 + (size_t)ne * 4 + ((size_t)ne * max_size + 1) / 2 * 4;
}

hipError_t prepare_expo_count(size_t lds_bytes) {
  return hipFuncSetAttribute((const void *)&expo_count_cached_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)lds_bytes);
}

// 8 slots per reduce block (the laboratory build: SPANAGG_XR = 16 / 32 / 64)
void launch_reduce_rescale(const ExpoParams &E, hipStream_t s) {
#ifdef SPANAGG_AB
  static const uint32_t xr = [] {
    const char *v = std::getenv("SPANAGG_XR");
    const uint32_t x = v ? (uint32_t)std::atoi(v) : 8u;
    return x == 16 || x == 32 || x == 64 ? x : 8u;
  }();
  const dim3 g((uint32_t)((E.cap + xr - 1) / xr));
  if (xr == 8) hipLaunchKernelGGL(expo_reduce_rescale_kernel<8>, g, dim3(1024), 0, s, E);
  else if (xr == 16) hipLaunchKernelGGL(expo_reduce_rescale_kernel<16>, g, dim3(1024), 0, s, E);
  else if (xr == 32) hipLaunchKernelGGL(expo_reduce_rescale_kernel<32>, g, dim3(1024), 0, s, E);
  else hipLaunchKernelGGL(expo_reduce_rescale_kernel<64>, g, dim3(1024), 0, s, E);
#else
  hipLaunchKernelGGL(expo_reduce_rescale_kernel<8>, dim3((uint32_t)((E.cap + 7) / 8)), dim3(1024), 0, s, E);
#endif
}

hipError_t launch_expo_ingest(const ExpoParams &E, hipStream_t s) {
  if (E.n == 0) return hipSuccess;
  if (E.xslab && E.xc_ne) {  // small table, slab counting (E.xG workgroups, <= kXcMaxSpans spans each)
    // (the selection's two slots per thread; the span records' 12-bit slots)
    if (E.cap > 2048) return hipErrorInvalidValue;
    launch_reduce_rescale(E, s);
    // (a multiple of 4: the counting kernel's 16-B loads of four spans)
    const uint64_t per_wg = ((E.n + E.xG - 1) / E.xG + 3) / 4 * 4;
    if (per_wg > kXcMaxSpans) return hipErrorInvalidValue;  // (the engine splits batches below this)
    const uint32_t grid = (uint32_t)((E.n + per_wg - 1) / per_wg);
#ifdef SPANAGG_AB  // (slots + times, span records: laboratory build only, SPANAGG_XREC=0 / 1)
    if (!E.xidx && !E.span_rec)
      hipLaunchKernelGGL(expo_count_slab_kernel<0>, dim3(grid), dim3(kXcBlock),
                         expo_slab_lds_bytes(E.cap, E.max_size, E.xc_ne), s, E, per_wg);
    else if (!E.xidx)
      hipLaunchKernelGGL(expo_count_slab_kernel<1>, dim3(grid), dim3(kXcBlock),
                         expo_slab_lds_bytes(E.cap, E.max_size, E.xc_ne), s, E, per_wg);
    else
#endif
      hipLaunchKernelGGL(expo_count_slab_kernel<2>, dim3(grid), dim3(kXcBlock),
                         expo_slab_lds_bytes(E.cap, E.max_size, E.xc_ne), s, E, per_wg);
    const uint32_t words = E.xc_ne * ((E.max_size + 1) / 2), slab_blocks = (words + 255) / 256;
    const uint32_t tail_blocks = E.xt_rec ? xt_bins(E.cap, E.max_size) : 0u;
    const size_t lds = std::max<size_t>(kXfPartBytes, tail_blocks ? (size_t)xt_bin_slots(E.max_size) * E.max_size * 4 : 0);
    hipLaunchKernelGGL(expo_fold_kernel, dim3(slab_blocks + tail_blocks), dim3(1024), lds, s, E, grid, slab_blocks);
    return hipGetLastError();
  }
  if (E.xslab) {  // small table: the ingest kernel left header partials and slots
    launch_reduce_rescale(E, s);
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

hipError_t launch_expo_init(ExpoHdr *hdr, int8_t *xscale, uint64_t cap, hipStream_t s) {
  hipLaunchKernelGGL(expo_init_kernel, dim3(grid_of(cap)), dim3(256), 0, s, hdr, xscale, cap);
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

// (tests) |v_log_f32(m) - log2(m)| over the floats m = 1 + i * 2^-23, i in
// [i0, i0 + n): the per-block maxima, as doubles
__global__ __launch_bounds__(256) void log2_err_probe_kernel(uint32_t i0, uint32_t n, double *block_max) {
  __shared__ double red[256];
  double mx = 0;
  for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
    const float m = 1.0f + (float)(i0 + i) * 0x1p-23f;
    const double err = fabs((double)__builtin_amdgcn_logf(m) - log2((double)m));
    mx = err > mx ? err : mx;
  }
  red[threadIdx.x] = mx;
  __syncthreads();
  for (uint32_t o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o && red[threadIdx.x + o] > red[threadIdx.x]) red[threadIdx.x] = red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) block_max[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(256) void expo_fast_probe_kernel(const uint64_t *d, const int32_t *scale, uint64_t n,
                                                             double div, int32_t l2d_q24, int32_t *fast,
                                                             int32_t *exact) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    int32_t ix;
    fast[i] = expo_index_fast(d[i], l2d_q24, scale[i], ix) ? ix : INT32_MIN;
    exact[i] = expo_index(expo_value(d[i], div), scale[i]);
  }
}

hipError_t launch_expo_fast_probe(const uint64_t *d, const int32_t *scale, uint64_t n, double div, int32_t *fast,
                                  int32_t *exact, hipStream_t s) {
  hipLaunchKernelGGL(expo_fast_probe_kernel, dim3(grid_of(n)), dim3(256), 0, s, d, scale, n, div, expo_l2d_q24(div), fast,
                     exact);
  return hipGetLastError();
}

hipError_t launch_log2_err_probe(uint32_t i0, uint32_t n, double *block_max, uint32_t blocks, hipStream_t s) {
  hipLaunchKernelGGL(log2_err_probe_kernel, dim3(blocks), dim3(256), 0, s, i0, n, block_max);
  return hipGetLastError();
}

hipError_t launch_expo_probe(const double *v, const int32_t *scale, int32_t *idx_out, double *log_out, uint64_t n,
                             hipStream_t s) {
  hipLaunchKernelGGL(expo_index_probe_kernel, dim3(grid_of(n)), dim3(256), 0, s, v, scale, idx_out, n);
  hipLaunchKernelGGL(go_log_probe_kernel, dim3(grid_of(n)), dim3(256), 0, s, v, log_out, n);
  return hipGetLastError();
}

}  // namespace sa
