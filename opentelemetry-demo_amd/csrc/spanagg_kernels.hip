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
#include <algorithm>
#include <cstdlib>

#include "sa_device.h"

namespace sa {
namespace {

// ---------------------------------------------------------------------------
// Small-table path.  LDS layout (dynamic, 16-B aligned):
//   lkeys [cap] u64   mirror of the HBM key table (same slot positions)
//   lsum  [cap] u64   per-slot ns sum of this epoch
//   lcnt  [cap][nw] u32, nw = ceil(nbk/2): two u16 bucket counters per word
// The workgroup's HBM slab is [cap][2*nw] u32 (+ [cap] u64 sums): LDS word w
// maps to slab cells 2w and 2w+1, so a pair of LDS words is one 16-B slab
// vector and the flush is a vectorised read-modify-write of touched cells.
__device__ __forceinline__ void flush_lds(const IngestParams &P, uint32_t cap, uint32_t nw,
                                          unsigned long long *lsum, uint32_t *lcnt) {
  if (P.diag & 8u) return;
  uint4 *scnt = reinterpret_cast<uint4 *>(P.slab_cnt + (uint64_t)blockIdx.x * cap * 2 * nw);
  uint2 *lw = reinterpret_cast<uint2 *>(lcnt);
  const uint32_t pairs = cap * nw / 2;
  constexpr int U = 5;  // two rounds of loads for cap 2048 x nw 9 at 1,024 threads
  for (uint32_t k0 = threadIdx.x; k0 < pairs; k0 += U * blockDim.x) {
    uint2 w[U];
    uint4 g[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t k = k0 + u * blockDim.x;
      w[u] = k < pairs ? lw[k] : make_uint2(0, 0);
      g[u] = (w[u].x | w[u].y) ? scnt[k] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t k = k0 + u * blockDim.x;
      if (w[u].x | w[u].y) {
        g[u].x += w[u].x & 0xFFFFu;
        g[u].y += w[u].x >> 16;
        g[u].z += w[u].y & 0xFFFFu;
        g[u].w += w[u].y >> 16;
        scnt[k] = g[u];
        lw[k] = make_uint2(0, 0);
      }
    }
  }
  ulonglong2 *ss = reinterpret_cast<ulonglong2 *>(P.slab_sum + (uint64_t)blockIdx.x * cap);
  ulonglong2 *ls = reinterpret_cast<ulonglong2 *>(lsum);
  for (uint32_t k = threadIdx.x; k < cap / 2; k += blockDim.x) {
    const ulonglong2 v = ls[k];
    if (v.x | v.y) {
      ulonglong2 g = ss[k];
      g.x += v.x;
      g.y += v.y;
      ss[k] = g;
      ls[k] = make_ulonglong2(0, 0);
    }
  }
}

// End-of-launch write-back of ingest_v2_kernel for a compile-time geometry
// (UPT slab-count pairs and SPT slab-sum pairs per thread), in two phases.
//
// v2_epi_pre runs in each wave right after its own loop, before the
// workgroup barrier: it loads the thread's slab-count and slab-sum words (all
// of them: which ones the launch touched is known only after the barrier) and
// the lower-bound sub-block of its wave.  The slabs are this workgroup's own
// (no other workgroup of the launch writes them; the previous launch of the
// slab set has completed), and a stale register read for the bound can only
// lower it, which keeps it a lower bound.  Waves end their loops up to ~10 us
// apart, so these loads land while the last waves still work.
//
// v2_epilogue runs after the barrier: LDS counters plus the prefetched words
// -> dependent stores of the touched words, the ERROR counts as no-return
// atomics on the workgroup's private ERROR slab, and the queued HLL raises as
// CAS from the register word each span saw in the loop (queued beside it), so
// the only memory round trip left after the barrier is a raise's CAS (one
// more when another workgroup changed the word since).  Before, the slab, ERROR
// and HLL words were read after the barrier: two round trips.  (The EXPO
// kernel's epilogue shares the raise and bound halves.)

// After the barrier: the queued HLL raises, each a CAS from the register word
// its span saw in the loop (hqv), and the bound from the prefetched quads.
template <uint32_t B, uint32_t Q, typename PT>
__device__ __forceinline__ void epi_raise_and_bound(const PT &P, const uint2 *hq, const uint32_t *hqv, uint32_t nq,
                                                    const uint4 (&lv)[4]) {
  const uint32_t tid = threadIdx.x;
  constexpr uint32_t kQ = Q / B;
#pragma unroll
  for (uint32_t i = 0; i < kQ; ++i) {
    if (tid + i * B >= nq) continue;
    const uint2 q = hq[tid + i * B];
    SA_GLOBAL uint32_t *word = gbl(reinterpret_cast<uint32_t *>(P.hll + (q.x & ~3u)));
    const uint32_t sh = (q.x & 3u) * 8;
    uint32_t old = hqv[tid + i * B];
    while (((old >> sh) & 0xFFu) < q.y) {  // a failed CAS refreshes `old`
      const uint32_t nw = (old & ~(0xFFu << sh)) | (q.y << sh);
      if (__hip_atomic_compare_exchange_strong(word, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT))
        break;
    }
  }
  hll_lb_finish<B>(P, lv);
}

template <int UPT, int SPT>
struct EpiPre {
  uint4 g[UPT];
  ulonglong2 sg[SPT];
  uint4 lv[4];
};

template <int UPT, int SPT, uint32_t B, typename PT>
__device__ __forceinline__ void v2_epi_pre(const PT &P, uint32_t cap, uint32_t nw, EpiPre<UPT, SPT> &x) {
  const uint32_t tid = threadIdx.x;
  const uint4 *scnt = reinterpret_cast<const uint4 *>(P.slab_cnt + (uint64_t)blockIdx.x * cap * 2 * nw);
#pragma unroll
  for (int u = 0; u < UPT; ++u) x.g[u] = scnt[tid + u * B];
  const ulonglong2 *ss = reinterpret_cast<const ulonglong2 *>(P.slab_sum + (uint64_t)blockIdx.x * cap);
#pragma unroll
  for (int u = 0; u < SPT; ++u) x.sg[u] = ss[tid + u * B];
  hll_lb_pre<B>(P, x.lv);
}

template <int UPT, int SPT, uint32_t B, uint32_t Q, typename PT>
__device__ __forceinline__ void v2_epilogue(const PT &P, uint32_t cap, uint32_t nw, uint32_t log2cap,
                                            const unsigned long long *lsum, const uint32_t *lcnt,
                                            const uint32_t *etab, bool err_lds, const uint2 *hq,
                                            const uint32_t *hqv, uint32_t nq, const EpiPre<UPT, SPT> &x) {
  const uint32_t tid = threadIdx.x;
  const bool slabs = !(P.diag & 8u);
  uint4 *scnt = reinterpret_cast<uint4 *>(P.slab_cnt + (uint64_t)blockIdx.x * cap * 2 * nw);
  const uint2 *lw = reinterpret_cast<const uint2 *>(lcnt);
#pragma unroll
  for (int u = 0; u < UPT; ++u) {
    const uint2 w = slabs ? lw[tid + u * B] : make_uint2(0, 0);
    if (w.x | w.y) {
      uint4 g = x.g[u];
      g.x += w.x & 0xFFFFu;
      g.y += w.x >> 16;
      g.z += w.y & 0xFFFFu;
      g.w += w.y >> 16;
      scnt[tid + u * B] = g;
    }
  }
  ulonglong2 *ss = reinterpret_cast<ulonglong2 *>(P.slab_sum + (uint64_t)blockIdx.x * cap);
  const ulonglong2 *ls = reinterpret_cast<const ulonglong2 *>(lsum);
#pragma unroll
  for (int u = 0; u < SPT; ++u) {
    const ulonglong2 sv = slabs ? ls[tid + u * B] : make_ulonglong2(0, 0);
    if (sv.x | sv.y) ss[tid + u * B] = make_ulonglong2(x.sg[u].x + sv.x, x.sg[u].y + sv.y);
  }
  constexpr uint32_t kE = kErrTab / B;  // ERROR table entries per thread
#pragma unroll
  for (uint32_t i = 0; i < kE; ++i) {
    const uint32_t e = err_lds ? etab[tid + i * B] : 0u;
    if (e)
      atomicAdd(P.errslab + (uint64_t)blockIdx.x * ((uint64_t)P.n_windows << log2cap) + ((e >> 16) - 1),
                e & 0xFFFFu);
  }
  epi_raise_and_bound<B, Q>(P, hq, hqv, nq, x.lv);
}

// Probe the LDS key mirror along the key's sequence from position i0 (the
// earlier positions are known not to hold `key`); returns the slot or
// kNotFound (empty slot reached / probe limit).
__device__ __forceinline__ uint32_t lds_probe_rest(const unsigned long long *lkeys, uint64_t key,
                                                   uint32_t log2cap, uint32_t i0,
                                                   uint32_t max_probe) {
  const ProbeSeq pr = probe_seq(key, log2cap);
  for (uint32_t i = i0; i < max_probe; ++i) {
    const uint32_t s = seq_slot(pr, i);
    const unsigned long long kk = lkeys[s];
    if (kk == key) return s;
    if (kk == 0) break;
  }
  return kNotFound;
}

// Small-table path (key table mirrored in LDS), 1,024 threads, S spans per
// lane per tile.  Per tile:
//   1. wait for the tile, compact it to (key, duration, bucket, HLL offset,
//      rho, window slot) -- the raw 44 B/span registers are then free;
//   2. S LDS key probes back to back -> key-table slots;
//   3. ERROR spans: one no-return atomic on the exact (window, slot) counter;
//   4. issue the S HLL register reads;
//   5. PF: prefetch the next tile into the freed tile registers, then the LDS
//      counter / sum atomics;
//   6. HLL compare (a counted vmcnt: the prefetch stays in flight); a register
//      that grows is queued in LDS and raised after the loop, so no returning
//      global atomic (and its vmcnt(0)) sits in the loop.
// BK: 1 = bucket by the LDS bin table, 0 = linear thresholds.  DIAG: honour
// the SA_DIAG_* ablation bits (profiling builds only).
// LDS: lkeys[cap] u64 | lsum[cap] u64 | lcnt[cap][nw] u32 | hq[kHllQueue] u64 |
//      hq_n (16 B) | bins[kBins]
template <int BK, int S, bool PF, bool DIAG, int AUX = 0>
__global__ __launch_bounds__(kLdsBlock) void ingest_lds_kernel(IngestParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (DIAG && P.dbg && threadIdx.x == 0) P.dbg[blockIdx.x * kDbgPerWg + 0] = __builtin_amdgcn_s_memrealtime();
  const uint32_t cap = 1u << P.log2cap;
  const uint32_t nbk = P.nbk;
  const uint32_t nw = (nbk + 1) >> 1;
  const uint32_t diag = DIAG ? P.diag : 0u;
  unsigned long long *lkeys = reinterpret_cast<unsigned long long *>(smem);
  unsigned long long *lsum = lkeys + cap;
  uint32_t *lcnt = reinterpret_cast<uint32_t *>(lsum + cap);
  uint2 *hq = reinterpret_cast<uint2 *>(lcnt + cap * nw);
  uint32_t *hq_n = reinterpret_cast<uint32_t *>(hq + kHllQueue);
  BinEntry *lbins = reinterpret_cast<BinEntry *>(hq_n + 4);

  uint64_t lo, hi;
  wg_range(P.n, lo, hi);
  const Cols c = make_cols(P, lo, hi);
  const uint32_t len = (uint32_t)(hi - lo);
  const uint32_t tile = kLdsBlock * S;
  uint32_t off = threadIdx.x * S;

  // Key-table (and bin-table) loads first, then the first tile's loads: the
  // LDS setup waits only for the keys (vmcnt counts in issue order).
  unsigned long long kv[8];
  const uint32_t per = (cap + kLdsBlock - 1) / kLdsBlock;  // <= 8 for cap <= 8192
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const uint32_t i = threadIdx.x + u * kLdsBlock;
    kv[u] = (u < (int)per && i < cap)
                ? __hip_atomic_load(&P.gkeys[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                : 0ULL;
  }
  uint4 bv = make_uint4(0, 0, 0, 0);
  if (BK == 1 && threadIdx.x < kBins * 2) bv = reinterpret_cast<const uint4 *>(P.bintab)[threadIdx.x];
  SpanTile<S> cur;
  load_tile<S, AUX>(c, off, len, cur);
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const uint32_t i = threadIdx.x + u * kLdsBlock;
    if (u < (int)per && i < cap) {
      lkeys[i] = kv[u];
      lsum[i] = 0;
    }
  }
  if (BK == 1 && threadIdx.x < kBins * 2) reinterpret_cast<uint4 *>(lbins)[threadIdx.x] = bv;
  for (uint32_t i = threadIdx.x; i < cap * nw; i += kLdsBlock) lcnt[i] = 0;
  if (threadIdx.x == 0) *hq_n = 0;
  __syncthreads();
  if (DIAG && P.dbg && threadIdx.x == 0) P.dbg[blockIdx.x * kDbgPerWg + 1] = __builtin_amdgcn_s_memrealtime();

  LaneStats st{0, 0, 0, 0};
  uint32_t in_epoch = 0;
  for (uint32_t t0 = 0; t0 < len; t0 += tile, off += tile) {
    // 1. compact the landed tile; info = bucket | rho << 6 | err << 13 | ws << 14
    //    (bucket < 64, rho <= 65, ws < 4096 window slots)
    uint64_t key[S], dur[S];
    uint32_t hoff[S], info[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const bool valid = j < cur.cnt;
      key[j] = valid ? cur.key[j] : 0;
      st.zero_key += (valid && cur.key[j] == 0) ? 1u : 0u;
      dur[j] = cur.e[j] > cur.s[j] ? cur.e[j] - cur.s[j] : 0;
      const uint32_t bkt = bucket_lds<BK>(dur[j], lbins, P);
      const uint32_t svc = cur.meta[j] & 0xFFFFu;
      const bool svc_ok = svc < P.n_services;
      const uint32_t ws = window_slot(P, cur.e[j]);
      const bool win_ok = ws != 0xFFFFFFFFu;
      st.bad_svc += (valid && !svc_ok) ? 1u : 0u;
      st.oor += (valid && svc_ok && !win_ok) ? 1u : 0u;
      const bool sk = valid && svc_ok && win_ok;
      const uint32_t err = (sk && ((cur.meta[j] >> 19) & 3u) == 2u && !(diag & 4u)) ? 1u : 0u;
      uint32_t rho = 0;
      hoff[j] = 0;
      if (sk && !(diag & 2u)) {
        const uint64_t x = xxh64_16(cur.a[j], cur.b[j]);
        rho = (uint32_t)__clzll((long long)((x << P.p) | (1ULL << (P.p - 1)))) + 1;
        hoff[j] = (((ws * P.n_services + svc) << P.p) + (uint32_t)(x >> (64 - P.p)));
      }
      info[j] = bkt | (rho << 6) | (err << 13) | ((ws & 4095u) << 14);
    }
    // 2. RED lookup: S LDS probes back to back (key no longer needed after)
    uint32_t found[S];
    if (!(diag & 1u)) {
      uint32_t sl[S];
      unsigned long long k0[S];
#pragma unroll
      for (int j = 0; j < S; ++j) {
        sl[j] = probe_seq(key[j], P.log2cap).b1 * 4;
        k0[j] = lkeys[sl[j]];
      }
#pragma unroll
      for (int j = 0; j < S; ++j) {
        found[j] = kNotFound;
        if (key[j] != 0) {
          found[j] = k0[j] == key[j] ? sl[j]
                     : k0[j] == 0    ? kNotFound
                                     : lds_probe_rest(lkeys, key[j], P.log2cap, 1, P.max_probe);
          if (found[j] == kNotFound) {
            found[j] = g_find_insert(P.gkeys, key[j], P.log2cap, P.max_probe);
            if (found[j] != kNotFound) lkeys[found[j]] = key[j];
          }
          st.dropped += found[j] == kNotFound ? 1u : 0u;
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < S; ++j) {
        found[j] = kNotFound;
        st.dropped += (uint32_t)(((key[j] ^ dur[j] ^ info[j]) & 0xFFFFFFFFFFFFULL) == 0x123456789ABCULL);
      }
    }
    // 3. error counts: exact per (window, slot) -- one no-return atomic,
    //    issued before the prefetch so the loop-top wait never covers it;
    //    spans without a slot update the count-min cells directly
#pragma unroll
    for (int j = 0; j < S; ++j) {
      if (info[j] & (1u << 13)) {
        if (found[j] != kNotFound)
          atomicAdd(P.errcnt + (((uint64_t)(info[j] >> 14)) << P.log2cap) + found[j], 1ULL);
        else
          cms_add(P, info[j] >> 14, key[j], 1ULL);
      }
    }
    // 4. HLL register reads (unconditional: offset 0 when unused)
    uint32_t hv[S];
#pragma unroll
    for (int j = 0; j < S; ++j)
      hv[j] = *reinterpret_cast<const uint32_t *>(P.hll + (hoff[j] & ~3u));
    // 5. prefetch the next tile
    if constexpr (PF) {
      __builtin_amdgcn_sched_barrier(0);
      load_tile<S, AUX>(c, off + tile, len, cur);
      __builtin_amdgcn_sched_barrier(0);
    }
    // 5b. RED update: LDS u16 bucket counter + u64 ns sum
#pragma unroll
    for (int j = 0; j < S; ++j) {
      if (found[j] != kNotFound) {
        const uint32_t b = info[j] & 63u;
        atomicAdd(&lcnt[found[j] * nw + (b >> 1)], 1u << ((b & 1) * 16));
        atomicAdd(&lsum[found[j]], (unsigned long long)dur[j]);
      }
    }
    // 6. HLL: queue the registers that grow
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const uint32_t rho = (info[j] >> 6) & 127u;
      if ((hv[j] & 0xFFu) < rho) {
        const uint32_t q = atomicAdd(hq_n, 1u);
        if (q < kHllQueue) hq[q] = make_uint2(hoff[j], rho);
        else hll_raise(P.hll + hoff[j], rho);
      }
    }
    if constexpr (!PF) load_tile<S, AUX>(c, off + tile, len, cur);
    if (++in_epoch == P.epoch_tiles) {  // u16 LDS counters: flush before they can wrap
      __syncthreads();
      flush_lds(P, cap, nw, lsum, lcnt);
      __syncthreads();
      in_epoch = 0;
    }
  }
  if (DIAG && P.dbg && threadIdx.x == 0) P.dbg[blockIdx.x * kDbgPerWg + 2] = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  flush_lds(P, cap, nw, lsum, lcnt);
  const uint32_t nq = *hq_n < kHllQueue ? *hq_n : kHllQueue;
  for (uint32_t i = threadIdx.x; i < nq; i += kLdsBlock) hll_raise(P.hll + hq[i].x, hq[i].y);
  if (DIAG && P.dbg && threadIdx.x == 0) P.dbg[blockIdx.x * kDbgPerWg + 3] = __builtin_amdgcn_s_memrealtime();
  flush_stats(P, st);
}

// ---------------------------------------------------------------------------
// Small-table path, v2.  Same LDS layout and slab flush as ingest_lds_kernel;
// the span loop is rebuilt for latency tolerance at 16 waves per CU:
//   * NBUF tiles of S spans per lane in flight per wave (a register ring): a
//     tile is re-filled right after it is compacted, so every wave keeps
//     loads outstanding while it computes;
//   * the key lookup reads the key's two 4-slot buckets from the LDS mirror
//     (4 x 16-B reads, fixed cost, no probe loop); only keys outside their two
//     buckets (a few % of a 0.7-load table, none at all after the first
//     launch for C2) take the wave-uniform cold path;
//   * HLL register reads are issued one step ahead of their compare, so the
//     wait for them is a counted vmcnt that leaves two tiles in flight;
//   * event statistics are per-wave ballot counts (scalar registers).
// LDS: lkeys[cap] u64 | lsum[cap] u64 | lcnt[cap][nw] u32 | hq[kHllQueue] u64 |
//      hq_n (16 B) | bins[kBins]
// Wave-cooperative find-or-insert of ONE (wave-uniform) key: the 64 lanes
// test 64 consecutive positions of its probe sequence at once, first in the
// LDS mirror, then in the HBM table (where the first empty position is
// claimed by CAS).  No divergent loop, so no per-lane exec-mask nesting.
// Must be called with all lanes active; returns the slot (uniform) or
// kNotFound when the table is full.
__device__ __forceinline__ uint32_t wave_find_insert(unsigned long long *lkeys, uint64_t k,
                                                     uint32_t log2cap) {
  SA_CONST const IngestParams &Q = cold_params();
  const uint32_t lane = threadIdx.x & 63;
  const ProbeSeq pr = probe_seq(k, log2cap);
  const uint32_t maxp = Q.max_probe;
  for (uint32_t i0 = 0; i0 < maxp; i0 += 64) {  // LDS mirror
    const uint32_t pos = i0 + lane;
    const uint32_t sl = seq_slot(pr, pos < maxp ? pos : maxp - 1);
    const unsigned long long v = lkeys[sl];
    const uint64_t mh = __ballot(v == k), me = __ballot(v == 0);
    if (mh | me) {
      if (mh && (!me || __builtin_ctzll(mh) < __builtin_ctzll(me)))
        return (uint32_t)__builtin_amdgcn_readlane((int)sl, __builtin_ctzll(mh));
      break;
    }
  }
  SA_GLOBAL unsigned long long *gk = gbl(Q.gkeys);
  for (uint32_t i0 = 0; i0 < maxp;) {  // HBM table
    const uint32_t pos = i0 + lane;
    const uint32_t sl = seq_slot(pr, pos < maxp ? pos : maxp - 1);
    const unsigned long long v = __hip_atomic_load(&gk[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t mh = __ballot(v == k), me = __ballot(v == 0 && pos < maxp);
    if (!(mh | me)) {
      i0 += 64;
      continue;
    }
    const int first = __builtin_ctzll(mh | me);
    const uint32_t fsl = (uint32_t)__builtin_amdgcn_readlane((int)sl, first);
    if ((mh >> first) & 1) {
      lkeys[fsl] = k;
      return fsl;
    }
    unsigned long long prev = 0;
    if ((int)lane == first) {
      unsigned long long expect = 0;
      __hip_atomic_compare_exchange_strong(&gk[fsl], &expect, (unsigned long long)k,
                                           __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      prev = expect;
    }
    const uint32_t plo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)prev, first);
    const uint32_t phi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(prev >> 32), first);
    const uint64_t pv = ((uint64_t)phi << 32) | plo;
    if (pv == 0 || pv == k) {
      lkeys[fsl] = k;
      return fsl;
    }
    i0 += (uint32_t)first;  // lost the race for that slot: re-read from it
  }
  return kNotFound;
}

// Resolves the lanes with `need` one distinct key at a time (lanes sharing a
// key are resolved together); call with all lanes active.
__device__ __forceinline__ void cold_lookup_wave(unsigned long long *lkeys, bool need, uint64_t key,
                                                 uint32_t log2cap, uint32_t &found, uint32_t *ltag = nullptr) {
  uint64_t m = __ballot(need);
  while (m) {
    const int l = __builtin_ctzll(m);
    const uint32_t klo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, l);
    const uint32_t khi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(key >> 32), l);
    const uint64_t k = ((uint64_t)khi << 32) | klo;
    const uint32_t f = wave_find_insert(lkeys, k, log2cap);
    if (ltag && f != kNotFound && (threadIdx.x & 63u) == 0) ltag[f] = key_tag(k);  // (the mirror's tag of the slot)
    const bool same = need && key == k;
    found = same ? f : found;
    m &= ~__ballot(same);
  }
}

// Adds one ERROR span of (window slot, key slot) key `ek` (< 65535) to the
// workgroup's LDS table: 256 aligned groups of 4 entries {(ek + 1) << 16 |
// count}; false when the key's group is taken by other keys (the caller then
// falls back to a global atomic).  The common case -- the key already in its
// group -- is one ds_read_b128, four compares and one ds_add; the claim loop
// runs once per key per workgroup.  (A linear 4-probe loop with a CAS per
// probe compiled to ~100 mostly scalar instructions per wave step: 2 % of
// spans are ERROR, so nearly every 128-span wave step has one.)
__device__ __forceinline__ bool lds_err_add(uint32_t *etab, uint32_t ek) {
  const uint32_t tag = (ek + 1) << 16;
  uint32_t *grp = etab + ((ek * 0x9E3779B1u) >> (32 - 8)) * 4;  // kErrTab = 1024
  const uint4 v = *reinterpret_cast<const uint4 *>(grp);
  const int at = (v.x & 0xFFFF0000u) == tag   ? 0
                 : (v.y & 0xFFFF0000u) == tag ? 1
                 : (v.z & 0xFFFF0000u) == tag ? 2
                 : (v.w & 0xFFFF0000u) == tag ? 3
                                              : -1;
  if (__builtin_expect(at >= 0, 1)) {
    atomicAdd(grp + at, 1u);
    return true;
  }
  for (int q = 0; q < 4; ++q) {
    uint32_t w = grp[q];
    if (w == 0) {
      w = atomicCAS(grp + q, 0u, tag | 1u);
      if (w == 0) return true;
    }
    if ((w & 0xFFFF0000u) == tag) {
      atomicAdd(grp + q, 1u);
      return true;
    }
  }
  return false;
}

// LC / NWC / PC: table log2 capacity, counter words per slot and HLL precision
// fixed at compile time for the common geometry (0 = read from P).
// HAUX >= 0: HLL register reads as buffer loads with that cache policy (gfx950:
// 1 = sc0, 2 = nt, 16 = sc1); -1 = plain global loads.
// DYN: inside the workgroup's range, waves claim chunks of NBUF wave-tiles
// from an LDS counter instead of owning a fixed slice of every workgroup
// tile, so waves the memory arbiter serves late simply take fewer chunks and
// all 16 finish together (the fixed split left the 4 youngest waves of every
// workgroup streaming alone for the last ~25% of the launch).  A grid-wide
// counter in HBM was tried first: its returning atomic put a vmcnt(0) at the
// top of every round and ran 3.4x slower.
// OPT (DYN only): bit 0 = every wave issues its key-table loads before any
// wave issues tile loads (a workgroup barrier between them), so the LDS setup
// does not wait behind the other waves' first tiles; bit 1 = claims of one
// wave tile instead of NBUF (a round takes NBUF claims), halving the work a
// wave can still hold when its neighbours run out.
// LEAN: the span hash on 32-bit halves (xxh64_16_h), rho / register index
// without 64-bit shifts, the register row offset by a 24-bit multiply.
// EXPO: exponential-histogram engines (spanagg_expo.hip does the buckets).
// The RED update becomes per-slot LDS header partials -- count, zero count,
// ns sum, max of ~d and max d over positive durations (XHdr) -- in the space
// of lsum + lcnt (nw = 6: 32 B per slot), written to the workgroup's header
// slab at the end; every span's key slot goes to P.slot_of for the
// bucket-counting pass.
// A wave's claim of the next chunk from an LDS counter kept in units of
// 1/64 chunk.  Every lane adds the same 1 (no branch: a divergent claim made
// the compiler wait for it at the join), so the atomic optimizer issues one
// ds_add_rtn of popcount(exec) = 64 and hands the lanes base + rank; the first
// lane's base / 64 is the claim.  (A lane-varying addend -- 1 on lane 0, 0
// elsewhere -- compiled to a 64-iteration readlane/writelane scan loop per
// claim: ~140 scalar and ~30 vector instructions per span-lane of the C2 loop.)
// Requires a full wave at the call, which the claim loops have.
__device__ __forceinline__ uint32_t wave_claim(uint32_t *ctr) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)atomicAdd(ctr, 1u)) >> 6;
}

// the scale read of the index records (the laboratory's SPANAGG_XIDX_OFF=3
// ablation skips it; the product build always reads it)
#ifdef SPANAGG_AB
#define SA_XIDX_SCALE(P) ((P).xidx != 3)
#else
#define SA_XIDX_SCALE(P) true
#endif

//
// The kernel's template: its geometry (LC = log2 slots, NWC = counter words
// per slot, PC = HLL precision; 0 = read from P), EXPO, the block size and an
// option set O (S spans per lane per step, NBUF tiles in flight, AUX cache
// policy, DYN / OPT / EPI / LEAN above).  The product's two option sets are
// V2Lean (the default table and every EXPO engine) and V2Plain; the
// laboratory's switches (DIAG ablations, TAG, POOL, the A/B sets) are defined
// in lab/small_lab.inc, which only the laboratory build compiles.
struct V2Plain {  // variant 15: chunk claims only
  static constexpr int S = 2, NBUF = 2, AUX = 2, HAUX = -1, OPT = 0;
  static constexpr bool DYN = true, EPI = false, LEAN = false, DIAG = false, TAG = false, POOL = false;
};
struct V2Lean : V2Plain {  // variant 20: + prologue barrier, LDS event counters, lean hash, two-phase epilogue
  static constexpr int OPT = 1;
  static constexpr bool EPI = true, LEAN = true;
};
template <int LC, int NWC, int PC, bool EXPO, uint32_t BLK, typename O>
__global__ __launch_bounds__(BLK) void ingest_v2_kernel(IngestParams P) {
  constexpr int S = O::S, NBUF = O::NBUF, AUX = O::AUX, HAUX = O::HAUX, OPT = O::OPT;
  constexpr bool DYN = O::DYN, EPI = O::EPI, LEAN = O::LEAN, DIAG = O::DIAG, TAG = O::TAG, POOL = O::POOL;
#ifndef SPANAGG_AB
  static_assert(!DIAG && !TAG && !POOL, "laboratory switches: libspanagg_ab.so only");
#endif
  static_assert(BLK % 64 == 0 && kErrTab % BLK == 0 && kHllQueue % BLK == 0 && BLK * 4 >= kLbMaxSub, "block size");
  static_assert(!POOL || (DYN && !(OPT & 2)), "the tail pool extends the chunk claims");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (P.dbg && threadIdx.x == 0) P.dbg[blockIdx.x * kDbgPerWg + 0] = __builtin_amdgcn_s_memrealtime();
  const uint32_t log2cap = LC ? (uint32_t)LC : P.log2cap;
  const uint32_t cap = 1u << log2cap;
  const uint32_t nw = EXPO ? 6u : NWC ? (uint32_t)NWC : (P.nbk + 1) >> 1;
  const uint32_t hp = PC ? (uint32_t)PC : P.p;
  const uint32_t diag = DIAG ? P.diag : 0u;
  unsigned long long *lkeys = reinterpret_cast<unsigned long long *>(smem);
  unsigned long long *lsum = lkeys + cap;
  uint32_t *lcnt = reinterpret_cast<uint32_t *>(lsum + cap);
  uint2 *hq = reinterpret_cast<uint2 *>(lcnt + cap * nw);
  uint32_t *hq_n = reinterpret_cast<uint32_t *>(hq + kHllQueue);
  // the compile-time-geometry epilogue (v2_epilogue) raises from the word each
  // span saw: the queue region holds kQcap (hoff, rho) pairs, then their words
  constexpr bool kObs = (LC != 0 && NWC != 0 && EPI) || EXPO;
  constexpr uint32_t kQcap = kObs ? kHllQueue / 2 : kHllQueue;
  static_assert(!kObs || kQcap * 12 <= kHllQueue * 8, "queue region");
  uint32_t *hqv = reinterpret_cast<uint32_t *>(hq + kQcap);
  uint32_t *lstat = hq_n + 4;  // EPI: [4] event counts (zero key, bad service, out of ring, dropped)
  BinEntry *lbins = reinterpret_cast<BinEntry *>(hq_n + 8);
  uint32_t *etab = reinterpret_cast<uint32_t *>(lbins + kBins);  // [kErrTab]: (key+1) << 16 | count
  uint8_t *llb = reinterpret_cast<uint8_t *>(etab + kErrTab);       // [kLbMaxSub] HLL lower bounds
  uint32_t *ltag = reinterpret_cast<uint32_t *>(llb + kLbMaxSub);    // TAG: [cap] key_tag of each slot's key
  // POOL: [kPoolMaxSteal] the pool block behind this workgroup's k-th stolen
  // block (0 = not known yet, block + 1, or kPoolDone)
  uint32_t *pmap = ltag + (TAG ? cap : 0u);
  // EXPO with index records: [cap] each slot's scale when the kernel started
  int8_t *lsc = reinterpret_cast<int8_t *>(pmap + (POOL ? kPoolMaxSteal : 0u));
  const bool err_lds = P.errslab != nullptr;
  const bool lb_on = P.lb_n != 0 && !(diag & 2u);
  // EXPO header partials (zeroed with lsum / lcnt): lsum = ns sums
  unsigned long long *xminx = lsum + cap, *xmax = lsum + 2 * cap;
  uint32_t *xcnt = reinterpret_cast<uint32_t *>(lsum + 3 * cap), *xzero = xcnt + cap;

  uint64_t lo, hi;
  wg_range_p(P, lo, hi);
  const uint32_t len = (uint32_t)(hi - lo);
  // static: a step covers one workgroup tile (BLK * S spans, lane_off
  // by thread); DYN: one wave tile (64 * S spans, lane_off by lane) and a
  // claim is NBUF consecutive wave tiles
  constexpr uint32_t tile = DYN ? 64 * S : BLK * S;
  constexpr bool kTileClaims = DYN && (OPT & 2);
  constexpr uint32_t chunk = kTileClaims ? tile : NBUF * tile;
  const uint32_t lane_off = (DYN ? (threadIdx.x & 63u) : threadIdx.x) * S;
  constexpr uint32_t kWaves = BLK / 64;
  const uint32_t n_chunks = DYN ? (len + chunk - 1) / chunk : 0u;
  // wave-uniform by construction; readfirstlane keeps it (and every tile
  // base derived from it) in SGPRs for the buffer descriptors
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  // the first two chunks of every wave are fixed; claims continue after them
  uint32_t c0 = wave, c1 = wave + kWaves;
  // tile claims: cur[b] / nxt[b] = the tile in buffer b this round / the next
  // round; the first two rounds are fixed (tile (r * NBUF + b) * kWaves + wave)
  uint32_t cur[NBUF], nxt[NBUF];
#pragma unroll
  for (int b = 0; b < NBUF; ++b) {
    cur[b] = (uint32_t)b * kWaves + wave;
    nxt[b] = (uint32_t)(NBUF + b) * kWaves + wave;
  }
  auto tstart = [&](uint32_t unit, int b) -> uint32_t {  // step b's first span, relative to lo
    return kTileClaims ? unit * tile : DYN ? unit * chunk + (uint32_t)b * tile : unit + (uint32_t)b * tile;
  };
  // spans readable from lo: the workgroup's range, or (POOL) the rest of the
  // batch, which the workgroup's stolen pool blocks lie in (its own range is
  // whole 256-span chunks then, so only a pool block at the batch end is short)
  // (a launch too small for two fixed chunks per wave has no pool: pool_n 0)
  const bool pool_on = POOL && cold_params().pool_n != 0;
  const uint32_t lim = pool_on ? (uint32_t)(cold_params().n - lo) : len;
  auto tremain = [&](uint32_t t) -> uint32_t { return lim > t ? lim - t : 0u; };

  // Prologue: key-table loads (16 B per lane, <= 4 per lane for cap <= 8192)
  // and the bin table first, then the first NBUF tiles; the LDS setup then
  // waits only for the key-table loads (vmcnt counts in issue order).
  ulonglong2 kv[4];
  const uint32_t per = (cap + 2 * BLK - 1) / (2 * BLK);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const uint32_t i = 2 * (threadIdx.x + u * BLK);
    kv[u] = (u < (int)per && i < cap) ? *reinterpret_cast<const ulonglong2 *>(P.gkeys + i)
                                      : make_ulonglong2(0, 0);
  }
  uint4 bv = make_uint4(0, 0, 0, 0);
  if (!EXPO && threadIdx.x < kBins * 2) bv = reinterpret_cast<const uint4 *>(P.bintab)[threadIdx.x];  // (EXPO: no buckets)
  // EXPO with index records: the slots' scales (cap <= 2,048 bytes: a 16-bit
  // pair per thread), issued with the key table so the LDS setup waits for
  // them and not for the first tiles
  uint32_t xsc = 0;
  if constexpr (EXPO)
    if (P.xidx && SA_XIDX_SCALE(P) && 2 * threadIdx.x < cap) xsc = *reinterpret_cast<const uint16_t *>(P.xscale + 2 * threadIdx.x);
  uint32_t lbw = 0;
  if (lb_on && threadIdx.x * 4 < P.lb_n) lbw = *reinterpret_cast<const uint32_t *>(P.hll_lb + threadIdx.x * 4);
  if constexpr (DYN && (OPT & 1)) {
    // no wait here (gfx950 barriers do not drain vmcnt): only the issue order
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  // Issue order = the steady state's (tile, then S HLL reads, per step), so
  // the loop header's vmcnt accounting is the same from both predecessors;
  // the prologue's HLL reads seed `pend` (rho 0: never raised).
  SpanTile<S> buf[NBUF];
  Pending<S> pend;
#pragma unroll
  for (int b = 0; b < NBUF; ++b) {
    const uint32_t t = kTileClaims ? tstart(cur[b], b) : tstart(DYN ? c0 : 0u, b);
    load_tile_at<S, AUX>(P, (diag & 16u) ? t % (4 * tile) : lo + t, tremain(t), lane_off, buf[b]);
    if (b == NBUF - 1) {
      uint32_t z;  // a VGPR zero: keeps these vector loads (a uniform address would be s_load)
      asm volatile("v_mov_b32 %0, 0" : "=v"(z));
#pragma unroll
      for (int j = 0; j < S; ++j) pend.hv[j] = *reinterpret_cast<const uint32_t *>(P.hll + z);
    }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const uint32_t i = 2 * (threadIdx.x + u * BLK);
    if (u < (int)per && i < cap) {
      reinterpret_cast<ulonglong2 *>(lkeys)[i / 2] = kv[u];
      reinterpret_cast<ulonglong2 *>(lsum)[i / 2] = make_ulonglong2(0, 0);
      if constexpr (TAG) reinterpret_cast<uint2 *>(ltag)[i / 2] = make_uint2(key_tag(kv[u].x), key_tag(kv[u].y));
    }
  }
  if (threadIdx.x < kBins * 2) reinterpret_cast<uint4 *>(lbins)[threadIdx.x] = bv;
  for (uint32_t i = threadIdx.x * 4; i < cap * nw; i += BLK * 4)
    *reinterpret_cast<uint4 *>(lcnt + i) = make_uint4(0, 0, 0, 0);
  if (threadIdx.x == 0) {
    hq_n[0] = 0;
    // DYN: next unclaimed chunk of this workgroup's range, x 64 (see the claims)
    hq_n[1] = ((kTileClaims ? 2u * NBUF : 2u) * kWaves) << 6;
    hq_n[2] = 0;  // EPI: HLL updates the lower-bound filter skipped (summed over the waves)
  }
  if (threadIdx.x < 4) lstat[threadIdx.x] = 0;
  if (POOL && threadIdx.x < kPoolMaxSteal) pmap[threadIdx.x] = 0;
  if constexpr (EXPO)
    if (P.xidx && SA_XIDX_SCALE(P) && 2 * threadIdx.x < cap) *reinterpret_cast<uint16_t *>(lsc + 2 * threadIdx.x) = (uint16_t)xsc;
  // the pool counter of the launch nsets ahead (it starts after this one ends)
  if (POOL && blockIdx.x == 0 && threadIdx.x == 0) *cold_params().pool_next = 0;
  for (uint32_t i = threadIdx.x; i < kErrTab; i += BLK) etab[i] = 0;
  // (filter off: the first bound word stays 0, and every span's sub-block
  // index is 0 or 1 below, so no rho can be at or below it)
  if (threadIdx.x * 4 < (lb_on ? P.lb_n : 4u)) reinterpret_cast<uint32_t *>(llb)[threadIdx.x] = lbw;
  __syncthreads();
  if (P.dbg && threadIdx.x == 0) P.dbg[blockIdx.x * kDbgPerWg + 1] = __builtin_amdgcn_s_memrealtime();

  // diagnostic build: per-wave cycle sums of the step's segments (s_memtime;
  // the stamp's lgkmcnt(0) serialises LDS, so read shares, not lengths)
  uint64_t seg[6] = {0, 0, 0, 0, 0, 0}, t_prev = 0;
  auto stamp = [&](int i) {
    if (DIAG && P.dbg) {
      __builtin_amdgcn_sched_barrier(0);
      uint64_t t;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
      __builtin_amdgcn_sched_barrier(0);
      if (i >= 0) seg[i] += t - t_prev;
      t_prev = t;
    }
  };
  stamp(-1);
  const __amdgpu_buffer_rsrc_t hll_rsrc = rsrc(P.hll, 0xFFFFFFFFu);
  // the bound's shift as a VGPR operand (31 with the filter off): a loop-long
  // scalar here was one of the kernel's SGPR spills, read back by a
  // v_readlane on every span
  const uint32_t lbs_v = copy_u32(lb_on ? P.lb_shift : 31u);
  const uint32_t wmask_v = copy_u32(P.win_mask);  // (likewise the ring mask of every span's window slot)
  constexpr uint32_t kHotUnset = 0xFFFFFFFEu;
  uint32_t hot_slot = kHotUnset;  // wave-uniform (see step 5b)
  unsigned long long hot_sum = 0;
  // wave-uniform event counts (scalar registers)
  uint32_t n_zero = 0, n_badsvc = 0, n_oor = 0, n_drop = 0;
  uint32_t n_filt = 0;  // per lane: HLL updates the lower-bound filter skipped (EPI builds)
#pragma unroll
  for (int j = 0; j < S; ++j) pend.hoff[j] = pend.rho[j] = 0;

  // HLL compare of the previous step's reads; registers that grow are queued
  // in LDS and raised after the loop (no returning global atomic in the loop).
  auto hll_settle = [&](const Pending<S> &q) {
#pragma unroll
    for (int j = 0; j < S; ++j) {
      // hv: the aligned u32 word holding the register (a u8 load would be
      // zero-extended by a v_and at the loop-carried copy, which waits for it)
      if (((q.hv[j] >> ((q.hoff[j] & 3u) * 8)) & 0xFFu) < q.rho[j]) {
        const uint32_t slot = atomicAdd(hq_n, 1u);
        if (slot < kQcap) {
          hq[slot] = make_uint2(q.hoff[j], q.rho[j]);
          if constexpr (kObs) hqv[slot] = q.hv[j];
        } else {
          cold_hll_raise(q.hoff[j], q.rho[j]);
        }
      }
    }
  };

  // step: consume the landed tile T (first span toff) and re-fill its
  // registers with the tile at pf (relative to lo)
  auto step = [&](SpanTile<S> &T, uint32_t toff, uint32_t pf) {
    // 1. compact the landed tile (its registers are re-filled in step 3)
    uint64_t key[S], dur[S];
    uint32_t bkt[S], ws[S], hoff[S], rho[S];
    bool err[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const bool valid = lane_off + toff + (uint32_t)j < lim;
      // 0 past the range (buffer bounds check).  An explicit copy: the key is
      // used after the tile registers are re-filled, and sharing them would
      // make the allocator rotate the tile ring through copies that wait.
      key[j] = copy_u64(T.key[j]);
      if (!(diag & 128u) && !EPI) n_zero += wave_count(valid && key[j] == 0);
      dur[j] = T.e[j] > T.s[j] ? T.e[j] - T.s[j] : 0;
      bkt[j] = EXPO ? 0u : (diag & 32u) ? (uint32_t)dur[j] & 15u : bucket_lds<1>(dur[j], lbins, P);
      const uint32_t meta = copy_u32(T.meta[j]);  // see key
      const uint32_t svc = meta & 0xFFFFu;
      const bool svc_ok = svc < P.n_services;
      ws[j] = (diag & 64u) ? (uint32_t)(T.e[j] >> 34) & 7u : LEAN ? window_slot_lean(P, T.e[j], wmask_v) : window_slot(P, T.e[j]);
      const bool win_ok = ws[j] != 0xFFFFFFFFu;
      if (!(diag & 128u)) {
        if constexpr (EPI) {
          // rare events: LDS counters (no wave-uniform accumulators held in
          // scalar registers across the loop)
          const uint32_t ev = (valid && key[j] == 0 ? 1u : 0u) | (valid && !svc_ok ? 2u : 0u) |
                              (valid && svc_ok && !win_ok ? 4u : 0u);
          if (__builtin_expect(ev != 0, 0)) {
            if (ev & 1u) atomicAdd(&lstat[0], 1u);
            if (ev & 2u) atomicAdd(&lstat[1], 1u);
            if (ev & 4u) atomicAdd(&lstat[2], 1u);
          }
        } else {
          n_badsvc += wave_count(valid && !svc_ok);
          n_oor += wave_count(valid && svc_ok && !win_ok);
        }
      }
      const bool sk = valid && svc_ok && win_ok;
      err[j] = sk && ((meta >> 19) & 3u) == 2u && !(diag & 4u);
      rho[j] = 0;
      hoff[j] = 0;
      if (!(diag & 2u)) {
        uint32_t r, idx, row;
        if constexpr (LEAN) {
          const H64 x = xxh64_16_h(T.a[j], T.b[j]);
          const uint32_t yh = __builtin_amdgcn_alignbit(x.hi, x.lo, 32 - hp);  // (x << hp) >> 32
          const uint32_t yl = (x.lo << hp) | (1u << (hp - 1));
          r = (uint32_t)__clzll((long long)(((uint64_t)yh << 32) | yl)) + 1;  // 2 x v_ffbh, no 64-bit shift
          idx = x.hi >> (32 - hp);
          // ws < 2^12, n_services <= 2^16: a 24-bit multiply-add (LLVM picks
          // the quarter-rate v_mad_u64_u32 for the plain expression)
          asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(row) : "v"(ws[j]), "s"(P.n_services), "v"(svc));
        } else {
          // diag 16384: one 64-bit multiply instead of xxh64 (prices the hash's VALU)
          const uint64_t x = (DIAG && (diag & 16384u)) ? (T.a[j] ^ T.b[j]) * XP1 : xxh64_16(T.a[j], T.b[j]);
          r = (uint32_t)__clzll((long long)((x << hp) | (1ULL << (hp - 1)))) + 1;
          idx = (uint32_t)(x >> (64 - hp));
          row = ws[j] * P.n_services + svc;
        }
        const uint32_t ho = sk ? (row << hp) + idx : 0u;
        // a rho at or below the register sub-block's lower bound cannot raise it
        const bool up = sk && !(r <= llb[ho >> lbs_v]);
        if constexpr (EPI) n_filt += (sk && !up) ? 1u : 0u;
        rho[j] = up ? r : 0u;
        hoff[j] = up ? ho : 0u;
      }
    }
    stamp(0);
    // 2. this step's HLL register reads (unconditional: offset 0 when unused)
    uint32_t hv[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      if (DIAG && (diag & 512u)) {  // diag: blind byte store instead of the read
        P.hll[hoff[j]] = (uint8_t)rho[j];
        hv[j] = 0xFFFFFFFFu;
      } else if (DIAG && (diag & 1024u)) {  // diag: no read at all
        hv[j] = 0xFFFFFFFFu;
      } else {
        hv[j] = HAUX < 0 ? *reinterpret_cast<const uint32_t *>(P.hll + (hoff[j] & ~3u))
                         : (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(
                               hll_rsrc, (int)(hoff[j] & ~3u), 0, HAUX < 0 ? 0 : HAUX);
      }
    }
    // 3. re-fill the tile registers with the tile NBUF steps ahead
    __builtin_amdgcn_sched_barrier(0);
    load_tile_at<S, AUX>(P, (diag & 16u) ? pf % (4 * tile) : lo + pf, tremain(pf), lane_off, T);
    __builtin_amdgcn_sched_barrier(0);
    stamp(1);
    // 4. key lookup: the two candidate buckets in the LDS mirror
    uint32_t found[S];
    if (!(diag & 1u)) {
      bool need[S];
#ifdef SPANAGG_AB
      if constexpr (TAG) {
#include "lab/v2_tag_lookup.inc"
      } else
#endif
      {
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const ProbeSeq pr = probe_seq(key[j], log2cap);
        const ulonglong2 *b1 = reinterpret_cast<const ulonglong2 *>(lkeys + pr.b1 * 4);
        const ulonglong2 *b2 = reinterpret_cast<const ulonglong2 *>(lkeys + pr.b2 * 4);
        const ulonglong2 q1a = b1[0], q1b = b1[1], q2a = b2[0], q2b = b2[1];
        const unsigned long long k = key[j];
        uint32_t f = kNotFound;
        f = q2b.y == k ? pr.b2 * 4 + 3 : f;
        f = q2b.x == k ? pr.b2 * 4 + 2 : f;
        f = q2a.y == k ? pr.b2 * 4 + 1 : f;
        f = q2a.x == k ? pr.b2 * 4 + 0 : f;
        f = q1b.y == k ? pr.b1 * 4 + 3 : f;
        f = q1b.x == k ? pr.b1 * 4 + 2 : f;
        f = q1a.y == k ? pr.b1 * 4 + 1 : f;
        f = q1a.x == k ? pr.b1 * 4 + 0 : f;
        found[j] = k != 0 ? f : kNotFound;
        need[j] = k != 0 && f == kNotFound;
      }
      }
      // 5. cold path (wave-uniform): keys outside their two buckets or not yet
      //    in this workgroup's mirror
#pragma unroll
      for (int j = 0; j < S; ++j) {
        if (__builtin_expect(__ballot(need[j]) != 0, 0)) {
          cold_lookup_wave(lkeys, need[j], key[j], log2cap, found[j], TAG ? ltag : nullptr);
          if constexpr (EPI) {
            if (need[j] && found[j] == kNotFound) atomicAdd(&lstat[3], 1u);
          } else {
            n_drop += wave_count(need[j] && found[j] == kNotFound);
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < S; ++j) {
        found[j] = kNotFound;
        n_drop += wave_count(((key[j] ^ dur[j] ^ bkt[j]) & 0xFFFFFFFFFFFFULL) == 0x123456789ABCULL);
      }
    }
    stamp(2);
    // wave-level key dedup (first step only): the wave's hot series is the
    // most common slot among four candidate lanes (ballot); its ns sum then
    // accumulates in a lane register instead of the LDS atomic that every lane
    // of that series would otherwise serialise on (summed once at the end)
    if (hot_slot == kHotUnset) {
      uint32_t best = kNotFound, nbest = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t cand = (uint32_t)__builtin_amdgcn_readlane((int)found[0], c * 16);
        const uint32_t n = wave_count(found[0] == cand);
        if (cand != kNotFound && n > nbest) {
          best = cand;
          nbest = n;
        }
      }
      hot_slot = best;
    }
    // 6. ERROR spans: exact per-(window, slot) counter (one no-return atomic);
    //    spans without a slot update the count-min cells directly
#pragma unroll
    for (int j = 0; j < S; ++j) {
      if (err[j]) {
        if (found[j] == kNotFound) {
          cold_cms_add(ws[j], key[j]);
        } else {
          const uint32_t ek = (ws[j] << log2cap) | found[j];
          if (!(err_lds && lds_err_add(etab, ek)))
            atomicAdd(cold_params().errcnt + ((uint64_t)ws[j] << log2cap) + found[j], 1ULL);
        }
      }
    }
    // 7. RED update: LDS u16 bucket counter + u64 ns sum.  LEAN: wave-level
    //    key dedup of the counter adds -- the lanes that hold the same
    //    (slot, bucket) as the wave's first lane of its hot series (a ballot
    //    on the readlane'd key) make one LDS add of their count, from the
    //    first of them; the other lanes add their own span.
    if constexpr (EXPO) {
      uint32_t xw[S] = {};
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const uint32_t f = found[j];
        if (f != kNotFound) {
          const unsigned long long d = dur[j];
          atomicAdd(&xcnt[f], 1u);
          if (f == hot_slot) hot_sum += d;
          else atomicAdd(&lsum[f], d);
          if (d == 0) {
            atomicAdd(&xzero[f], 1u);
          } else {
            atomicMax(&xminx[f], ~d);
            atomicMax(&xmax[f], d);
          }
        }
        if (!P.span_rec) {
          uint32_t w = f;
          if (P.xidx) {  // the index record: the bucket index at the slot's starting scale
            // (branch-free but for the rare long-duration store: every lane
            // computes the index, the record is picked by selects)
            const unsigned long long d = dur[j];
            const bool nf = f == kNotFound;
            const uint32_t fs = nf ? 0u : f;
#ifdef SPANAGG_AB
            const int32_t sc = P.xidx == 3 ? 0 : lsc[fs];
#else
            const int32_t sc = lsc[fs];
#endif
            int32_t ix = 0;
            bool ok;
#ifdef SPANAGG_AB
            if (P.xidx >= 2) ok = true, ix = (int32_t)(d & 7u);  // ablation (SPANAGG_XIDX_OFF): wrong buckets
            else
#endif
            ok = expo_index_fast(d ? d : 1u, P.l2d_q24, sc, ix) && ix >= kIxMin && ix <= kIxMax;
            w = nf ? kSpanRecNoSlot << kIxSlotShift
                   : d == 0 ? (f << kIxSlotShift | kIxZero)
                            : ok ? ixrec_of(f, sc, ix) : (f << kIxSlotShift | kIxLong);
            if (!nf && d != 0 && !ok && lane_off + toff + (uint32_t)j < lim) P.span_long[lo + toff + lane_off + j] = d;
          }
          xw[j] = w;
        }
      }
      // the lane's slots / index records: one 8-B store for its two spans
      // (lo, toff and lane_off are even)
      if (!P.span_rec) {
        const uint32_t i0 = toff + lane_off;
        uint32_t *wp = P.slot_of + lo + i0;
        if constexpr (S == 2) {
          if (i0 + 1 < lim) *reinterpret_cast<uint2 *>(wp) = make_uint2(xw[0], xw[1]);
          else if (i0 < lim) wp[0] = xw[0];
        } else {
#pragma unroll
          for (int j = 0; j < S; ++j)
            if (i0 + (uint32_t)j < lim) wp[j] = xw[j];
        }
      }
      // the lane's span records: one 16-B store for its two spans (two 8-B
      // stores per lane cost the kernel ~24 us per 10 M spans)
      if (P.span_rec) {
        const uint32_t i0 = toff + lane_off;
        unsigned long long *rp = P.span_rec + lo + i0;
        if constexpr (S == 2) {
          if (i0 + 1 < lim) {
            *reinterpret_cast<ulonglong2 *>(rp) =
                make_ulonglong2(span_rec_of(found[0], dur[0]), span_rec_of(found[1], dur[1]));
          } else if (i0 < lim) {
            rp[0] = span_rec_of(found[0], dur[0]);
          }
        } else {
#pragma unroll
          for (int j = 0; j < S; ++j)
            if (i0 + (uint32_t)j < lim) rp[j] = span_rec_of(found[j], dur[j]);
        }
        // (durations past the record's field, 52 days or more: in full beside it)
#pragma unroll
        for (int j = 0; j < S; ++j)
          if (dur[j] >= kSpanRecDurMask && i0 + (uint32_t)j < lim) P.span_long[lo + i0 + j] = dur[j];
      }
    } else if constexpr (LEAN) {
      const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const uint32_t key = (found[j] << 6) | bkt[j];  // found < 2^11 or kNotFound, bucket < 64
        const uint64_t hm = __ballot(found[j] == hot_slot && found[j] != kNotFound);
        uint32_t lead = 64u, ndup = 0u, kk = 0xFFFFFFFFu;
        if (hm) {  // wave-uniform
          lead = (uint32_t)__builtin_ctzll(hm);
          kk = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)lead);
          ndup = (uint32_t)__popcll(__ballot(key == kk));
        }
        const bool dup = key == kk;
        if (found[j] != kNotFound && (!dup || lane == lead)) {
          const uint32_t b = bkt[j];
          atomicAdd(&lcnt[found[j] * nw + (b >> 1)], (dup ? ndup : 1u) << ((b & 1) * 16));
        }
        if (found[j] == hot_slot) hot_sum += dur[j];
        else if (found[j] != kNotFound) atomicAdd(&lsum[found[j]], (unsigned long long)dur[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < S && !LEAN && !EXPO; ++j) {
      if (found[j] != kNotFound) {
        const uint32_t b = bkt[j];
        // diag 4096: spread the atomics over slots by lane (prices same-address
        // serialisation of hot keys; counts are wrong)
        const uint32_t fs = (DIAG && (diag & 4096u)) ? (found[j] + (threadIdx.x & 63u) * 29u) & (cap - 1u)
                                                     : found[j];
        atomicAdd(&lcnt[fs * nw + (b >> 1)], 1u << ((b & 1) * 16));
        if (found[j] == hot_slot) hot_sum += dur[j];
        else atomicAdd(&lsum[fs], (unsigned long long)dur[j]);
      }
    }
    stamp(3);
    // 8. settle the previous step's HLL reads, keep this step's for the next
    hll_settle(pend);
#pragma unroll
    for (int j = 0; j < S; ++j) {
      pend.hoff[j] = hoff[j];
      pend.rho[j] = rho[j];
      pend.hv[j] = hv[j];
    }
    stamp(4);
  };

  // Whole rounds of NBUF steps (a step past the range sees only zero-filled
  // lanes and does nothing): no exit between the steps of a round, so the
  // register allocator keeps each in-flight tile in one set of registers
  // across the back-edge instead of copying it (a copy waits for the loads).
  const uint32_t loop_len = (diag & 256u) ? 0u : len;  // diag: prologue/epilogue only
  if constexpr (kTileClaims) {
    // NBUF claims per round, each returning while the round runs; claims of a
    // wave increase, so cur[0] is its smallest outstanding tile
    while (cur[0] * tile < len) {
      uint32_t nw_[NBUF];
#pragma unroll
      for (int b = 0; b < NBUF; ++b) nw_[b] = wave_claim(&hq_n[1]);
#pragma unroll
      for (int b = 0; b < NBUF; ++b) step(buf[b], tstart(cur[b], b), tstart(nxt[b], b));
#pragma unroll
      for (int b = 0; b < NBUF; ++b) {
        cur[b] = nxt[b];
        nxt[b] = nw_[b];
      }
    }
  } else if constexpr (DYN) {
    // c0: this round's chunk (its tiles are in buf), c1: the next round's
    // (prefetched during this round), c2: claimed now for the round after.
    // The claim returns while the round runs; its result is read at the end.
    // (POOL, the laboratory's tail pool, has its own loop: lab/v2_pool_loop.inc.)
    if constexpr (!POOL) {
      while (c0 < n_chunks) {
        const uint32_t c2 = wave_claim(&hq_n[1]);
#pragma unroll
        for (int b = 0; b < NBUF; ++b) step(buf[b], tstart(c0, b), tstart(c1, b));
        c0 = c1;
        c1 = c2;
      }
    }
#ifdef SPANAGG_AB
    if constexpr (POOL) {
#include "lab/v2_pool_loop.inc"
    }
#endif
  } else {
    for (uint32_t t0 = 0; t0 < loop_len; t0 += NBUF * tile) {
#pragma unroll
      for (int b = 0; b < NBUF; ++b) step(buf[b], t0 + b * tile, t0 + (NBUF + b) * tile);
    }
  }
  hll_settle(pend);
  if (hot_slot < cap) {  // the hot series' ns sum: one add per wave
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
      hot_sum += (unsigned long long)(uint32_t)__shfl_xor((int)(uint32_t)hot_sum, o, 64) |
                 ((unsigned long long)(uint32_t)__shfl_xor((int)(uint32_t)(hot_sum >> 32), o, 64) << 32);
    if ((threadIdx.x & 63u) == 0 && hot_sum) atomicAdd(&lsum[hot_slot], hot_sum);
  }
  if constexpr (EPI) {  // one LDS add per wave; one global add per workgroup after the epilogue
    n_filt = wave_sum(n_filt);
    if ((threadIdx.x & 63) == 0 && n_filt) atomicAdd(&hq_n[2], n_filt);
  }
  // (parameters used only after the loop are read through the laundered
  // kernarg pointer, so they do not hold SGPRs across it)
  unsigned long long *const dbg = cold_params().dbg;
  const uint64_t wave_loop_end = dbg ? __builtin_amdgcn_s_memrealtime() : 0;
  if (dbg && threadIdx.x == 0) dbg[blockIdx.x * kDbgPerWg + 2] = __builtin_amdgcn_s_memrealtime();
  // the two-phase epilogues' loads, before the barrier (v2_epi_pre)
  constexpr bool kSlabPre = LC != 0 && NWC != 0 && EPI && !EXPO;
  constexpr uint32_t kCapC = 1u << (LC ? LC : 1);
  constexpr int kUpt = kSlabPre ? (int)(kCapC * NWC / 2 / BLK) : 1, kSpt = kSlabPre ? (int)(kCapC / 2 / BLK) : 1;
  EpiPre<kUpt, kSpt> epre;
  if constexpr (kSlabPre) {
    static_assert((kCapC * NWC / 2) % BLK == 0 && (kCapC / 2) % BLK == 0, "epilogue geometry");
    v2_epi_pre<kUpt, kSpt, BLK>(cold_params(), cap, nw, epre);
  } else if constexpr (EXPO) {
    hll_lb_pre<BLK>(cold_params(), epre.lv);
  }
  __syncthreads();
  const uint32_t nq = *hq_n < kQcap ? *hq_n : kQcap;
  if constexpr (EXPO) {
    // this workgroup's header partials -> its slab, every slot (untouched ones
    // as zeros: the reduce pass reads the slab and leaves it as it is, no
    // zeroing stores behind its reads)
    XHdr *xs = P.xslab + (uint64_t)blockIdx.x * cap;
    for (uint32_t sl = threadIdx.x; sl < cap; sl += BLK) xs[sl] = XHdr{xcnt[sl], xzero[sl], lsum[sl], xminx[sl], xmax[sl]};
    if (err_lds) {  // this workgroup's ERROR counts -> its private slab (no-return atomics)
      for (uint32_t t = threadIdx.x; t < kErrTab; t += BLK) {
        const uint32_t e = etab[t];
        if (e) atomicAdd(P.errslab + (uint64_t)blockIdx.x * ((uint64_t)P.n_windows << log2cap) + ((e >> 16) - 1),
                         e & 0xFFFFu);
      }
    }
    epi_raise_and_bound<BLK, kQcap>(cold_params(), hq, hqv, nq, epre.lv);
  } else if constexpr (LC != 0 && NWC != 0 && EPI) {
    // compile-time geometry: the two-phase epilogue (words prefetched above)
    v2_epilogue<kUpt, kSpt, BLK, kQcap>(cold_params(), cap, nw, log2cap, lsum, lcnt, etab, err_lds, hq, hqv, nq,
                                        epre);
  } else {
    flush_lds(P, cap, nw, lsum, lcnt);
    if (err_lds) {  // this workgroup's ERROR counts -> its private slab (plain RMW)
      for (uint32_t t = threadIdx.x; t < kErrTab; t += BLK) {
        const uint32_t e = etab[t];
        if (e) {
          uint32_t *cell = P.errslab + (uint64_t)blockIdx.x * ((uint64_t)P.n_windows << log2cap) + ((e >> 16) - 1);
          *cell += e & 0xFFFFu;
        }
      }
    }
    for (uint32_t i = threadIdx.x; i < nq; i += BLK) hll_raise(P.hll + hq[i].x, hq[i].y);
    hll_lb_refresh(P, threadIdx.x >> 6, kWaves);
  }
  if (dbg && threadIdx.x == 0) dbg[blockIdx.x * kDbgPerWg + 3] = __builtin_amdgcn_s_memrealtime();
  if (dbg && (threadIdx.x & 63) == 0) {
    for (int i = 0; i < 6 && DIAG; ++i) dbg[blockIdx.x * kDbgPerWg + 8 + (threadIdx.x >> 6) * 8 + i] = seg[i];
    dbg[blockIdx.x * kDbgPerWg + 8 + (threadIdx.x >> 6) * 8 + 6] = wave_loop_end;
  }
  if constexpr (EPI) {  // (lstat is final: the epilogue follows a workgroup barrier)
    if (threadIdx.x < 4 && lstat[threadIdx.x]) {
      constexpr uint32_t kIdx[4] = {kStatZeroKey, kStatInvalidService, kStatWindowOOR, kStatDropped};
      atomicAdd(&cold_params().stats[kIdx[threadIdx.x]], (unsigned long long)lstat[threadIdx.x]);
    }
    // (a slot per workgroup: thousands of same-address atomics at the end of
    // every launch would serialise its tail)
    if (threadIdx.x == 0 && hq_n[2])
      atomicAdd(&cold_params().hll_filt[blockIdx.x & (kFiltSlots - 1)], (unsigned long long)hq_n[2]);
  }
  if ((threadIdx.x & 63) == 0) {
    unsigned long long *const stats = cold_params().stats;
    if (n_zero) atomicAdd(&stats[kStatZeroKey], (unsigned long long)n_zero);
    if (n_badsvc) atomicAdd(&stats[kStatInvalidService], (unsigned long long)n_badsvc);
    if (n_oor) atomicAdd(&stats[kStatWindowOOR], (unsigned long long)n_oor);
    if (n_drop) atomicAdd(&stats[kStatDropped], (unsigned long long)n_drop);
  }
}

// ---------------------------------------------------------------------------
// HBM-table path (table larger than LDS): CAS insert + u64 atomics per span.
template <int NB, int S, bool PF, int BLOCK>
__global__ __launch_bounds__(BLOCK) void ingest_hbm_kernel(IngestParams P) {
  LaneStats st{0, 0, 0, 0};
  const uint32_t nbk = NB >= 0 ? (uint32_t)NB + 1 : P.nbk;
  const uint32_t stride = row_stride(nbk);
  uint64_t lo, hi;
  wg_range(P.n, lo, hi);
  const Cols c = make_cols(P, lo, hi);
  const uint32_t len = (uint32_t)(hi - lo);
  const uint32_t tile = BLOCK * S;
  uint32_t off = threadIdx.x * S;
  SpanTile<S> cur;
  load_tile<S>(c, off, len, cur);
  for (uint32_t t0 = 0; t0 < len; t0 += tile, off += tile) {
    SketchPre<S> k;
    sketch_pre<S>(P, cur, k, st);
    SpanTile<S> nxt;
    if constexpr (PF) {
      __builtin_amdgcn_sched_barrier(0);
      load_tile<S>(c, off + tile, len, nxt);
      __builtin_amdgcn_sched_barrier(0);
    }
    uint32_t slot[S], bk[S];
    uint64_t dd[S];
#pragma unroll
    for (int j = 0; j < S; ++j) {
      slot[j] = kNotFound;
      bk[j] = 0;
      dd[j] = 0;
      if (j < cur.cnt) {
        const uint64_t key = cur.key[j];
        const uint64_t d = cur.e[j] > cur.s[j] ? cur.e[j] - cur.s[j] : 0;
        st.zero_key += key == 0 ? 1u : 0u;
        if (key != 0 && !(P.diag & 1u)) {
          bk[j] = bucket_of<NB>(d, P);
          dd[j] = d;
          const uint32_t found = g_find_insert(P.gkeys, key, P.log2cap, P.max_probe);
          st.dropped += found == kNotFound ? 1u : 0u;
          slot[j] = found;
        }
      }
    }
    // Counter atomics in lane pairs: lanes 2i and 2i+1 each add the count of
    // one span and the sum of the other's, so one instruction carries both
    // cells of a span -- one 64-B segment, one memory-side atomic request
    // (the requests, not the bytes, bound this path: tools/atomic_probe.hip).
    if (!(P.diag & 2048u)) {  // diag 2048: lookups only
      const bool even = (threadIdx.x & 1u) == 0;
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const uint32_t os = (uint32_t)__shfl_xor((int)slot[j], 1);
        const uint32_t ob = (uint32_t)__shfl_xor((int)bk[j], 1);
        const uint64_t od = (uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)dd[j], 1) |
                            ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(dd[j] >> 32), 1) << 32);
        // instruction 1: even lane -> its count, odd lane -> the even lane's sum
        const uint32_t s1 = even ? slot[j] : os, b1 = even ? bk[j] : ob;
        if (s1 != kNotFound)
          atomicAdd(P.gcounts + (uint64_t)s1 * stride + (even ? row_count_cell(b1) : row_sum_cell(b1)),
                    even ? 1ULL : (unsigned long long)od);
        // instruction 2: odd lane -> its count, even lane -> the odd lane's sum
        const uint32_t s2 = even ? os : slot[j], b2 = even ? ob : bk[j];
        if (s2 != kNotFound)
          atomicAdd(P.gcounts + (uint64_t)s2 * stride + (even ? row_sum_cell(b2) : row_count_cell(b2)),
                    even ? (unsigned long long)od : 1ULL);
      }
    }
    sketch_post<S>(P, cur, k, slot);
    if constexpr (PF) {
      cur = nxt;
    } else {
      load_tile<S>(c, off + tile, len, cur);
    }
  }
  flush_stats(P, st);
}

// ---------------------------------------------------------------------------
// Partitioned HBM-table path.  Random per-span lookups and counter atomics
// into a table far larger than LDS bound ingest_hbm_kernel (10 M spans over
// 1 M keys: 552 us).  Here every span is first written as a 16-B record into
// the bin of its key (top 11 bits), then one workgroup per bin aggregates its
// records in an LDS table (~490 keys per bin at 1 M keys) and adds each key's
// row to the HBM counters once, with plain read-modify-write: a key belongs
// to one bin, so its row has one writer per launch.  Records that do not fit
// (a bin beyond its capacity, durations >= 2^57 ns, an LDS table past its
// probe limit) take the direct path: lookup + counter atomics, as in
// ingest_hbm_kernel.  Stats, HLL and ERROR spans are handled in the scatter.

typedef unsigned long long nt_u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void direct_red(const IngestParams &P, uint64_t key, uint64_t d,
                                           uint32_t bk, uint32_t stride, LaneStats &st) {
  const uint32_t s = g_find_insert(P.gkeys, key, P.log2cap, P.max_probe);
  if (s == kNotFound) {
    st.dropped += 1u;
    return;
  }
  atomicAdd(P.gcounts + (uint64_t)s * stride + row_count_cell(bk), 1ULL);
  atomicAdd(P.gcounts + (uint64_t)s * stride + row_sum_cell(bk), (unsigned long long)d);
}

#ifndef PART_U
#define PART_U 4
#endif
// STAGE: records go through a kPartStage-record LDS stage per bin and leave
// as whole chunks (runs are reserved in multiples of kPartStage records, so
// chunks stay aligned); without it each record is its own 16-B store.
#ifndef SA_PART_SKIP_USED
#define SA_PART_SKIP_USED 1
#endif
#ifndef SA_PART_WAVES_EU
#define SA_PART_WAVES_EU 1  // 8 caps VGPRs at 64: two 1,024-thread workgroups per CU
#endif
template <int NB, bool STAGE>
__global__ __launch_bounds__(kPartBlock, SA_PART_WAVES_EU) void part_scatter_kernel(IngestParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t *cur = reinterpret_cast<uint32_t *>(smem);  // phase 1: counts; then next record index
  uint32_t *lim = cur + kPartBins;                      // end of this workgroup's run in the bin
  uint32_t *scnt = lim + kPartBins;                     // STAGE: records staged per bin
  ulonglong2 *stage = reinterpret_cast<ulonglong2 *>(scnt + kPartBins);  // [kPartBins][kPartStage]
  unsigned long long *hkey = reinterpret_cast<unsigned long long *>(stage + kPartBins * kPartStage);
  unsigned long long *hsum = hkey + kPartHot;                           // overflow table
  uint32_t *hcnt = reinterpret_cast<uint32_t *>(hsum + kPartHot);       // [kPartHot][kPartMaxBk]
  LaneStats st{0, 0, 0, 0};
  const uint32_t nbk = NB >= 0 ? (uint32_t)NB + 1 : P.nbk;
  const uint32_t stride = row_stride(nbk);
  uint64_t lo, hi;
  wg_range(P.n, lo, hi);
  for (uint32_t b = threadIdx.x; b < kPartBins; b += blockDim.x) cur[b] = scnt[b] = 0;
  for (uint32_t h = threadIdx.x; h < kPartHot; h += blockDim.x) hkey[h] = hsum[h] = 0;
  for (uint32_t h = threadIdx.x; h < kPartHot * kPartMaxBk; h += blockDim.x) hcnt[h] = 0;
  __syncthreads();
  // 1. records per bin in this workgroup's range (key column only; 8 loads
  //    in flight per thread)
  constexpr int U1 = 8;
  for (uint64_t i0 = lo + threadIdx.x; i0 < hi; i0 += (uint64_t)U1 * blockDim.x) {
    uint64_t k[U1];
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      const uint64_t i = i0 + (uint64_t)u * blockDim.x;
      k[u] = i < hi ? P.key[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < U1; ++u)
      if (k[u] != 0) atomicAdd(&cur[part_bin(k[u])], 1u);
  }
  __syncthreads();
  // 2. reserve one contiguous run per bin (one returning atomic per bin)
  for (uint32_t b = threadIdx.x; b < kPartBins; b += blockDim.x) {
    const uint32_t c = STAGE ? (cur[b] + kPartStage - 1) & ~(kPartStage - 1) : cur[b];
    uint32_t base = 0;
    if (c) base = atomicAdd(&P.part_fill[b], c);
    const uint64_t b0 = (uint64_t)b * P.part_cap;
    cur[b] = (uint32_t)(b0 + min(base, P.part_cap));
    lim[b] = (uint32_t)(b0 + min(base + c, P.part_cap));
  }
  __syncthreads();
  // a span whose bin run is full: into the overflow table (hot keys of a
  // skewed mix overfill their bins; per-span global atomics on one row would
  // serialise), else the direct path
  auto spill = [&](uint64_t key, uint64_t d, uint32_t bk) {
    uint32_t h = ((uint32_t)key * 0x9E3779B1u) >> (32 - kPartHotBits);
    for (int pr = 0; pr < 8; ++pr, h = (h + 1) & (kPartHot - 1)) {
      unsigned long long k = hkey[h];
      if (k == 0) k = atomicCAS(&hkey[h], 0ULL, (unsigned long long)key);
      if (k == 0 || k == key) {
        atomicAdd(&hcnt[h * kPartMaxBk + bk], 1u);
        atomicAdd(&hsum[h], (unsigned long long)d);
        return;
      }
    }
    direct_red(P, key, d, bk, stride, st);
  };
  auto put = [&](uint32_t b, const ulonglong2 &rec, uint64_t d, uint32_t bk) {  // one record, now
    const uint32_t r = atomicAdd(&cur[b], 1u);
    if (r < lim[b]) P.part_rec[r] = rec;  // write-back: partial lines merge in L2
    else spill(rec.x, d, bk);
  };
  // 3. every span: stats, sketches, and its record (or the direct path);
  //    U spans per thread with all their loads issued first; rounds are
  //    workgroup-uniform (STAGE flushes between them)
  constexpr int U = PART_U;
  for (uint64_t r0 = lo; r0 < hi; r0 += (uint64_t)U * blockDim.x) {
   const uint64_t i0 = r0 + threadIdx.x;
   uint64_t K[U], S0[U], E0[U], A[U], B[U];
   uint32_t M[U];
#pragma unroll
   for (int u = 0; u < U; ++u) {
     const uint64_t i = i0 + (uint64_t)u * blockDim.x;
     const bool ok = i < hi;
     K[u] = ok ? P.key[i] : 0;
     S0[u] = ok ? P.start[i] : 0;
     E0[u] = ok ? P.end[i] : 0;
     A[u] = ok ? P.w0[i] : 0;
     B[u] = ok ? P.w1[i] : 0;
     M[u] = ok ? P.meta[i] : 0xFFFFu;  // padding lanes are skipped below
   }
   // sketch phase A for all U spans: the HLL register reads are issued
   // together (unconditional: a skipped span reads the first byte)
   uint32_t WS[U], RHO[U], CUR[U];
   uint8_t *REG[U];
#pragma unroll
   for (int u = 0; u < U; ++u) {
    const bool in = i0 + (uint64_t)u * blockDim.x < hi;
    const uint32_t svc = M[u] & 0xFFFFu;
    const bool svc_ok = svc < P.n_services;
    const uint64_t win = fast_div(E0[u], P.window_ns, P.win_magic);
    const bool win_ok = win - P.win_base < (uint64_t)P.n_windows;
    if (in) {
      st.zero_key += K[u] == 0 ? 1u : 0u;
      st.bad_svc += svc_ok ? 0u : 1u;
      st.oor += (svc_ok && !win_ok) ? 1u : 0u;
    }
    WS[u] = in && svc_ok && win_ok ? (uint32_t)(win & P.win_mask) : 0xFFFFFFFFu;
    RHO[u] = 0;
    REG[u] = P.hll;
    if (WS[u] != 0xFFFFFFFFu && !(P.diag & 2u)) {
      const uint64_t x = xxh64_16(A[u], B[u]);
      RHO[u] = (uint32_t)__clzll((long long)((x << P.p) | (1ULL << (P.p - 1)))) + 1;
      REG[u] = P.hll + ((((uint64_t)WS[u] * P.n_services + svc) << P.p) + (x >> (64 - P.p)));
    }
   }
#pragma unroll
   for (int u = 0; u < U; ++u) CUR[u] = *REG[u];
#pragma unroll
   for (int u = 0; u < U; ++u) {
    if (i0 + (uint64_t)u * blockDim.x >= hi) continue;
    const uint64_t key = K[u], s0 = S0[u], e0 = E0[u];
    const uint32_t meta = M[u];
    const uint64_t d = e0 > s0 ? e0 - s0 : 0;
    const uint32_t bk = bucket_of<NB>(d, P);
    const uint32_t ws = WS[u];
    if (key != 0 && !(P.diag & 1u)) {
      const uint32_t b = part_bin(key);
      const ulonglong2 rec = make_ulonglong2(key, (d << 7) | bk);
      if (d >= (1ULL << 57)) {
        direct_red(P, key, d, bk, stride, st);
      } else if (SA_PART_SKIP_USED && cur[b] >= lim[b]) {  // run used up (stays so): no stage, no cur atomic
        spill(key, d, bk);
      } else if (STAGE) {
        const uint32_t slot = atomicAdd(&scnt[b], 1u);
        if (slot < kPartStage) stage[b * kPartStage + slot] = rec;
        else put(b, rec, d, bk);
      } else {
        put(b, rec, d, bk);
      }
    }
    // ERROR spans: the exact per-(window, slot) counter (count-min cells are
    // folded from it); no slot (key 0, table full): the cells directly
    if (ws != 0xFFFFFFFFu && ((meta >> 19) & 3u) == 2u && !(P.diag & 4u)) {
      const uint32_t slot = key != 0 ? g_find_insert(P.gkeys, key, P.log2cap, P.max_probe) : kNotFound;
      if (slot != kNotFound) atomicAdd(P.errcnt + ((uint64_t)ws << P.log2cap) + slot, 1ULL);
      else cms_add(P, ws, key, 1ULL);
    }
   }
#pragma unroll
   for (int u = 0; u < U; ++u)
     if ((CUR[u] & 0xFFu) < RHO[u]) hll_raise(REG[u], RHO[u]);
   if constexpr (STAGE) {  // full stages leave as one 64-B chunk
     __syncthreads();
     for (uint32_t b = threadIdx.x; b < kPartBins; b += blockDim.x) {
       if (scnt[b] < kPartStage) continue;
       const uint32_t r = cur[b];
       cur[b] = r + kPartStage;
       scnt[b] = 0;
#pragma unroll
       for (int j = 0; j < (int)kPartStage; ++j) {
         const ulonglong2 rec = stage[b * kPartStage + j];
         if (r + j < lim[b]) P.part_rec[r + j] = rec;
         else spill(rec.x, rec.y >> 7, (uint32_t)(rec.y & 127u));
       }
     }
     __syncthreads();
   }
  }
  // partial stages, then zero records over the run's unused tail (the
  // padding, and the slots of spans that took the direct path)
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < kPartBins; b += blockDim.x) {
    if constexpr (STAGE) {
      for (uint32_t j = 0; j < scnt[b]; ++j) {
        const ulonglong2 rec = stage[b * kPartStage + j];
        put(b, rec, rec.y >> 7, (uint32_t)(rec.y & 127u));
      }
    }
    for (uint32_t r = cur[b]; r < lim[b]; ++r) P.part_rec[r] = make_ulonglong2(0, 0);
  }
  // the overflow table: one atomic per non-zero cell per key (the aggregate
  // kernel's plain row updates come after this kernel)
  __syncthreads();
  for (uint32_t h = threadIdx.x; h < kPartHot; h += blockDim.x) {
    const unsigned long long key = hkey[h];
    if (key == 0) continue;
    const uint32_t g = g_find_insert(P.gkeys, key, P.log2cap, P.max_probe);
    if (g == kNotFound) {
      for (uint32_t b = 0; b < nbk; ++b) st.dropped += hcnt[h * kPartMaxBk + b];
      continue;
    }
    unsigned long long *row = P.gcounts + (uint64_t)g * stride;
    for (uint32_t b = 0; b < nbk; ++b)
      if (const uint32_t c = hcnt[h * kPartMaxBk + b]) atomicAdd(row + row_count_cell(b), (unsigned long long)c);
    atomicAdd(row + row_sum_cell(0), hsum[h]);
  }
  flush_stats(P, st);
}

// One workgroup per bin: LDS table of kPartSlots keys (linear probing from a
// hash of the key's low bits; the bin fixes its top bits), u16 bucket-count
// pairs (a bin holds < 2^16 records) and u64 ns sums -- 52 KiB, three
// workgroups per CU -- then one read-modify-write of each key's HBM row.
__global__ __launch_bounds__(kPartAggBlock) void part_aggregate_kernel(IngestParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned long long *lkeys = reinterpret_cast<unsigned long long *>(smem);
  unsigned long long *lsum = lkeys + kPartSlots;
  uint32_t *lcnt = reinterpret_cast<uint32_t *>(lsum + kPartSlots);  // [kPartSlots][kPartWords]
  const uint32_t nbk = P.nbk, stride = row_stride(nbk);
  auto cnt = [&](uint32_t s, uint32_t b) -> uint32_t {
    return (lcnt[s * kPartWords + (b >> 1)] >> ((b & 1u) * 16)) & 0xFFFFu;
  };
  LaneStats st{0, 0, 0, 0};
  __shared__ uint32_t spilled;  // direct-path atomics from this workgroup
  if (threadIdx.x == 0) spilled = 0;
  const uint32_t bin = blockIdx.x;
  const uint32_t n = (P.diag & 1u) ? 0u : min(P.part_fill[bin], P.part_cap);  // diag 1: no records
  for (uint32_t i = threadIdx.x; i < kPartSlots; i += blockDim.x) lkeys[i] = lsum[i] = 0;
  for (uint32_t i = threadIdx.x; i < kPartSlots * kPartWords; i += blockDim.x) lcnt[i] = 0;
  __syncthreads();
  const ulonglong2 *rec = P.part_rec + (uint64_t)bin * P.part_cap;
  constexpr int R = 8;  // records in flight per thread
  for (uint32_t i0 = 0; i0 < n; i0 += R * blockDim.x) {
    ulonglong2 v[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const uint32_t i = i0 + u * blockDim.x + threadIdx.x;
      v[u] = i < n ? rec[i] : make_ulonglong2(0, 0);
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const unsigned long long key = v[u].x;
      if (key == 0) continue;
      const uint64_t d = v[u].y >> 7;
      const uint32_t bk = (uint32_t)(v[u].y & 127u);
      uint32_t s = ((uint32_t)key * 0x9E3779B1u) >> (32 - kPartSlotBits), found = kNotFound;
      for (int pr = 0; pr < 64; ++pr, s = (s + 1) & (kPartSlots - 1)) {
        unsigned long long k = lkeys[s];
        if (k == 0) k = atomicCAS(&lkeys[s], 0ULL, key);
        if (k == 0 || k == key) {
          found = s;
          break;
        }
      }
      if (found != kNotFound) {
        atomicAdd(&lcnt[found * kPartWords + (bk >> 1)], 1u << ((bk & 1u) * 16));
        atomicAdd(&lsum[found], (unsigned long long)d);
      } else {
        direct_red(P, key, d, bk, stride, st);
        spilled = 1;
      }
    }
  }
  __syncthreads();
  // Row updates below use plain loads: a row belongs to this workgroup's bin,
  // so in this launch only this workgroup writes it (earlier launches' writes
  // are visible at the kernel boundary).  After a direct-path spill the
  // row may also hold this launch's atomics, which are performed beyond the
  // XCD's L2: then fence and read at agent scope.
  const bool coherent = spilled != 0;
  if (coherent) {
    __threadfence();
    __syncthreads();
  }
  if (threadIdx.x == 0) P.part_fill[bin] = 0;  // ready for the next launch
  for (uint32_t s = threadIdx.x; s < kPartSlots && !(P.diag & 8u); s += blockDim.x) {
    const unsigned long long key = lkeys[s];
    if (key == 0) continue;
    // the key's first-choice bucket in four independent loads (most keys sit
    // there); the full probe sequence only for the rest
    const ProbeSeq pr = probe_seq(key, P.log2cap);
    const ulonglong2 *bq = reinterpret_cast<const ulonglong2 *>(P.gkeys + pr.b1 * 4);
    const ulonglong2 qa = bq[0], qb = bq[1];  // stale reads just miss: see g_find_insert
    const unsigned long long q[4] = {qa.x, qa.y, qb.x, qb.y};
    uint32_t g = kNotFound;
#pragma unroll
    for (int j = 3; j >= 0; --j) g = q[j] == key ? pr.b1 * 4 + j : g;
    if (g == kNotFound) g = g_find_insert(P.gkeys, key, P.log2cap, P.max_probe);
    if (g == kNotFound) {
      uint32_t calls = 0;
      for (uint32_t b = 0; b < nbk; ++b) calls += cnt(s, b);
      st.dropped += calls;
      continue;
    }
    unsigned long long *row = P.gcounts + (uint64_t)g * stride;
    // every load issued before any store (no wait per cell)
    unsigned long long old[kPartMaxBk + 1];
    if (coherent) {
#pragma unroll
      for (uint32_t b = 0; b < kPartMaxBk; ++b)  // unconditional (in-row address), no branch per load
        old[b] = __hip_atomic_load(row + (b < nbk ? row_count_cell(b) : 0u), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
      old[kPartMaxBk] = __hip_atomic_load(row + row_sum_cell(0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      // the row's (<= 3) 64-B segments as 16-B loads
      constexpr uint32_t kSeg = (kPartMaxBk + kSegBuckets - 1) / kSegBuckets;
      const uint32_t nseg = stride / 8;
      ulonglong2 v[kSeg * 4];
#pragma unroll
      for (uint32_t k = 0; k < kSeg * 4; ++k)
        v[k] = reinterpret_cast<const ulonglong2 *>(row)[(k / 4 < nseg ? k : k % 4)];
      auto cell = [&](uint32_t c) -> unsigned long long { return (c & 1u) ? v[c / 2].y : v[c / 2].x; };
#pragma unroll
      for (uint32_t b = 0; b < kPartMaxBk; ++b) old[b] = b < nbk ? cell(row_count_cell(b)) : 0ULL;
      old[kPartMaxBk] = cell(row_sum_cell(0));
    }
#pragma unroll
    for (uint32_t b = 0; b < kPartMaxBk; ++b)
      if (b < nbk && cnt(s, b)) row[row_count_cell(b)] = old[b] + cnt(s, b);
    row[row_sum_cell(0)] = old[kPartMaxBk] + lsum[s];
  }
  flush_stats(P, st);
}

// ---------------------------------------------------------------------------
// Flush-time kernels.
// slabs -> counters.  blockIdx.y takes a group of kSlabGroup workgroup slabs;
// each thread sums one 4-cell quad of them and adds the partial into the u64
// counters (coalesced no-return atomics, G / kSlabGroup per cell).  The slabs
// are cleared by a memset afterwards.
constexpr uint32_t kSlabGroup = 16;
__global__ void reduce_slabs_kernel(const uint32_t *slab_cnt, const unsigned long long *slab_sum,
                                    unsigned long long *gcounts, uint32_t G, uint64_t cap,
                                    uint32_t nbk) {
  const uint32_t srow = (nbk + 1) & ~1u;  // 2 * ceil(nbk / 2)
  const uint64_t cells = cap * srow, quads = cells / 4;
  const uint32_t stride = row_stride(nbk);
  const uint32_t g0 = blockIdx.y * kSlabGroup, g1 = min(G, g0 + kSlabGroup);
  const uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (q < quads) {
    unsigned long long acc[4] = {0, 0, 0, 0};
    for (uint32_t g = g0; g < g1; ++g) {
      const uint4 v = reinterpret_cast<const uint4 *>(slab_cnt + (uint64_t)g * cells)[q];
      acc[0] += v.x;
      acc[1] += v.y;
      acc[2] += v.z;
      acc[3] += v.w;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t c = q * 4 + i, slot = c / srow, b = c - slot * srow;
      if (acc[i] && b < nbk) atomicAdd(gcounts + slot * stride + row_count_cell((uint32_t)b), acc[i]);
    }
  } else if (q < quads + cap) {
    const uint64_t slot = q - quads;
    unsigned long long acc = 0;
    for (uint32_t g = g0; g < g1; ++g) acc += slab_sum[(uint64_t)g * cap + slot];
    if (acc) atomicAdd(gcounts + slot * stride + row_sum_cell(0), acc);
  }
}

// One counter row in the external layout [nbk bucket counts, ns sum] (u64),
// from either row layout (u64 segment rows, or the binned path's 32-B u8 rows
// + the u64 spill array).
__device__ __forceinline__ bool row_nonzero(const unsigned long long *gcounts, uint64_t s, const RowGeom &g) {
  if (g.row8) {
    const uint4 *row = reinterpret_cast<const uint4 *>(gcounts) + s * (kRowBytes / 16);
    const uint4 a = row[0], b = row[1];
    if (a.x | a.y | a.z | a.w | b.x | b.y | b.z | b.w) return true;
    for (uint32_t c = 0; c <= g.nbk; ++c)
      if (g.base64[s * (g.nbk + 1) + c]) return true;
    return false;
  }
  const uint32_t stride = row_stride(g.nbk);
  const unsigned long long *row = gcounts + s * stride;
  for (uint32_t c = 0; c < stride; ++c)
    if (row[c]) return true;
  return false;
}

__device__ __forceinline__ void row_emit(const unsigned long long *gcounts, uint64_t s, const RowGeom &g,
                                         unsigned long long *out) {
  const uint32_t nbk = g.nbk;
  if (g.row8) {
    const unsigned long long *row = gcounts + s * (kRowBytes / 8);
    const uint8_t *cnt = reinterpret_cast<const uint8_t *>(row + 1);
    const unsigned long long *b64 = g.base64 + s * (nbk + 1);
    for (uint32_t b = 0; b < nbk; ++b) out[b] = cnt[b] + b64[b];
    out[nbk] = row[0] + b64[nbk];
    return;
  }
  const uint32_t stride = row_stride(nbk);
  const unsigned long long *row = gcounts + s * stride;
  unsigned long long sum = 0;
  for (uint32_t c = 0; c < stride; c += 8) sum += row[c];
  for (uint32_t b = 0; b < nbk; ++b) out[b] = row[row_count_cell(b)];
  out[nbk] = sum;
}

__device__ __forceinline__ void row_zero(unsigned long long *gcounts, uint64_t s, const RowGeom &g) {
  if (g.row8) {
    uint4 *row = reinterpret_cast<uint4 *>(gcounts) + s * (kRowBytes / 16);
    row[0] = row[1] = make_uint4(0, 0, 0, 0);
    for (uint32_t c = 0; c <= g.nbk; ++c) g.base64[s * (g.nbk + 1) + c] = 0;
    return;
  }
  const uint32_t stride = row_stride(g.nbk);
  for (uint32_t c = 0; c < stride; ++c) gcounts[s * stride + c] = 0;
}

// Compacts occupied slots with a non-zero row into (out_keys, out_rows); order
// is arrival order of the atomic ticket (the host sorts by key).  Keys leave
// as the host's series ids (stored id * kinv), rows in the external layout.
__global__ void compact_kernel(const unsigned long long *gkeys, unsigned long long *gcounts,
                               uint64_t cap, RowGeom g, unsigned long long *out_keys,
                               unsigned long long *out_rows, unsigned long long *out_n,
                               uint64_t out_cap, int reset) {
  const uint32_t ostride = g.nbk + 1;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap;
       s += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long k = gkeys[s];
    if (!k) continue;
    if (!row_nonzero(gcounts, s, g)) continue;
    // one returning atomic per wave for its emitting lanes (a million lanes
    // on one counter serialised the compaction of a 1 M-series table)
    const uint64_t m = __ballot(true);
    const int leader = __builtin_ctzll(m);
    unsigned long long base = 0;
    if ((int)(threadIdx.x & 63u) == leader) base = atomicAdd(out_n, (unsigned long long)__popcll(m));
    base = ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(base >> 32), leader) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)base, leader);
    const unsigned long long pos =
        base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (pos < out_cap) {
      if (out_keys) out_keys[pos] = k * g.kinv;
      if (out_rows) row_emit(gcounts, s, g, out_rows + pos * ostride);
    }
    if (reset) row_zero(gcounts, s, g);
  }
}

__device__ __forceinline__ uint32_t geom_find(const unsigned long long *gkeys, uint64_t m, const RowGeom &g) {
  if (g.binned) {
    const BtSeq q = bt_seq(m, g.log2sb);
    const uint32_t base = (uint32_t)(m >> kBinShift) << g.log2sb;
    for (uint32_t i = 0; i < bt_probe_max(g.log2sb); ++i) {
      const uint32_t s = base | bt_pos(q, i);
      const unsigned long long k = gkeys[s];
      if (k == m) return s;
      if (k == 0) return kNotFound;
    }
    return kNotFound;
  }
  return g_find(gkeys, m, g.log2cap, g.max_probe);
}

// rows[i] = [nbk bucket counts, ns sum] of keys[i] (zeros if absent).  One
// 32-lane half wave per key: every lane probes the same key (one broadcast
// load per probe), then lane c moves cells c, c + 32, ... so a row's reads
// and its dense output row are contiguous across the lanes.
__global__ void gather_dense_kernel(const unsigned long long *gkeys, const unsigned long long *gcounts,
                                    RowGeom g, const uint64_t *keys, uint64_t n, uint64_t *rows) {
  const uint32_t nbk = g.nbk, ostride = nbk + 1, c0 = threadIdx.x & 31u;
  for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 5; i < n;
       i += ((uint64_t)gridDim.x * blockDim.x) >> 5) {
    const uint64_t k = keys[i];
    const uint32_t s = k ? geom_find(gkeys, k * g.kmul, g) : kNotFound;
    unsigned long long *out = reinterpret_cast<unsigned long long *>(rows) + i * ostride;
    for (uint32_t c = c0; c < ostride; c += 32) {
      unsigned long long v = 0;
      if (s != kNotFound) {
        if (g.row8) {
          const unsigned long long *row = gcounts + (uint64_t)s * (kRowBytes / 8);
          v = g.base64[(uint64_t)s * ostride + c] +
              (c < nbk ? (unsigned long long)reinterpret_cast<const uint8_t *>(row + 1)[c] : row[0]);
        } else {
          const uint32_t stride = row_stride(nbk);
          const unsigned long long *row = gcounts + (uint64_t)s * stride;
          if (c < nbk) {
            v = row[row_count_cell(c)];
          } else {
            for (uint32_t q = 0; q < stride; q += 8) v += row[q];
          }
        }
      }
      out[c] = v;
    }
  }
}

// errcnt[ws][slot] += sum over workgroups of errslab[g][ws << log2cap | slot]
// (blockIdx.y = a group of kSlabGroup workgroups; no-return u64 atomics).
__global__ void reduce_errslab_kernel(const uint32_t *errslab, uint32_t G, uint64_t per_wg,
                                      uint64_t ws, uint32_t log2cap,
                                      unsigned long long *errcnt_ws) {
  const uint64_t cap = 1ULL << log2cap;
  const uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (s >= cap) return;
  const uint32_t g0 = blockIdx.y * kSlabGroup, g1 = min(G, g0 + kSlabGroup);
  unsigned long long acc = 0;
  for (uint32_t g = g0; g < g1; ++g) acc += errslab[g * per_wg + (ws << log2cap) + s];
  if (acc) atomicAdd(errcnt_ws + s, acc);
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

// Window read: add the exact per-slot error counts of window slot `ws` into
// its count-min cells, then clear them (so reads are idempotent).
__global__ void fold_errcnt_kernel(const unsigned long long *gkeys, unsigned long long *errcnt,
                                   uint64_t cap, unsigned long long *cms, uint32_t d, uint32_t w,
                                   uint32_t shift, const uint64_t *seeds, uint64_t kinv) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap;
       s += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long c = errcnt[s];
    if (!c) continue;
    const uint64_t key = gkeys[s] * kinv;
    for (uint32_t r = 0; r < d; ++r) {
      const uint64_t col = splitmix64(key ^ seeds[r]) >> shift;
      atomicAdd(cms + (uint64_t)r * w + col, c);
    }
    errcnt[s] = 0;
  }
}

uint32_t grid_for(uint64_t work, uint32_t block, uint32_t cap_blocks) {
  uint64_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap_blocks) g = cap_blocks;
  return (uint32_t)g;
}

// Small-table kernels.  Product build: the v2 kernel specialised for the
// default geometry (variant 20: 2,048 slots, 17 buckets, HLL p 14, LEAN), the
// generic v2 kernel with 512-thread workgroups (variant 26, two per CU) for
// other geometries whose LDS state fits a CU twice and with 1,024 threads
// (variant 15) for the rest with a bucket bin table, and the
// linear-threshold kernel for bounds no bin table can hold.
// The laboratory build (SPANAGG_AB) keeps every variant and the diagnostic
// (ablation) kernels.
#ifndef SPANAGG_AB
static const void *small_fn(bool bt, int v, bool diag) {
  (void)diag;
  if (!bt) return (const void *)&ingest_lds_kernel<0, 4, true, false>;
  if (v == 20) return (const void *)&ingest_v2_kernel<11, 9, 14, false, 1024, V2Lean>;
  if (v == kLdsHalfBlockVariant) return (const void *)&ingest_v2_kernel<0, 0, 0, false, 512, V2Lean>;
  return (const void *)&ingest_v2_kernel<0, 0, 0, false, 1024, V2Plain>;
}
constexpr int kSmallFnVariants[] = {15, 20, kLdsHalfBlockVariant};
#else
// every variant and the diagnostic kernels (tools/ A/B runs)
#include "lab/small_lab.inc"
#endif

template <int NB>
static void launch_hbm_nb(const IngestParams &P, uint32_t grid, hipStream_t s, int v) {
#ifndef SPANAGG_AB
  (void)v;
  hipLaunchKernelGGL((ingest_hbm_kernel<NB, 4, false, 256>), dim3(grid), dim3(256), 0, s, P);
#else
  switch (v) {
    case 1: hipLaunchKernelGGL((ingest_hbm_kernel<NB, 2, true, 256>), dim3(grid), dim3(256), 0, s, P); break;
    case 2: hipLaunchKernelGGL((ingest_hbm_kernel<NB, 4, true, 256>), dim3(grid), dim3(256), 0, s, P); break;
    case 3: hipLaunchKernelGGL((ingest_hbm_kernel<NB, 2, false, 256>), dim3(grid), dim3(256), 0, s, P); break;
    default: hipLaunchKernelGGL((ingest_hbm_kernel<NB, 4, false, 256>), dim3(grid), dim3(256), 0, s, P); break;
  }
#endif
}

}  // namespace

hipError_t prepare_ingest_small(size_t lds_bytes) {
#ifndef SPANAGG_AB
  for (int bt = 0; bt < 2; ++bt)
    for (int v : kSmallFnVariants) {
      hipError_t e = hipFuncSetAttribute(small_fn(bt, v, false), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)lds_bytes);
      if (e != hipSuccess) return e;
    }
#else
  for (int bt = 0; bt < 2; ++bt)
    for (int v = 0; v < kNumLdsVariants; ++v)
      for (int d = 0; d < 2; ++d) {
        hipError_t e = hipFuncSetAttribute(small_fn(bt, v, d),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
        if (e != hipSuccess) return e;
      }
#endif
  return hipSuccess;
}

// the variant that runs for a geometry: the specialised v2 builds are only
// valid for their compile-time geometry (2,048 slots, 17 buckets, HLL p 14)
static int small_variant(int variant, uint32_t log2cap, uint32_t nbk, uint32_t p) {
  if ((variant == 12 || variant == 13 || (variant >= 14 && variant != 25 && variant != 26)) &&
      !(log2cap == 11 && (nbk + 1) / 2 == 9 && p == 14))
    variant = variant == 12 ? 8 : variant == 13 ? 11 : 15;
  return variant;
}
// (the linear-threshold kernel, for bounds no bin table holds, is 1,024 threads)
static uint32_t small_block(bool bt, int variant) { return bt ? lds_variant_block(variant) : kLdsBlock; }

hipError_t launch_ingest_small(const IngestParams &P, uint32_t grid, size_t lds_bytes,
                               hipStream_t s, int variant) {
  variant = small_variant(variant, P.log2cap, P.nbk, P.p);
  // (the lean window quotient of variant 20 needs window_ns < 2^56, which
  // sa_create enforces; SA_OPT_STAMPS engines keep the production v2 kernels:
  // their workgroup and wave-end stamps are written whenever P.dbg is set)
  const bool bt = P.bintab != nullptr;
  const void *fn = small_fn(bt, variant, P.diag != 0 || (P.dbg != nullptr && variant < 8));
  void *args[] = {const_cast<IngestParams *>(&P)};
  return hipLaunchKernel(fn, dim3(grid), dim3(small_block(bt, variant)), args, lds_bytes, s);
}

// The same launch as a HIP graph kernel node (sa_ingest_device_many): the
// kernel, its geometry and `args` (args[0] = &P, owned by the caller, read
// when the node is added or its parameters set).
void ingest_small_node(const IngestParams &P, uint32_t grid, size_t lds_bytes, int variant, void **args,
                       hipKernelNodeParams *np) {
  variant = small_variant(variant, P.log2cap, P.nbk, P.p);
  const bool bt = P.bintab != nullptr;
  *np = hipKernelNodeParams{};
  np->func = const_cast<void *>(small_fn(bt, variant, P.diag != 0 || (P.dbg != nullptr && variant < 8)));
  np->gridDim = dim3(grid);
  np->blockDim = dim3(small_block(bt, variant));
  np->sharedMemBytes = (unsigned int)lds_bytes;
  np->kernelParams = args;
  np->extra = nullptr;
}

uint32_t ingest_small_block(bool bt, int variant, uint32_t log2cap, uint32_t nbk, uint32_t p) {
  return small_block(bt, small_variant(variant, log2cap, nbk, p));
}

// workgroups of the small-table kernel resident per CU (registers and LDS);
// 0 when the runtime cannot tell.  After prepare_ingest_small.
uint32_t ingest_small_blocks_per_cu(bool bt, int variant, uint32_t log2cap, uint32_t nbk, uint32_t p,
                                    size_t lds_bytes) {
  variant = small_variant(variant, log2cap, nbk, p);
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, small_fn(bt, variant, false), (int)small_block(bt, variant),
                                                   lds_bytes) != hipSuccess)
    return 0;
  return n > 0 ? (uint32_t)n : 0u;
}

// the EXPO kernel: specialised for the default small table (2,048 slots, HLL
// p = 14: C2's geometry) like variant 20, generic otherwise
static const void *expo_small_fn(bool spec) {
  return spec ? (const void *)&ingest_v2_kernel<11, 0, 14, true, 1024, V2Lean>
              : (const void *)&ingest_v2_kernel<0, 0, 0, true, 1024, V2Lean>;
}

hipError_t prepare_ingest_expo_small(size_t lds_bytes) {
  for (bool spec : {false, true})
    if (hipError_t e = hipFuncSetAttribute(expo_small_fn(spec), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes);
        e != hipSuccess)
      return e;
  return hipSuccess;
}
// workgroups of the EXPO kernel resident per CU; 0 when the runtime cannot
// tell.  After prepare_ingest_expo_small.
uint32_t ingest_expo_blocks_per_cu(uint32_t log2cap, uint32_t p, size_t lds_bytes) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, expo_small_fn(log2cap == 11 && p == 14), (int)kLdsBlock,
                                                   lds_bytes) != hipSuccess)
    return 0;
  return n > 0 ? (uint32_t)n : 0u;
}

hipError_t launch_ingest_expo_small(const IngestParams &P, uint32_t grid, size_t lds_bytes, hipStream_t s) {
  void *args[] = {const_cast<IngestParams *>(&P)};
  return hipLaunchKernel(expo_small_fn(P.log2cap == 11 && P.p == 14), dim3(grid), dim3(kLdsBlock), args, lds_bytes, s);
}

hipError_t launch_ingest_part(const IngestParams &P, hipStream_t s) {
#ifdef SPANAGG_AB
  static const uint32_t max_grid = [] {
    const char *v = std::getenv("SPANAGG_PART_GRID");  // laboratory knob
    return v ? (uint32_t)std::max(1, std::atoi(v)) : 256u;
  }();
  static const bool stage = [] {
    const char *v = std::getenv("SPANAGG_PART_STAGE");  // laboratory knob
    return !(v && std::atoi(v) == 0);
  }();
#else
  constexpr uint32_t max_grid = 256u;
  constexpr bool stage = true;
#endif
  const uint32_t grid = (uint32_t)std::min<uint64_t>(max_grid, (P.n + kPartBlock - 1) / kPartBlock);
  const bool b16 = P.nneg == 0 && P.npos == 16;
#ifdef SPANAGG_AB
  const void *fn = stage ? (b16 ? (const void *)&part_scatter_kernel<16, true> : (const void *)&part_scatter_kernel<-1, true>)
                         : (b16 ? (const void *)&part_scatter_kernel<16, false> : (const void *)&part_scatter_kernel<-1, false>);
#else
  (void)stage;
  const void *fn = b16 ? (const void *)&part_scatter_kernel<16, true> : (const void *)&part_scatter_kernel<-1, true>;
#endif
  void *args[] = {const_cast<IngestParams *>(&P)};
  if (hipError_t e = hipLaunchKernel(fn, dim3(grid), dim3(kPartBlock), args, kPartScatterLds, s); e != hipSuccess)
    return e;
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  hipLaunchKernelGGL(part_aggregate_kernel, dim3(kPartBins), dim3(kPartAggBlock), kPartLdsBytes, s, P);
  return hipGetLastError();
}

hipError_t prepare_ingest_part() {
#ifdef SPANAGG_AB
  for (const void *fn : {(const void *)&part_scatter_kernel<16, true>, (const void *)&part_scatter_kernel<-1, true>,
                         (const void *)&part_scatter_kernel<16, false>, (const void *)&part_scatter_kernel<-1, false>})
#else
  for (const void *fn : {(const void *)&part_scatter_kernel<16, true>, (const void *)&part_scatter_kernel<-1, true>})
#endif
    if (hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPartScatterLds);
        e != hipSuccess)
      return e;
  return hipFuncSetAttribute((const void *)&part_aggregate_kernel,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPartLdsBytes);
}

hipError_t launch_ingest_hbm(const IngestParams &P, uint32_t grid, hipStream_t s, int variant) {
  if (P.nneg == 0 && P.npos == 16) launch_hbm_nb<16>(P, grid, s, variant);
  else launch_hbm_nb<-1>(P, grid, s, variant);
  return hipGetLastError();
}


hipError_t launch_reduce_slabs(uint32_t *slab_cnt, unsigned long long *slab_sum,
                               unsigned long long *gcounts, uint32_t G, uint64_t cap,
                               uint32_t nbk, hipStream_t s) {
  const uint32_t block = 256;
  const uint64_t srow = (nbk + 1) & ~1u, work = cap * srow / 4 + cap;
  const dim3 grid((uint32_t)((work + block - 1) / block), (G + kSlabGroup - 1) / kSlabGroup);
  hipLaunchKernelGGL(reduce_slabs_kernel, grid, dim3(block), 0, s, slab_cnt, slab_sum, gcounts, G,
                     cap, nbk);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  if (hipError_t e = hipMemsetAsync(slab_cnt, 0, (size_t)G * cap * srow * 4, s); e != hipSuccess)
    return e;
  return hipMemsetAsync(slab_sum, 0, (size_t)G * cap * 8, s);
}

hipError_t launch_compact(const unsigned long long *gkeys, unsigned long long *gcounts,
                          uint64_t cap, const RowGeom &g, unsigned long long *out_keys,
                          unsigned long long *out_rows, unsigned long long *out_n,
                          uint64_t out_cap, int reset, hipStream_t s) {
  const uint32_t block = 256;
  hipLaunchKernelGGL(compact_kernel, dim3(grid_for(cap, block, 4096)), dim3(block), 0, s, gkeys,
                     gcounts, cap, g, out_keys, out_rows, out_n, out_cap, reset);
  return hipGetLastError();
}

hipError_t launch_gather_dense(const unsigned long long *gkeys, const unsigned long long *gcounts,
                               const RowGeom &g, const uint64_t *keys, uint64_t n, uint64_t *rows,
                               hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t block = 256;
  hipLaunchKernelGGL(gather_dense_kernel, dim3(grid_for(n * 32, block, 8192)), dim3(block), 0, s,  // (32 lanes a key)
                     gkeys, gcounts, g, keys, n, rows);
  return hipGetLastError();
}

hipError_t launch_fold_errcnt(const unsigned long long *gkeys, unsigned long long *errcnt,
                              uint64_t cap, unsigned long long *cms, uint32_t d, uint32_t w,
                              uint32_t shift, const uint64_t *seeds, uint64_t kinv, hipStream_t s) {
  const uint32_t block = 256;
  hipLaunchKernelGGL(fold_errcnt_kernel, dim3(grid_for(cap, block, 2048)), dim3(block), 0, s, gkeys,
                     errcnt, cap, cms, d, w, shift, seeds, kinv);
  return hipGetLastError();
}

hipError_t launch_reduce_errslab(uint32_t *errslab, uint32_t G, uint64_t per_wg, uint64_t ws,
                                 uint32_t log2cap, unsigned long long *errcnt_ws, hipStream_t s) {
  const uint32_t block = 256;
  const uint64_t cap = 1ULL << log2cap;
  const dim3 grid((uint32_t)((cap + block - 1) / block), (G + kSlabGroup - 1) / kSlabGroup);
  hipLaunchKernelGGL(reduce_errslab_kernel, grid, dim3(block), 0, s, errslab, G, per_wg, ws, log2cap,
                     errcnt_ws);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  // clear window ws's cells of every workgroup slab (a strided 2-D memset)
  return hipMemset2DAsync(errslab + (ws << log2cap), per_wg * 4, 0, cap * 4, G, s);
}

hipError_t launch_count_keys(const unsigned long long *gkeys, uint64_t cap,
                             unsigned long long *out, hipStream_t s) {
  const uint32_t block = 256;
  hipLaunchKernelGGL(count_keys_kernel, dim3(grid_for(cap, block, 2048)), dim3(block), 0, s,
                     gkeys, cap, out);
  return hipGetLastError();
}

}  // namespace sa
