// spanagg_binned.hip -- the binned-table high-cardinality path of libspanagg
// (gfx950).  BASELINE config 4: ~1 M series, too many for an LDS-resident key
// table, so every span is first routed to the bin of its series and each bin
// is then aggregated by one workgroup that owns the bin's whole slice of the
// key table and counter rows.  Replaces, for that geometry, the per-span body
// of the connector's aggregateMetrics ([UPSTREAM] spanmetricsconnector
// connector.go: buildKey -> map lookup, Sum.Add(1), explicitHistogram.Observe)
// and adds the sketch updates.
//
// Two kernels per launch:
//   bt_scatter2_kernel (one 1,024-thread workgroup per CU, ~160 KiB LDS)
//     streams the SoA batch once (register tile ring, 16-B nt buffer loads:
//     the C2 kernel's skeleton), does the per-span stats and HLL work, and
//     writes one 16-B record {m's low 53 bits | ERROR flag | window slot,
//     duration} per span into the region of (its bin, this workgroup),
//     through 4-record LDS stages that leave as aligned 64-B chunks.  Hot keys
//     are pre-aggregated in an LDS overflow table; past that, the direct path
//     (key-table CAS + atomics into the spill array).
//   bt_aggregate3_kernel (one 512-thread workgroup per bin; the laboratory
//   build, lab/binned_lab.inc, also keeps bt_aggregate2_kernel, the earlier
//   form, SPANAGG_BT_AGG=2)
//     loads the bin's 2^log2sb key slots into LDS at the same positions,
//     aggregates the bin's records there (u16 bucket-count pairs, u64 ns
//     sums, an ERROR table keyed by (window slot, key slot)), then writes the
//     new keys and read-modify-writes each touched 32-B row of the bin (one
//     owner, no atomics).
// Rows hold u8 bucket counts (sa_internal.h kRowBytes); a count that would
// pass 255 moves the row's counts into the u64 spill array base64.
#include <algorithm>
#include <cstdlib>

#include "sa_device.h"

namespace sa {
namespace {

__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

// Find-or-insert m in its bin's sub-table (HBM, CAS); kNotFound when the
// bin is full.  Plain probe reads, as g_find_insert (a stale 0 is corrected
// by the CAS).
__device__ __forceinline__ uint32_t bt_find_insert(unsigned long long *keys, uint64_t m, uint32_t log2sb) {
  const BtSeq q = bt_seq(m, log2sb);
  const uint32_t base = (uint32_t)(m >> kBinShift) << log2sb;
  for (uint32_t i = 0; i < bt_probe_max(log2sb); ++i) {
    const uint32_t s = base | bt_pos(q, i);
    unsigned long long k = keys[s];
    if (k == m) return s;
    if (k == 0) {
      const unsigned long long prev = atomicCAS(&keys[s], 0ULL, (unsigned long long)m);
      if (prev == 0 || prev == m) return s;
    }
  }
  return kNotFound;
}

// Adds cnt spans of bucket bk and an ns sum to key slot s in the u64 spill
// array with atomics (the direct path and the overflow table's rows).
__device__ __forceinline__ void spill_add(unsigned long long *base64, uint32_t nbk, uint32_t s, uint32_t bk,
                                          uint32_t cnt, unsigned long long dsum) {
  unsigned long long *row = base64 + (uint64_t)s * (nbk + 1);
  if (cnt) atomicAdd(row + bk, (unsigned long long)cnt);
  if (dsum) atomicAdd(row + nbk, dsum);
}

// The kernel's parameters in the kernarg segment.  Taken in the kernel body
// and passed to the cold paths below (which are real calls, where
// __builtin_amdgcn_kernarg_segment_ptr -- cold_params -- is not valid), so
// the fields only they use do not occupy scalar registers in the span loop.
typedef SA_CONST const IngestParams *KParams;
__device__ __forceinline__ KParams kernel_params() {
  return (KParams)__builtin_amdgcn_kernarg_segment_ptr();
}

// Count-min cells of one ERROR span without a key-table slot (d atomics).
template <typename QP>
__device__ __forceinline__ void bt_cms_add(QP Q, uint32_t ws, uint64_t key) {
  SA_GLOBAL unsigned long long *row0 = gbl(Q->cms) + (uint64_t)ws * Q->cms_d * Q->cms_w;
  for (uint32_t r = 0; r < Q->cms_d; ++r) {
    const uint64_t col = splitmix64(key ^ Q->seeds[r]) >> Q->cms_shift;
    __hip_atomic_fetch_add(row0 + (uint64_t)r * Q->cms_w + col, 1ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Cold paths of the scatter.
__device__ __noinline__ void bt_cold_err(KParams Q, uint64_t m, uint32_t ws) {
  const uint32_t s = bt_find_insert(Q->gkeys, m, Q->log2sb);
  if (s != kNotFound) atomicAdd(Q->errcnt + ((uint64_t)ws << Q->log2cap) + s, 1ULL);
  else bt_cms_add(Q, ws, m * Q->kinv);
}

// returns 1 when the span was dropped (its bin is full)
__device__ __noinline__ uint32_t bt_cold_direct(KParams Q, uint64_t m, uint64_t d, uint32_t bk, bool err,
                                                uint32_t ws) {
  const uint32_t s = bt_find_insert(Q->gkeys, m, Q->log2sb);
  if (s == kNotFound) {
    if (err) bt_cms_add(Q, ws, m * Q->kinv);
    return 1u;
  }
  spill_add(Q->base64, Q->nbk, s, bk, 1u, d);
  if (err) atomicAdd(Q->errcnt + ((uint64_t)ws << Q->log2cap) + s, 1ULL);
  return 0u;
}

// Diagnostic per-workgroup timestamps (SPANAGG_STAMPS builds of the engine):
// s_memrealtime (100 MHz, comparable across CUs) into dbg[base + k].
__device__ __forceinline__ void bt_stamp(const IngestParams &P, uint64_t base, uint32_t k) {
  if (P.dbg && threadIdx.x == 0) P.dbg[base + k] = __builtin_amdgcn_s_memrealtime();
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// Round-synchronous scatter.  The workgroup takes its span range in rounds of
// 2,048 spans (one 128-span tile per wave, two rounds of tiles in flight);
// every span claims a slot of its bin's 4-record LDS stage with one LDS
// atomic.  After a barrier each wave collects the full stages of the 128 bins
// it owns into a list and writes them out four lanes per stage, so every
// stage leaves as one aligned 64-B piece of a single store instruction; a
// second barrier frees the stages for the next round.  Keys already in the
// overflow table (the hot keys of a skewed mix) are added there directly;
// a span whose stage is full in its round, or whose region is used up, goes
// to the overflow table, past that the direct path.  The record layout
// ({m's low 53 bits | ERROR flag | window slot, duration} per (bin,
// workgroup) region) is the one bt_aggregate3_kernel reads.
// MODE (ablation): 1 = no records, 2 = no HLL, 4 = overflow-table adds
// skipped, 8 = overflow-table ERROR counts skipped.
template <int MODE = 0>
__global__ __launch_bounds__(kBtBlock) void bt_scatter2_kernel(IngestParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr uint32_t kWaves = kBtBlock / 64;
  ulonglong2 *stage = reinterpret_cast<ulonglong2 *>(smem);                          // [bins][4]
  uint32_t *fillw = reinterpret_cast<uint32_t *>(stage + kPartBins * kBtStage);      // [bins / 2] u16 pairs
  uint32_t *rcnw = fillw + kPartBins / 2;                                            // [bins / 2] region fills
  uint16_t *flist = reinterpret_cast<uint16_t *>(rcnw + kPartBins / 2);              // [waves][128]
  unsigned long long *hkey = reinterpret_cast<unsigned long long *>(flist + kWaves * 128);
  unsigned long long *hsum = hkey + kBt2Hot;
  uint32_t *hcnt = reinterpret_cast<uint32_t *>(hsum + kBt2Hot);  // [kBt2Hot][kPartWords] u16 pairs
  uint2 *hq = reinterpret_cast<uint2 *>(hcnt + kBt2Hot * kPartWords);
  uint32_t *hq_n = reinterpret_cast<uint32_t *>(hq + kBtHq);
  BinEntry *lbins = reinterpret_cast<BinEntry *>(hq_n + 4);
  uint2 *herr = reinterpret_cast<uint2 *>(lbins + kBins);  // [kBt2HotErr] {(ws << 8 | entry) + 1, count}
  uint8_t *llb = reinterpret_cast<uint8_t *>(herr + kBt2HotErr);
  const KParams kp = kernel_params();
  const uint64_t sbase = (uint64_t)kPartBins * 8 + blockIdx.x * 8;
  bt_stamp(P, sbase, 0);

  uint64_t lo, hi;
  wg_range_p(P, lo, hi);
  const uint32_t len = (uint32_t)(hi - lo);
  constexpr uint32_t kRound = kBtBlock * 2;
  const uint32_t lane = threadIdx.x & 63u, lane_off = lane * 2;
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t rounds = (len + kRound - 1) / kRound;
  auto tstart = [&](uint32_t r) -> uint32_t { return r * kRound + wave * 128; };
  auto tremain = [&](uint32_t t) -> uint32_t { return len > t ? len - t : 0u; };

  // prologue: bin table and bounds, the first two rounds' tiles, LDS setup
  uint4 bv = make_uint4(0, 0, 0, 0);
  if (threadIdx.x < kBins * 2) bv = reinterpret_cast<const uint4 *>(P.bintab)[threadIdx.x];
  const uint32_t lb_on = P.lb_n != 0 && !(MODE & 2);
  uint32_t lbw = 0;
  if (lb_on && threadIdx.x * 4 < P.lb_n) lbw = *reinterpret_cast<const uint32_t *>(P.hll_lb + threadIdx.x * 4);
  SpanTile<2> buf[2];
  Pending<2> pend, pend2;  // HLL reads of the last two rounds (compared two rounds later:
                           // the flush stores between a read and its compare would
                           // otherwise make that wait drain the prefetched tiles too)
  load_tile_at<2, 2>(P, lo + tstart(0), tremain(tstart(0)), lane_off, buf[0]);
  load_tile_at<2, 2>(P, lo + tstart(1), tremain(tstart(1)), lane_off, buf[1]);
  {
    uint32_t z;  // a VGPR zero keeps these vector loads
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
#pragma unroll
    for (int j = 0; j < 2; ++j) pend.hv[j] = pend2.hv[j] = *reinterpret_cast<const uint32_t *>(P.hll + z);
  }
  for (uint32_t b = threadIdx.x; b < kPartBins / 2; b += kBtBlock) fillw[b] = rcnw[b] = 0;
  for (uint32_t h = threadIdx.x; h < kBt2Hot; h += kBtBlock) hkey[h] = hsum[h] = 0;
  for (uint32_t h = threadIdx.x; h < kBt2Hot * kPartWords; h += kBtBlock) hcnt[h] = 0;
  if (threadIdx.x < kBt2HotErr) herr[threadIdx.x] = make_uint2(0, 0);
  if (threadIdx.x < kBins * 2) reinterpret_cast<uint4 *>(lbins)[threadIdx.x] = bv;
  if (lb_on && threadIdx.x * 4 < P.lb_n) reinterpret_cast<uint32_t *>(llb)[threadIdx.x] = lbw;
  if (threadIdx.x == 0) hq_n[0] = 0;
  __syncthreads();
  bt_stamp(P, sbase, 1);

  uint32_t n_zero = 0, n_badsvc = 0, n_oor = 0;  // wave-uniform (SGPR)
  uint32_t n_drop = 0;                           // per lane
  uint32_t n_filt = 0;                           // per lane: HLL updates the lower-bound filter skipped
#pragma unroll
  for (int j = 0; j < 2; ++j) pend.hoff[j] = pend.rho[j] = pend2.hoff[j] = pend2.rho[j] = 0;
  const uint32_t region = P.bt_region;
  ulonglong2 *my_rec = P.bt_rec + (uint64_t)blockIdx.x * region;  // + bin * grid * region
  const uint64_t bin_stride = (uint64_t)P.bt_grid * region;

  // overflow-table home: an even entry, probed as a pair first
  auto hot_home = [&](uint64_t m) -> uint32_t {
    return (uint32_t)(((uint64_t)(uint32_t)(m >> 21) * (kBt2Hot / 2)) >> 32) * 2;
  };
  auto hot_acc = [&](uint32_t h, uint64_t m, uint64_t d, bool err, uint32_t ws) {
    if (MODE & 4) return;
    const uint32_t bk = bucket_lds<1>(d, lbins, P);
    atomicAdd(&hcnt[h * kPartWords + (bk >> 1)], 1u << ((bk & 1u) * 16));
    atomicAdd(&hsum[h], (unsigned long long)d);
    if (err && !(MODE & 8)) {  // ERROR count per (window slot, entry); a full table takes the key-table path
      const uint32_t ek = ((ws << 8) | h) + 1;
      uint32_t e = (ek * 0x9E3779B1u) >> 25;  // kBt2HotErr = 128
      for (int pr = 0; pr < 4; ++pr, e = (e + 1) & (kBt2HotErr - 1)) {
        uint32_t k = herr[e].x;
        if (k == 0) k = atomicCAS(&herr[e].x, 0u, ek);
        if (k == 0 || k == ek) {
          atomicAdd(&herr[e].y, 1u);
          return;
        }
      }
      bt_cold_err(kp, m, ws);
    }
  };
  // the overflow table: false when the key is not in it and its 8 probes
  // are taken
  auto hot_try = [&](uint64_t m, uint64_t d, bool err, uint32_t ws) -> bool {
    uint32_t h = hot_home(m);
    for (int pr = 0; pr < 8; ++pr) {
      unsigned long long k = hkey[h];
      if (k == 0) k = atomicCAS(&hkey[h], 0ULL, (unsigned long long)m);
      if (k == 0 || k == m) {
        hot_acc(h, m, d, err, ws);
        return true;
      }
      h = h + 1 == kBt2Hot ? 0u : h + 1;
    }
    return false;
  };
  // a span its region cannot take: the overflow table, else the direct path
  auto hot_add = [&](uint64_t m, uint64_t d, bool err, uint32_t ws) {
    if (hot_try(m, d, err, ws)) return;
    const uint32_t bk = bucket_lds<1>(d, lbins, P);
    n_drop += bt_cold_direct(kp, m, d, bk, err, ws);
  };
  auto hot_rec = [&](uint32_t b, const ulonglong2 &r) {
    const uint64_t m = ((uint64_t)b << kBinShift) | (r.x & kBinRest);
    hot_add(m, r.y & kRecDurMask, (r.x >> 63) != 0, (uint32_t)(r.x >> kBinShift) & 1023u);
  };
  // claims n record positions of bin b's region (u16 pairs); positions at or
  // past the region's end take the overflow table instead
  auto claim = [&](uint32_t b, uint32_t n) -> uint32_t {
    const uint32_t sh = (b & 1u) * 16;
    return (atomicAdd(&rcnw[b >> 1], n << sh) >> sh) & 0xFFFFu;
  };
  auto place = [&](uint64_t m, uint64_t d, bool err, uint32_t ws) {
    const uint32_t h0 = hot_home(m);
    const ulonglong2 hk = *reinterpret_cast<const ulonglong2 *>(hkey + h0);
    if (hk.x == m || hk.y == m) {
      hot_acc(h0 + (hk.x == m ? 0u : 1u), m, d, err, ws);
      return;
    }
    const uint32_t bk = bucket_lds<1>(d, lbins, P);
    if (__builtin_expect(d > kRecDurMask, 0)) {  // beyond the record's duration bits: the direct path
      n_drop += bt_cold_direct(kp, m, d, bk, err, ws);
      return;
    }
    const uint32_t b = (uint32_t)(m >> kBinShift), sh = (b & 1u) * 16;
    const uint32_t c = (atomicAdd(&fillw[b >> 1], 1u << sh) >> sh) & 0xFFFFu;
    const ulonglong2 rec = make_ulonglong2((m & kBinRest) | (err ? (1ULL << 63) | ((uint64_t)ws << kBinShift) : 0ULL),
                                           d | ((uint64_t)bk << kRecDurBits));
    if (c < kBtStage) {
      stage[b * kBtStage + c] = rec;
      return;
    }
    // the stage is full this round.  A key that holds two or more of its
    // slots is frequent (a hot key of a skewed mix): it moves to the overflow
    // table; any other record is stored on its own.  (The slots may hold this
    // round's records or, not yet overwritten, an earlier round's: either way
    // records of this bin, which is all the test needs.)
    uint32_t same = 0;
#pragma unroll
    for (uint32_t q = 0; q < kBtStage; ++q) same += ((stage[b * kBtStage + q].x ^ rec.x) & kBinRest) == 0 ? 1u : 0u;
    // (a frequent key the full overflow table cannot take stays a record:
    // the per-span direct path is only for a region that is used up)
    if (same >= 2 && hot_try(m, d, err, ws)) return;
    const uint32_t at = claim(b, 1);
    if (at < region) my_rec[b * bin_stride + at] = rec;
    else hot_add(m, d, err, ws);
  };
  auto hll_settle = [&](const Pending<2> &q) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (((q.hv[j] >> ((q.hoff[j] & 3u) * 8)) & 0xFFu) < q.rho[j]) {
        const uint32_t slot = atomicAdd(&hq_n[0], 1u);
        if (slot < kBtHq) hq[slot] = make_uint2(q.hoff[j], q.rho[j]);
        else hll_raise(kp->hll + q.hoff[j], q.rho[j]);
      }
    }
  };

  const uint32_t hp = P.p, lbs = P.lb_shift;
  auto step = [&](SpanTile<2> &T, uint32_t toff, uint32_t pf) {
    uint64_t m[2], d[2];
    uint32_t ws[2], hoff[2], rho[2];
    bool err[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool valid = lane_off + toff + (uint32_t)j < len;
      const uint64_t key = copy_u64(T.key[j]);  // 0 past the range
      n_zero += wave_count(valid && key == 0);
      d[j] = T.e[j] > T.s[j] ? T.e[j] - T.s[j] : 0;
      const uint32_t meta = copy_u32(T.meta[j]);
      const uint32_t svc = meta & 0xFFFFu;
      const bool svc_ok = svc < P.n_services;
      ws[j] = window_slot_lean(P, T.e[j]);
      const bool win_ok = ws[j] != 0xFFFFFFFFu;
      n_badsvc += wave_count(valid && !svc_ok);
      n_oor += wave_count(valid && svc_ok && !win_ok);
      const bool sk = valid && svc_ok && win_ok;
      err[j] = sk && ((meta >> 19) & 3u) == 2u;
      // the span hash on 32-bit halves, rho without 64-bit shifts, the
      // register row by a 24-bit multiply-add (as the lean C2 kernel)
      const H64 x = xxh64_16_h(T.a[j], T.b[j]);
      const uint32_t yh = __builtin_amdgcn_alignbit(x.hi, x.lo, 32 - hp), yl = (x.lo << hp) | (1u << (hp - 1));
      const uint32_t r = (uint32_t)__clzll((long long)(((uint64_t)yh << 32) | yl)) + 1;
      uint32_t row;
      asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(row) : "v"(ws[j]), "s"(P.n_services), "v"(svc));
      const uint32_t ho = sk ? (row << hp) + (x.hi >> (32 - hp)) : 0u;
      bool up = sk && !(MODE & 2);
      if (lb_on) {
        const bool f = r <= llb[ho >> lbs];
        n_filt += (up && f) ? 1u : 0u;
        up = up && !f;
      }
      rho[j] = up ? r : 0u;
      hoff[j] = up ? ho : 0u;
      m[j] = key * P.kmul;
    }
    uint32_t hv[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
      hv[j] = (MODE & 2) ? 0xFFFFFFFFu : *reinterpret_cast<const uint32_t *>(P.hll + (hoff[j] & ~3u));
    __builtin_amdgcn_sched_barrier(0);
    load_tile_at<2, 2>(P, lo + pf, tremain(pf), lane_off, T);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (MODE & 1) n_drop += (uint32_t)((m[j] ^ d[j]) == 0x123456789ABCULL);  // keep the values live
      else if (m[j] != 0) place(m[j], d[j], err[j], ws[j]);
    }
    hll_settle(pend2);
    pend2 = pend;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      pend.hoff[j] = hoff[j];
      pend.rho[j] = rho[j];
      pend.hv[j] = hv[j];
    }
  };
  // the waves write out the full stages of their 128 bins (4 lanes a stage)
  uint16_t *wl = flist + wave * 128;
  auto flush = [&]() {
    const uint32_t fw = fillw[threadIdx.x];  // bins 2t, 2t + 1
    const bool f0 = (fw & 0xFFFFu) >= kBtStage, f1 = (fw >> 16) >= kBtStage;
    if (f0 || f1) fillw[threadIdx.x] = (f0 ? 0u : (fw & 0xFFFFu)) | (f1 ? 0u : (fw & 0xFFFF0000u));
    const uint64_t m0 = __ballot(f0), m1 = __ballot(f1);
    const uint32_t n0 = (uint32_t)__popcll(m0), nf = n0 + (uint32_t)__popcll(m1);
    if (f0) wl[lane_rank(m0)] = (uint16_t)(2 * threadIdx.x);
    if (f1) wl[n0 + lane_rank(m1)] = (uint16_t)(2 * threadIdx.x + 1);
    compiler_fence();  // one wave's LDS operations complete in order
    for (uint32_t i0 = 0; i0 < nf; i0 += 16) {  // wave-uniform
      const uint32_t i = i0 + (lane >> 2), q = lane & 3u;
      const bool act = i < nf;
      const uint32_t b = act ? wl[i] : 0u;
      const ulonglong2 r = stage[b * kBtStage + q];
      uint32_t at = act && q == 0 ? claim(b, kBtStage) : 0u;
      at = (uint32_t)__shfl((int)at, (int)(lane & ~3u), 64);
      if (act) {
        if (MODE & 16) my_rec[(uint64_t)threadIdx.x * 64 + ((i0 + at) & 63)] = r;  // ablation: no scatter
        else if (MODE & 32) (void)0;                                          // ablation: no store
        else if (at + q < region) my_rec[b * bin_stride + at + q] = r;
        else hot_rec(b, r);
      }
    }
  };

  // Stage flushes: after every round, or -- once the first two rounds have
  // put 32 or more keys in the overflow table (a skewed mix, whose hot keys
  // bypass the stages) -- after every second round, which halves the
  // barriers (for uniform keys the fuller stages would spill more records).
  bool sparse = false;  // workgroup-uniform: read from LDS after a barrier
  for (uint32_t r = 0; r < rounds; r += 2) {
    step(buf[0], tstart(r), tstart(r + 2));
    if (!sparse) {
      __syncthreads();
      if (!(MODE & 1)) flush();
      __syncthreads();
    }
    if (r + 1 < rounds) step(buf[1], tstart(r + 1), tstart(r + 3));
    __syncthreads();
    if (!(MODE & 1)) flush();
    if (r == 0 && wave == 0) {
      uint32_t used = 0;
      for (uint32_t h = lane; h < kBt2Hot; h += 64) used += wave_count(hkey[h] != 0);
      if (lane == 0) hq_n[2] = used >= 32 ? 1u : 0u;
    }
    __syncthreads();
    if (r == 0) sparse = (MODE & 64) ? true : hq_n[2] != 0;
  }
  hll_settle(pend2);
  hll_settle(pend);
  // the wave's bound sub-block, loaded now (hll_lb_pre): it lands during the
  // stage flush and the overflow table's key lookups below
  uint4 lbv[4];
  hll_lb_pre<kBtBlock>(P, lbv);
  bt_stamp(P, sbase, 2);
  // partial stages, then this workgroup's region fills
  for (uint32_t b = threadIdx.x; b < kPartBins; b += kBtBlock) {
    const uint32_t c = (fillw[b >> 1] >> ((b & 1u) * 16)) & 0xFFFFu;  // < kBtStage after the last flush
    const uint32_t at = c ? claim(b, c) : 0u;
    for (uint32_t q = 0; q < c; ++q) {
      if (at + q < region) my_rec[b * bin_stride + at + q] = stage[b * kBtStage + q];
      else hot_rec(b, stage[b * kBtStage + q]);
    }
  }
  __syncthreads();
  // the queued HLL raises' register words, read now (the queue is final after
  // the barrier above) and CAS-raised at the end: the reads overlap the
  // overflow table's lookups instead of adding a round trip
  const uint32_t nq = min(hq_n[0], kBtHq);
  constexpr uint32_t kQ = (kBtHq + kBtBlock - 1) / kBtBlock;
  uint32_t qv[kQ];
#pragma unroll
  for (uint32_t i = 0; i < kQ; ++i) {
    const uint32_t t = threadIdx.x + i * kBtBlock;
    qv[i] = t < nq ? __hip_atomic_load(reinterpret_cast<const uint32_t *>(P.hll + (hq[t].x & ~3u)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT)
                   : 0u;
  }
  for (uint32_t b = threadIdx.x; b < kPartBins; b += kBtBlock)
    P.bt_cnt[(uint64_t)b * P.bt_grid + blockIdx.x] = min((rcnw[b >> 1] >> ((b & 1u) * 16)) & 0xFFFFu, region);
  __syncthreads();
  // the overflow table: each entry's key slot (find-or-insert, one lane per
  // entry) into the LDS of the flush lists (the stages are all out) ...
  uint32_t *hslot = reinterpret_cast<uint32_t *>(flist);  // [kBt2Hot]
  for (uint32_t h = threadIdx.x; h < kBt2Hot; h += kBtBlock) {
    const unsigned long long m = hkey[h];
    uint32_t s = kNotFound;
    if (m != 0) {
      s = bt_find_insert(P.gkeys, m, P.log2sb);
      if (s == kNotFound)
        for (uint32_t b = 0; b < P.nbk; ++b) n_drop += (hcnt[h * kPartWords + (b >> 1)] >> ((b & 1u) * 16)) & 0xFFFFu;
    }
    hslot[h] = s;
  }
  __syncthreads();
  // ... then its row added to the spill array (atomics: the entries of one key
  // come from every workgroup), two entries per wave instruction and one cell
  // per lane: an entry's nbk counts and ns sum are contiguous in base64, so it
  // leaves as three 64-B atomic requests, where one lane's nbk + 1 serial
  // atomics made a Zipf mix's epilogue (hundreds of hot keys in every
  // workgroup's table) the scatter's longest phase
  {
    const uint32_t half = lane >> 5, cell = lane & 31u, nc = P.nbk + 1;
    static_assert(kBt2Hot % 2 == 0 && kPartMaxBk + 1 <= 32, "overflow flush geometry");
    for (uint32_t h0 = wave * 2; h0 < kBt2Hot; h0 += kWaves * 2) {
      const uint32_t h = h0 + half;
      const uint32_t s = hslot[h];
      if (s == kNotFound || cell >= nc) continue;
      const unsigned long long v = cell == P.nbk ? hsum[h]
                                                 : (hcnt[h * kPartWords + (cell >> 1)] >> ((cell & 1u) * 16)) & 0xFFFFu;
      if (v) atomicAdd(P.base64 + (uint64_t)s * nc + cell, v);
    }
  }
  if (threadIdx.x < kBt2HotErr) {
    const uint2 e = herr[threadIdx.x];
    if (e.x) {
      const uint32_t ws = (e.x - 1) >> 8, h = (e.x - 1) & 0xFFu;
      const uint32_t s = hslot[h];
      if (s != kNotFound) atomicAdd(P.errcnt + ((uint64_t)ws << P.log2cap) + s, (unsigned long long)e.y);
      else
        for (uint32_t i = 0; i < e.y; ++i) bt_cms_add(kp, ws, hkey[h] * P.kinv);
    }
  }
#pragma unroll
  for (uint32_t i = 0; i < kQ; ++i) {
    const uint32_t t = threadIdx.x + i * kBtBlock;
    if (t >= nq) continue;
    const uint2 q = hq[t];
    SA_GLOBAL uint32_t *word = gbl(reinterpret_cast<uint32_t *>(P.hll + (q.x & ~3u)));
    const uint32_t sh = (q.x & 3u) * 8;
    uint32_t old = qv[i];
    while (((old >> sh) & 0xFFu) < q.y) {  // a failed CAS refreshes `old`
      const uint32_t nw = (old & ~(0xFFu << sh)) | (q.y << sh);
      if (__hip_atomic_compare_exchange_strong(word, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT))
        break;
    }
  }
  n_drop = wave_sum(n_drop);
  n_filt = wave_sum(n_filt);
  if (lane == 0) {
    // a slot per workgroup (same-address atomics from every wave would
    // serialise the tail of the launch)
    if (n_filt) atomicAdd(&P.hll_filt[blockIdx.x & (kFiltSlots - 1)], (unsigned long long)n_filt);
    if (n_zero) atomicAdd(&P.stats[kStatZeroKey], (unsigned long long)n_zero);
    if (n_badsvc) atomicAdd(&P.stats[kStatInvalidService], (unsigned long long)n_badsvc);
    if (n_oor) atomicAdd(&P.stats[kStatWindowOOR], (unsigned long long)n_oor);
    if (n_drop) atomicAdd(&P.stats[kStatDropped], (unsigned long long)n_drop);
  }
  hll_lb_finish<kBtBlock>(P, lbv);
  bt_stamp(P, sbase, 3);
}

// Aggregate geometry (bt_aggregate3_kernel; the laboratory build's earlier
// form bt_aggregate2_kernel shares it).  One 512-thread workgroup per bin;
// its LDS holds the bin's key slots (mirror), u64 ns sums and u16 bucket
// counts (17 per slot, packed), an ERROR table and the region fills: 53 KiB
// at 1,024 slots, so three workgroups share a CU.  No prefix scan: each
// wave-instruction reads two regions (lanes 0-31 and 32-63, one record per
// lane), a wave takes every eighth region pair and issues its loads in
// batches of eight before it aggregates them.  Then each touched slot's u32
// row is read, added to and written back (all reads first).
constexpr uint32_t kBtAgg2Block = 512;
constexpr uint32_t kBtAgg2Err = 128;
__host__ __device__ inline uint32_t bt_agg2_cnt_words(uint32_t sb) { return (sb * kPartMaxBk + 1) / 2; }
__host__ __device__ inline uint32_t bt_agg2_off_err(uint32_t sb) { return (sb * 16 + bt_agg2_cnt_words(sb) * 4 + 7) & ~7u; }
__host__ __device__ inline uint32_t bt_agg2_off_reg(uint32_t sb) { return bt_agg2_off_err(sb) + kBtAgg2Err * 8; }



// Aggregate, third form (the default).  The layout, phases and row
// write-back of bt_aggregate2_kernel; the records go through the LDS two per
// lane at a time with every LDS access of the pair issued before the first
// one is waited for -- both records' two key buckets (4 x ds_read_b128 each),
// then the compares, then both records' counter atomics -- instead of one
// record's dependent chain after another (a record costs ~6 LDS round trips
// in sequence there).  Records carry their bucket (the scatter's bin table),
// so there is no per-record bucketing.  A key missing from its two buckets
// (new in the bin, or placed past them) takes the probe loop, rare after the
// first launches.  ERROR records append (window slot, key slot) to an LDS
// list, added to errcnt after the records (global atomics past the list's
// 255).  The record loop keeps its VALU lean -- 32-bit key arithmetic
// (records carry m's low 53 bits, so m's high word is (x.hi & 0x1FFFFF) |
// bin << 21), load offsets stepped per batch, the in-bucket slot picked as an
// index 0-7 by inline-constant selects -- and its batches of two region pairs
// are double-buffered: the next batch's loads are issued before this one goes
// through the LDS.
// MODE (ablation): 1 = no records aggregated, 2 = no key / row write-back,
// 16 = no lookup reads, 32 = no counter atomics.
template <int MODE = 0, int MAXPER = 2, int BLOCK = 512>
__global__ __launch_bounds__(BLOCK, BLOCK == 1024 ? 8 : 6) void bt_aggregate3_kernel(IngestParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t log2sb = P.log2sb, sb = 1u << log2sb;
  // record sets: one, or two (P.bt_rec2: two launches' scatters aggregated
  // together, so the bin's setup and row write-back serve both)
  const uint32_t nrs = cold_params().bt_rec2 ? 2u : 1u;
  const uint32_t Gmax = nrs == 2 && cold_params().bt_grid2 > P.bt_grid ? cold_params().bt_grid2 : P.bt_grid;
  const uint32_t bin = blockIdx.x;
  unsigned long long *lkeys = reinterpret_cast<unsigned long long *>(smem);
  unsigned long long *lsum = lkeys + sb;
  uint32_t *lcnt = reinterpret_cast<uint32_t *>(lsum + sb);  // u16 [sb][17], packed
  constexpr uint32_t kErrL = kBtAgg2Err * 2;                  // u32 words in the etab space
  uint32_t *errl = reinterpret_cast<uint32_t *>(smem + bt_agg2_off_err(sb));  // [0] count, [1..] ek + 1
  uint32_t *rcnt = reinterpret_cast<uint32_t *>(smem + bt_agg2_off_reg(sb));  // [G] region fills (the set's)
  uint32_t *misc = rcnt + Gmax;  // [0] dropped
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  unsigned long long *gk = P.gkeys + ((uint64_t)bin << log2sb);
  bt_stamp(P, (uint64_t)bin * 8, 0);

  // 1. the bin's key slots (kept in registers to find the new ones later),
  //    region fills, zeroed counters
  constexpr int kMaxPer = MAXPER;
  unsigned long long orig[kMaxPer];
#pragma unroll
  for (int u = 0; u < kMaxPer; ++u) {
    const uint32_t s = tid + u * BLOCK;
    orig[u] = s < sb ? gk[s] : 0ULL;
  }
  for (uint32_t g = tid; g < P.bt_grid; g += BLOCK) rcnt[g] = P.bt_cnt[(uint64_t)bin * P.bt_grid + g];
#pragma unroll
  for (int u = 0; u < kMaxPer; ++u) {
    const uint32_t s = tid + u * BLOCK;
    if (s < sb) {
      lkeys[s] = orig[u];
      lsum[s] = 0;
    }
  }
  const uint32_t cw = bt_agg2_cnt_words(sb);
  for (uint32_t i = tid; i < cw; i += BLOCK) lcnt[i] = 0;
  if (tid == 0) errl[0] = misc[0] = 0;
  __syncthreads();
  bt_stamp(P, (uint64_t)bin * 8, 1);

  // 2. the records, set by set
  const uint32_t half = lane >> 5, r0 = lane & 31u;
  const uint32_t pmax = bt_probe_max(log2sb);
  uint32_t n_drop = 0;
  const ulonglong2 *lk2 = reinterpret_cast<const ulonglong2 *>(lkeys);
  const uint32_t binhi = bin << (kBinShift - 32);
  const uint32_t sh = 34 - log2sb;  // bt_seq: the top (log2sb - 2) bits
  // two records (ok: valid) through the LDS together
  auto agg_pair = [&](const ulonglong2 (&v)[2], const bool (&ok)[2]) {
    uint32_t mlo[2], mhi[2], b1[2], b2[2];
    ulonglong2 q[2][4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      mlo[k] = (uint32_t)v[k].x;
      mhi[k] = (((uint32_t)(v[k].x >> 32)) & ((1u << (kBinShift - 32)) - 1)) | binhi;
      // bt_seq on the 32-bit halves
      const uint32_t h1 = (mlo[k] ^ __builtin_amdgcn_alignbit(mhi[k], mlo[k], 29)) * 0x9E3779B1u;
      const uint32_t h2 = (h1 ^ (h1 >> 16)) * 0x85EBCA6Bu;
      b1[k] = h1 >> sh;
      b2[k] = h2 >> sh;
      if (MODE & 16) {  // ablation: no lookup reads (every key taken as slot 0 of its first bucket)
        q[k][0] = make_ulonglong2(((uint64_t)mhi[k] << 32) | mlo[k], 0);
        q[k][1] = q[k][2] = q[k][3] = make_ulonglong2(0, 0);
        continue;
      }
      q[k][0] = lk2[b1[k] * 2];
      q[k][1] = lk2[b1[k] * 2 + 1];
      q[k][2] = lk2[b2[k] * 2];
      q[k][3] = lk2[b2[k] * 2 + 1];
    }
    // position in the two buckets (8: not there)
    uint32_t s[2], j[2] = {8u, 8u};
    uint64_t mm[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) mm[k] = ((uint64_t)mhi[k] << 32) | mlo[k];
#pragma unroll
    for (int i = 7; i >= 0; --i) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const unsigned long long w = (i & 1) ? q[k][i >> 1].y : q[k][i >> 1].x;
        j[k] = w == mm[k] ? (uint32_t)i : j[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t sl = ((j[k] < 4 ? b1[k] : b2[k]) << 2) | (j[k] & 3u);
      s[k] = j[k] < 8 ? sl : kNotFound;
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (__builtin_expect(ok[k] && s[k] == kNotFound, 0)) {  // probe / insert in the mirror
        const BtSeq bq = bt_seq(mm[k], log2sb);
        uint32_t i = 0, sl = kNotFound;
        for (; i < pmax; ++i) {
          sl = bt_pos(bq, i);
          unsigned long long kk = lkeys[sl];
          if (kk == 0) kk = atomicCAS(&lkeys[sl], 0ULL, (unsigned long long)mm[k]);
          if (kk == 0 || kk == mm[k]) break;
        }
        s[k] = i == pmax ? kNotFound - 1 : sl;  // kNotFound - 1: the bin's sub-table is full
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (!ok[k]) continue;
      const uint32_t xhi = (uint32_t)(v[k].x >> 32);
      const bool err = (int32_t)xhi < 0;
      const uint32_t ws = (xhi >> (kBinShift - 32)) & 1023u;
      if (__builtin_expect(s[k] == kNotFound - 1, 0)) {  // dropped
        ++n_drop;
        if (err) bt_cms_add(kernel_params(), ws, mm[k] * P.kinv);
        continue;
      }
      const uint32_t yhi = (uint32_t)(v[k].y >> 32);
      uint32_t h;  // the (slot, bucket) u16 counter: s * 17 + bucket
      asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(h) : "v"(s[k]), "i"(kPartMaxBk), "v"(yhi >> (kRecDurBits - 32)));
      if (MODE & 32) {  // ablation: no counter atomics
        n_drop += (h == 0xFFFFFFFu) ? 1u : 0u;
      } else {
        atomicAdd(&lcnt[h >> 1], 1u << ((h & 1u) << 4));
        atomicAdd(&lsum[s[k]], ((unsigned long long)(yhi & ((1u << (kRecDurBits - 32)) - 1)) << 32) | (uint32_t)v[k].y);
      }
      if (err) {
        const uint32_t ek = (ws << log2sb) | s[k];
        const uint32_t at = atomicAdd(&errl[0], 1u);
        if (at + 1 < kErrL) errl[at + 1] = ek;
        // past the LDS list: the key's canonical HBM slot (find-or-insert), so
        // the count stays right if the write-back relocates the key
        else bt_cold_err(kernel_params(), mm[k], ws);
      }
    }
  };
  constexpr uint32_t kWaves = BLOCK / 64;
#pragma unroll 1
  for (uint32_t rs = 0; rs < nrs; ++rs) {
    // (the second set's parameters through the kernarg pointer: read where
    // they are used, so they hold no scalar registers across the first set)
    SA_CONST const IngestParams &Q = cold_params();
    const uint32_t G = rs ? Q.bt_grid2 : P.bt_grid, region = rs ? Q.bt_region2 : P.bt_region;
    if (rs) {  // the second set's region fills (every wave is past the first set's records)
      __syncthreads();
      for (uint32_t g = tid; g < G; g += BLOCK) rcnt[g] = Q.bt_cnt2[(uint64_t)bin * G + g];
      __syncthreads();
    }
    const ulonglong2 *bin_rec = (rs ? Q.bt_rec2 : P.bt_rec) + (uint64_t)bin * G * region;
    const __amdgpu_buffer_rsrc_t rrec = rsrc(bin_rec, G * region * 16);
    const uint32_t pairs = (G + 1) / 2;
    if (!(MODE & 1)) {
      // the wave's region pairs p = wave + 8 j; this lane's region g = 2 p +
      // half, its byte offset stepped by 16 regions per pair.  Batches of two
      // pairs, double-buffered (a batch past the bin's regions loads nothing
      // and adds nothing).
      const uint32_t g0 = 2 * wave + half;
      const uint32_t rstep = 2 * kWaves * region * 16;
      uint32_t roff = (g0 * region + r0) * 16;
      uint32_t goff = g0;
      auto issue = [&](ulonglong2 (&v)[2], bool (&ok)[2]) {
#pragma unroll
        for (uint32_t b = 0; b < 2; ++b) {
          const uint32_t g = goff + b * 2 * kWaves;
          const uint32_t c = rcnt[g < G ? g : 0u];
          ok[b] = g < G && r0 < c;
          const auto x = __builtin_amdgcn_raw_buffer_load_b128(rrec, (int)(ok[b] ? roff + b * rstep : 0xFFFFFFF0u), 0, 2);
          v[b] = make_ulonglong2((uint64_t)x[0] | ((uint64_t)x[1] << 32), (uint64_t)x[2] | ((uint64_t)x[3] << 32));
        }
        roff += 2 * rstep;
        goff += 4 * kWaves;
      };
      ulonglong2 va[2], vb[2];
      bool oka[2], okb[2];
      issue(va, oka);
      for (uint32_t p0 = wave; p0 < pairs; p0 += kWaves * 4) {
        issue(vb, okb);
        agg_pair(va, oka);
        issue(va, oka);
        agg_pair(vb, okb);
      }
      // regions longer than 32 records: the rest, one record per lane
#pragma unroll 1
      for (uint32_t p = wave; p < pairs; p += kWaves) {
        const uint32_t g = 2 * p + half;
        const uint32_t c = g < G ? rcnt[g] : 0u;
        for (uint32_t r = 32 + r0; r < c; r += 32) {
          const ulonglong2 vv[2] = {bin_rec[(uint64_t)g * region + r], make_ulonglong2(0, 0)};
          const bool ok[2] = {true, false};
          agg_pair(vv, ok);
        }
      }
    }
  }
  // the rows of the slots the bin held at setup, loaded by each wave right
  // after its records, before the barrier: waves end their records at
  // different times, so these loads land while the last ones work, and the
  // write-back below reads HBM only for keys new to the bin (a slot that held
  // a key keeps it; the rows are this aggregate's alone)
  uint4 *rows = reinterpret_cast<uint4 *>(P.gcounts) + ((uint64_t)bin << log2sb) * (kRowBytes / 16);
  uint4 rpre[kMaxPer][2];
#pragma unroll
  for (int u = 0; u < kMaxPer; ++u) {
    const uint32_t s = tid + u * BLOCK;
#pragma unroll
    for (uint32_t q = 0; q < 2; ++q)
      rpre[u][q] = s < sb && orig[u] != 0 && !(MODE & 2) ? rows[(uint64_t)s * 2 + q] : make_uint4(0, 0, 0, 0);
  }
  n_drop = wave_sum(n_drop);
  if (lane == 0 && n_drop) atomicAdd(&misc[0], n_drop);
  __syncthreads();
  bt_stamp(P, (uint64_t)bin * 8, 2);

  // 3. new keys and touched rows of the bin (one owner: plain stores; every
  //    row read is issued before the first row is written); the ERROR list.
  //    The next launch's scatter may run beside this aggregate (the engine
  //    overlaps them, section "launch pipeline" of spanagg_engine.cpp) and
  //    CAS-insert keys into this bin's HBM sub-table meanwhile, so a key this
  //    aggregate added to its LDS mirror is inserted into HBM by the same
  //    find-or-insert the scatter uses: slots never empty and every inserter
  //    probes one sequence, so the HBM table stays free of duplicates.  When
  //    the key lands in another slot than its LDS one (a concurrent insert
  //    took that slot or an earlier one of the key's sequence), its counts go
  //    to that slot's spill-array cells by atomics and the LDS slot's row is
  //    left alone; lsum[s] then carries the relocated slot for the ERROR list.
  if (MODE & 2) return;
  const uint32_t nbk = P.nbk;
  constexpr unsigned long long kMoved = 1ULL << 63;  // lsum[s] after the write-back: kMoved | new slot (or kNotFound)
  uint4 rv[kMaxPer][2];
  bool touched[kMaxPer];
  uint32_t hs[kMaxPer];  // the HBM slot (in the whole table) holding lkeys[s]
#pragma unroll
  for (int u = 0; u < kMaxPer; ++u) {
    const uint32_t s = tid + u * BLOCK;
    hs[u] = (bin << log2sb) | s;
    if (s < sb && lkeys[s] != orig[u]) {
      const uint32_t f = bt_find_insert(P.gkeys, lkeys[s], log2sb);
      hs[u] = f;  // kNotFound: the bin's HBM sub-table filled meanwhile
    }
    touched[u] = s < sb && lsum[s] != 0;
    if (s < sb && !touched[u]) {  // a zero ns sum: look at the counts
      uint32_t any = 0;
      for (uint32_t b = 0; b < nbk; ++b) {
        const uint32_t h = s * kPartMaxBk + b;
        any |= (lcnt[h >> 1] >> ((h & 1u) * 16)) & 0xFFFFu;
      }
      touched[u] = any != 0;
    }
    const bool own = hs[u] == ((bin << log2sb) | s);
#pragma unroll
    for (uint32_t q = 0; q < 2; ++q)
      rv[u][q] = !(touched[u] && own) ? make_uint4(0, 0, 0, 0)
                 : orig[u] != 0  ? rpre[u][q]
                                 : rows[(uint64_t)s * 2 + q];
  }
  uint32_t n_lost = 0;
#pragma unroll
  for (int u = 0; u < kMaxPer; ++u) {
    const uint32_t s = tid + u * BLOCK;
    if (s >= sb) continue;
    const bool own = hs[u] == ((bin << log2sb) | s);
    const unsigned long long ls = lsum[s];
    lsum[s] = own ? 0ULL : kMoved | hs[u];
    if (!touched[u]) continue;
    if (!own) {  // relocated (or lost): the counts by atomics into the spill array
      for (uint32_t b = 0; b < nbk; ++b) {
        const uint32_t h = s * kPartMaxBk + b;
        const uint32_t c = (lcnt[h >> 1] >> ((h & 1u) * 16)) & 0xFFFFu;
        if (hs[u] == kNotFound) n_lost += c;
        else if (c) atomicAdd(P.base64 + (uint64_t)hs[u] * (nbk + 1) + b, (unsigned long long)c);
      }
      if (hs[u] != kNotFound && ls) atomicAdd(P.base64 + (uint64_t)hs[u] * (nbk + 1) + nbk, ls);
      continue;
    }
    const uint32_t w[8] = {rv[u][0].x, rv[u][0].y, rv[u][0].z, rv[u][0].w,
                           rv[u][1].x, rv[u][1].y, rv[u][1].z, rv[u][1].w};
    const unsigned long long sum = ((unsigned long long)w[1] << 32 | w[0]) + ls;  // (lsum[s] now holds the relocation mark)
    uint32_t c[kPartMaxBk];
    bool spill = false;
#pragma unroll
    for (uint32_t b = 0; b < kPartMaxBk; ++b) {
      const uint32_t h = s * kPartMaxBk + b;
      c[b] = b < nbk ? ((w[2 + b / 4] >> ((b & 3u) * 8)) & 0xFFu) + ((lcnt[h >> 1] >> ((h & 1u) * 16)) & 0xFFFFu)
                     : 0u;
      spill |= c[b] > 0xFFu;
    }
    uint32_t o[6] = {0, 0, 0, 0, 0, 0};
    if (spill) {  // the row's counts move to the spill array (atomics: the scatter adds there too)
      unsigned long long *sp = P.base64 + ((uint64_t)bin << log2sb | s) * (nbk + 1);
#pragma unroll
      for (uint32_t b = 0; b < kPartMaxBk; ++b)
        if (c[b]) atomicAdd(sp + b, (unsigned long long)c[b]);
    } else {
#pragma unroll
      for (uint32_t b = 0; b < kPartMaxBk; ++b) o[b / 4] |= c[b] << ((b & 3u) * 8);
    }
    rows[(uint64_t)s * 2] = make_uint4((uint32_t)sum, (uint32_t)(sum >> 32), o[0], o[1]);
    rows[(uint64_t)s * 2 + 1] = make_uint4(o[2], o[3], o[4], o[5]);
  }
  n_lost = wave_sum(n_lost);
  if (lane == 0 && n_lost) atomicAdd(&misc[0], n_lost);
  __syncthreads();  // lsum carries the relocations for the ERROR list
  const uint32_t ne = min(errl[0], kErrL - 1);
  for (uint32_t i = tid; i < ne; i += BLOCK) {
    const uint32_t ek = errl[i + 1], ws = ek >> log2sb, s = ek & (sb - 1);
    const unsigned long long mv = lsum[s];
    const uint32_t slot = (mv & kMoved) ? (uint32_t)mv : ((bin << log2sb) | s);
    if (slot != kNotFound) atomicAdd(P.errcnt + ((uint64_t)ws << P.log2cap) + slot, 1ULL);
    else bt_cms_add(kernel_params(), ws, lkeys[s] * P.kinv);
  }
  if (tid == 0 && misc[0]) atomicAdd(&P.stats[kStatDropped], (unsigned long long)misc[0]);
  bt_stamp(P, (uint64_t)bin * 8, 3);
}

}  // namespace

#ifdef SPANAGG_AB
// the laboratory build's earlier aggregate form, ablation instances and
// kernel selection (tools/ A/B runs; never in libspanagg.so)
#include "lab/binned_lab.inc"
#else
// Product build: one scatter and one aggregate (bins of up to 1,024 slots, or
// the wide form for 2,048).
static const void *bt_scatter2_fn(uint32_t) { return (const void *)&bt_scatter2_kernel<0>; }
constexpr uint32_t kDiagBtAggWide = 1u << 30;
static const void *bt_agg_fn(uint32_t diag) {
  return (diag & kDiagBtAggWide) ? (const void *)&bt_aggregate3_kernel<0, 4> : (const void *)&bt_aggregate3_kernel<0, 2>;
}
hipError_t prepare_ingest_bt(size_t agg_lds) {
  if (hipError_t e = hipFuncSetAttribute(bt_scatter2_fn(0), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)kBt2ScatterLds);
      e != hipSuccess)
    return e;
  for (uint32_t v : {0u, kDiagBtAggWide})
    if (hipError_t e = hipFuncSetAttribute(bt_agg_fn(v), hipFuncAttributeMaxDynamicSharedMemorySize, (int)agg_lds);
        e != hipSuccess)
      return e;
  return hipSuccess;
}
constexpr uint32_t kDiagBtNoScatter = 0, kDiagBtNoAgg = 0;
static uint32_t bt_agg_block() { return kBtAgg2Block; }
#endif

hipError_t launch_bt_scatter(const IngestParams &P, hipStream_t s) {
  if (P.diag & kDiagBtNoScatter) return hipSuccess;
  void *args[] = {const_cast<IngestParams *>(&P)};
  return hipLaunchKernel(bt_scatter2_fn(P.diag), dim3(P.bt_grid), dim3(kBtBlock), args, kBt2ScatterLds, s);
}

hipError_t launch_bt_aggregate(const IngestParams &P, hipStream_t s) {
  if (P.diag & kDiagBtNoAgg) return hipSuccess;
  void *args[] = {const_cast<IngestParams *>(&P)};
  const uint32_t diag = P.diag | (P.log2sb > 10 ? kDiagBtAggWide : 0u);
  // (two record sets: the region-fill array holds the larger set's)
  const uint32_t g = P.bt_rec2 && P.bt_grid2 > P.bt_grid ? P.bt_grid2 : P.bt_grid;
  return hipLaunchKernel(bt_agg_fn(diag), dim3(kPartBins), dim3(bt_agg_block()), args, bt_agg2_lds_bytes(P.log2sb, g),
                         s);
}

size_t bt_agg2_lds_bytes(uint32_t log2sb, uint32_t grid) {
  return bt_agg2_off_reg(1u << log2sb) + (size_t)grid * 4 + 16;
}

}  // namespace sa
