// sa_device.h -- device-side helpers shared by the gfx950 kernels of libspanagg
// (spanagg_kernels.hip: small-table, HBM-table and round-1 partitioned paths;
// spanagg_binned.hip: the binned-table high-cardinality path).
#pragma once
#include "sa_internal.h"

namespace sa {
namespace {

constexpr uint64_t XP1 = 0x9E3779B185EBCA87ULL;
constexpr uint64_t XP2 = 0xC2B2AE3D27D4EB4FULL;
constexpr uint64_t XP3 = 0x165667B19E3779F9ULL;
constexpr uint64_t XP4 = 0x85EBCA77C2B2AE63ULL;
constexpr uint64_t XP5 = 0x27D4EB2F165667C5ULL;

__device__ __forceinline__ uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// Fast path of the bucket index of a duration d > 0 ns at `scale`: log2 of the
// value from d's exponent, v_log_f32 of its leading 24 bits (as a mantissa in
// [1, 2)) and log2(div), all exact or nearly so (the hardware log2 over every
// float in [1, 2) is within 2^-20, measured exhaustively by test_gpu_expo.py's
// test_fast_log2_error_bound; d's rounding to a float and the fixed-point
// conversions add the rest of kFastFxErr).  When the scaled value is farther than its error bound from an
// integer, its floor is the index Go's math.Log computation gives (that one is
// within ~1e-9 of the exact value at any scale <= 20); otherwise -- including
// every power of two and every value near a bucket boundary -- false, and the
// caller takes the exact path.
// 32-bit arithmetic only: z = log2(d / div) in 8.24 fixed point (l2d_q24 =
// log2(div) * 2^24 rounded; d as a float, split by frexp; the mantissa's log2
// converted with 24 fraction bits),
// so the scaled value's integer part is z's bits above 24 - scale and its
// distance to an integer is read from the bits below.  kFastFxErr, in units
// of 2^-24: the hardware log2's 2^-20 (16), d as a float (|f / d - 1| <=
// 2^-23: <= 2.9 in log2), the mantissa log's and log2(div)'s conversions
// (< 1.5), rounded up with margin.
constexpr int32_t kFastFxErr = 24;
__device__ __forceinline__ bool expo_index_fast(uint64_t d, int32_t l2d_q24, int32_t scale, int32_t &idx) {
  // d as a float: the high word exactly below 2^24 (else rounded), the low
  // word rounded, one rounding of the sum -- |f / d - 1| <= 2^-23
  const float f = __builtin_fmaf((float)(uint32_t)(d >> 32), 0x1p32f, (float)(uint32_t)d);
  int32_t ef;
  const float m = frexpf(f, &ef) * 2.0f;  // f = m * 2^(ef - 1), m in [1, 2)
  const int32_t e = ef - 1;
  const int32_t t = (int32_t)(__builtin_amdgcn_logf(m) * 0x1p24f);  // log2(m) < 1, 24 fraction bits
  const int32_t z = (e << 24) - l2d_q24 + t;                         // ~ log2(d / div) * 2^24
  const int32_t sh = scale > 0 ? 24 - scale : 24;
  const int32_t one = 1 << sh, fr = z & (one - 1);
  if (fr <= kFastFxErr || one - fr <= kFastFxErr) return false;  // near a bucket boundary / power of two
  const int32_t fl = z >> sh;                                     // floor of the scaled value
  if (scale <= 0) {
    idx = fl >> (-scale);  // Go: exponent >> -scale (z is not an integer)
    return true;
  }
  const int32_t max_index = (1024 << scale) - 1;
  idx = fl >= max_index ? max_index : fl;
  return true;
}
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

// The same hash on 32-bit halves (the lean C2 kernel): each 64-bit multiply by
// a constant is one v_mad_u64_u32 and two v_mul_lo_u32 (three quarter-rate
// ops, the minimum for a 64 x 64 -> 64 product) and each rotate a pair of
// v_alignbit.  Written on u64 values, LLVM turns rotl(x * C, 31) into a second
// multiply by C << 31 (five quarter-rate ops instead of three plus two
// alignbits) and 64-bit shifts into v_lshlrev_b64.
struct H64 {
  uint32_t lo, hi;
};
__device__ __forceinline__ H64 h64(uint64_t x) { return H64{(uint32_t)x, (uint32_t)(x >> 32)}; }
__device__ __forceinline__ H64 h64_mulc(H64 x, uint64_t c) {
  const uint32_t cl = (uint32_t)c, ch = (uint32_t)(c >> 32);
  const uint64_t p = (uint64_t)x.lo * cl;
  return H64{(uint32_t)p, (uint32_t)(p >> 32) + x.lo * ch + x.hi * cl};
}
__device__ __forceinline__ H64 h64_rotl(H64 x, int r) {  // 0 < r < 32
  return H64{__builtin_amdgcn_alignbit(x.lo, x.hi, 32 - r), __builtin_amdgcn_alignbit(x.hi, x.lo, 32 - r)};
}
__device__ __forceinline__ H64 h64_xor(H64 a, H64 b) { return H64{a.lo ^ b.lo, a.hi ^ b.hi}; }
__device__ __forceinline__ H64 h64_addc(H64 a, uint64_t c) {
  return h64((((uint64_t)a.hi << 32) | a.lo) + c);
}
__device__ __forceinline__ H64 xxh64_16_h(uint64_t a, uint64_t b) {
  H64 h = h64_xor(h64_mulc(h64_rotl(h64_mulc(h64(a), XP2), 31), XP1), h64(XP5 + 16));
  h = h64_addc(h64_mulc(h64_rotl(h, 27), XP1), XP4);
  h = h64_xor(h, h64_mulc(h64_rotl(h64_mulc(h64(b), XP2), 31), XP1));
  h = h64_addc(h64_mulc(h64_rotl(h, 27), XP1), XP4);
  h.lo ^= h.hi >> 1;  // h ^= h >> 33
  h = h64_mulc(h, XP2);
  h = H64{h.lo ^ __builtin_amdgcn_alignbit(h.hi, h.lo, 29), h.hi ^ (h.hi >> 29)};  // h ^= h >> 29
  h = h64_mulc(h, XP3);
  h.lo ^= h.hi;  // h ^= h >> 32
  return h;
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// floor(n / d) with magic = floor((2^64-1)/d): the estimate is low by at most
// 2, fixed by two branch-free correction steps.
__device__ __forceinline__ uint64_t fast_div(uint64_t n, uint64_t d, uint64_t magic) {
  uint64_t q = __umul64hi(n, magic);
  uint64_t r = n - q * d;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const bool c = r >= d;
    q += c ? 1 : 0;
    r -= c ? d : 0;
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

// Find-or-insert along the key's probe sequence (sa_internal.h), starting at
// sequence position i0; kNotFound when the table is full.  Slots only ever go
// from 0 to a key, so a plain (possibly stale, L2-cached) read is safe: a
// stale 0 is corrected by the CAS, which returns the slot's real key.
// (Agent-scope loads bypass the XCD's L2 on gfx950 and made every probe a
// memory round trip.)  SA_AGENT_PROBE restores them for A/B runs.
__device__ __forceinline__ uint32_t g_find_insert(unsigned long long *keys, uint64_t key,
                                                  uint32_t log2cap, uint32_t max_probe,
                                                  uint32_t i0 = 0) {
  const ProbeSeq pr = probe_seq(key, log2cap);
  for (uint32_t i = i0; i < max_probe; ++i) {
    const uint32_t s = seq_slot(pr, i);
#ifdef SA_AGENT_PROBE
    unsigned long long k = __hip_atomic_load(&keys[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    unsigned long long k = keys[s];
#endif
    if (k == key) return s;
    if (k == 0) {
      unsigned long long prev = atomicCAS(&keys[s], 0ULL, (unsigned long long)key);
      if (prev == 0 || prev == key) return s;
    }
  }
  return kNotFound;
}

__device__ __forceinline__ uint32_t g_find(const unsigned long long *keys, uint64_t key,
                                           uint32_t log2cap, uint32_t max_probe) {
  const ProbeSeq pr = probe_seq(key, log2cap);
  for (uint32_t i = 0; i < max_probe; ++i) {
    const uint32_t s = seq_slot(pr, i);
    unsigned long long k = keys[s];
    if (k == key) return s;
    if (k == 0) return kNotFound;
  }
  return kNotFound;
}

// Raise one u8 HLL register to rho (CAS on the containing aligned u32).
// Address-space-qualified views (so cold paths use global_/s_load forms, not
// flat: flat ops count in both vmcnt and lgkmcnt and complete out of order,
// which makes every later wait in the loop conservative).
#define SA_GLOBAL __attribute__((address_space(1)))
#define SA_CONST __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ SA_GLOBAL T *gbl(T *p) {
  return (SA_GLOBAL T *)p;
}

__device__ __forceinline__ void hll_raise(uint8_t *reg, uint32_t rho) {
  SA_GLOBAL uint32_t *word =
      gbl(reinterpret_cast<uint32_t *>(reinterpret_cast<uintptr_t>(reg) & ~uintptr_t(3)));
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(reg) & 3) * 8;
  uint32_t old = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (((old >> sh) & 0xFFu) < rho) {  // a failed CAS refreshes `old`
    const uint32_t nw = (old & ~(0xFFu << sh)) | (rho << sh);
    if (__hip_atomic_compare_exchange_strong(word, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      break;
  }
}

// Per-lane event counters, updated arithmetically (no addressable struct, so
// the compiler keeps them in VGPRs instead of scratch).
struct LaneStats {
  uint32_t zero_key, bad_svc, oor, dropped;
};

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

// Per-workgroup buffer descriptors over the SoA columns of its span range
// [lo, hi).  Loads are bounds-checked by the hardware (out-of-range dwords
// read as 0), so every lane issues the same loads -- also in the last tile --
// and the compiler's vmcnt accounting stays exact across the prefetch.
struct Cols {
  __amdgpu_buffer_rsrc_t key, start, end, w0, w1, meta;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ Cols make_cols(const IngestParams &P, uint64_t lo, uint64_t hi) {
  const uint32_t b8 = (uint32_t)((hi - lo) * 8), b4 = (uint32_t)((hi - lo) * 4);
  Cols c;
  c.key = rsrc(P.key + lo, b8);
  c.start = rsrc(P.start + lo, b8);
  c.end = rsrc(P.end + lo, b8);
  c.w0 = rsrc(P.w0 + lo, b8);
  c.w1 = rsrc(P.w1 + lo, b8);
  c.meta = rsrc(P.meta + lo, b4);
  return c;
}

// S consecutive spans per lane per tile: each u64 column is read with S/2
// 16-B loads (one wave-instruction = 1 KiB), meta with one 4*S-B load.
template <int S>
struct SpanTile {
  uint64_t key[S], s[S], e[S], a[S], b[S];
  uint32_t meta[S];
  int cnt;
};

template <int AUX = 0>
__device__ __forceinline__ void u64x2(__amdgpu_buffer_rsrc_t r, int off, uint64_t &x, uint64_t &y) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
  x = (uint64_t)v[0] | ((uint64_t)v[1] << 32);
  y = (uint64_t)v[2] | ((uint64_t)v[3] << 32);
}

// AUX: buffer-load cache policy (gfx950: 2 = nt, streamed once; keeps the
// key table / HLL registers resident in L2 instead of the span stream).
template <int S, int AUX = 0>
__device__ __forceinline__ void load_tile(const Cols &c, uint32_t off, uint32_t len,
                                          SpanTile<S> &v) {
  static_assert(S == 2 || S == 4, "2 or 4 spans per lane");
#pragma unroll
  for (int h = 0; h < S / 2; ++h) {
    const int ob = (int)(off * 8 + 16 * h);
    u64x2<AUX>(c.key, ob, v.key[2 * h], v.key[2 * h + 1]);
    u64x2<AUX>(c.start, ob, v.s[2 * h], v.s[2 * h + 1]);
    u64x2<AUX>(c.end, ob, v.e[2 * h], v.e[2 * h + 1]);
    u64x2<AUX>(c.w0, ob, v.a[2 * h], v.a[2 * h + 1]);
    u64x2<AUX>(c.w1, ob, v.b[2 * h], v.b[2 * h + 1]);
  }
  if constexpr (S == 4) {
    const auto m = __builtin_amdgcn_raw_buffer_load_b128(c.meta, (int)(off * 4), 0, AUX);
    v.meta[0] = m[0]; v.meta[1] = m[1]; v.meta[2] = m[2]; v.meta[3] = m[3];
  } else {
    const auto m = __builtin_amdgcn_raw_buffer_load_b64(c.meta, (int)(off * 4), 0, AUX);
    v.meta[0] = m[0]; v.meta[1] = m[1];
  }
  v.cnt = off < len ? ((len - off) < (uint32_t)S ? (int)(len - off) : S) : 0;
}

// Tile loads with per-tile buffer descriptors: the descriptors are rebuilt
// from the column pointers at every tile (a few SALU), so only the six 64-bit
// column bases stay live across the loop instead of six 4-SGPR descriptors.
// `first` = first span of the tile (absolute), `remain` = spans of the
// workgroup's range from `first` on (0 when past the end).
template <int S, int AUX = 0>
__device__ __forceinline__ void load_tile_at(const IngestParams &P, uint64_t first, uint32_t remain,
                                             uint32_t lane_off, SpanTile<S> &v) {
  Cols c;
  // readfirstlane: hipcc lowers the caller's saturating subtract to a VALU
  // op, and a descriptor word in a VGPR turns every load into a waterfall loop
  remain = (uint32_t)__builtin_amdgcn_readfirstlane((int)remain);
  const uint32_t b8 = remain * 8, b4 = remain * 4;
  c.key = rsrc(P.key + first, b8);
  c.start = rsrc(P.start + first, b8);
  c.end = rsrc(P.end + first, b8);
  c.w0 = rsrc(P.w0 + first, b8);
  c.w1 = rsrc(P.w1 + first, b8);
  c.meta = rsrc(P.meta + first, b4);
  load_tile<S, AUX>(c, lane_off, remain, v);
}

// Sketch phase A: validate service / window, hash the trace id and issue the
// HLL register read (consumed in phase B, after the RED work, so the read's
// latency hides under it).
template <int S>
struct SketchPre {
  uint8_t *reg[S];
  uint32_t rho[S];   // 0 = no HLL update for this span
  uint32_t cur[S];
  uint32_t ws[S];    // window slot, 0xFFFFFFFF = no sketch update
};

template <int S>
__device__ __forceinline__ void sketch_pre(const IngestParams &P, const SpanTile<S> &v,
                                           SketchPre<S> &k, LaneStats &st) {
#pragma unroll
  for (int j = 0; j < S; ++j) {
    k.rho[j] = 0;
    k.ws[j] = 0xFFFFFFFFu;
    k.reg[j] = P.hll;
    if (j < v.cnt) {
      const uint32_t svc = v.meta[j] & 0xFFFFu;
      const bool svc_ok = svc < P.n_services;
      const uint64_t win = fast_div(v.e[j], P.window_ns, P.win_magic);
      const bool win_ok = win - P.win_base < (uint64_t)P.n_windows;
      st.bad_svc += svc_ok ? 0u : 1u;
      st.oor += (svc_ok && !win_ok) ? 1u : 0u;
      if (svc_ok && win_ok) {
        const uint32_t ws = (uint32_t)(win & P.win_mask);
        k.ws[j] = ws;
        if (!(P.diag & 2u)) {
          const uint64_t x = xxh64_16(v.a[j], v.b[j]);
          const uint64_t idx = x >> (64 - P.p);
          k.rho[j] = (uint32_t)__clzll((long long)((x << P.p) | (1ULL << (P.p - 1)))) + 1;
          k.reg[j] = P.hll + ((((uint64_t)ws * P.n_services + svc) << P.p) + idx);
        }
      }
    }
  }
  // Unconditional reads (a skipped span reads the array's first byte): a
  // per-span "load or constant" makes hipcc branch around each load with its
  // own vmcnt(0), serialising the reads and draining any prefetch in flight.
#pragma unroll
  for (int j = 0; j < S; ++j) k.cur[j] = *k.reg[j];
}

// Direct count-min update of one ERROR span (d atomics).
__device__ __forceinline__ void cms_add(const IngestParams &P, uint32_t ws, uint64_t key,
                                        unsigned long long c) {
  unsigned long long *row = P.cms + (uint64_t)ws * P.cms_d * P.cms_w;
  for (uint32_t r = 0; r < P.cms_d; ++r) {
    const uint64_t col = splitmix64(key ^ P.seeds[r]) >> P.cms_shift;
    atomicAdd(row + (uint64_t)r * P.cms_w + col, c);
  }
}

// Sketch phase B: raise HLL registers that grew; count ERROR spans.  A span
// whose series has a key-table slot adds 1 to the exact per-(window, slot)
// error counter (one atomic); the count-min cells are derived from those
// counters when the window is read (fold_errcnt_kernel).  Because the sketch
// is linear in its inputs this is bit-identical to d per-span cell updates.
// Spans without a slot (key 0, table full) update the cells directly.
// The no-return error atomics are issued before the HLL compare, so the wait
// for the register reads is a counted vmcnt behind the prefetch.
template <int S>
__device__ __forceinline__ void sketch_post(const IngestParams &P, const SpanTile<S> &v,
                                            const SketchPre<S> &k, const uint32_t (&slot)[S]) {
#pragma unroll
  for (int j = 0; j < S; ++j) {
    if (k.ws[j] != 0xFFFFFFFFu && ((v.meta[j] >> 19) & 3u) == 2u && !(P.diag & 4u)) {
      if (slot[j] != kNotFound)
        atomicAdd(P.errcnt + ((uint64_t)k.ws[j] << P.log2cap) + slot[j], 1ULL);
      else
        cms_add(P, k.ws[j], v.key[j], 1ULL);
    }
  }
#pragma unroll
  for (int j = 0; j < S; ++j)
    if ((k.cur[j] & 0xFFu) < k.rho[j]) hll_raise(k.reg[j], k.rho[j]);
}

// Contiguous per-workgroup span range [lo, hi) from the host-computed chunk
// (scalar arithmetic only: no 64-bit division in the kernel).
__device__ __forceinline__ void wg_range_p(const IngestParams &P, uint64_t &lo, uint64_t &hi) {
  lo = (uint64_t)blockIdx.x * P.wg_chunk;
  if (lo > P.n) lo = P.n;
  hi = lo + P.wg_chunk < P.n ? lo + P.wg_chunk : P.n;
}

// Contiguous per-workgroup span range [lo, hi), lo a multiple of 4.
__device__ __forceinline__ void wg_range(uint64_t n, uint64_t &lo, uint64_t &hi) {
  uint64_t chunk = (n + gridDim.x - 1) / gridDim.x;
  chunk = (chunk + 3) / 4 * 4;
  lo = (uint64_t)blockIdx.x * chunk;
  if (lo > n) lo = n;
  hi = lo + chunk < n ? lo + chunk : n;
}

constexpr uint32_t kLdsBlock = 1024;

// Window slot of `end` in the resident ring, or 0xFFFFFFFF when outside it:
// q = (end - base_ns) / window_ns from a float estimate (|error| <= 1 for
// q < 2^22) fixed by one signed correction each way -- 2 integer multiplies
// instead of a 64-bit magic division.
__device__ __forceinline__ uint32_t window_slot(const IngestParams &P, uint64_t end) {
  const uint64_t delta = end - P.base_ns;  // wraps (huge) for end < base
  const float f = (float)(uint32_t)(delta >> 32) * 4294967296.0f + (float)(uint32_t)delta;
  uint32_t q = (uint32_t)(f * P.inv_window);
  long long r = (long long)(delta - (uint64_t)q * P.window_ns);
  const bool lo = r < 0;
  q -= lo ? 1u : 0u;
  r += lo ? (long long)P.window_ns : 0;
  q += r >= (long long)P.window_ns ? 1u : 0u;
  return delta < P.ring_ns ? ((P.base_slot + q) & P.win_mask) : 0xFFFFFFFFu;
}

// window_slot on 32-bit pieces (the lean C2 kernel): the float estimate from
// two v_cvt_f32_u32 (written as a 64-bit conversion LLVM expands a generic
// normalising sequence with a 64-bit shift), q * window_ns as one
// v_mad_u64_u32 plus a 24-bit multiply-add for the high word (q < 2^24 inside
// the ring, window_ns < 2^56 -- checked by the host), and the +-1 correction
// from the remainder's sign and size.
//
// Most spans skip the correction: inside the ring the estimate t = delta / W
// is below n_windows, and its three roundings (the two conversions folded by
// the fma, the multiply, 1 / W itself) put it within ~5 * 2^-24 * t of the
// true quotient.  So when t's fraction is more than n_windows * 2^-20 from
// an integer (|fract(t) - 1/2| < P.win_ok), floor(t) is the exact quotient;
// the other lanes (~2^-15 of the spans at 16 windows) take the correction.
// Out-of-ring spans return 0xFFFFFFFF whichever path they take.
__device__ __forceinline__ uint32_t window_slot_lean(const IngestParams &P, uint64_t end, uint32_t win_mask) {
  const uint64_t delta = end - P.base_ns;  // wraps (huge) for end < base
  float fh, fl;
  asm("v_cvt_f32_u32 %0, %1" : "=v"(fh) : "v"((uint32_t)(delta >> 32)));
  asm("v_cvt_f32_u32 %0, %1" : "=v"(fl) : "v"((uint32_t)delta));
  const float t = __builtin_fmaf(fh, 4294967296.0f, fl) * P.inv_window;
  uint32_t q = (uint32_t)t;
  if (__builtin_expect(!(__builtin_fabsf(__builtin_amdgcn_fractf(t) - 0.5f) < P.win_ok), 0)) {
    const uint64_t lo = (uint64_t)q * (uint32_t)P.window_ns;  // v_mad_u64_u32
    uint32_t qh;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(qh) : "v"(q), "s"((uint32_t)(P.window_ns >> 32)), "v"((uint32_t)(lo >> 32)));
    const uint64_t r = delta - (((uint64_t)qh << 32) | (uint32_t)lo);
    const uint32_t neg = (uint32_t)((int32_t)(r >> 32) >> 31);  // r < 0: q one too high (then r >= W too)
    const uint32_t big = r >= P.window_ns ? 1u : 0u;            // r >= W: q one too low
    q = q + big + (neg << 1);
  }
  return delta < P.ring_ns ? ((P.base_slot + q) & win_mask) : 0xFFFFFFFFu;
}
__device__ __forceinline__ uint32_t window_slot_lean(const IngestParams &P, uint64_t end) {
  return window_slot_lean(P, end, P.win_mask);
}

// Bucket via the LDS bin table (BK = 1) or linear thresholds (BK = 0).
template <int BK>
__device__ __forceinline__ uint32_t bucket_lds(uint64_t d, const BinEntry *bins,
                                               const IngestParams &P) {
  if constexpr (BK == 1) {
    const uint32_t bin = d ? 63u - (uint32_t)__clzll((long long)d) : 64u;
    const BinEntry &e = bins[bin];
    return e.base + (d > e.ta ? 1u : 0u) + (d > e.tb ? 1u : 0u);
  } else {
    return bucket_of<-1>(d, P);
  }
}

// Cold paths of ingest_v2_kernel.  They are inlined, but read the kernel
// parameters they need through a laundered kernarg pointer inside the cold
// block: those loads cannot be hoisted to kernel entry, so the parameters only
// the cold paths use do not occupy scalar registers across the span loop.
__device__ __forceinline__ SA_CONST const IngestParams &cold_params() {
  SA_CONST const IngestParams *kp =
      (SA_CONST const IngestParams *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(kp));
  return *kp;
}

__device__ __forceinline__ void cold_cms_add(uint32_t ws, uint64_t key) {
  SA_CONST const IngestParams &Q = cold_params();
  SA_GLOBAL unsigned long long *row0 = gbl(Q.cms) + (uint64_t)ws * Q.cms_d * Q.cms_w;
  const SA_GLOBAL uint64_t *seeds = gbl(Q.seeds);
  for (uint32_t r = 0; r < Q.cms_d; ++r) {
    const uint64_t col = splitmix64(key ^ seeds[r]) >> Q.cms_shift;
    __hip_atomic_fetch_add(row0 + (uint64_t)r * Q.cms_w + col, 1ULL, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
}

__device__ __forceinline__ void cold_hll_raise(uint32_t hoff, uint32_t rho) {
  hll_raise(cold_params().hll + hoff, rho);
}

template <int S>
struct Pending {  // one step's HLL reads, compared one step later
  uint32_t hoff[S], rho[S], hv[S];
};

// 32-bit tag of a series id in the small-table LDS mirror (TAG kernels); the
// same fold probe_seq hashes, so the two share the XOR
__device__ __forceinline__ uint32_t key_tag(uint64_t k) { return (uint32_t)k ^ (uint32_t)(k >> 32); }

__device__ __forceinline__ uint64_t copy_u64(uint64_t x) {
  uint32_t lo, hi;
  asm volatile("v_mov_b32 %0, %1" : "=v"(lo) : "v"((uint32_t)x));
  asm volatile("v_mov_b32 %0, %1" : "=v"(hi) : "v"((uint32_t)(x >> 32)));
  return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t copy_u32(uint32_t x) {
  uint32_t y;
  asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}

__device__ __forceinline__ uint32_t wave_count(bool p) {
  return (uint32_t)__popcll(__ballot(p));
}

__device__ __forceinline__ uint32_t min_bytes(uint4 v) {
  uint32_t m = 0xFFu;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < 32; s += 8) m = min(m, (w[i] >> s) & 0xFFu);
  return m;
}

// One wave recomputes the lower bound of one HLL sub-block per launch
// (rotating over launches when there are more sub-blocks than waves).
__device__ __forceinline__ void hll_lb_refresh(const IngestParams &P, uint32_t wave, uint32_t waves) {
  if (!P.lb_n) return;
  const uint32_t total = min(P.lb_n, gridDim.x * waves), gi = blockIdx.x * waves + wave;
  if (gi >= total) return;
  const uint32_t sb = (uint32_t)(((uint64_t)P.lb_seq * total + gi) % P.lb_n);
  const uint32_t lane = threadIdx.x & 63u, quads = (1u << P.lb_shift) / 16;
  const uint4 *src = reinterpret_cast<const uint4 *>(P.hll + ((uint64_t)sb << P.lb_shift));
  uint32_t mn = 0xFFu;
  for (uint32_t o = lane; o < quads; o += 64) mn = min(mn, min_bytes(src[o]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
  if (lane == 0) P.hll_lb[sb] = (uint8_t)mn;
}

// hll_lb_refresh in two phases, for epilogues that issue their loads early:
// hll_lb_pre loads the wave's sub-block (up to 4 quads per lane; a stale
// register read can only lower the bound, which keeps it a lower bound),
// hll_lb_finish reduces it (reading any quads past the first 256) and stores
// the bound.  B = the workgroup's threads.
template <uint32_t B, typename PT>
__device__ __forceinline__ void hll_lb_pre(const PT &P, uint4 (&lv)[4]) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t lbt = P.lb_n ? min(P.lb_n, gridDim.x * (B / 64)) : 0u, gi = blockIdx.x * (B / 64) + wave;
  const uint32_t sb = gi < lbt ? (uint32_t)(((uint64_t)P.lb_seq * lbt + gi) % P.lb_n) : 0u;
  const uint32_t quads = gi < lbt ? (1u << P.lb_shift) / 16 : 0u;
  const uint4 *src = reinterpret_cast<const uint4 *>(P.hll + ((uint64_t)sb << P.lb_shift));
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i)
    lv[i] = lane + i * 64 < quads ? src[lane + i * 64] : make_uint4(~0u, ~0u, ~0u, ~0u);
}
template <uint32_t B, typename PT>
__device__ __forceinline__ void hll_lb_finish(const PT &P, const uint4 (&lv)[4]) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t lbt = P.lb_n ? min(P.lb_n, gridDim.x * (B / 64)) : 0u, gi = blockIdx.x * (B / 64) + wave;
  if (gi >= lbt) return;
  const uint32_t sb = (uint32_t)(((uint64_t)P.lb_seq * lbt + gi) % P.lb_n);
  const uint32_t quads = (1u << P.lb_shift) / 16;
  const uint4 *src = reinterpret_cast<const uint4 *>(P.hll + ((uint64_t)sb << P.lb_shift));
  uint32_t mn = 0xFFu;
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) mn = min(mn, min_bytes(lv[i]));
  for (uint32_t o = lane + 256; o < quads; o += 64) mn = min(mn, min_bytes(src[o]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
  if (lane == 0) P.hll_lb[sb] = (uint8_t)mn;
}

}  // namespace
}  // namespace sa
