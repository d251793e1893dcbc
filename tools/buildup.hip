// buildup.hip -- build the ingest loop up from the pure streaming probe, one
// ingredient at a time, on C2-like data, to find which ingredient stops the
// per-span work from hiding under the 44 B/span HBM stream.
// Build: hipcc --offload-arch=gfx950 -O3 -I opentelemetry-demo_amd/csrc tools/buildup.hip -o build/buildup
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "sa_internal.h"
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)
using u64 = unsigned long long;
constexpr u64 XP1 = 0x9E3779B185EBCA87ULL, XP2 = 0xC2B2AE3D27D4EB4FULL, XP3 = 0x165667B19E3779F9ULL, XP4 = 0x85EBCA77C2B2AE63ULL, XP5 = 0x27D4EB2F165667C5ULL;
__device__ __forceinline__ u64 rotl(u64 x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ u64 xxh(u64 a, u64 b) {
  u64 h = XP5 + 16;
  h ^= rotl(a * XP2, 31) * XP1; h = rotl(h, 27) * XP1 + XP4;
  h ^= rotl(b * XP2, 31) * XP1; h = rotl(h, 27) * XP1 + XP4;
  h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; h ^= h >> 32; return h;
}
struct Args {
  const u64 *k, *s, *e, *a, *b; const unsigned *m; u64 n;
  const u64 *gkeys; const u64 *bins;  // [65][4] {ta, tb, base, 0}
  unsigned char *hll; u64 *errcnt; unsigned *slab; u64 *stats;
  u64 base_ns, window_ns; float inv_w;
};
enum : int { F_BIN = 1, F_LOOKUP = 2, F_ATOM = 4, F_HLL = 8, F_ERR = 16, F_STAT = 32, F_PRO = 64, F_FLUSH = 128, F_WIN = 256, F_PHASED = 512, F_ERRQ = 1024, F_GIND = 2048, F_GONLY = 4096 };
constexpr int CAP = 2048, NW = 9;
template <int F>
__global__ __launch_bounds__(1024) void kern(Args A) {
  __shared__ __attribute__((aligned(16))) u64 lkeys[CAP];
  __shared__ __attribute__((aligned(16))) u64 lsum[CAP];
  __shared__ __attribute__((aligned(16))) unsigned lcnt[CAP * NW];
  __shared__ __attribute__((aligned(16))) u64 lbins[65 * 4];
  __shared__ unsigned eq[4096];
  __shared__ unsigned eq_n;
  if (threadIdx.x == 0) eq_n = 0;
  if (F & F_PRO) {
    for (int i = threadIdx.x; i < CAP; i += 1024) { lkeys[i] = A.gkeys[i]; lsum[i] = 0; }
    for (int i = threadIdx.x; i < CAP * NW; i += 1024) lcnt[i] = 0;
    for (int i = threadIdx.x; i < 65 * 4; i += 1024) lbins[i] = A.bins[i];
    __syncthreads();
  }
  u64 chunk = (A.n + gridDim.x - 1) / gridDim.x; chunk = (chunk + 3) / 4 * 4;
  const u64 lo = blockIdx.x * chunk, hi = lo + chunk < A.n ? lo + chunk : A.n;
  unsigned acc = threadIdx.x, nz = 0;
  for (u64 i = lo + threadIdx.x * 4; i < hi; i += 4096) {
    u64 kk[4], ss[4], ee[4], aa[4], bb[4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const ulonglong2 k = *reinterpret_cast<const ulonglong2 *>(A.k + i + 2 * h);
      const ulonglong2 s = *reinterpret_cast<const ulonglong2 *>(A.s + i + 2 * h);
      const ulonglong2 e = *reinterpret_cast<const ulonglong2 *>(A.e + i + 2 * h);
      const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(A.a + i + 2 * h);
      const ulonglong2 b = *reinterpret_cast<const ulonglong2 *>(A.b + i + 2 * h);
      kk[2 * h] = k.x; kk[2 * h + 1] = k.y; ss[2 * h] = s.x; ss[2 * h + 1] = s.y; ee[2 * h] = e.x; ee[2 * h + 1] = e.y;
      aa[2 * h] = a.x; aa[2 * h + 1] = a.y; bb[2 * h] = b.x; bb[2 * h + 1] = b.y;
    }
    const uint4 m4 = *reinterpret_cast<const uint4 *>(A.m + i);
    const unsigned mm[4] = {m4.x, m4.y, m4.z, m4.w};
    if (F & (F_GIND | F_GONLY)) {  // random 1-B gathers whose addresses do not depend on the tile
      unsigned g = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const unsigned h = ((unsigned)(i + j) * 0x9E3779B1u) ^ ((unsigned)(i >> 7) * 0x85EBCA6Bu);
        g += A.hll[(h >> 6) % (16u * 20u << 14)];
      }
      if (F & F_GONLY) { acc += g; continue; }
      acc += g + (unsigned)(kk[0] ^ ss[1] ^ ee[2] ^ aa[3] ^ bb[0]) + mm[0] + mm[3];
      continue;
    }
    if (F & F_PHASED) {
      // phase A: window, service, hash -> issue the 4 HLL gathers
      unsigned ws[4], hoff[4], rho[4], hv[4]; bool sk[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const u64 delta = ee[j] - A.base_ns;
        const float f = (float)(unsigned)(delta >> 32) * 4294967296.0f + (float)(unsigned)delta;
        unsigned q = (unsigned)(f * A.inv_w);
        long long r = (long long)(delta - (u64)q * A.window_ns);
        q -= r < 0 ? 1u : 0u; r += r < 0 ? (long long)A.window_ns : 0;
        q += r >= (long long)A.window_ns ? 1u : 0u;
        ws[j] = delta < 16 * A.window_ns ? (q & 15u) : 0xFFFFFFFFu;
        const unsigned svc = mm[j] & 0xFFFFu;
        sk[j] = svc < 20 && ws[j] != 0xFFFFFFFFu;
        const u64 x = xxh(aa[j], bb[j]);
        rho[j] = sk[j] ? (unsigned)__clzll((long long)((x << 14) | (1ULL << 13))) + 1 : 0u;
        hoff[j] = sk[j] ? ((ws[j] * 20 + svc) << 14) + (unsigned)(x >> 50) : 0u;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) hv[j] = A.hll[hoff[j]];
      // phase B: bucket, lookup, LDS counters
      unsigned found[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const u64 d = ee[j] > ss[j] ? ee[j] - ss[j] : 0;
        const unsigned bin = d ? 63u - (unsigned)__clzll((long long)d) : 64u;
        const ulonglong2 t = *reinterpret_cast<const ulonglong2 *>(&lbins[bin * 4]);
        const unsigned bkt = (unsigned)lbins[bin * 4 + 2] + (d > t.x) + (d > t.y);
        const sa::ProbeSeq pr = sa::probe_seq(kk[j], 11);
        const ulonglong2 *b1 = reinterpret_cast<const ulonglong2 *>(lkeys + pr.b1 * 4);
        const ulonglong2 *b2 = reinterpret_cast<const ulonglong2 *>(lkeys + pr.b2 * 4);
        const ulonglong2 q1a = b1[0], q1b = b1[1], q2a = b2[0], q2b = b2[1];
        const u64 k = kk[j];
        unsigned fnd = 0xFFFFFFFFu;
        fnd = q2b.y == k ? pr.b2 * 4 + 3 : fnd; fnd = q2b.x == k ? pr.b2 * 4 + 2 : fnd;
        fnd = q2a.y == k ? pr.b2 * 4 + 1 : fnd; fnd = q2a.x == k ? pr.b2 * 4 + 0 : fnd;
        fnd = q1b.y == k ? pr.b1 * 4 + 3 : fnd; fnd = q1b.x == k ? pr.b1 * 4 + 2 : fnd;
        fnd = q1a.y == k ? pr.b1 * 4 + 1 : fnd; fnd = q1a.x == k ? pr.b1 * 4 + 0 : fnd;
        found[j] = fnd;
        if (fnd != 0xFFFFFFFFu) {
          atomicAdd(&lcnt[fnd * NW + (bkt >> 1)], 1u << ((bkt & 1) * 16));
          atomicAdd(&lsum[fnd], d);
        }
        if (F & F_STAT) nz += (unsigned)__popcll(__ballot(kk[j] == 0)) + (unsigned)__popcll(__ballot(!sk[j]));
      }
      // phase C: HLL compare (consume), phase D: errors
#pragma unroll
      for (int j = 0; j < 4; ++j) if (hv[j] < rho[j]) acc += 1;
      if (F & F_ERR) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (sk[j] && ((mm[j] >> 19) & 3u) == 2u && found[j] != 0xFFFFFFFFu) {
            if (F & F_ERRQ) {  // LDS queue instead of a global atomic in the loop
              const unsigned slot = atomicAdd(&eq_n, 1u);
              if (slot < 4096) eq[slot] = (ws[j] << 11) | found[j];
            } else {
              atomicAdd(A.errcnt + ((u64)ws[j] << 11) + found[j], 1ULL);
            }
          }
      }
      continue;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u64 d = ee[j] > ss[j] ? ee[j] - ss[j] : 0;
      unsigned bkt = (unsigned)d & 15u;
      if (F & F_BIN) {
        const unsigned bin = d ? 63u - (unsigned)__clzll((long long)d) : 64u;
        const ulonglong2 t = *reinterpret_cast<const ulonglong2 *>(&lbins[bin * 4]);
        bkt = (unsigned)lbins[bin * 4 + 2] + (d > t.x) + (d > t.y);
      }
      unsigned ws = (unsigned)(ee[j] >> 34) & 15u;
      if (F & F_WIN) {
        const u64 delta = ee[j] - A.base_ns;
        const float f = (float)(unsigned)(delta >> 32) * 4294967296.0f + (float)(unsigned)delta;
        unsigned q = (unsigned)(f * A.inv_w);
        long long r = (long long)(delta - (u64)q * A.window_ns);
        q -= r < 0 ? 1u : 0u; r += r < 0 ? (long long)A.window_ns : 0;
        q += r >= (long long)A.window_ns ? 1u : 0u;
        ws = delta < 16 * A.window_ns ? (q & 15u) : 0xFFFFFFFFu;
      }
      const unsigned svc = mm[j] & 0xFFFFu;
      const bool sk = svc < 20 && ws != 0xFFFFFFFFu;
      unsigned found = (unsigned)kk[j] & (CAP - 1);
      if (F & F_LOOKUP) {
        const sa::ProbeSeq pr = sa::probe_seq(kk[j], 11);
        const ulonglong2 *b1 = reinterpret_cast<const ulonglong2 *>(lkeys + pr.b1 * 4);
        const ulonglong2 *b2 = reinterpret_cast<const ulonglong2 *>(lkeys + pr.b2 * 4);
        const ulonglong2 q1a = b1[0], q1b = b1[1], q2a = b2[0], q2b = b2[1];
        const u64 k = kk[j];
        unsigned f = 0xFFFFFFFFu;
        f = q2b.y == k ? pr.b2 * 4 + 3 : f; f = q2b.x == k ? pr.b2 * 4 + 2 : f;
        f = q2a.y == k ? pr.b2 * 4 + 1 : f; f = q2a.x == k ? pr.b2 * 4 + 0 : f;
        f = q1b.y == k ? pr.b1 * 4 + 3 : f; f = q1b.x == k ? pr.b1 * 4 + 2 : f;
        f = q1a.y == k ? pr.b1 * 4 + 1 : f; f = q1a.x == k ? pr.b1 * 4 + 0 : f;
        found = f;
      }
      if (F & F_ATOM) {
        if (found != 0xFFFFFFFFu) {
          atomicAdd(&lcnt[found * NW + (bkt >> 1)], 1u << ((bkt & 1) * 16));
          atomicAdd(&lsum[found], d);
        }
      } else {
        acc += found + bkt;
      }
      if (F & F_HLL) {
        const u64 x = xxh(aa[j], bb[j]);
        const unsigned rho = (unsigned)__clzll((long long)((x << 14) | (1ULL << 13))) + 1;
        const unsigned hoff = sk ? ((ws * 20 + svc) << 14) + (unsigned)(x >> 50) : 0u;
        const unsigned hv = A.hll[hoff];
        if (hv < rho && sk) acc += 1;  // (a real raise is queued; here just consume)
      }
      if (F & F_ERR) {
        if (sk && ((mm[j] >> 19) & 3u) == 2u && found != 0xFFFFFFFFu)
          atomicAdd(A.errcnt + ((u64)ws << 11) + found, 1ULL);
      }
      if (F & F_STAT) nz += (unsigned)__popcll(__ballot(kk[j] == 0)) + (unsigned)__popcll(__ballot(!sk));
    }
  }
  if (F & F_FLUSH) {
    __syncthreads();
    uint4 *sc = reinterpret_cast<uint4 *>(A.slab + (u64)blockIdx.x * CAP * NW * 2);
    const uint2 *lw = reinterpret_cast<const uint2 *>(lcnt);
    for (int k = threadIdx.x; k < CAP * NW / 2; k += 1024) {
      const uint2 w = lw[k];
      if (w.x | w.y) { uint4 g = sc[k]; g.x += w.x & 0xFFFF; g.y += w.x >> 16; g.z += w.y & 0xFFFF; g.w += w.y >> 16; sc[k] = g; }
    }
  }
  if (F & F_ERRQ) {
    __syncthreads();
    const unsigned ne = eq_n < 4096 ? eq_n : 4096;
    for (unsigned i = threadIdx.x; i < ne; i += 1024)
      atomicAdd(A.errcnt + ((u64)(eq[i] >> 11) << 11) + (eq[i] & 2047u), 1ULL);
  }
  if (acc == 0x12345678u || nz == 0x7654321u) A.stats[0] = acc + nz;
}
template <typename Fn> float time_it(Fn f, int reps) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize()); CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f();
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}
int main() {
  const u64 n = 10000000ULL;
  int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // C2-like data: 1500 keys (Zipf 1.1 over 500 pairs x status 88/10/2 %), lognormal durations,
  // ~10 spans per trace, 20 services, 60 s of end times
  std::mt19937_64 rng(42);
  std::vector<u64> keys(1500); for (auto &k : keys) k = rng() | 1;
  std::vector<double> cdf(500); double acc = 0; for (int i = 0; i < 500; ++i) { acc += 1.0 / std::pow(i + 1, 1.1); cdf[i] = acc; }
  std::vector<u64> K(n), S(n), E(n), A(n), B(n); std::vector<unsigned> M(n);
  const u64 T0 = 1767225600ULL * 1000000000ULL;
  std::vector<u64> ta(n / 10 + 1), tb(n / 10 + 1); for (auto &t : ta) t = rng(); for (auto &t : tb) t = rng();
  std::uniform_real_distribution<double> U(0, 1); std::normal_distribution<double> N(std::log(5e6), 1.5);
  for (u64 i = 0; i < n; ++i) {
    const double u = U(rng) * acc; int p = (int)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin()); if (p > 499) p = 499;
    const double v = U(rng); const int st = v < 0.02 ? 2 : v < 0.12 ? 1 : 0;
    K[i] = keys[p * 3 + st]; S[i] = T0 + (u64)(U(rng) * 60e9);
    double d = std::exp(N(rng)); if (d > 60e9) d = 60e9; E[i] = S[i] + (u64)d;
    const u64 t = rng() % ta.size(); A[i] = ta[t]; B[i] = tb[t];
    M[i] = (unsigned)(p / 25) | (2u << 16) | ((unsigned)st << 19);
  }
  // key table in the engine's bucketed layout
  std::vector<u64> gk(CAP, 0);
  for (u64 k : keys) { const sa::ProbeSeq pr = sa::probe_seq(k, 11); for (unsigned i = 0;; ++i) { const unsigned s = sa::seq_slot(pr, i); if (!gk[s]) { gk[s] = k; break; } } }
  std::vector<u64> bins(65 * 4, 0);
  const u64 thr[16] = {2000000, 4000000, 6000000, 8000000, 10000000, 50000000, 100000000, 200000000, 400000000, 800000000, 1000000000, 1400000000, 2000000000, 5000000000ULL, 10000000000ULL, 15000000000ULL};
  for (int k = 0; k < 65; ++k) { bins[k * 4] = bins[k * 4 + 1] = ~0ULL; if (k == 64) continue; const u64 lo = 1ULL << k, hi = k == 63 ? ~0ULL : (2ULL << k) - 1; unsigned below = 0, in = 0; for (u64 t : thr) { if (t < lo) ++below; else if (t < hi) bins[k * 4 + in++] = t; } bins[k * 4 + 2] = below; }
  Args a{};
  void *buf; CK(hipMalloc(&buf, n * 44 + 4096));
  u64 *dk = (u64 *)buf, *ds = dk + n, *de = ds + n, *da = de + n, *db = da + n; unsigned *dm = (unsigned *)(db + n);
  CK(hipMemcpy(dk, K.data(), n * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(ds, S.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(de, E.data(), n * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(da, A.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(db, B.data(), n * 8, hipMemcpyHostToDevice)); CK(hipMemcpy(dm, M.data(), n * 4, hipMemcpyHostToDevice));
  a.k = dk; a.s = ds; a.e = de; a.a = da; a.b = db; a.m = dm; a.n = n;
  u64 *g; CK(hipMalloc(&g, CAP * 8)); CK(hipMemcpy(g, gk.data(), CAP * 8, hipMemcpyHostToDevice)); a.gkeys = g;
  u64 *bb; CK(hipMalloc(&bb, bins.size() * 8)); CK(hipMemcpy(bb, bins.data(), bins.size() * 8, hipMemcpyHostToDevice)); a.bins = bb;
  CK(hipMalloc(&a.hll, 16 * 20 << 14)); CK(hipMemset(a.hll, 0, 16 * 20 << 14));
  CK(hipMalloc(&a.errcnt, 16 * CAP * 8)); CK(hipMalloc(&a.slab, (u64)cus * CAP * NW * 8)); CK(hipMalloc(&a.stats, 64));
  CK(hipMemset(a.slab, 0, (u64)cus * CAP * NW * 8));
  a.base_ns = (T0 / 10000000000ULL) * 10000000000ULL; a.window_ns = 10000000000ULL; a.inv_w = 1e-10f;
#define R(F, name) std::printf("{\"case\": \"%s\", \"flags\": %d, \"us\": %.2f}\n", name, F, time_it([&] { kern<F><<<cus, 1024>>>(a); }, 20));
  R(0, "stream")
  R(F_PRO, "+prologue")
  R(F_PRO | F_BIN, "+bins")
  R(F_PRO | F_BIN | F_WIN, "+window")
  R(F_PRO | F_BIN | F_WIN | F_LOOKUP, "+lookup")
  R(F_PRO | F_BIN | F_WIN | F_LOOKUP | F_ATOM, "+lds_atomics")
  R(F_PRO | F_BIN | F_WIN | F_LOOKUP | F_ATOM | F_HLL, "+hll")
  R(F_PRO | F_BIN | F_WIN | F_LOOKUP | F_ATOM | F_HLL | F_ERR, "+err")
  R(F_PRO | F_BIN | F_WIN | F_LOOKUP | F_ATOM | F_HLL | F_ERR | F_STAT, "+stats")
  R(F_PRO | F_BIN | F_WIN | F_LOOKUP | F_ATOM | F_HLL | F_ERR | F_STAT | F_FLUSH, "+flush")
  R(F_PRO | F_HLL, "hll_only")
  R(F_GIND, "stream44+indep_gather")
  R(F_GONLY, "indep_gather_only")
  R(F_PRO | F_PHASED, "phased")
  R(F_PRO | F_PHASED | F_STAT, "phased+stats")
  R(F_PRO | F_PHASED | F_STAT | F_ERR, "phased+stats+err")
  R(F_PRO | F_PHASED | F_STAT | F_ERR | F_ERRQ, "phased+stats+errq")
  R(F_PRO | F_PHASED | F_STAT | F_ERR | F_ERRQ | F_FLUSH, "phased+stats+errq+flush")
  R(F_PRO | F_PHASED | F_STAT | F_ERR | F_FLUSH, "phased+stats+err+flush")
  R(F_PRO | F_LOOKUP | F_ATOM, "red_only")
  R(F_PRO | F_ATOM, "atomics_only")
  return 0;
}
