// spanagg_engine.cpp -- C-ABI of libspanagg (include/spanagg.h): engine state in
// HBM, staging, flush/compaction and the multi-GPU merge hooks.  One engine owns
// one gfx950 device; the product path has no CPU fallback -- sa_create fails with
// SA_EDEVICE when no gfx950 device is usable.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "sa_group_hooks.h"
#include "sa_internal.h"
#include "sa_results.h"
#include "spanagg.h"
#include "spanagg_diag.h"

using sa::IngestParams;

namespace {

constexpr double kDefaultBounds[16] = {2,   4,   6,    8,    10,   50,   100,   200,
                                       400, 800, 1000, 1400, 2000, 5000, 10000, 15000};
constexpr uint64_t kCmsSeed[8] = {0x9E3779B97F4A7C15ULL, 0xBF58476D1CE4E5B9ULL,
                                  0x94D049BB133111EBULL, 0xD6E8FEB86659FD93ULL,
                                  0xA0761D6478BD642FULL, 0xE7037ED1A0B428DBULL,
                                  0x8EBC6AF09C88C6E3ULL, 0x589965CC75374CC3ULL};
constexpr size_t kLdsBudget = 144 * 1024;  // small-table path LDS ceiling per workgroup
constexpr uint64_t kSlabLimit = 1ULL << 31;  // per-workgroup spans between slab reductions
// small path: ingest_v2_kernel variant 20 (19 LEAN: the span hash on 32-bit
// halves and the wave-level (slot, bucket) dedup of the hot series' counter
// adds); SPANAGG_VARIANT overrides in the laboratory build
constexpr int kDefaultVariant = 20;
constexpr uint32_t kMaxSlabSets = 4;      // per-workgroup slab sets (small path)
constexpr uint32_t kDefaultSlabSets = 2;  // SPANAGG_SLAB_SETS overrides (laboratory build)
// exponential slab path: what the ingest kernel hands the counting pass per
// span (expo_rec_mode): 0 the key slot (the pass reads both times too), 1 an
// 8-B span record (slot | duration), 2 an index record (slot | scale | bucket
// index, ixrec_of) -- DESIGN.md section 4
constexpr int kExpoRecMode = 2;

// Laboratory knobs: the SPANAGG_AB build (`make ab` -> libspanagg_ab.so, used
// by tools/ for A/B runs and ablations) reads them from the environment; the
// product library reads no environment at all.
#ifdef SPANAGG_AB
const char *ab_env(const char *name) { return std::getenv(name); }
#else
constexpr const char *ab_env(const char *) { return nullptr; }
#endif

// The engine's ordering events only order its own launches, copies and
// reads on this device (cross-stream waits, slab-set and record-set reuse),
// so they release at device scope: a default event ends with a system-scope
// fence (L2 write-back and invalidate) that the next launch on the stream
// waits behind and starts cold after.  (Laboratory build: SPANAGG_EV_SYS=1
// restores the default for A/B runs.)
unsigned ev_flags() {
  static const unsigned f = [] {
    const char *v = ab_env("SPANAGG_EV_SYS");
    return (v && std::atoi(v) != 0) ? hipEventDisableTiming : (hipEventDisableTiming | hipEventReleaseToDevice);
  }();
  return f;
}

bool is_pow2(uint64_t x) { return x && !(x & (x - 1)); }
uint32_t log2u(uint64_t x) { return 63u - (uint32_t)__builtin_clzll(x); }
uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace

struct sa_engine {
  sa_config cfg{};
  std::vector<double> bounds;
  int dev = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev_a = nullptr, ev_b = nullptr;
  // Slab sets: the small-table path keeps two sets of per-workgroup slabs and
  // alternates launches between them, so a launch only has to wait for the
  // launch two back (the previous user of its set), not the previous one.
  // Launches on different streams can then overlap: the next batch's
  // workgroups start on the CUs that the current batch's workgroups leave.
  // ev_set[i] marks the completion of the last launch that used set i (on
  // set_stream[i]); non-ingest operations join every set onto the engine
  // stream first, and the next launch orders after them through ev_ctl.
  uint32_t nsets = 1, set = 0;
  hipEvent_t ev_set[kMaxSlabSets] = {}, ev_ctl = nullptr;
  hipStream_t set_stream[kMaxSlabSets] = {};
  // sa_ingest_device_many: two instantiated graphs of K small-table launches,
  // used in turn; a graph's kernel nodes are re-pointed at the next K batches
  // (hipGraphExecKernelNodeSetParams) only after its previous launch finished
  // (gx_done), so no launch in flight sees its arguments change
  struct GraphIngest {
    hipGraph_t g = nullptr;
    hipGraphExec_t x = nullptr;
    hipEvent_t done = nullptr;
    bool launched = false;
    std::vector<hipGraphNode_t> nodes;
    const void *fn = nullptr;
    dim3 block{};
    size_t lds = 0;
  } gi[2];
  uint32_t gi_next = 0;
  bool ctl_dirty = true;
  uint32_t nbk = 0, npos = 0, nneg = 0;
  uint64_t thr[sa::kMaxBounds]{};
  uint32_t log2cap = 0;
  uint64_t cap = 0;
  bool small = false;
  int variant = 0;
  uint32_t spl = 4;
  uint32_t G = 0, block = 0, cus = 0;
  size_t lds_bytes = 0;
  unsigned long long *gkeys = nullptr, *gcounts = nullptr, *slab_sum = nullptr, *cms = nullptr,
                     *stats = nullptr, *out_keys = nullptr, *out_rows = nullptr, *scratch = nullptr,
                     *errcnt = nullptr;
  uint64_t *d_seeds = nullptr;
  sa::BinEntry *d_bins = nullptr;  // bucket bin table (nullptr: linear thresholds)
  unsigned long long *dbg = nullptr;  // SPANAGG_STAMPS diagnostic timestamps
  uint32_t *slab_cnt = nullptr;
  uint32_t *errslab = nullptr;  // v2: [G][n_windows << log2cap] per-workgroup ERROR counts
  uint8_t *hll = nullptr;
  // HLL lower bounds per sub-block of 2^lb_shift registers (IngestParams::hll_lb)
  uint8_t *hll_lb = nullptr;
  uint32_t lb_shift = 0, lb_n = 0, lb_seq = 0;
  unsigned long long *hll_filt = nullptr;  // [kFiltSlots] filtered HLL updates per workgroup slot
  // exponential-histogram mode (cfg.exp_max_size > 0): the HBM-table path
  // runs the sketches, spanagg_expo.hip the histograms
  bool expo = false;
  // exponential engines whose key table fits LDS: the small-table kernel in
  // EXPO mode (per-workgroup header partials in xslab [G][cap], per-span slots)
  bool expo_small = false;
  sa::XHdr *xslab = nullptr;
  // slab bucket counting of small expo tables (spanagg_expo.hip expo_count_slab_kernel)
  uint32_t xc_ne = 0;
  uint32_t *xc_lcount = nullptr, *xc_slot_of_entry = nullptr, *xcslab = nullptr;
  // the counting kernel's entry selections, double-buffered by launch parity
  // (xc_sel): each launch counts with the selection the previous one made
  // from its counts -- slot_of_entry [2][xc_ne], entry of each slot [2][cap]
  int32_t *xc_ent = nullptr;
  uint32_t xc_sel = 0;
  bool xc_sel_made = false;
  uint32_t *xt_rec = nullptr, *xt_off = nullptr;  // the counting kernel's tail records (ExpoParams::xt_*)
  sa::ExpoHdr *expo_hdr = nullptr;
  int8_t *expo_xscale = nullptr;  // [cap] the slots' scales for the ingest kernel (index records)
  uint32_t *expo_buckets = nullptr, *expo_slot = nullptr;
  uint64_t expo_slot_cap = 0;  // spans per set of expo_slot ([nsets][cap], 8 B each)
  // Small-table exponential engines run launch k + 1's ingest kernel beside
  // launch k's reduce / count / fold (two slab sets of header partials and
  // span slots); launch k + 1's reduce waits for ev_expo, launch k's fold
  // (the headers and buckets have one owner at a time)
  hipEvent_t ev_expo = nullptr;
  hipStream_t expo_last = nullptr;
  // Laboratory build (SPANAGG_XSTREAM=1): with span records the histogram
  // kernels read no caller memory, so they can run on an engine stream after
  // an event on the launch's ingest kernel (ev_ing[set]); slower than the
  // caller's stream by A/B (the ingest kernel starves them), so off
  hipStream_t xstream = nullptr;
  hipEvent_t ev_ing[kMaxSlabSets] = {};
  unsigned long long *expo_out_keys = nullptr;
  sa::ExpoRow *expo_out_rows = nullptr;
  uint32_t *expo_out_buckets = nullptr;
  // partitioned HBM-table path (lazily allocated on the first launch)
  bool part = false;
  ulonglong2 *part_rec = nullptr;
  uint32_t *part_fill = nullptr;
  // binned-table path (spanagg_binned.hip): bin-local key sub-tables of
  // 2^log2sb slots, stored ids m = key * kmul, 32-B u8-count rows plus the u64
  // spill array base64 [cap][nbk + 1], span records in per-(bin, scatter
  // workgroup) regions (lazily allocated)
  bool bt = false;
  uint32_t log2sb = 0, bt_grid = 0;
  uint64_t kmul = 1, kinv = 1;
  size_t agg_lds = 0;
  // Launch pipeline of the binned path: launch k's scatter runs on the
  // caller's stream; the aggregate runs on agg_stream (after the scatters'
  // events), so later scatters overlap it.  Launches are aggregated in pairs:
  // launch k's records wait (bt_pend) until launch k + 1's scatter, then one
  // aggregate takes both record sets -- a bin's setup and row write-back
  // serve two launches.  A pending set is aggregated alone before anything
  // reads (join_sets, sa_join).  Four record sets (records + region fills):
  // a scatter waits only for the aggregate that last read its set.  The
  // aggregate's key write-back is safe against the concurrent scatters' key
  // inserts (spanagg_binned.hip bt_aggregate3_kernel step 3).
  static constexpr int kBtSets = 4;
  ulonglong2 *bt_rec[kBtSets] = {};
  uint32_t *bt_cnt[kBtSets] = {};
  hipStream_t agg_stream = nullptr;
  hipEvent_t ev_scat[kBtSets] = {}, ev_agg[kBtSets] = {};
  bool agg_used[kBtSets] = {};
  uint32_t bt_set = 0;
  int bt_pend = -1;              // the set whose records await the next launch's (or a join)
  int sticky_rc = 0;             // a pending aggregate that failed to launch (join_checked)
  sa::IngestParams bt_pend_P{};  // its launch parameters
  unsigned long long *base64 = nullptr;
  size_t hll_slot_bytes = 0, cms_slot_elems = 0;
  // sa_ingest: two pinned host slots and their HBM copies; a slot is refilled
  // once its event (H2D copy + aggregation of the previous use) has passed
  void *pin[2] = {nullptr, nullptr}, *dstage[2] = {nullptr, nullptr};
  hipEvent_t pin_ev[2] = {nullptr, nullptr};
  bool pin_used[2] = {false, false};
  // sa_ingest_async: the event after the last async call's copies (its
  // columns are the caller's until that event completes)
  hipEvent_t ev_async = nullptr;
  bool async_pending = false;
  int pin_cur = 0;
  uint64_t win_base = 0, spans = 0, slab_load = 0, dropped_seen = 0;
  bool unflushed = false;   // spans ingested since the RED counters were last reset
  uint64_t reclaims = 0;    // key-table reclamations (sa_reclaim_keys)
  // small-table kernel with the tail pool (sa::kLdsPoolVariant): per-launch
  // pool counters [kPoolRing] (launch k zeroes launch k + nsets's)
  bool pool = false;
  uint32_t *pool_ring = nullptr;
  uint32_t pool_seq = 0;
  std::string err;
};

namespace {

int fail(sa_engine *e, int code, const std::string &msg) {
  if (e) e->err = msg;
  return code;
}

#define SA_HIP(e, call)                                                                   \
  do {                                                                                    \
    hipError_t _st = (call);                                                              \
    if (_st != hipSuccess)                                                                \
      return fail((e), SA_EDEVICE, std::string(#call) + ": " + hipGetErrorString(_st));  \
  } while (0)

int set_dev(sa_engine *e) {
  SA_HIP(e, hipSetDevice(e->dev));
  return SA_OK;
}

int validate_config(const sa_config *c, std::string &why) {
  if (!c) return why = "null config", SA_EINVAL;
  if (c->n_bounds > SA_MAX_BOUNDS) return why = "too many histogram bounds", SA_EINVAL;
  if (c->n_bounds && !c->bounds) return why = "bounds pointer is null", SA_EINVAL;
  if (c->unit > SA_UNIT_S) return why = "unit must be ms or s", SA_EINVAL;
  if (c->hll_p < 4 || c->hll_p > 18) return why = "hll_p must be in 4..18", SA_EINVAL;
  if (c->cms_d < 1 || c->cms_d > 8) return why = "cms_d must be in 1..8", SA_EINVAL;
  if (c->cms_w < 2 || !is_pow2(c->cms_w)) return why = "cms_w must be a power of two >= 2", SA_EINVAL;
  if (c->window_ns == 0) return why = "window_ns must be > 0", SA_EINVAL;
  if (c->window_ns >> 56) return why = "window_ns must stay below 2^56 ns (~2.3 years)", SA_EINVAL;
  if (!is_pow2(c->n_windows) || c->n_windows > 4096)
    return why = "n_windows must be a power of two <= 4096", SA_EINVAL;
  if (c->n_services < 1 || c->n_services > 65536)
    return why = "n_services must be in 1..65536", SA_EINVAL;
  if (c->key_capacity < 1 || c->key_capacity > (1ULL << 30))
    return why = "key_capacity must be in 1..2^30", SA_EINVAL;
  if (c->window_ns >= (1ULL << 63) / c->n_windows)
    return why = "n_windows * window_ns must stay below 2^63 ns", SA_EINVAL;
  if (((uint64_t)c->n_windows * c->n_services << c->hll_p) >= (1ULL << 32))
    return why = "n_windows * n_services * 2^hll_p must stay below 2^32 registers", SA_EINVAL;
  if (c->exp_max_size == 1 || c->exp_max_size > sa::kExpoMaxSize)
    return why = "exp_max_size must be 0 (explicit buckets) or 2..4096", SA_EINVAL;
  if (c->options & ~SA_OPT_ALL) return why = "unknown bits in options", SA_EINVAL;
#ifndef SPANAGG_AB
  if (c->flags) return why = "SA_DIAG_* flags need the laboratory build (libspanagg_ab.so)", SA_EINVAL;
#endif
  return SA_OK;
}

}  // namespace

// Bucket bin table for the LDS kernels: bin k = floor(log2 d) (64 for d = 0).
// Returns false (use linear thresholds) if any bin holds more than 2 of them.
static bool build_bins(const sa_engine *e, sa::BinEntry (&bins)[sa::kBins]) {
  for (int k = 0; k < sa::kBins; ++k) {
    bins[k] = sa::BinEntry{UINT64_MAX, UINT64_MAX, e->nneg, {0, 0, 0}};
    if (k == 64) continue;  // d = 0: no u64 threshold is below 0
    const uint64_t lo = 1ULL << k, hi = k == 63 ? UINT64_MAX : (2ULL << k) - 1;
    uint32_t below = 0, inside = 0;
    for (uint32_t i = 0; i < e->npos; ++i) {
      const uint64_t t = e->thr[i];
      if (t < lo) ++below;                  // every d in the bin exceeds it
      else if (t < hi) {                    // decided per span
        if (inside == 0) bins[k].ta = t;
        else if (inside == 1) bins[k].tb = t;
        ++inside;
      }
    }
    if (inside > 2) return false;
    bins[k].base = e->nneg + below;
  }
  return true;
}

static size_t counts_bytes(const sa_engine *e) {
  return e->bt ? (size_t)e->cap * sa::kRowBytes : (size_t)e->cap * sa::row_stride(e->nbk) * 8;
}

static sa::RowGeom geom(const sa_engine *e) {
  sa::RowGeom g{};
  g.nbk = e->nbk;
  g.row8 = e->bt ? 1u : 0u;
  g.binned = e->bt ? 1u : 0u;
  g.log2cap = e->log2cap;
  g.log2sb = e->log2sb;
  g.max_probe = sa::max_probe_of(e->log2cap);
  g.kmul = e->kmul;
  g.kinv = e->kinv;
  g.base64 = e->base64;
  return g;
}

extern "C" {

int sa_abi_version(void) { return SA_ABI_VERSION; }

void sa_config_default(sa_config *c) {
  if (!c) return;
  std::memset(c, 0, sizeof *c);
  c->bounds = kDefaultBounds;
  c->n_bounds = 16;
  c->unit = SA_UNIT_MS;
  c->hll_p = 14;
  c->cms_d = 4;
  c->cms_w = 2048;
  c->window_ns = 10ULL * 1000000000ULL;
  c->n_windows = 8;
  c->n_services = 64;
  c->key_capacity = 1000;  // the connector's dimensions_cache_size default
  c->device = 0;
}

int sa_bucket_thresholds(const double *bounds, uint32_t n, uint32_t unit, uint64_t *thr,
                         uint32_t *n_neg) {
  if (n > SA_MAX_BOUNDS || (n && (!bounds || !thr)) || !n_neg || unit > SA_UNIT_S)
    return SA_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    if (std::isnan(bounds[i])) return SA_EINVAL;
    if (i && !(bounds[i - 1] <= bounds[i])) return SA_EINVAL;
  }
  const double div = unit == SA_UNIT_S ? 1e9 : 1e6;
  uint32_t neg = 0;
  while (neg < n && bounds[neg] < 0.0) ++neg;
  for (uint32_t i = neg; i < n; ++i) {
    const double b = bounds[i];
    // T = max{d in u64 : float64(d)/div <= b}; f(d) is monotone non-decreasing.
    auto f_le = [&](uint64_t d) { return (double)d / div <= b; };
    uint64_t t;
    if (f_le(UINT64_MAX)) {
      t = UINT64_MAX;
    } else {
      uint64_t lo = 0, hi = UINT64_MAX;  // f_le(lo) holds since b >= 0
      while (hi - lo > 1) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (f_le(mid)) lo = mid;
        else hi = mid;
      }
      t = lo;
    }
    thr[i - neg] = t;
  }
  *n_neg = neg;
  return SA_OK;
}

double sa_hll_estimate(const uint8_t *regs, uint32_t p) {
  if (!regs || p < 4 || p > 18) return -1.0;
  const uint32_t m = 1u << p;
  double sum = 0.0;
  uint32_t zeros = 0;
  for (uint32_t j = 0; j < m; ++j) {
    sum += std::ldexp(1.0, -(int)regs[j]);
    zeros += regs[j] == 0;
  }
  const double alpha = m == 16 ? 0.673 : m == 32 ? 0.697 : m == 64 ? 0.709
                                                                  : 0.7213 / (1.0 + 1.079 / m);
  double est = alpha * (double)m * (double)m / sum;
  if (est <= 2.5 * m && zeros) est = (double)m * std::log((double)m / (double)zeros);
  return est;
}

int sa_create(const sa_config *cfg, sa_engine **out) {
  if (!out) return SA_EINVAL;
  *out = nullptr;
  std::string why;
  if (int rc = validate_config(cfg, why)) {
    std::fprintf(stderr, "sa_create: %s\n", why.c_str());
    return rc;
  }
  auto *e = new sa_engine();
  e->cfg = *cfg;
  e->bounds.assign(cfg->bounds, cfg->bounds + cfg->n_bounds);
  e->cfg.bounds = e->bounds.data();
  e->nbk = cfg->n_bounds + 1;
  if (sa_bucket_thresholds(e->bounds.data(), cfg->n_bounds, cfg->unit, e->thr, &e->nneg) != SA_OK) {
    std::fprintf(stderr, "sa_create: histogram bounds must be sorted ascending and not NaN\n");
    delete e;
    return SA_EINVAL;
  }
  e->npos = cfg->n_bounds - e->nneg;

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || cfg->device < 0 ||
      cfg->device >= ndev) {
    std::fprintf(stderr, "sa_create: no HIP device %d (found %d)\n", cfg->device, ndev);
    delete e;
    return SA_EDEVICE;
  }
  e->dev = cfg->device;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, e->dev) != hipSuccess ||
      std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    std::fprintf(stderr, "sa_create: device %d is not gfx950 (%s)\n", e->dev, prop.gcnArchName);
    delete e;
    return SA_EDEVICE;
  }
  e->cus = (uint32_t)prop.multiProcessorCount;

  auto bail = [&](int rc) {
    std::fprintf(stderr, "sa_create: %s\n", e->err.c_str());
    sa_destroy(e);
    return rc;
  };
  if (int rc = set_dev(e)) return bail(rc);
  // A blocking stream: it orders against the legacy null stream, so callers
  // that produce batches on the null stream (stream == NULL) stay race-free.
  if (hipStreamCreateWithFlags(&e->stream, hipStreamDefault) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_a, ev_flags()) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_b, ev_flags()) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_ctl, ev_flags()) != hipSuccess)
    return bail(fail(e, SA_EDEVICE, "stream/event creation failed"));
  for (hipEvent_t &ev : e->ev_set)
    if (hipEventCreateWithFlags(&ev, ev_flags()) != hipSuccess)
      return bail(fail(e, SA_EDEVICE, "event creation failed"));

  // buckets of 4 slots with two choices stay well-behaved up to ~90% load:
  // size for 80% at the declared capacity (the LDS mirror path needs cap <= 2048)
  e->cap = std::max<uint64_t>(16, next_pow2(cfg->key_capacity + (cfg->key_capacity + 3) / 4));
  e->log2cap = log2u(e->cap);
  const uint32_t nw = (e->nbk + 1) / 2;
  // lkeys + lsum + lcnt + deferred-HLL queue (+ its counter), see ingest_lds_kernel
  e->lds_bytes = (size_t)e->cap * 16 + (size_t)e->cap * nw * 4 + sa::kLdsExtraBytes;
  e->expo = cfg->exp_max_size != 0;
  e->small = e->lds_bytes <= kLdsBudget && !e->expo;
  if (e->expo) {  // key mirror + 32-B header partials per slot (nw = 6 counter words)
    // (+ cap: the index records' per-slot scales)
    const size_t xl = (size_t)e->cap * 8 + (size_t)e->cap * 32 + sa::kLdsExtraBytes + (size_t)e->cap;
    e->expo_small = xl <= kLdsBudget && !(cfg->options & SA_OPT_EXPO_HBM);
    if (e->expo_small) e->lds_bytes = xl;
  }
  e->variant = e->small ? kDefaultVariant : 0;
  if (const char *v = ab_env("SPANAGG_VARIANT"))
    e->variant = std::max(0, std::min((e->small ? sa::kNumLdsVariants : sa::kNumVariants) - 1,
                                      std::atoi(v)));
  // the laboratory TAG variant also keeps a u32 key tag per slot in LDS; a
  // table whose tags do not fit stays on the default variant
  if (e->small && e->variant == sa::kLdsTagVariant) {
    if (e->lds_bytes + (size_t)e->cap * sa::kLdsTagBytesPerSlot <= kLdsBudget)
      e->lds_bytes += (size_t)e->cap * sa::kLdsTagBytesPerSlot;
    else
      e->variant = kDefaultVariant;
  }
  if (e->small) {
    sa::BinEntry bins_probe[sa::kBins];
    const bool bins_ok = build_bins(e, bins_probe);
    // a table other than the specialised default geometry whose LDS state
    // fits a CU twice: 512-thread workgroups, two per CU, so one workgroup's
    // prologue and write-back overlap the other's loop
    if (e->variant == kDefaultVariant && bins_ok && 2 * e->lds_bytes <= (size_t)160 * 1024 &&
        !(e->log2cap == 11 && nw == 9 && cfg->hll_p == 14))
      e->variant = sa::kLdsHalfBlockVariant;
    e->spl = (uint32_t)sa::kLdsSpl[e->variant];
    e->block = sa::ingest_small_block(bins_ok, e->variant, e->log2cap, e->nbk, cfg->hll_p);
    if (hipError_t st = sa::prepare_ingest_small(e->lds_bytes); st != hipSuccess)
      return bail(fail(e, SA_EDEVICE, std::string("LDS attribute: ") + hipGetErrorString(st)));
    // one resident round of workgroups (registers and LDS decide how many
    // share a CU; a second round would repeat every workgroup's prologue)
    uint32_t per_cu = sa::ingest_small_blocks_per_cu(bins_ok, e->variant, e->log2cap, e->nbk, cfg->hll_p,
                                                     e->lds_bytes);
    if (per_cu == 0)
      per_cu = std::max<uint32_t>(1, std::min<uint32_t>(2048 / e->block, (uint32_t)((160 * 1024) / e->lds_bytes)));
    e->G = e->cus * per_cu;
  } else if (e->expo_small) {
    e->block = 1024;
    e->spl = 2;
    if (hipError_t st = sa::prepare_ingest_expo_small(e->lds_bytes); st != hipSuccess)
      return bail(fail(e, SA_EDEVICE, std::string("LDS attribute: ") + hipGetErrorString(st)));
    // one resident round of workgroups (registers and LDS), as the small tables
    uint32_t per_cu = sa::ingest_expo_blocks_per_cu(e->log2cap, cfg->hll_p, e->lds_bytes);
    if (per_cu == 0) per_cu = std::max<uint32_t>(1, (uint32_t)((160 * 1024) / e->lds_bytes));
    e->G = e->cus * per_cu;
    if (hipError_t st = sa::prepare_expo_count(sa::expo_count_lds_bytes(e->cap, cfg->exp_max_size)); st != hipSuccess)
      return bail(fail(e, SA_EDEVICE, std::string("LDS attribute: ") + hipGetErrorString(st)));
    // slab counting: its workgroups (one per ingest workgroup) share a CU as the
    // ingest ones do; SA_OPT_EXPO_CACHED keeps the cached-probe kernel
    const size_t budget = (size_t)160 * 1024 * e->cus / e->G - 1024;
    e->xc_ne = (cfg->options & SA_OPT_EXPO_CACHED) ? 0u : sa::expo_slab_entries(e->cap, cfg->exp_max_size, budget);
    if (e->xc_ne)
      if (hipError_t st = sa::prepare_expo_slab(sa::expo_slab_lds_bytes(e->cap, cfg->exp_max_size, e->xc_ne));
          st != hipSuccess)
        return bail(fail(e, SA_EDEVICE, std::string("LDS attribute: ") + hipGetErrorString(st)));
  } else {
    e->block = sa::kHbmBlock;
    e->spl = (uint32_t)sa::kVariants[e->variant].spl;
    e->G = e->cus * 8;
    // partitioned path unless the LDS counter row is too small for the
    // buckets (SA_OPT_ATOMIC_TABLE: per-span atomics)
    e->part = e->nbk <= sa::kPartMaxBk && !(cfg->options & SA_OPT_ATOMIC_TABLE) && !e->expo;
    if (e->part)
      if (hipError_t st = sa::prepare_ingest_part(); st != hipSuccess)
        return bail(fail(e, SA_EDEVICE, std::string("LDS attribute: ") + hipGetErrorString(st)));
    // binned-table path where each bin's sub-table fits an aggregate
    // workgroup's LDS (256..2048 slots per bin: 2^19..2^22 table slots), the
    // window slot fits the record (<= 1024 windows) and buckets come from the
    // bin table (SA_OPT_PARTITIONED: the partitioned path)
    sa::BinEntry bins_probe[sa::kBins];  // the binned kernels bucket by the bin table
    e->bt = e->part && e->log2cap >= sa::kPartBinBits + 8 && e->log2cap <= sa::kPartBinBits + 11 &&
            cfg->n_windows <= 1024 && build_bins(e, bins_probe) && !(cfg->options & SA_OPT_PARTITIONED);
  }

  const uint64_t S = cfg->n_services, W = cfg->n_windows;
  e->hll_slot_bytes = (size_t)S << cfg->hll_p;
  e->cms_slot_elems = (size_t)cfg->cms_d * cfg->cms_w;
  auto alloc = [&](void **p, size_t bytes) -> int {
    if (hipMalloc(p, bytes) != hipSuccess) return fail(e, SA_ENOMEM, "hipMalloc failed");
    if (hipMemset(*p, 0, bytes) != hipSuccess) return fail(e, SA_EDEVICE, "hipMemset failed");
    return SA_OK;
  };
  int rc = SA_OK;
  if ((rc = alloc((void **)&e->gkeys, e->cap * 8)) ||
      (rc = alloc((void **)&e->gcounts, counts_bytes(e))) ||
      (rc = alloc((void **)&e->hll, e->hll_slot_bytes * W)) ||
      (rc = alloc((void **)&e->cms, e->cms_slot_elems * W * 8)) ||
      (rc = alloc((void **)&e->errcnt, (size_t)W * e->cap * 8)) ||
      (rc = alloc((void **)&e->d_seeds, sizeof kCmsSeed)) ||
      (rc = alloc((void **)&e->stats, 64)) || (rc = alloc((void **)&e->scratch, 64)) ||
      (rc = alloc((void **)&e->hll_filt, sa::kFiltSlots * 8)))
    return bail(rc);
  {
    // bound sub-blocks: as small as kLbMinShift allows within kLbMaxSub of them
    // (SA_OPT_NO_HLL_FILTER turns the filter off)
    const uint64_t regs = W * S << cfg->hll_p;
    uint32_t sh = sa::kLbMinShift;
    while (sh < cfg->hll_p && (regs >> sh) > sa::kLbMaxSub) ++sh;
    if ((regs >> sh) <= sa::kLbMaxSub && sh <= cfg->hll_p && !(cfg->options & SA_OPT_NO_HLL_FILTER)) {
      e->lb_shift = sh;
      e->lb_n = (uint32_t)(regs >> sh);
      if ((rc = alloc((void **)&e->hll_lb, ((size_t)e->lb_n + 15) & ~(size_t)15))) return bail(rc);
    }
  }
  if (e->expo) {
    if ((rc = alloc((void **)&e->expo_hdr, (size_t)e->cap * sizeof(sa::ExpoHdr))) ||
        (rc = alloc((void **)&e->expo_buckets, (size_t)2 * e->cap * cfg->exp_max_size * 4)))
      return bail(rc);
    if (e->expo_small && (rc = alloc((void **)&e->expo_xscale, (size_t)e->cap))) return bail(rc);
    if (sa::launch_expo_init(e->expo_hdr, e->expo_xscale, e->cap, nullptr) != hipSuccess)
      return bail(fail(e, SA_EDEVICE, "expo state init failed"));
    if (e->expo_small) {
      e->nsets = kDefaultSlabSets;
      if (const char *v = ab_env("SPANAGG_SLAB_SETS"))
        e->nsets = (uint32_t)std::max(1, std::min((int)kMaxSlabSets, std::atoi(v)));
      if ((rc = alloc((void **)&e->xslab, (size_t)e->nsets * e->G * e->cap * sizeof(sa::XHdr)))) return bail(rc);
      if (hipEventCreateWithFlags(&e->ev_expo, ev_flags()) != hipSuccess)
        return bail(fail(e, SA_EDEVICE, "event creation failed"));
      // (laboratory build, SPANAGG_XSTREAM=1: the histogram kernels on an
      // engine stream -- slower by A/B)
      if (const char *v = ab_env("SPANAGG_XSTREAM"); v && std::atoi(v) != 0) {
        if (hipStreamCreateWithFlags(&e->xstream, hipStreamNonBlocking) != hipSuccess)
          return bail(fail(e, SA_EDEVICE, "histogram stream creation failed"));
        for (hipEvent_t &ev : e->ev_ing)
          if (hipEventCreateWithFlags(&ev, ev_flags()) != hipSuccess)
            return bail(fail(e, SA_EDEVICE, "event creation failed"));
      }
      if (e->xc_ne &&
          ((rc = alloc((void **)&e->xc_lcount, e->cap * 12)) ||  // lcount [cap], then xmeta [cap]
           (rc = alloc((void **)&e->xc_slot_of_entry, (size_t)e->xc_ne * 8)) ||
           (rc = alloc((void **)&e->xc_ent, (size_t)e->cap * 8)) ||
           (rc = alloc((void **)&e->xcslab, (size_t)e->G * sa::xc_slab_stride(e->xc_ne, cfg->exp_max_size) * 4)) ||
           (rc = alloc((void **)&e->xt_rec, (size_t)e->G * sa::xt_bins(e->cap, cfg->exp_max_size) * sa::kXtRun * 4)) ||
           (rc = alloc((void **)&e->xt_off, (size_t)e->G * (sa::xt_bins(e->cap, cfg->exp_max_size) + 1) * 4))))
        return bail(rc);
      // no selection yet: no entries (the first launch counts every span through the tail)
      if (e->xc_ne && (hipMemset(e->xc_slot_of_entry, 0xFF, (size_t)e->xc_ne * 8) != hipSuccess ||
                       hipMemset(e->xc_ent, 0xFF, (size_t)e->cap * 8) != hipSuccess))
        return bail(fail(e, SA_EDEVICE, "hipMemset failed"));
      // (window, slot) keys of the LDS ERROR table are 16-bit
      if ((uint64_t)cfg->n_windows * e->cap < 65535 &&
          (rc = alloc((void **)&e->errslab, (size_t)e->nsets * e->G * cfg->n_windows * e->cap * 4)))
        return bail(rc);
    }
  }
  if ((cfg->options & SA_OPT_STAMPS) && (rc = alloc((void **)&e->dbg, (size_t)e->G * sa::kDbgPerWg * 8)))
    return bail(rc);
  {
    sa::BinEntry bins[sa::kBins];
    if (build_bins(e, bins)) {
      if ((rc = alloc((void **)&e->d_bins, sizeof bins))) return bail(rc);
      if (hipMemcpy(e->d_bins, bins, sizeof bins, hipMemcpyHostToDevice) != hipSuccess)
        return bail(fail(e, SA_EDEVICE, "bin table upload failed"));
    }
  }
  if (e->bt) {
    // one scatter workgroup per CU (~160 KiB LDS); 512-thread aggregate
    // workgroups sized for the bin's sub-table
    e->log2sb = e->log2cap - sa::kPartBinBits;
    e->bt_grid = e->cus;
    e->agg_lds = sa::bt_agg2_lds_bytes(e->log2sb, e->bt_grid);
    const size_t spill = (size_t)e->cap * (e->nbk + 1) * 8;
    if ((rc = alloc((void **)&e->base64, spill))) return bail(rc);  // (zeroed)
    if (hipError_t st = sa::prepare_ingest_bt(e->agg_lds); st != hipSuccess)
      return bail(fail(e, SA_EDEVICE, std::string("LDS attribute: ") + hipGetErrorString(st)));
    // the aggregate stream of the launch pipeline (ordered by events only)
    if (hipStreamCreateWithFlags(&e->agg_stream, hipStreamNonBlocking) != hipSuccess)
      return bail(fail(e, SA_EDEVICE, "aggregate stream creation failed"));
    for (int k = 0; k < sa_engine::kBtSets; ++k)
      if (hipEventCreateWithFlags(&e->ev_scat[k], ev_flags()) != hipSuccess ||
          hipEventCreateWithFlags(&e->ev_agg[k], ev_flags()) != hipSuccess)
        return bail(fail(e, SA_EDEVICE, "event creation failed"));
    // a random odd multiplier per engine: series ids -> stored ids (bins and
    // home slots), so bin occupancy does not depend on ids a sender chooses
    std::random_device rd;
    uint64_t r = ((uint64_t)rd() << 32) ^ rd();
    if (cfg->options & SA_OPT_IDENTITY_IDS) r = 1;  // stored id = series id (tests of a full bin)
    if (const char *kv = ab_env("SPANAGG_KMUL")) r = std::strtoull(kv, nullptr, 0);  // fixed, for A/B runs
    e->kmul = r | 1ULL;
    uint64_t x = e->kmul;  // Newton: x = x (2 - a x) doubles the correct low bits
    for (int i = 0; i < 6; ++i) x *= 2 - e->kmul * x;
    e->kinv = x;
  }
  if (hipMemcpy(e->d_seeds, kCmsSeed, sizeof kCmsSeed, hipMemcpyHostToDevice) != hipSuccess)
    return bail(fail(e, SA_EDEVICE, "seed upload failed"));
  if (e->small) {
    e->nsets = kDefaultSlabSets;
    if (const char *v = ab_env("SPANAGG_SLAB_SETS"))
      e->nsets = (uint32_t)std::max(1, std::min((int)kMaxSlabSets, std::atoi(v)));
    const size_t srow = (e->nbk + 1) & ~1u;  // slab row = 2 * ceil(nbk/2) u32 cells
    const size_t gs = (size_t)e->G * e->nsets;  // slabs of all sets, set-major
    if ((rc = alloc((void **)&e->slab_cnt, gs * e->cap * srow * 4)) ||
        (rc = alloc((void **)&e->slab_sum, gs * e->cap * 8)))
      return bail(rc);
    // (window, slot) keys of the v2 kernels' LDS ERROR table are 16-bit
    if (e->variant >= 8 && (uint64_t)cfg->n_windows * e->cap < 65535 &&
        (rc = alloc((void **)&e->errslab, gs * cfg->n_windows * e->cap * 4)))
      return bail(rc);
  }
  // the tail pool: only the specialised default geometry has a POOL kernel
  e->pool = e->small && e->variant == sa::kLdsPoolVariant && e->d_bins && e->log2cap == 11 &&
            (e->nbk + 1) / 2 == 9 && cfg->hll_p == 14;
  if (e->pool && (rc = alloc((void **)&e->pool_ring, sa::kPoolRing * 4))) return bail(rc);
  if (hipDeviceSynchronize() != hipSuccess) return bail(fail(e, SA_EDEVICE, "device sync failed"));
  *out = e;
  return SA_OK;
}

static void join_sets(sa_engine *e);

void sa_destroy(sa_engine *e) {
  if (!e) return;
  (void)hipSetDevice(e->dev);
  if (e->stream) {
    join_sets(e);
    (void)hipStreamSynchronize(e->stream);
  }
  for (void *p : {(void *)e->gkeys, (void *)e->gcounts, (void *)e->slab_sum, (void *)e->cms,
                  (void *)e->stats, (void *)e->out_keys, (void *)e->out_rows, (void *)e->scratch,
                  (void *)e->slab_cnt, (void *)e->hll, (void *)e->errcnt, (void *)e->d_seeds,
                  (void *)e->dbg, (void *)e->d_bins, (void *)e->errslab, (void *)e->part_rec,
                  (void *)e->part_fill, (void *)e->base64, (void *)e->hll_lb,
                  (void *)e->expo_hdr, (void *)e->expo_xscale, (void *)e->expo_buckets, (void *)e->expo_slot,
                  (void *)e->expo_out_keys,
                  (void *)e->expo_out_rows, (void *)e->expo_out_buckets, (void *)e->hll_filt, (void *)e->xslab,
                  (void *)e->xc_lcount, (void *)e->xc_slot_of_entry, (void *)e->xc_ent, (void *)e->xcslab, (void *)e->pool_ring,
                  (void *)e->xt_rec, (void *)e->xt_off,
                  e->dstage[0], e->dstage[1]})
    if (p) (void)hipFree(p);
  for (int k = 0; k < sa_engine::kBtSets; ++k)
    for (void *p : {(void *)e->bt_rec[k], (void *)e->bt_cnt[k]})
      if (p) (void)hipFree(p);
  for (int k = 0; k < 2; ++k) {
    if (e->pin[k]) (void)hipHostFree(e->pin[k]);
    if (e->pin_ev[k]) (void)hipEventDestroy(e->pin_ev[k]);
  }
  if (e->ev_async) (void)hipEventDestroy(e->ev_async);
  for (auto &g : e->gi) {
    if (g.x) (void)hipGraphExecDestroy(g.x);
    if (g.g) (void)hipGraphDestroy(g.g);
    if (g.done) (void)hipEventDestroy(g.done);
  }
  if (e->ev_a) (void)hipEventDestroy(e->ev_a);
  if (e->ev_b) (void)hipEventDestroy(e->ev_b);
  for (hipEvent_t ev : e->ev_set)
    if (ev) (void)hipEventDestroy(ev);
  if (e->ev_ctl) (void)hipEventDestroy(e->ev_ctl);
  if (e->ev_expo) (void)hipEventDestroy(e->ev_expo);
  for (hipEvent_t ev : e->ev_ing)
    if (ev) (void)hipEventDestroy(ev);
  if (e->xstream) {
    (void)hipStreamSynchronize(e->xstream);
    (void)hipStreamDestroy(e->xstream);
  }
  for (int k = 0; k < sa_engine::kBtSets; ++k) {
    if (e->ev_scat[k]) (void)hipEventDestroy(e->ev_scat[k]);
    if (e->ev_agg[k]) (void)hipEventDestroy(e->ev_agg[k]);
  }
  if (e->agg_stream) {
    (void)hipStreamSynchronize(e->agg_stream);
    (void)hipStreamDestroy(e->agg_stream);
  }
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
}

const char *sa_last_error(const sa_engine *e) { return e ? e->err.c_str() : "null engine"; }

// Orders the engine stream after every outstanding launch (each set's last
// user); the next launch then orders after whatever the caller enqueues on the
// engine stream now (ev_ctl, recorded lazily by that launch).
static int bt_aggregate_pending(sa_engine *e);
static void join_sets(sa_engine *e) {
  // a pending binned record set is aggregated first; a failed launch is
  // kept (sticky_rc, bt_aggregate_pending) and returned by join_checked, so
  // no read goes on without it
  (void)bt_aggregate_pending(e);
  for (uint32_t i = 0; i < e->nsets; ++i)
    if (e->set_stream[i] && e->set_stream[i] != e->stream)
      (void)hipStreamWaitEvent(e->stream, e->ev_set[i], 0);
  for (int k = 0; k < sa_engine::kBtSets; ++k)  // the binned path's aggregates
    if (e->agg_used[k]) (void)hipStreamWaitEvent(e->stream, e->ev_agg[k], 0);
  e->ctl_dirty = true;
}

// join_sets for the calls that read or reorder: SA_EDEVICE (with e->err) when
// a pending aggregate could not be launched
static int join_checked(sa_engine *e) {
  join_sets(e);
  return e->sticky_rc;
}

static int reduce_slabs(sa_engine *e, hipStream_t s) {
  if (!e->small || e->slab_load == 0) return SA_OK;
  SA_HIP(e, sa::launch_reduce_slabs(e->slab_cnt, e->slab_sum, e->gcounts, e->G * e->nsets, e->cap,
                                    e->nbk, s));
  e->slab_load = 0;
  return SA_OK;
}

static int ingest_launch(sa_engine *e, const sa_span_batch *b, hipStream_t s);

// Splits a batch so that each workgroup's range stays addressable by a 32-bit
// buffer offset (< 2^27 spans per workgroup per launch).
static int ingest_on(sa_engine *e, const sa_span_batch *b, hipStream_t s) {
  // v2 small-table kernels keep u16 LDS counters for the whole launch: at most
  // 65532 spans per workgroup per launch (ingest_v2_kernel has no epoch flush)
  const uint64_t max_n = e->bt     ? (uint64_t)e->bt_grid * sa::kBtMaxWgSpans
                         : e->part ? sa::kPartMaxSpans
                                   : e->pool ? (uint64_t)e->G * sa::kPoolMaxWgSpans
                         : (uint64_t)e->G * (((e->small && e->variant >= 8) || e->expo_small) ? sa::kMaxWgSpans
                                                                                                       : (1u << 27));
  for (uint64_t off = 0; off < b->n; off += max_n) {
    const uint64_t m = std::min(max_n, b->n - off);
    sa_span_batch sub{b->key_hash + off, b->start_ns + off, b->end_ns + off, b->trace_w0 + off,
                      b->trace_w1 + off, b->meta + off, m};
    if (int rc = ingest_launch(e, &sub, s)) return rc;
  }
  return SA_OK;
}

// Binned path: launch geometry, record regions (allocated once for the
// largest launch).  Region capacity: the mean records
// per (bin, scatter workgroup) plus 4 standard deviations and 8, in whole
// 4-record chunks; records beyond it take the scatter's overflow table.
static uint32_t bt_region_for(uint64_t wg_chunk) {
  const double mu = (double)wg_chunk / sa::kPartBins;
  return ((uint32_t)std::ceil(mu + 4.0 * std::sqrt(mu) + 8.0) + sa::kBtStage - 1) & ~(sa::kBtStage - 1);
}

static int bt_prepare_launch(sa_engine *e, uint64_t n, IngestParams &P, hipStream_t s) {
  const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(e->bt_grid, (n + 4095) / 4096));
  P.bt_grid = grid;
  P.wg_chunk = ((n + grid - 1) / grid + 3) / 4 * 4;
  P.bt_region = bt_region_for(P.wg_chunk);
  if (!e->bt_rec[0]) {
    const size_t recs = (size_t)sa::kPartBins * e->bt_grid * bt_region_for(sa::kBtMaxWgSpans);
    for (int k = 0; k < sa_engine::kBtSets; ++k)
      if (hipMalloc((void **)&e->bt_rec[k], recs * sizeof(ulonglong2)) != hipSuccess ||
          hipMalloc((void **)&e->bt_cnt[k], (size_t)e->bt_grid * sa::kPartBins * 4) != hipSuccess)
        return fail(e, SA_ENOMEM, "binned-path record buffers hipMalloc failed");
  }
  P.log2sb = e->log2sb;
  P.kmul = e->kmul;
  P.kinv = e->kinv;
  P.bt_rec = e->bt_rec[e->bt_set];
  P.bt_cnt = e->bt_cnt[e->bt_set];
  P.bt_rec2 = nullptr;
  P.bt_cnt2 = nullptr;
  return SA_OK;
}

// The aggregate of record set k alone (pend < 0), or of the pending set and k
// together (the pending set's records first), on `as` after both scatters.
static int bt_launch_aggregate(sa_engine *e, int pend, const sa::IngestParams &Pp, int k,
                               const sa::IngestParams &Pk, hipStream_t as) {
  sa::IngestParams A = pend >= 0 ? Pp : Pk;
  if (pend >= 0) {
    A.bt_rec2 = Pk.bt_rec;
    A.bt_cnt2 = Pk.bt_cnt;
    A.bt_grid2 = Pk.bt_grid;
    A.bt_region2 = Pk.bt_region;
  }
  for (int j : {pend, k})
    if (j >= 0) SA_HIP(e, hipStreamWaitEvent(as, e->ev_scat[j], 0));
  {
    // laboratory build: SPANAGG_FAIL_AGG=n fails the n-th aggregate launch of
    // the process (tests of the pending-set error path)
    static const long fail_at = [] {
      const char *v = ab_env("SPANAGG_FAIL_AGG");
      return v ? std::atol(v) : 0L;
    }();
    static long n_agg = 0;
    if (fail_at > 0 && ++n_agg == fail_at) return fail(e, SA_EDEVICE, "aggregate launch: injected failure");
  }
  if (hipError_t st = sa::launch_bt_aggregate(A, as); st != hipSuccess)
    return fail(e, SA_EDEVICE, std::string("aggregate launch: ") + hipGetErrorString(st));
  for (int j : {pend, k})
    if (j >= 0) {
      SA_HIP(e, hipEventRecord(e->ev_agg[j], as));
      e->agg_used[j] = true;
    }
  return SA_OK;
}

// Every launch of an aggregate that takes a pending record set goes through
// here: the pending set belongs to an ingest that already returned SA_OK, so a
// failure is kept (sticky_rc) and returned by every later read instead of
// results without those records.
static int bt_launch_with_pending(sa_engine *e, const sa::IngestParams &Pk, int k, hipStream_t as) {
  const int pend = e->bt_pend;
  e->bt_pend = -1;
  const int rc = bt_launch_aggregate(e, pend, e->bt_pend_P, k, Pk, as);
  if (rc && pend >= 0 && !e->sticky_rc) e->sticky_rc = rc;
  return rc;
}

static int bt_aggregate_pending(sa_engine *e) {
  if (!e->bt || e->bt_pend < 0) return SA_OK;
  const int k = e->bt_pend;
  e->bt_pend = -1;
  const int rc = bt_launch_aggregate(e, -1, e->bt_pend_P, k, e->bt_pend_P, e->agg_stream);
  if (rc && !e->sticky_rc) e->sticky_rc = rc;
  return rc;
}


// The exponential slab path's span words (kExpoRecMode; laboratory build:
// SPANAGG_XREC=0 / 1 / 2 picks, for A/B runs); slab counting only
static int expo_rec_mode(const sa_engine *e) {
  static const int knob = [] {
    const char *v = ab_env("SPANAGG_XREC");
    return v ? std::atoi(v) : -1;
  }();
  if (!e->expo_small || !e->xc_ne) return 0;
  return knob >= 0 && knob <= 2 ? knob : kExpoRecMode;
}
static bool expo_span_recs(const sa_engine *e) { return expo_rec_mode(e) == 1; }

static sa::ExpoParams expo_params(sa_engine *e, const sa_span_batch *b, uint32_t set = 0) {
  sa::ExpoParams E{};
  if (b) {
    E.key = b->key_hash;
    E.start = b->start_ns;
    E.end = b->end_ns;
    E.n = b->n;
  }
  E.gkeys = e->gkeys;
  E.log2cap = e->log2cap;
  E.max_probe = sa::max_probe_of(e->log2cap);
  E.cap = e->cap;
  E.hdr = e->expo_hdr;
  E.xscale = e->expo_xscale;
  E.buckets = e->expo_buckets;
  E.max_size = e->cfg.exp_max_size;
  E.div = e->cfg.unit == SA_UNIT_S ? 1e9 : 1e6;
  E.log2div_q24 = sa::expo_l2d_q24(E.div);
  {
    static const uint32_t diag = [] {
      const char *v = ab_env("SPANAGG_XC_DIAG");
      return v ? (uint32_t)std::strtoul(v, nullptr, 0) : 0u;
    }();
    E.diag = diag;
  }
  // (this launch's set of span slots / records and header partials)
  // (per set: n span records or u32 slots, then n long durations)
  E.slot_of = e->expo_slot ? e->expo_slot + 4 * (size_t)set * e->expo_slot_cap : nullptr;
  E.span_rec = expo_span_recs(e) ? reinterpret_cast<const unsigned long long *>(E.slot_of) : nullptr;
  E.xidx = expo_rec_mode(e) == 2 ? 1u : 0u;
  E.span_long = (E.span_rec || E.xidx) && e->expo_slot
                    ? reinterpret_cast<const unsigned long long *>(E.slot_of) + e->expo_slot_cap
                    : nullptr;
  E.dropped = e->stats + sa::kStatDropped;
  E.xslab = e->expo_small ? e->xslab + (size_t)set * e->G * e->cap : nullptr;
  // the workgroups whose header partials this launch wrote (ingest_launch's
  // grid: each writes every slot of its slab row; rows past it are stale)
  E.xG = b ? (uint32_t)std::min<uint64_t>((b->n + (uint64_t)e->block * e->spl - 1) / ((uint64_t)e->block * e->spl), e->G)
           : e->G;
  E.xc_ne = e->expo_small ? e->xc_ne : 0u;
  E.lcount = E.xc_ne ? e->xc_lcount : nullptr;
  E.xmeta = E.xc_ne ? reinterpret_cast<int2 *>(e->xc_lcount + e->cap) : nullptr;
  // (compact passes no batch and reads none of these)
  const uint32_t cur = e->xc_sel & 1u, nxt = cur ^ 1u;
  E.slot_of_entry = e->xc_slot_of_entry ? e->xc_slot_of_entry + (size_t)cur * e->xc_ne : nullptr;
  E.soe_next = e->xc_slot_of_entry ? e->xc_slot_of_entry + (size_t)nxt * e->xc_ne : nullptr;
  E.xent = e->xc_ent ? e->xc_ent + (size_t)cur * e->cap : nullptr;
  E.xent_next = e->xc_ent ? e->xc_ent + (size_t)nxt * e->cap : nullptr;
  if (!e->xc_sel_made) {  // the first launch: its own selection, in every counting workgroup
    E.xent = nullptr;
    E.slot_of_entry = E.soe_next;
  }
  E.xcslab = e->xcslab;
  {
    // laboratory build: SPANAGG_XT=0 sends the counting kernel's tail to HBM
    // atomics (the earlier form), for A/B runs
    static const bool xt = [] {
      const char *v = ab_env("SPANAGG_XT");
      return !(v && std::atoi(v) == 0);
    }();
    E.xt_rec = xt && E.xc_ne ? e->xt_rec : nullptr;
    E.xt_off = e->xt_off;
  }
  E.dbg = e->dbg;
  return E;
}

// The launch parameters of one ingest of batch b into slab set `set` (the
// workgroup ranges, pool and tables; every path's kernels read from these).
static void fill_params(sa_engine *e, const sa_span_batch *b, uint32_t set, uint64_t wg_chunk,
                        uint64_t pool_base, uint32_t pool_n, IngestParams &P) {
  const size_t srow = (e->nbk + 1) & ~1u;
  P.key = b->key_hash;
  P.start = b->start_ns;
  P.end = b->end_ns;
  P.w0 = b->trace_w0;
  P.w1 = b->trace_w1;
  P.meta = b->meta;
  P.n = b->n;
  P.wg_chunk = wg_chunk;
  P.pool_base = pool_base;
  P.pool_n = pool_n;
  if (e->pool) {
    P.pool_ctr = e->pool_ring + e->pool_seq % sa::kPoolRing;
    P.pool_next = e->pool_ring + (e->pool_seq + e->nsets) % sa::kPoolRing;
    ++e->pool_seq;
  }
  P.gkeys = e->gkeys;
  P.log2cap = e->log2cap;
  P.max_probe = sa::max_probe_of(e->log2cap);
  P.slab_cnt = e->slab_cnt ? e->slab_cnt + (size_t)set * e->G * e->cap * srow : nullptr;
  P.slab_sum = e->slab_sum ? e->slab_sum + (size_t)set * e->G * e->cap : nullptr;
  P.gcounts = e->gcounts;
  P.base64 = e->base64;
  std::memcpy(P.thr, e->thr, sizeof e->thr);
  P.npos = e->npos;
  P.nneg = e->nneg;
  P.nbk = e->nbk;
  P.epoch_tiles = (uint32_t)(65535 / ((uint64_t)e->block * e->spl));  // (the launch's tile)
  P.hll = e->hll;
  P.cms = e->cms;
  P.errcnt = e->errcnt;
  P.errslab = e->errslab ? e->errslab + (size_t)set * e->G * e->cfg.n_windows * e->cap : nullptr;
  P.window_ns = e->cfg.window_ns;
  P.win_magic = UINT64_MAX / e->cfg.window_ns;
  P.win_base = e->win_base;
  P.base_ns = e->win_base * e->cfg.window_ns;  // < 2^64: checked in sa_window_advance
  P.ring_ns = (uint64_t)e->cfg.n_windows * e->cfg.window_ns;
  P.inv_window = (float)(1.0 / (double)e->cfg.window_ns);
  P.win_ok = (float)(0.5 - (double)e->cfg.n_windows * 0x1p-20);  // n_windows <= 4096: >= 0.496
  P.base_slot = (uint32_t)(e->win_base & (e->cfg.n_windows - 1));
  P.bintab = e->d_bins;
  P.win_mask = e->cfg.n_windows - 1;
  P.n_windows = e->cfg.n_windows;
  P.p = e->cfg.hll_p;
  P.n_services = e->cfg.n_services;
  P.cms_d = e->cfg.cms_d;
  P.cms_w = e->cfg.cms_w;
  P.cms_shift = 64 - log2u(e->cfg.cms_w);
  P.seeds = e->d_seeds;
  P.stats = e->stats;
  P.diag = e->cfg.flags;
  P.dbg = e->dbg;
  P.hll_lb = e->hll_lb;
  P.lb_shift = e->lb_shift;
  P.lb_n = e->lb_n;  // read (and refreshed) by the v2 and binned kernels; the others ignore it
  P.lb_seq = e->lb_seq++;
  P.hll_filt = e->hll_filt;
}

static int ingest_launch(sa_engine *e, const sa_span_batch *b, hipStream_t s) {
  if (b->n == 0) return SA_OK;
  const uint64_t tile = (uint64_t)e->block * e->spl;
  const uint64_t tiles = (b->n + tile - 1) / tile;
  // each workgroup gets one contiguous range of >= one tile (kernel: wg_range)
  const uint32_t grid = (uint32_t)std::min<uint64_t>(tiles, e->G);
  // tail pool (POOL kernel): each workgroup's static share is 7/8 of the
  // average in whole 256-span chunks, the rest is the pool the workgroups
  // that finish first take in blocks of kPoolSpans (a launch too small for two
  // fixed chunks per wave has no pool)
  uint64_t wg_chunk = ((b->n + grid - 1) / grid + 3) / 4 * 4, pool_base = 0;
  uint32_t pool_n = 0;
  if (e->pool) {
    const uint64_t per = (b->n + grid - 1) / grid;
    const uint64_t wc = std::min<uint64_t>(per * 7 / 8 / 256 * 256, sa::kPoolMaxStatic);
    if (wc >= sa::kPoolMinStatic) {
      wg_chunk = wc;
      pool_base = grid * wc;
      pool_n = (uint32_t)((b->n - pool_base + sa::kPoolSpans - 1) / sa::kPoolSpans);
      if (pool_n > (uint64_t)grid * sa::kPoolMaxSteal) return fail(e, SA_EINVAL, "tail pool above the steal limits");
    }
  }
  if (e->small) {
    const uint64_t per_wg = pool_n ? wg_chunk + sa::kPoolMaxSteal * sa::kPoolSpans : wg_chunk;
    if (e->slab_load + per_wg > kSlabLimit) {  // fold every set into the counters first
      if (int rc = join_checked(e)) return rc;
      if (int rc = reduce_slabs(e, e->stream)) return rc;
    }
    e->slab_load += per_wg;
  }
  // order: after the engine stream's work so far (ev_ctl, re-recorded after
  // each join) and after the previous launch that used this slab set
  if (e->ctl_dirty) {
    SA_HIP(e, hipEventRecord(e->ev_ctl, e->stream));
    e->ctl_dirty = false;
  }
  if (s != e->stream) SA_HIP(e, hipStreamWaitEvent(s, e->ev_ctl, 0));
  const uint32_t set = e->set;
  if (e->set_stream[set] && e->set_stream[set] != s) SA_HIP(e, hipStreamWaitEvent(s, e->ev_set[set], 0));
  IngestParams P{};
  fill_params(e, b, set, wg_chunk, pool_base, pool_n, P);
  hipError_t st;
  hipStream_t hs = s;  // the stream the launch's last kernel runs on (expo: the histogram kernels')
  if (e->small) {
    st = sa::launch_ingest_small(P, grid, e->lds_bytes, s, e->variant);
  } else if (e->bt) {
    if (int rc = bt_prepare_launch(e, b->n, P, s)) return rc;
    // the pipeline (sa_engine::bt_rec): scatter here, aggregate on agg_stream
    const int k = (int)e->bt_set;
    if (e->agg_used[k]) SA_HIP(e, hipStreamWaitEvent(s, e->ev_agg[k], 0));  // set k's last reader
    // (laboratory build: SPANAGG_BT_PIPE=0 runs each launch's aggregate right
    // after its scatter on the caller's stream; SPANAGG_BT_PAIR=0 aggregates
    // every launch alone on the aggregate stream)
    static const bool pipe = [] {
      const char *v = ab_env("SPANAGG_BT_PIPE");
      return !(v && std::atoi(v) == 0);
    }();
    static const bool pair = [] {
      const char *v = ab_env("SPANAGG_BT_PAIR");
      return !(v && std::atoi(v) == 0);
    }();
    st = sa::launch_bt_scatter(P, s);
    if (st == hipSuccess) st = hipEventRecord(e->ev_scat[k], s);
    if (st != hipSuccess) return fail(e, SA_EDEVICE, std::string("ingest launch: ") + hipGetErrorString(st));
    if (!pipe) {
      if (int rc = bt_launch_aggregate(e, -1, P, k, P, s)) return rc;
    } else if (pair && e->bt_pend < 0) {
      e->bt_pend = k;  // aggregated with the next launch's records, or at the next join
      e->bt_pend_P = P;
    } else {
      if (int rc = bt_launch_with_pending(e, P, k, e->agg_stream)) return rc;
    }
    e->bt_set = (e->bt_set + 1) % sa_engine::kBtSets;
  } else if (e->part) {
    // records per bin: 1.25x the mean plus slack; a fuller bin spills to the
    // direct path, so this bounds memory, not correctness
    const uint64_t per_bin_max = sa::kPartMaxCap;
    if (!e->part_rec) {
      if (hipMalloc((void **)&e->part_rec, sa::kPartBins * per_bin_max * sizeof(ulonglong2)) != hipSuccess ||
          hipMalloc((void **)&e->part_fill, sa::kPartBins * 4) != hipSuccess ||
          hipMemset(e->part_fill, 0, sa::kPartBins * 4) != hipSuccess)
        return fail(e, SA_ENOMEM, "partition buffers hipMalloc failed");
    }
    P.part_rec = e->part_rec;
    P.part_fill = e->part_fill;
    // a multiple of 4 records: staged 64-B chunks stay segment-aligned
    P.part_cap = (uint32_t)std::min<uint64_t>(
        per_bin_max, ((b->n + sa::kPartBins - 1) / sa::kPartBins * 5 / 4 + 64 + sa::kPartStage - 1) &
                         ~(uint64_t)(sa::kPartStage - 1));
    st = sa::launch_ingest_part(P, s);
  } else if (e->expo) {
    if (e->expo_slot_cap < b->n) {  // (hipFree waits for the device)
      if (e->expo_slot) (void)hipFree(e->expo_slot);
      e->expo_slot = nullptr;
      e->expo_slot_cap = 0;
      // (16 B per span and set: span records or u32 slots, then long durations)
      if (hipMalloc((void **)&e->expo_slot, (size_t)e->nsets * b->n * 16) != hipSuccess)
        return fail(e, SA_ENOMEM, "expo slot buffer");
      e->expo_slot_cap = b->n;
    }
    uint32_t *slots = e->expo_slot + 4 * (size_t)set * e->expo_slot_cap;
    if (e->expo_small) {
      // the small-table kernel in EXPO mode: sketches, key slots, header partials
      const int mode = expo_rec_mode(e);
      const bool recs = mode == 1;
      if (recs) {
        P.span_rec = reinterpret_cast<unsigned long long *>(slots);
        P.span_long = P.span_rec + e->expo_slot_cap;
      } else {
        P.slot_of = slots;
        if (mode == 2) {
          P.xidx = 1;
          if (const char *v = ab_env("SPANAGG_XIDX_OFF")) P.xidx = std::atoi(v) == 2 ? 3 : 2;  // (ablation: results wrong)
          P.xscale = e->expo_xscale;
          P.l2d_q24 = sa::expo_l2d_q24(e->cfg.unit == SA_UNIT_S ? 1e9 : 1e6);
          P.span_long = reinterpret_cast<unsigned long long *>(slots) + e->expo_slot_cap;
        }
      }
      P.xslab = e->xslab + (size_t)set * e->G * e->cap;
      st = sa::launch_ingest_expo_small(P, grid, e->lds_bytes, s);
      if (recs && e->xstream) {
        // the histogram kernels on the engine's xstream, after this ingest kernel
        hs = e->xstream;
        if (st == hipSuccess) st = hipEventRecord(e->ev_ing[set], s);
        if (st == hipSuccess) st = hipStreamWaitEvent(hs, e->ev_ing[set], 0);
      } else if (st == hipSuccess && e->expo_last && e->expo_last != s) {
        // on the caller's stream, after the previous launch's histogram kernels
        // (one owner of the headers and buckets at a time)
        st = hipStreamWaitEvent(s, e->ev_expo, 0);
      }
    } else {
      // sketches (and the zero-key / service / window counters) through the
      // HBM-table kernel with its RED part off
      P.diag |= SA_DIAG_NO_RED;
      st = sa::launch_ingest_hbm(P, grid, s, e->variant);
    }
    // then the histogram kernels
    if (st == hipSuccess) st = sa::launch_expo_ingest(expo_params(e, b, set), hs);
    if (st == hipSuccess && e->expo_small && e->xc_ne) {  // (the next launch counts with this one's selection)
      e->xc_sel ^= 1u;
      e->xc_sel_made = true;
    }
    if (st == hipSuccess && e->ev_expo) {
      st = hipEventRecord(e->ev_expo, hs);
      e->expo_last = hs;
    }
  } else {
    st = sa::launch_ingest_hbm(P, grid, s, e->variant);
  }
  if (st != hipSuccess) return fail(e, SA_EDEVICE, std::string("ingest launch: ") + hipGetErrorString(st));
  // (laboratory build: SPANAGG_NO_SETEV=1 skips the slab-set event -- only
  // valid when every launch uses one stream; it prices the event's cost)
  static const bool no_setev = ab_env("SPANAGG_NO_SETEV") != nullptr;
  if (!no_setev) SA_HIP(e, hipEventRecord(e->ev_set[set], hs));
  e->set_stream[set] = hs;
  e->set = (set + 1) % e->nsets;
  e->spans += b->n;
  e->unflushed = true;
  return SA_OK;
}

static int check_batch(sa_engine *e, const sa_span_batch *b, bool device) {
  if (!e) return SA_EINVAL;
  if (!b) return fail(e, SA_EINVAL, "null batch");
  if (b->n == 0) return SA_OK;
  const void *cols[5] = {b->key_hash, b->start_ns, b->end_ns, b->trace_w0, b->trace_w1};
  for (const void *c : cols) {
    if (!c) return fail(e, SA_EINVAL, "null batch column");
    if (device && (reinterpret_cast<uintptr_t>(c) & 15))
      return fail(e, SA_EINVAL, "device batch u64 columns must be 16-byte aligned");
  }
  if (!b->meta) return fail(e, SA_EINVAL, "null meta column");
  if (device && (reinterpret_cast<uintptr_t>(b->meta) & 7))
    return fail(e, SA_EINVAL, "device batch meta column must be 8-byte aligned");
  return SA_OK;
}

int sa_ingest_device(sa_engine *e, const sa_span_batch *b, void *stream) {
  if (int rc = check_batch(e, b, true)) return rc;
  if (int rc = set_dev(e)) return rc;
  // stream-ordered on `stream`: after the engine's earlier work, before the
  // caller's later work on the same stream; launches on other streams may
  // overlap it (see sa_engine::nsets)
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
  return ingest_on(e, b, s);
}

// k device batches in order on `stream`, as k sa_ingest_device calls would
// ingest them.  Small-table engines (no tail pool, no diagnostics) launch the
// k kernels as one HIP graph: no per-launch dispatch gap between them.  Any
// other engine, a batch that would split, or a slab reduction due inside the
// k launches takes the stream path, one launch after another.
int sa_ingest_device_many(sa_engine *e, const sa_span_batch *bs, uint32_t k, void *stream) {
  if (!e) return SA_EINVAL;
  if (k && !bs) return fail(e, SA_EINVAL, "null batch array");
  for (uint32_t i = 0; i < k; ++i)
    if (int rc = check_batch(e, &bs[i], true)) return rc;
  if (int rc = set_dev(e)) return rc;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
  bool graph = k > 1 && e->small && !e->expo && !e->bt && !e->part && !e->pool && !e->dbg && e->cfg.flags == 0;
  const uint64_t tile = (uint64_t)e->block * e->spl;
  const uint64_t max_wg = e->variant >= 8 ? sa::kMaxWgSpans : (1u << 27);
  std::vector<uint32_t> grid(k);
  std::vector<uint64_t> chunk(k);
  uint64_t load = 0;
  for (uint32_t i = 0; graph && i < k; ++i) {
    const uint64_t n = bs[i].n;
    if (n == 0 || n > (uint64_t)e->G * max_wg) {
      graph = false;
      break;
    }
    grid[i] = (uint32_t)std::min<uint64_t>((n + tile - 1) / tile, e->G);
    chunk[i] = ((n + grid[i] - 1) / grid[i] + 3) / 4 * 4;
    load += chunk[i];
  }
  if (graph && e->slab_load + load > kSlabLimit) {  // fold every set into the counters first
    if (int rc = join_checked(e)) return rc;
    if (int rc = reduce_slabs(e, e->stream)) return rc;
    graph = load <= kSlabLimit;
  }
  if (!graph) {
    for (uint32_t i = 0; i < k; ++i)
      if (int rc = ingest_on(e, &bs[i], s)) return rc;
    return SA_OK;
  }
  // the ordering ingest_launch gives each launch, once for the k
  if (e->ctl_dirty) {
    SA_HIP(e, hipEventRecord(e->ev_ctl, e->stream));
    e->ctl_dirty = false;
  }
  if (s != e->stream) SA_HIP(e, hipStreamWaitEvent(s, e->ev_ctl, 0));
  for (uint32_t j = 0; j < e->nsets && j < k; ++j) {
    const uint32_t set = (e->set + j) % e->nsets;
    if (e->set_stream[set] && e->set_stream[set] != s) SA_HIP(e, hipStreamWaitEvent(s, e->ev_set[set], 0));
  }
  sa_engine::GraphIngest &g = e->gi[e->gi_next];
  if (g.launched) SA_HIP(e, hipEventSynchronize(g.done));  // its previous launch is over
  std::vector<IngestParams> P(k);
  std::vector<void *> args(k);
  std::vector<hipKernelNodeParams> np(k);
  for (uint32_t i = 0; i < k; ++i) {
    fill_params(e, &bs[i], (e->set + i) % e->nsets, chunk[i], 0, 0, P[i]);
    args[i] = &P[i];
    sa::ingest_small_node(P[i], grid[i], e->lds_bytes, e->variant, &args[i], &np[i]);
  }
  const bool reuse = g.x && g.nodes.size() == k && g.fn == np[0].func && g.lds == e->lds_bytes &&
                     g.block.x == np[0].blockDim.x;
  if (reuse) {
    for (uint32_t i = 0; i < k; ++i) SA_HIP(e, hipGraphExecKernelNodeSetParams(g.x, g.nodes[i], &np[i]));
  } else {
    if (g.x) (void)hipGraphExecDestroy(g.x);
    if (g.g) (void)hipGraphDestroy(g.g);
    g.x = nullptr;
    g.g = nullptr;
    g.nodes.assign(k, nullptr);
    SA_HIP(e, hipGraphCreate(&g.g, 0));
    for (uint32_t i = 0; i < k; ++i)
      SA_HIP(e, hipGraphAddKernelNode(&g.nodes[i], g.g, i ? &g.nodes[i - 1] : nullptr, i ? 1 : 0, &np[i]));
    SA_HIP(e, hipGraphInstantiate(&g.x, g.g, nullptr, nullptr, 0));
    if (!g.done) SA_HIP(e, hipEventCreateWithFlags(&g.done, hipEventDisableTiming));
    g.fn = np[0].func;
    g.lds = e->lds_bytes;
    g.block = np[0].blockDim;
  }
  if (hipError_t st = hipGraphLaunch(g.x, s); st != hipSuccess)
    return fail(e, SA_EDEVICE, std::string("ingest graph launch: ") + hipGetErrorString(st));
  SA_HIP(e, hipEventRecord(g.done, s));
  g.launched = true;
  e->gi_next ^= 1u;
  for (uint32_t j = 0; j < e->nsets && j < k; ++j) {
    const uint32_t set = (e->set + j) % e->nsets;
    SA_HIP(e, hipEventRecord(e->ev_set[set], s));
    e->set_stream[set] = s;
  }
  e->set = (e->set + k) % e->nsets;
  for (uint32_t i = 0; i < k; ++i) e->spans += bs[i].n;
  e->slab_load += load;
  e->unflushed = true;
  return SA_OK;
}

int sa_host_alloc(size_t bytes, void **out) {
  if (!out) return SA_EINVAL;
  *out = nullptr;
  if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    return SA_ENOMEM;
  }
  return SA_OK;
}

void sa_host_free(void *p) {
  if (p) (void)hipHostFree(p);
}

// true when every column of the batch lies in page-locked host memory
static bool batch_pinned(const sa_span_batch *b) {
  const void *cols[6] = {b->key_hash, b->start_ns, b->end_ns, b->trace_w0, b->trace_w1, b->meta};
  for (const void *c : cols) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, c) != hipSuccess) {
      (void)hipGetLastError();  // pageable memory: an error the runtime must not keep
      return false;
    }
    if (a.type != hipMemoryTypeHost) return false;
  }
  return true;
}

// Host batches: each chunk is packed into a pinned slot (CPU copy, 44 B/span),
// copied to HBM by DMA and aggregated on the engine stream; the call returns
// once the batch has been copied out of the caller's buffers, so the caller
// builds the next batch while this one is in flight (two slots).
static int ingest_host(sa_engine *e, const sa_span_batch *b, bool async) {
  if (int rc = check_batch(e, b, false)) return rc;
  if (b->n == 0) return SA_OK;
  if (int rc = set_dev(e)) return rc;
  // No join: ingest_launch orders each launch itself (slab-set and record-set
  // events), so a binned record set still pending from an earlier call --
  // host or device ingest -- pairs with this call's first launch instead of
  // being aggregated alone.  A pending aggregate that failed earlier is
  // reported here as at every read.
  if (e->sticky_rc) return e->sticky_rc;
  if (!e->ev_async) SA_HIP(e, hipEventCreateWithFlags(&e->ev_async, hipEventDisableTiming));
  constexpr uint64_t kChunk = sa::kHostChunkSpans;
  constexpr size_t kSlotBytes = kChunk * 44 + 256;
  if (!e->pin[0]) {
    for (int k = 0; k < 2; ++k) {
      if (hipHostMalloc(&e->pin[k], kSlotBytes, hipHostMallocDefault) != hipSuccess ||
          hipMalloc(&e->dstage[k], kSlotBytes) != hipSuccess)
        return fail(e, SA_ENOMEM, "ingest staging allocation failed");
      SA_HIP(e, hipEventCreateWithFlags(&e->pin_ev[k], hipEventDisableTiming));
    }
  }
  const bool pinned = batch_pinned(b);
  // page-locked columns are copied asynchronously: an error return after the
  // first copy still waits for the copies in flight (the caller may reuse or
  // free its columns as soon as the call returns, whatever it returned)
  struct CopyGuard {
    hipStream_t s;
    bool armed;
    ~CopyGuard() {
      if (armed) (void)hipStreamSynchronize(s);
    }
  } guard{e->stream, pinned};
  for (uint64_t off = 0; off < b->n; off += kChunk) {
    const uint64_t m = std::min(kChunk, b->n - off);
    const uint64_t ms = (m + 1) & ~1ULL;  // column stride: u64 columns stay 16-byte aligned
    const int k = e->pin_cur;
    e->pin_cur ^= 1;
    // the packing path rewrites the pinned slot: its last reader (the copy of
    // two chunks back) must be done.  The other paths only reuse the device
    // slot, which stream order protects.
    if (e->pin_used[k] && !pinned && m < sa::kHostPageableMin) SA_HIP(e, hipEventSynchronize(e->pin_ev[k]));
    char *h = static_cast<char *>(e->pin[k]);
    const uint64_t *src[5] = {b->key_hash + off, b->start_ns + off, b->end_ns + off, b->trace_w0 + off,
                              b->trace_w1 + off};
    char *d = static_cast<char *>(e->dstage[k]);
    if (pinned) {
      // page-locked columns (sa_host_alloc): DMA straight from them, no
      // packing; the copies are waited for after the last chunk
      for (int c = 0; c < 5; ++c)
        SA_HIP(e, hipMemcpyAsync(d + c * ms * 8, src[c], m * 8, hipMemcpyHostToDevice, e->stream));
      SA_HIP(e, hipMemcpyAsync(d + 5 * ms * 8, b->meta + off, m * 4, hipMemcpyHostToDevice, e->stream));
      SA_HIP(e, hipEventRecord(e->ev_b, e->stream));
    } else if (m >= sa::kHostPageableMin) {
      // large chunks: the runtime's own staging of pageable memory copies
      // faster than one host thread packing the pinned slot.  HIP does not
      // promise that an asynchronous copy from pageable memory has taken the
      // caller's bytes when it returns, so wait for these copies (not for the
      // aggregation) before the caller may reuse or free its columns.
      for (int c = 0; c < 5; ++c)
        SA_HIP(e, hipMemcpyAsync(d + c * ms * 8, src[c], m * 8, hipMemcpyHostToDevice, e->stream));
      SA_HIP(e, hipMemcpyAsync(d + 5 * ms * 8, b->meta + off, m * 4, hipMemcpyHostToDevice, e->stream));
      SA_HIP(e, hipEventRecord(e->ev_b, e->stream));
      SA_HIP(e, hipEventSynchronize(e->ev_b));
    } else {
      for (int c = 0; c < 5; ++c) std::memcpy(h + c * ms * 8, src[c], m * 8);
      std::memcpy(h + 5 * ms * 8, b->meta + off, m * 4);
      SA_HIP(e, hipMemcpyAsync(d, h, 5 * ms * 8 + m * 4, hipMemcpyHostToDevice, e->stream));
    }
    const uint64_t *dc = reinterpret_cast<const uint64_t *>(d);
    sa_span_batch sub{dc, dc + ms, dc + 2 * ms, dc + 3 * ms, dc + 4 * ms,
                      reinterpret_cast<const uint32_t *>(d + 5 * ms * 8), m};
    if (int rc = ingest_on(e, &sub, e->stream)) return rc;
    SA_HIP(e, hipEventRecord(e->pin_ev[k], e->stream));
    e->pin_used[k] = true;
  }
  // page-locked columns: every chunk's copies are done (stream order) once
  // the last chunk's are, before the caller may reuse the arrays -- or, for
  // sa_ingest_async, the previous async call's copies (earlier on the stream)
  if (pinned && async) {
    if (e->async_pending) SA_HIP(e, hipEventSynchronize(e->ev_async));
    SA_HIP(e, hipEventRecord(e->ev_async, e->stream));
    e->async_pending = true;
  } else if (pinned) {
    SA_HIP(e, hipEventSynchronize(e->ev_b));
  }
  guard.armed = false;
  return SA_OK;
}

int sa_ingest(sa_engine *e, const sa_span_batch *b) { return ingest_host(e, b, false); }
int sa_ingest_async(sa_engine *e, const sa_span_batch *b) { return ingest_host(e, b, true); }

int sa_join(sa_engine *e, void *stream) {
  if (!e) return SA_EINVAL;
  if (int rc = set_dev(e)) return rc;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
  if (int rc = bt_aggregate_pending(e)) return rc;
  if (e->sticky_rc) return e->sticky_rc;
  for (uint32_t i = 0; i < e->nsets; ++i)
    if (e->set_stream[i] && e->set_stream[i] != s) SA_HIP(e, hipStreamWaitEvent(s, e->ev_set[i], 0));
  for (int k = 0; k < sa_engine::kBtSets; ++k)
    if (e->agg_used[k]) SA_HIP(e, hipStreamWaitEvent(s, e->ev_agg[k], 0));
  return SA_OK;
}

int sa_sync(sa_engine *e) {
  if (!e) return SA_EINVAL;
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  SA_HIP(e, hipStreamSynchronize(e->stream));
  return SA_OK;
}

static int ensure_out(sa_engine *e) {
  if (e->out_keys) return SA_OK;
  const uint32_t stride = e->nbk + 1;
  if (hipMalloc((void **)&e->out_keys, e->cap * 8) != hipSuccess ||
      hipMalloc((void **)&e->out_rows, e->cap * stride * 8) != hipSuccess)
    return fail(e, SA_ENOMEM, "flush buffers hipMalloc failed");
  return SA_OK;
}

static int read_stats(sa_engine *e, uint64_t out[sa::kNumStats]) {
  SA_HIP(e, hipMemcpyAsync(out, e->stats, sa::kNumStats * 8, hipMemcpyDeviceToHost, e->stream));
  SA_HIP(e, hipStreamSynchronize(e->stream));
  return SA_OK;
}

static int fold_window(sa_engine *e, uint64_t ws, hipStream_t s);

// Empties the key table.  Keys are a cache of the series seen: after a flush
// every row is zero, so a forgotten key costs nothing and is re-inserted by its
// next span (the delta histograms do not depend on the slot).  Window error
// counts are kept per slot, so every resident window's are folded into its
// count-min first.
static int reclaim_now(sa_engine *e) {
  for (uint32_t ws = 0; ws < e->cfg.n_windows; ++ws)
    if (int rc = fold_window(e, ws, e->stream)) return rc;
  SA_HIP(e, hipMemsetAsync(e->gkeys, 0, e->cap * 8, e->stream));
  ++e->reclaims;
  return SA_OK;
}

// Flush-time policy: reclaim once more than half the table is resident, so a
// collector whose series churn (new pods, restarts) keeps room for the next
// interval's series instead of dropping their spans.  Binned tables reclaim
// past 35 %: their bins are as small as 256 slots, and a fully churned next
// interval doubles the load, which must stay near 70 % for no bin to fill
// (at 76 % of a 2^19-slot table, 2,048 bins of 256, P(some bin full) = 2.8 %).
static int reclaim_if_full(sa_engine *e) {
  SA_HIP(e, hipMemsetAsync(e->scratch, 0, 8, e->stream));
  SA_HIP(e, sa::launch_count_keys(e->gkeys, e->cap, e->scratch, e->stream));
  uint64_t nk = 0;
  SA_HIP(e, hipMemcpyAsync(&nk, e->scratch, 8, hipMemcpyDeviceToHost, e->stream));
  SA_HIP(e, hipStreamSynchronize(e->stream));
  return sa_grp::over_reclaim_threshold(e, nk) ? reclaim_now(e) : SA_OK;
}

}  // extern "C"

namespace sa_grp {
bool over_reclaim_threshold(const sa_engine *e, uint64_t nk) {
  return e->bt ? 20 * nk > 7 * (uint64_t)e->cap : 2 * nk > e->cap;
}

int export_keys_async(sa_engine *e, uint64_t *d_keys, uint64_t cap, uint64_t *h_n, uint64_t *h_dropped,
                      hipStream_t s) {
  if (!e || !h_n || !h_dropped || (cap && !d_keys)) return SA_EINVAL;
  if (e->expo) return fail(e, SA_ESTATE, "merge hooks cover explicit-bucket engines only");
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  SA_HIP(e, hipEventRecord(e->ev_a, e->stream));
  SA_HIP(e, hipStreamWaitEvent(s, e->ev_a, 0));
  if (int rc = reduce_slabs(e, s)) return rc;
  SA_HIP(e, hipMemsetAsync(e->scratch, 0, 8, s));
  SA_HIP(e, sa::launch_compact(e->gkeys, e->gcounts, e->cap, geom(e), reinterpret_cast<unsigned long long *>(d_keys),
                               nullptr, e->scratch, cap, 0, s));
  SA_HIP(e, hipMemcpyAsync(h_n, e->scratch, 8, hipMemcpyDeviceToHost, s));
  SA_HIP(e, hipMemcpyAsync(h_dropped, e->stats + sa::kStatDropped, 8, hipMemcpyDeviceToHost, s));
  // later engine work (the gather's counter reset) orders after these reads
  SA_HIP(e, hipEventRecord(e->ev_b, s));
  SA_HIP(e, hipStreamWaitEvent(e->stream, e->ev_b, 0));
  return SA_OK;
}

int count_keys_async(sa_engine *e, uint64_t *h_n) {
  if (!e || !h_n) return SA_EINVAL;
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  SA_HIP(e, hipMemsetAsync(e->scratch + 1, 0, 8, e->stream));
  SA_HIP(e, sa::launch_count_keys(e->gkeys, e->cap, e->scratch + 1, e->stream));
  SA_HIP(e, hipMemcpyAsync(h_n, e->scratch + 1, 8, hipMemcpyDeviceToHost, e->stream));
  return SA_OK;
}

int reclaim_async(sa_engine *e) {
  if (!e) return SA_EINVAL;
  if (e->unflushed) return fail(e, SA_ESTATE, "reclaim: spans ingested since the last flush");
  if (int rc = set_dev(e)) return rc;
  return reclaim_now(e);
}

uint64_t table_capacity(const sa_engine *e) { return e ? e->cap : 0; }

int sync_stream(sa_engine *e) {
  if (!e) return SA_EINVAL;
  if (int rc = set_dev(e)) return rc;
  SA_HIP(e, hipStreamSynchronize(e->stream));
  return SA_OK;
}
}  // namespace sa_grp

extern "C" {

int sa_reclaim_keys(sa_engine *e, int force) {
  if (!e) return SA_EINVAL;
  if (e->unflushed) return fail(e, SA_ESTATE, "sa_reclaim_keys: spans ingested since the last flush");
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  if (int rc = force ? reclaim_now(e) : reclaim_if_full(e)) return rc;
  SA_HIP(e, hipStreamSynchronize(e->stream));
  return SA_OK;
}

int sa_flush(sa_engine *e, sa_red_result **out) {
  if (!e || !out) return SA_EINVAL;
  *out = nullptr;
  if (e->expo) return fail(e, SA_ESTATE, "exponential-histogram engine: use sa_flush_exp");
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  if (int rc = ensure_out(e)) return rc;
  if (int rc = reduce_slabs(e, e->stream)) return rc;
  const uint32_t stride = e->nbk + 1;
  SA_HIP(e, hipMemsetAsync(e->scratch, 0, 8, e->stream));
  SA_HIP(e, sa::launch_compact(e->gkeys, e->gcounts, e->cap, geom(e), e->out_keys, e->out_rows,
                               e->scratch, e->cap, 1, e->stream));
  uint64_t n = 0;
  SA_HIP(e, hipMemcpyAsync(&n, e->scratch, 8, hipMemcpyDeviceToHost, e->stream));
  SA_HIP(e, hipStreamSynchronize(e->stream));
  std::vector<uint64_t> k(n), rows(n * stride);
  if (n) {
    SA_HIP(e, hipMemcpyAsync(k.data(), e->out_keys, n * 8, hipMemcpyDeviceToHost, e->stream));
    SA_HIP(e, hipMemcpyAsync(rows.data(), e->out_rows, n * stride * 8, hipMemcpyDeviceToHost, e->stream));
    SA_HIP(e, hipStreamSynchronize(e->stream));
  }
  std::vector<uint64_t> ord(n);
  std::iota(ord.begin(), ord.end(), 0);
  std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) { return k[a] < k[b]; });
  auto *h = new red_holder();
  h->keys.resize(n);
  h->counts.resize(n * e->nbk);
  h->calls.resize(n);
  h->sum_ns.resize(n);
  h->sum.resize(n);
  const double div = e->cfg.unit == SA_UNIT_S ? 1e9 : 1e6;
  for (uint64_t r = 0; r < n; ++r) {
    const uint64_t i = ord[r];
    h->keys[r] = k[i];
    uint64_t c = 0;
    for (uint32_t b = 0; b < e->nbk; ++b) {
      h->counts[r * e->nbk + b] = rows[i * stride + b];
      c += rows[i * stride + b];
    }
    h->calls[r] = c;
    h->sum_ns[r] = rows[i * stride + e->nbk];
    h->sum[r] = (double)h->sum_ns[r] / div;
  }
  h->r.n_series = n;
  h->r.n_buckets = e->nbk;
  h->r.key_hash = h->keys.data();
  h->r.bucket_counts = h->counts.data();
  h->r.calls = h->calls.data();
  h->r.sum_ns = h->sum_ns.data();
  h->r.sum = h->sum.data();
  *out = &h->r;
  e->unflushed = false;
  if (int rc = reclaim_if_full(e)) return rc;
  uint64_t st[sa::kNumStats];
  if (int rc = read_stats(e, st)) return rc;
  if (st[sa::kStatDropped] != e->dropped_seen) {
    e->dropped_seen = st[sa::kStatDropped];
    return fail(e, SA_EFULL, "key table full: spans were dropped since the previous flush");
  }
  return SA_OK;
}

void sa_red_result_free(sa_red_result *r) { delete reinterpret_cast<red_holder *>(r); }

int sa_flush_exp(sa_engine *e, sa_exp_result **out) {
  if (!e || !out) return SA_EINVAL;
  *out = nullptr;
  if (!e->expo) return fail(e, SA_ESTATE, "explicit-bucket engine: use sa_flush");
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  const uint32_t M = e->cfg.exp_max_size;
  if (!e->expo_out_keys &&
      (hipMalloc((void **)&e->expo_out_keys, e->cap * 8) != hipSuccess ||
       hipMalloc((void **)&e->expo_out_rows, e->cap * sizeof(sa::ExpoRow)) != hipSuccess ||
       hipMalloc((void **)&e->expo_out_buckets, e->cap * (size_t)M * 4) != hipSuccess))
    return fail(e, SA_ENOMEM, "expo flush buffers hipMalloc failed");
  SA_HIP(e, hipMemsetAsync(e->scratch, 0, 8, e->stream));
  SA_HIP(e, sa::launch_expo_compact(expo_params(e, nullptr), e->expo_out_keys, e->expo_out_rows,
                                    e->expo_out_buckets, e->scratch, e->stream));
  uint64_t n = 0;
  SA_HIP(e, hipMemcpyAsync(&n, e->scratch, 8, hipMemcpyDeviceToHost, e->stream));
  SA_HIP(e, hipStreamSynchronize(e->stream));
  std::vector<uint64_t> k(n);
  std::vector<sa::ExpoRow> rows(n);
  std::vector<uint32_t> bk(n * M);
  if (n) {
    SA_HIP(e, hipMemcpyAsync(k.data(), e->expo_out_keys, n * 8, hipMemcpyDeviceToHost, e->stream));
    SA_HIP(e, hipMemcpyAsync(rows.data(), e->expo_out_rows, n * sizeof(sa::ExpoRow), hipMemcpyDeviceToHost, e->stream));
    SA_HIP(e, hipMemcpyAsync(bk.data(), e->expo_out_buckets, n * (size_t)M * 4, hipMemcpyDeviceToHost, e->stream));
    SA_HIP(e, hipStreamSynchronize(e->stream));
  }
  std::vector<uint64_t> ord(n);
  std::iota(ord.begin(), ord.end(), 0);
  std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) { return k[a] < k[b]; });
  auto *h = new exp_holder();
  h->keys.resize(n);
  h->count.resize(n);
  h->zero.resize(n);
  h->sum_ns.resize(n);
  h->sum.resize(n);
  h->min.resize(n);
  h->max.resize(n);
  h->scale.resize(n);
  h->offset.resize(n);
  h->nb.resize(n);
  h->buckets.assign(n * M, 0);
  const double div = e->cfg.unit == SA_UNIT_S ? 1e9 : 1e6;
  for (uint64_t r = 0; r < n; ++r) {
    const uint64_t i = ord[r];
    const sa::ExpoRow &x = rows[i];
    h->keys[r] = k[i];
    h->count[r] = x.count;
    h->zero[r] = x.zero;
    h->sum_ns[r] = x.sum_ns;
    h->sum[r] = (double)x.sum_ns / div;
    h->min[r] = (double)x.min_ns / div;
    h->max[r] = (double)x.max_ns / div;
    h->scale[r] = x.scale;
    h->offset[r] = x.offset;
    h->nb[r] = x.n;
    for (uint32_t j = 0; j < x.n && j < M; ++j) h->buckets[r * M + j] = bk[i * M + j];
  }
  h->r.n_series = n;
  h->r.max_size = M;
  h->r.unit = e->cfg.unit;
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
  e->unflushed = false;
  if (int rc = reclaim_if_full(e)) return rc;
  uint64_t st[sa::kNumStats];
  if (int rc = read_stats(e, st)) return rc;
  if (st[sa::kStatDropped] != e->dropped_seen) {
    e->dropped_seen = st[sa::kStatDropped];
    return fail(e, SA_EFULL, "key table full: spans were dropped since the previous flush");
  }
  return SA_OK;
}

void sa_exp_result_free(sa_exp_result *r) { delete reinterpret_cast<exp_holder *>(r); }

int sa_expo_probe(sa_engine *e, const double *v, const int32_t *scale, uint64_t n, int32_t *out, double *logs) {
  if (!e || (n && (!v || !scale || !out || !logs)) || n > (1ULL << 20)) return SA_EINVAL;
  if (n == 0) return SA_OK;
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  void *buf = nullptr;
  if (hipMalloc(&buf, n * 24) != hipSuccess) return fail(e, SA_ENOMEM, "probe buffer");
  double *dv = static_cast<double *>(buf), *dl = dv + n;
  int32_t *ds = reinterpret_cast<int32_t *>(dl + n), *di = ds + n;
  hipError_t st = hipMemcpyAsync(dv, v, n * 8, hipMemcpyHostToDevice, e->stream);
  if (st == hipSuccess) st = hipMemcpyAsync(ds, scale, n * 4, hipMemcpyHostToDevice, e->stream);
  if (st == hipSuccess) st = sa::launch_expo_probe(dv, ds, di, dl, n, e->stream);
  if (st == hipSuccess) st = hipMemcpyAsync(out, di, n * 4, hipMemcpyDeviceToHost, e->stream);
  if (st == hipSuccess) st = hipMemcpyAsync(logs, dl, n * 8, hipMemcpyDeviceToHost, e->stream);
  if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
  (void)hipFree(buf);
  return st == hipSuccess ? SA_OK : fail(e, SA_EDEVICE, std::string("expo probe: ") + hipGetErrorString(st));
}

int sa_key_union_probe(sa_engine *e, const uint64_t *in, uint64_t n, uint64_t *out, uint64_t *n_out) {
  if (!e || !n_out || (n && (!in || !out)) || n > (1ULL << 28)) return SA_EINVAL;
  *n_out = 0;
  if (n == 0) return SA_OK;
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  void *buf = nullptr;
  const size_t scratch = sa::key_union_scratch_bytes(n);
  if (hipMalloc(&buf, n * 16 + scratch + 64) != hipSuccess) return fail(e, SA_ENOMEM, "probe buffer");
  auto *din = static_cast<uint64_t *>(buf), *dout = din + n;
  auto *dtot = reinterpret_cast<uint32_t *>(dout + n);
  void *dscr = reinterpret_cast<char *>(dtot) + 64;
  uint64_t *big = nullptr;
  size_t big_bytes = 0;
  uint32_t tot = 0;
  hipError_t st = hipMemcpyAsync(din, in, n * 8, hipMemcpyHostToDevice, e->stream);
  if (st == hipSuccess) st = sa::key_union(din, n, dout, dtot, dscr, &big, &big_bytes, e->stream);
  if (st == hipSuccess) st = hipMemcpyAsync(&tot, dtot, 4, hipMemcpyDeviceToHost, e->stream);
  if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
  if (st == hipSuccess && tot) st = hipMemcpy(out, dout, (size_t)tot * 8, hipMemcpyDeviceToHost);
  if (big) (void)hipFree(big);
  (void)hipFree(buf);
  if (st != hipSuccess) return fail(e, SA_EDEVICE, std::string("key union probe: ") + hipGetErrorString(st));
  *n_out = tot;
  return SA_OK;
}

int sa_expo_fast_probe(sa_engine *e, const uint64_t *d_ns, const int32_t *scale, uint64_t n, int32_t *fast,
                       int32_t *exact, double *log2_err) {
  if (!e || (n && (!d_ns || !scale || !fast || !exact)) || n > (1ULL << 20)) return SA_EINVAL;
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  constexpr uint32_t kBlocks = 2048;
  void *buf = nullptr;
  if (hipMalloc(&buf, n * 20 + kBlocks * 8) != hipSuccess) return fail(e, SA_ENOMEM, "probe buffer");
  double *bmax = static_cast<double *>(buf);
  uint64_t *dd = reinterpret_cast<uint64_t *>(bmax + kBlocks);
  int32_t *ds = reinterpret_cast<int32_t *>(dd + n), *df = ds + n, *dx = df + n;
  hipError_t st = hipSuccess;
  if (n) {
    st = hipMemcpyAsync(dd, d_ns, n * 8, hipMemcpyHostToDevice, e->stream);
    if (st == hipSuccess) st = hipMemcpyAsync(ds, scale, n * 4, hipMemcpyHostToDevice, e->stream);
    if (st == hipSuccess)
      st = sa::launch_expo_fast_probe(dd, ds, n, e->cfg.unit == SA_UNIT_S ? 1e9 : 1e6, df, dx, e->stream);
    if (st == hipSuccess) st = hipMemcpyAsync(fast, df, n * 4, hipMemcpyDeviceToHost, e->stream);
    if (st == hipSuccess) st = hipMemcpyAsync(exact, dx, n * 4, hipMemcpyDeviceToHost, e->stream);
  }
  std::vector<double> hm(kBlocks);
  if (log2_err) {
    if (st == hipSuccess) st = sa::launch_log2_err_probe(0, 1u << 23, bmax, kBlocks, e->stream);
    if (st == hipSuccess) st = hipMemcpyAsync(hm.data(), bmax, kBlocks * 8, hipMemcpyDeviceToHost, e->stream);
  }
  if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
  (void)hipFree(buf);
  if (st != hipSuccess) return fail(e, SA_EDEVICE, std::string("expo fast probe: ") + hipGetErrorString(st));
  if (log2_err) *log2_err = *std::max_element(hm.begin(), hm.end());
  return SA_OK;
}

static bool resident(const sa_engine *e, uint64_t w) {
  return w >= e->win_base && w - e->win_base < e->cfg.n_windows;
}

// Derive the count-min cells of window slot ws from its exact per-slot error
// counts (see sketch_post in spanagg_kernels.hip).
static int fold_errslab(sa_engine *e, uint64_t ws, hipStream_t s) {
  if (!e->errslab) return SA_OK;
  SA_HIP(e, sa::launch_reduce_errslab(e->errslab, e->G * e->nsets, (uint64_t)e->cfg.n_windows * e->cap, ws,
                                      e->log2cap, e->errcnt + ws * e->cap, s));
  return SA_OK;
}

static int fold_window(sa_engine *e, uint64_t ws, hipStream_t s) {
  if (int rc = fold_errslab(e, ws, s)) return rc;
  SA_HIP(e, sa::launch_fold_errcnt(e->gkeys, e->errcnt + ws * e->cap, e->cap,
                                   e->cms + ws * e->cms_slot_elems, e->cfg.cms_d, e->cfg.cms_w,
                                   64 - log2u(e->cfg.cms_w), e->d_seeds, e->kinv, s));
  return SA_OK;
}

int sa_window_read(sa_engine *e, uint64_t window_id, sa_sketch_result **out) {
  if (!e || !out) return SA_EINVAL;
  *out = nullptr;
  if (!resident(e, window_id)) return fail(e, SA_ERANGE, "window not resident");
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  const uint64_t ws = window_id & (e->cfg.n_windows - 1);
  if (int rc = fold_window(e, ws, e->stream)) return rc;
  auto *h = new sketch_holder();
  h->hll.resize(e->hll_slot_bytes);
  std::vector<uint64_t> cms64(e->cms_slot_elems);
  hipError_t a = hipMemcpyAsync(h->hll.data(), e->hll + ws * e->hll_slot_bytes, e->hll_slot_bytes,
                                hipMemcpyDeviceToHost, e->stream);
  hipError_t b = hipMemcpyAsync(cms64.data(), e->cms + ws * e->cms_slot_elems,
                                e->cms_slot_elems * 8, hipMemcpyDeviceToHost, e->stream);
  hipError_t c = hipStreamSynchronize(e->stream);
  if (a != hipSuccess || b != hipSuccess || c != hipSuccess) {
    delete h;
    return fail(e, SA_EDEVICE, "window read failed");
  }
  h->cms.resize(e->cms_slot_elems);
  for (size_t i = 0; i < cms64.size(); ++i)
    h->cms[i] = cms64[i] > UINT32_MAX ? UINT32_MAX : (uint32_t)cms64[i];
  h->r.window_id = window_id;
  h->r.n_services = e->cfg.n_services;
  h->r.hll_p = e->cfg.hll_p;
  h->r.hll = h->hll.data();
  h->r.cms_d = e->cfg.cms_d;
  h->r.cms_w = e->cfg.cms_w;
  h->r.cms = h->cms.data();
  *out = &h->r;
  return SA_OK;
}

void sa_sketch_result_free(sa_sketch_result *r) { delete reinterpret_cast<sketch_holder *>(r); }

int sa_window_advance(sa_engine *e, uint64_t new_base) {
  if (!e) return SA_EINVAL;
  if (new_base < e->win_base) return fail(e, SA_EINVAL, "window base cannot move backwards");
  if (new_base > UINT64_MAX / e->cfg.window_ns)
    return fail(e, SA_EINVAL, "window base beyond the u64 nanosecond range");
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  const uint64_t n = std::min<uint64_t>(new_base - e->win_base, e->cfg.n_windows);
  for (uint64_t k = 0; k < n; ++k) {
    const uint64_t ws = (e->win_base + k) & (e->cfg.n_windows - 1);
    SA_HIP(e, hipMemsetAsync(e->hll + ws * e->hll_slot_bytes, 0, e->hll_slot_bytes, e->stream));
    if (e->hll_lb) {  // the window's bounds go back to 0 with its registers
      const size_t per = e->hll_slot_bytes >> e->lb_shift;
      SA_HIP(e, hipMemsetAsync(e->hll_lb + ws * per, 0, per, e->stream));
    }
    SA_HIP(e, hipMemsetAsync(e->cms + ws * e->cms_slot_elems, 0, e->cms_slot_elems * 8, e->stream));
    if (int rc = fold_errslab(e, ws, e->stream)) return rc;  // clears the slab cells
    SA_HIP(e, hipMemsetAsync(e->errcnt + ws * e->cap, 0, e->cap * 8, e->stream));
  }
  e->win_base = new_base;
  return SA_OK;
}

int sa_debug_stamps(sa_engine *e, uint64_t *out, uint64_t cap, uint64_t *n_out) {
  if (!e || !n_out) return SA_EINVAL;
  *n_out = e->dbg ? (uint64_t)e->G * sa::kDbgPerWg : 0;
  if (!e->dbg || !out) return SA_OK;
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  SA_HIP(e, hipStreamSynchronize(e->stream));
  SA_HIP(e, hipMemcpy(out, e->dbg, std::min<uint64_t>(cap, *n_out) * 8, hipMemcpyDeviceToHost));
  return SA_OK;
}

int sa_get_stats(sa_engine *e, sa_stats *o) {
  if (!e || !o) return SA_EINVAL;
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  uint64_t st[sa::kNumStats];
  SA_HIP(e, hipMemsetAsync(e->scratch, 0, 8, e->stream));
  SA_HIP(e, sa::launch_count_keys(e->gkeys, e->cap, e->scratch, e->stream));
  uint64_t nk = 0;
  SA_HIP(e, hipMemcpyAsync(&nk, e->scratch, 8, hipMemcpyDeviceToHost, e->stream));
  if (int rc = read_stats(e, st)) return rc;
  std::memset(o, 0, sizeof *o);
  o->spans = e->spans;
  o->zero_key = st[sa::kStatZeroKey];
  o->invalid_service = st[sa::kStatInvalidService];
  o->window_out_of_range = st[sa::kStatWindowOOR];
  o->dropped_table_full = st[sa::kStatDropped];
  o->n_keys = nk;
  o->table_capacity = e->cap;
  o->window_base = e->win_base;
  o->small_table = (e->small || e->expo_small) ? 1 : 0;
  {
    std::vector<uint64_t> f(sa::kFiltSlots);
    SA_HIP(e, hipMemcpyAsync(f.data(), e->hll_filt, sa::kFiltSlots * 8, hipMemcpyDeviceToHost, e->stream));
    SA_HIP(e, hipStreamSynchronize(e->stream));
    o->hll_filtered = std::accumulate(f.begin(), f.end(), (uint64_t)0);
  }
  return SA_OK;
}

int sa_export_keys(sa_engine *e, uint64_t *d_keys, uint64_t cap, uint64_t *n_out, void *stream) {
  if (!e || !n_out || (cap && !d_keys)) return SA_EINVAL;
  if (e->expo) return fail(e, SA_ESTATE, "merge hooks cover explicit-bucket engines only");
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
  if (s != e->stream) {
    SA_HIP(e, hipEventRecord(e->ev_a, e->stream));
    SA_HIP(e, hipStreamWaitEvent(s, e->ev_a, 0));
  }
  if (int rc = reduce_slabs(e, s)) return rc;
  SA_HIP(e, hipMemsetAsync(e->scratch, 0, 8, s));
  SA_HIP(e, sa::launch_compact(e->gkeys, e->gcounts, e->cap, geom(e),
                               reinterpret_cast<unsigned long long *>(d_keys), nullptr, e->scratch,
                               cap, 0, s));
  SA_HIP(e, hipMemcpyAsync(n_out, e->scratch, 8, hipMemcpyDeviceToHost, s));
  SA_HIP(e, hipStreamSynchronize(s));
  return SA_OK;
}

int sa_gather_dense(sa_engine *e, const uint64_t *d_keys, uint64_t n, uint64_t *d_rows, int reset,
                    void *stream) {
  if (!e || (n && (!d_keys || !d_rows))) return SA_EINVAL;
  if (e->expo) return fail(e, SA_ESTATE, "merge hooks cover explicit-bucket engines only");
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
  if (s != e->stream) {
    SA_HIP(e, hipEventRecord(e->ev_a, e->stream));
    SA_HIP(e, hipStreamWaitEvent(s, e->ev_a, 0));
  }
  if (int rc = reduce_slabs(e, s)) return rc;
  SA_HIP(e, sa::launch_gather_dense(e->gkeys, e->gcounts, geom(e), d_keys, n, d_rows, s));
  if (reset) {
    e->unflushed = false;
    SA_HIP(e, hipMemsetAsync(e->gcounts, 0, counts_bytes(e), s));
    if (e->base64) SA_HIP(e, hipMemsetAsync(e->base64, 0, (size_t)e->cap * (e->nbk + 1) * 8, s));
  }
  if (s != e->stream) {
    SA_HIP(e, hipEventRecord(e->ev_b, s));
    SA_HIP(e, hipStreamWaitEvent(e->stream, e->ev_b, 0));
  }
  return SA_OK;
}

int sa_window_export(sa_engine *e, uint64_t window_id, uint8_t *d_hll, uint64_t *d_cms,
                     void *stream) {
  if (!e) return SA_EINVAL;
  if (!resident(e, window_id)) return fail(e, SA_ERANGE, "window not resident");
  if (int rc = set_dev(e)) return rc;
  if (int rc = join_checked(e)) return rc;
  hipStream_t s = stream ? static_cast<hipStream_t>(stream) : e->stream;
  if (s != e->stream) {
    SA_HIP(e, hipEventRecord(e->ev_a, e->stream));
    SA_HIP(e, hipStreamWaitEvent(s, e->ev_a, 0));
  }
  const uint64_t ws = window_id & (e->cfg.n_windows - 1);
  if (int rc = fold_window(e, ws, s)) return rc;
  if (d_hll)
    SA_HIP(e, hipMemcpyAsync(d_hll, e->hll + ws * e->hll_slot_bytes, e->hll_slot_bytes,
                             hipMemcpyDeviceToDevice, s));
  if (d_cms)
    SA_HIP(e, hipMemcpyAsync(d_cms, e->cms + ws * e->cms_slot_elems, e->cms_slot_elems * 8,
                             hipMemcpyDeviceToDevice, s));
  if (s != e->stream) {
    SA_HIP(e, hipEventRecord(e->ev_b, s));
    SA_HIP(e, hipStreamWaitEvent(e->stream, e->ev_b, 0));
  }
  return SA_OK;
}

}  // extern "C"
