// sa_internal.h -- shared definitions between the HIP kernels and the C-ABI
// engine of libspanagg (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

namespace sa {

constexpr int kMaxBounds = 62;          // SA_MAX_BOUNDS
constexpr uint32_t kNotFound = 0xFFFFFFFFu;
constexpr uint64_t kPhi = 0x9E3779B97F4A7C15ULL;  // Fibonacci hashing multiplier

// stats slots (device array of u64)
enum : int {
  kStatZeroKey = 0,
  kStatInvalidService = 1,
  kStatWindowOOR = 2,
  kStatDropped = 3,
  kNumStats = 4
};
// HLL updates skipped by the lower-bound filter (sa_stats.hll_filtered): one
// u64 slot per workgroup index (mod kFiltSlots), summed when stats are read
constexpr uint32_t kFiltSlots = 1024;

// Bucket lookup table: bin k = floor(log2 d) (k = 64 for d = 0).  For d in
// bin k, bucket = base + [d > ta] + [d > tb] (ta/tb = UINT64_MAX when absent);
// valid when no bin holds more than two thresholds.
struct BinEntry {
  unsigned long long ta, tb;
  uint32_t base, pad[3];
};
constexpr int kBins = 65;

struct XHdr;
struct ExpoHdr;
// Everything the ingest kernels need, passed by value (kernel-argument segment,
// read through the scalar cache).
struct IngestParams {
  // SoA v1 batch (device pointers, 16-B aligned)
  const uint64_t *key, *start, *end, *w0, *w1;
  const uint32_t *meta;
  uint64_t n;
  uint64_t wg_chunk;  // spans per workgroup (multiple of 4; host-computed, = kernel wg_range)
  // key table (open addressing, linear probing, EMPTY = 0)
  unsigned long long *gkeys;
  uint32_t log2cap;
  uint32_t max_probe;
  // small-table path: per-workgroup slabs [G][cap][nbk] u32 and [G][cap] u64
  uint32_t *slab_cnt;
  unsigned long long *slab_sum;
  // HBM-table path: counters [cap][nbk+1] u64 (last = sum_ns); binned path:
  // 32-B rows (kRowBytes) plus the u64 spill array base64 [cap][nbk + 1]
  unsigned long long *gcounts;
  unsigned long long *base64;
  // histogram: bucket(d) = nneg + #{i < npos : d > thr[i]}
  uint64_t thr[kMaxBounds];
  uint32_t npos, nneg, nbk;
  uint32_t epoch_tiles;  // small path: LDS u16 counters flushed every epoch_tiles tiles
  // sketches
  uint8_t *hll;                 // [W][S][2^p]
  unsigned long long *cms;      // [W][d][w]
  unsigned long long *errcnt;   // [W][cap] exact ERROR-span counts per (window, key slot)
  // v2 kernels: per-workgroup ERROR counts [G][W << log2cap] u32, gathered in an
  // LDS table during the launch and added here at its end (nullptr: errcnt atomics)
  uint32_t *errslab;
  uint64_t window_ns, win_magic, win_base;
  uint64_t base_ns, ring_ns;  // win_base * window_ns, n_windows * window_ns (< 2^63)
  float inv_window;           // 1 / window_ns
  // 0.5 - n_windows * 2^-20: a quotient estimate inside the ring whose
  // fraction lies within this of 1/2 has the exact floor (window_slot_lean)
  float win_ok;
  uint32_t base_slot;         // win_base & win_mask
  const BinEntry *bintab;     // [kBins] or nullptr (linear thresholds)
  uint32_t win_mask, n_windows;
  uint32_t p, n_services, cms_d, cms_shift, cms_w;
  uint32_t diag;  // SA_DIAG_* ablation bits (0 in production)
  const uint64_t *seeds;  // [8] count-min row seeds (device memory)
  unsigned long long *stats;
  unsigned long long *dbg;  // diagnostic timestamps [G][8] (nullptr in production)
  // partitioned HBM-table path: span records binned by key ([kPartBins][part_cap]
  // of {key, ns << 7 | bucket}) and the per-bin fill counters
  ulonglong2 *part_rec;
  uint32_t *part_fill;
  uint32_t part_cap;
  // binned-table path (spanagg_binned.hip): key table split into kPartBins
  // bin-local sub-tables of 2^log2sb slots, keys stored as m = key * kmul,
  // u32 count rows; records in per-(bin, scatter workgroup) regions of
  // bt_region records, region fills in bt_cnt [bin][scatter workgroup]
  uint32_t log2sb;
  uint32_t bt_region;
  uint64_t kmul, kinv;
  ulonglong2 *bt_rec;
  uint32_t *bt_cnt;
  uint32_t bt_grid;  // scatter workgroups (regions per bin)
  // the aggregate's second record set (nullptr: one): the next launch's
  // scatter output, aggregated with this one (sa_engine::bt_pend)
  ulonglong2 *bt_rec2;
  uint32_t *bt_cnt2;
  uint32_t bt_grid2, bt_region2;
  // HLL lower bounds: hll_lb[j] <= every register of sub-block j (registers
  // [j << lb_shift, (j + 1) << lb_shift)), so a span whose rho is at most its
  // sub-block's bound cannot raise a register and skips the register read.
  // lb_n sub-blocks (0: no filter); lb_seq rotates which sub-blocks a launch
  // refreshes (registers only grow between window clears, which zero the
  // window's bounds, so a bound read at any time stays a lower bound).
  uint8_t *hll_lb;
  uint32_t lb_shift, lb_n, lb_seq;
  unsigned long long *hll_filt;  // [kFiltSlots] (sa_stats.hll_filtered)
  // exponential-histogram engines on the small-table kernel (EXPO): the key
  // slot of every span (for the bucket-counting pass) and the per-workgroup
  // header slabs [G][cap] (XHdr) the rescale pass reduces
  uint32_t *slot_of;  // EXPO mode: [n] key slot of each span (kNotFound without one)
  // EXPO mode with slab counting: [n] span records instead (span_rec_of), so
  // the counting pass reads 8 B per span instead of the slot and both times
  unsigned long long *span_rec;
  unsigned long long *span_long;  // [n]: the duration of each span whose record holds kSpanRecDurMask
  // EXPO mode, index records (xidx != 0): slot_of holds ixrec words -- each
  // span's bucket index at the scale its series had when the kernel started
  // (xscale[], read in the prologue) -- and span_long the durations the
  // fast index path declined
  const int8_t *xscale;  // [cap] each slot's scale (expo_reduce_rescale_kernel keeps it)
  int32_t l2d_q24;  // log2(div) * 2^24 rounded (expo_index_fast)
  uint32_t xidx;
  XHdr *xslab;
  // Small-table kernels with the tail pool (POOL): every workgroup owns the
  // static range [b * wg_chunk, (b + 1) * wg_chunk); spans [pool_base, n)
  // form pool_n blocks of kPoolSpans that workgroups take from *pool_ctr
  // (x 64: one wave's claim) once their own range is claimed, so fast
  // workgroups (and XCDs) finish the slow ones' share of the launch.
  // pool_next: the counter of the launch nsets ahead (same slab set, so it
  // starts after this one ends), zeroed here.
  uint64_t pool_base;
  uint32_t pool_n;
  uint32_t *pool_ctr, *pool_next;
};
// the tail pool (IngestParams::pool_*): blocks of 8 claim chunks (2 x 128
// spans each), at most kPoolMaxSteal of them per workgroup (its u16 LDS
// counters bound the spans of one launch)
constexpr uint32_t kPoolSpans = 2048;
constexpr uint32_t kPoolMaxSteal = 8;
constexpr uint32_t kPoolRing = 8;  // per-launch pool counters per engine
// One workgroup's exponential-histogram header partial for one key slot
// (EXPO kernel -> expo_reduce_rescale_kernel): counts, exact ns sum, the
// largest ~d over positive durations (so the minimum starts from a zeroed
// slab) and the largest positive duration.
struct XHdr {
  uint32_t cnt, zero;
  unsigned long long sum, minx, max;
};

// Exponential-histogram mode (spanagg_expo.hip): per key slot a header and
// max_size u32 buckets kept circularly (index mod max_size), two buffers so a
// downscale can merge from one into the other.
struct ExpoHdr {
  unsigned long long count, zero, sum_ns, min_ns, max_ns, minpos_ns, maxpos_ns;
  int32_t scale, lo, hi;  // the kept buckets' scale and positive index range (lo = INT32_MAX: none)
  uint32_t cur;           // which bucket buffer holds them
};
struct ExpoRow {  // one flushed series
  unsigned long long count, zero, sum_ns, min_ns, max_ns;
  int32_t scale, offset;
  uint32_t n, pad;
};
struct ExpoParams {
  const uint64_t *key, *start, *end;
  uint64_t n;
  unsigned long long *gkeys;
  uint32_t log2cap, max_probe;
  uint64_t cap;
  ExpoHdr *hdr;
  uint32_t *buckets;  // [2][cap][max_size]
  uint32_t max_size;
  double div;         // 1e6 (ms) or 1e9 (s)
  int32_t log2div_q24;  // log2(div) * 2^24 rounded, for the bucket index's fast path
  uint32_t diag;      // ablation bits (SPANAGG_XC_DIAG, profiling only; results wrong when set):
                      // 1 no HBM bucket atomics, 2 no LDS cache, 4 exact index path only, 8 no index
  uint32_t *slot_of;  // [n] key slot of each span (pass 1 / the small-table ingest kernel -> counting)
  const unsigned long long *span_rec;  // [n] span records (slab counting: the small-table kernel -> counting)
  const unsigned long long *span_long;  // [n] durations of the records holding kSpanRecDurMask
  uint32_t xidx;  // slot_of holds index records (ixrec), the counting pass shifts them to the new scale
  int8_t *xscale;  // [cap] each slot's scale as the reduce pass left it, for the ingest kernel (nullptr: none)
  unsigned long long *dropped;
  XHdr *xslab;        // small-table engines: [xG][cap] per-workgroup header partials (nullptr: pass 1 atomics)
  uint32_t xG;
  // small-table bucket counting (expo_count_slab with its entry selection / expo_fold_slab):
  uint32_t *lcount;         // [cap] this launch's positive durations per slot (reduce -> selection)
  int2 *xmeta;              // [cap] {scale | buffer << 8, lo - (lo mod max_size)} per slot (reduce -> counting)
  uint32_t *slot_of_entry;  // [xc_ne] the entry's slot, ~0u: unused (this launch's selection)
  int32_t *xent;            // [cap] each slot's entry, -1: none (this launch's selection)
  int32_t *xent_next;       // [cap] and the next launch's, by the counting kernel's workgroup 0
  uint32_t *soe_next;       // [xc_ne] the next launch's slot_of_entry
  uint32_t *xcslab;         // [xG][xc_slab_stride] per-workgroup u16 bucket-count pairs ([xc_ne][(max_size + 1) / 2])
  uint32_t xc_ne;           // LDS entries of the counting kernel (0: the cached-probe kernel)
  // the counting kernel's tail (spans of series without an LDS entry): each
  // workgroup's (slot << 12 | bucket) records, sorted by fold bin of
  // xt_bin_slots slots, each bin's run at a fixed place [xG][nbins][kXtRun],
  // and the runs' lengths [xG][nbins + 1];
  // expo_fold_kernel sums them per bin (nullptr: HBM atomics)
  uint32_t *xt_rec, *xt_off;  // (records past kXtCap, or past a full run, take an HBM atomic)
  // SA_OPT_STAMPS: the counting kernel's per-workgroup s_memrealtime stamps,
  // in the ingest kernel's stamp rows (kDbgPerWg per workgroup; slots
  // kXcStamp.. are the counting kernel's); nullptr: none
  unsigned long long *dbg;
};
// A span record of the exponential-histogram slab path: the key slot in the
// top 12 bits (kSpanRecNoSlot: none; slab tables have <= 2,048 slots) and the
// duration in ns below; a duration of 2^52 - 1 ns (52 days) or more is stored
// as kSpanRecDurMask and in full at the span's index of span_long (so the
// counting pass reads no caller memory).
constexpr uint32_t kSpanRecShift = 52;
constexpr uint32_t kSpanRecNoSlot = 0xFFFu;
constexpr unsigned long long kSpanRecDurMask = (1ull << kSpanRecShift) - 1;
__host__ __device__ inline unsigned long long span_rec_of(uint32_t slot, unsigned long long d) {
  return (unsigned long long)(slot < kSpanRecNoSlot ? slot : kSpanRecNoSlot) << kSpanRecShift |
         (d < kSpanRecDurMask ? d : kSpanRecDurMask);
}
// An index record (the exponential slab path's span word, u32): the key slot
// in the top 12 bits (kSpanRecNoSlot: none), the scale the ingest kernel read
// for the slot + 10 (5 bits), the bucket index at that scale (14 bits,
// signed) and a flag bit.  Flag with index field 0: the duration is in
// span_long (the fast path declined, or the index needs more bits); flag with
// index field 1: zero duration.  A series' scale only falls within a flush
// interval, so the counting pass gets the index at the scale the reduce pass
// settled on by an arithmetic shift (go-expohisto: bucket i at scale s - 1
// holds buckets 2i and 2i + 1 at scale s).
constexpr uint32_t kIxSlotShift = 20, kIxScaleShift = 15, kIxScaleBias = 10;
constexpr int32_t kIxMin = -(1 << 13), kIxMax = (1 << 13) - 1;
constexpr uint32_t kIxLong = 1u, kIxZero = 3u;  // flag | index field 0 / 1
__host__ __device__ inline uint32_t ixrec_of(uint32_t slot, int32_t scale, int32_t ix) {
  return slot << kIxSlotShift | (uint32_t)(scale + (int32_t)kIxScaleBias) << kIxScaleShift | ((uint32_t)ix & 0x3FFFu) << 1;
}
// log2(div) in the fast bucket index's 8.24 fixed point (expo_index_fast)
__host__ inline int32_t expo_l2d_q24(double div) { return (int32_t)std::llround(std::log2(div) * 16777216.0); }
constexpr uint32_t kXtCap = 4096;       // tail records per counting workgroup (16 KiB of LDS)
constexpr uint32_t kXtRun = 64;         // a counting workgroup's records of one fold bin (C2: ~23 on average)
// slots per tail fold bin: 16 (a fold workgroup counts [16][max_size] u32 in
// LDS), 8 past max_size 2,048; one fold round at C2's 2,048 slots (128 bins)
constexpr uint32_t kXtBinSlotsMax = 16;
__host__ __device__ inline uint32_t xt_bin_slots(uint32_t max_size) { return max_size <= 2048 ? 16u : 8u; }
__host__ __device__ inline uint32_t xt_bins(uint64_t cap, uint32_t max_size) {
  return (uint32_t)((cap + xt_bin_slots(max_size) - 1) / xt_bin_slots(max_size));
}
// the counting slab's words per workgroup: xc_ne entries of (max_size + 1) / 2
// u16 pairs, padded to 16 B (the fold reads four words a lane)
__host__ __device__ inline uint32_t xc_slab_stride(uint32_t ne, uint32_t max_size) {
  return (ne * ((max_size + 1) / 2) + 3u) & ~3u;
}
__host__ __device__ ExpoHdr expo_hdr_empty();
constexpr uint32_t kExpoMaxSize = 4096;

// HLL bound sub-blocks: 2^kLbMinShift registers or more, at most kLbMaxSub of
// them per engine (the kernels keep the bounds in LDS)
constexpr uint64_t kHostChunkSpans = 1ull << 20;  // sa_ingest pinned slot (44 MiB)
constexpr uint64_t kHostPageableMin = 1ull << 18;  // chunks from here on: the runtime's pageable staging
constexpr uint32_t kLbMinShift = 10;
constexpr uint32_t kLbMaxSub = 2048;


// Partitioned HBM-table path (high cardinality): part_scatter_kernel bins
// every span's record by the top 11 bits of its key, part_aggregate_kernel
// aggregates one bin per workgroup in an LDS table and adds it to the HBM
// counters once per key.
#ifndef SA_PART_BIN_BITS
#define SA_PART_BIN_BITS 11
#endif
constexpr uint32_t kPartBinBits = SA_PART_BIN_BITS;
constexpr uint32_t kPartBins = 1u << kPartBinBits;
// LDS table slots per bin: ~2x the mean keys per bin at 1 M keys
constexpr uint32_t kPartSlotBits = 21 - kPartBinBits;
constexpr uint32_t kPartSlots = 1u << kPartSlotBits;
// records staged per bin in the scatter's LDS (one chunk = kPartStage x 16 B)
#ifndef SA_PART_STAGE
#define SA_PART_STAGE (SA_PART_BIN_BITS >= 11 ? 2 : 8)  // 2: LDS left for a 512-entry overflow table
#endif
constexpr uint32_t kPartStage = SA_PART_STAGE;
constexpr uint32_t kPartMaxBk = 17;       // LDS counter row: nbk <= 17 (default buckets)
constexpr uint32_t kPartBlock = 1024;     // scatter
constexpr uint32_t kPartAggBlock = kPartSlots >= 2048 ? 1024 : 512;  // aggregate workgroup
constexpr uint64_t kPartMaxSpans = 1ULL << 24;  // spans per partitioned launch
// records per bin: 1.25x the mean plus slack (a fuller bin spills to the direct path)
constexpr uint64_t kPartMaxCap = kPartMaxSpans / kPartBins * 5 / 4 + 64;  // a multiple of kPartStage
// a bin holds < 2^16 records, so its LDS bucket counters are u16 pairs
static_assert(kPartMaxCap < 65536, "u16 LDS counters");
constexpr uint32_t kPartWords = (kPartMaxBk + 1) / 2;
__host__ __device__ inline uint32_t part_bin(uint64_t key) { return (uint32_t)(key >> (64 - kPartBinBits)); }
constexpr size_t kPartLdsBytes = (size_t)kPartSlots * (16 + 4 * kPartWords);  // 52 KiB at 1,024 slots
// scatter: cur, lim, stage counts (u32 per bin) + a 4-record stage per bin
// scatter overflow table: spans whose bin run is full are pre-aggregated per
// workgroup (key, ns sum, u32 bucket counts) and leave as one row update each
#ifndef SA_PART_HOT_BITS
#define SA_PART_HOT_BITS 9
#endif
constexpr uint32_t kPartHotBits = SA_PART_HOT_BITS;
constexpr uint32_t kPartHot = 1u << kPartHotBits;
constexpr size_t kPartScatterLds =
    (size_t)kPartBins * (12 + kPartStage * 16) + (size_t)kPartHot * (16 + 4 * kPartMaxBk);  // 130 KiB

// Counter row layout (gcounts, one row per key slot): 64-B segments of 8 u64
// cells -- cell 0 holds that segment's share of the ns sum, cells 1..7 seven
// bucket counts.  A span's count cell and sum cell share a segment, so when
// one wave instruction carries both (two adjacent lanes) the memory side
// handles them as one atomic request (tools/atomic_probe.hip: 2x the rate).
// The row's ns sum is the sum of its segments' cells.
constexpr uint32_t kSegBuckets = 7;
__host__ __device__ inline uint32_t row_stride(uint32_t nbk) {
  return (nbk + kSegBuckets - 1) / kSegBuckets * 8;
}
__host__ __device__ inline uint32_t row_count_cell(uint32_t b) {
  return b / kSegBuckets * 8 + 1 + b % kSegBuckets;
}
__host__ __device__ inline uint32_t row_sum_cell(uint32_t b) { return b / kSegBuckets * 8; }

// ---------------------------------------------------------------------------
// Binned key table (high-cardinality path, spanagg_binned.hip).
// The table of cap = 2^log2cap slots is split into kPartBins bins of
// SB = 2^log2sb slots: a key lives in the bin given by the top kPartBinBits
// bits of m = key * kmul (kmul odd, so the map is a bijection and 0 stays the
// EMPTY marker).  Within the bin the sub-table is buckets of 4 slots with two
// choices, as the small table (probe_seq): positions 0-3 are bucket b1,
// then bucket b2 and the buckets after it in order (wrapping inside the bin),
// so a lookup is two 32-B bucket reads for nearly every key.  One aggregate
// workgroup per bin mirrors the whole sub-table in LDS at the same positions,
// so the bin's keys and counter rows are read and written as one contiguous
// block.
constexpr uint32_t kBinShift = 64 - kPartBinBits;          // bin = m >> kBinShift
constexpr uint64_t kBinRest = (1ULL << kBinShift) - 1;     // m's bits below the bin
struct BtSeq {
  uint32_t b1, b2, nbmask;
};
__host__ __device__ inline BtSeq bt_seq(uint64_t m, uint32_t log2sb) {
  const uint32_t h1 = ((uint32_t)m ^ (uint32_t)(m >> 29)) * 0x9E3779B1u;
  const uint32_t h2 = (h1 ^ (h1 >> 16)) * 0x85EBCA6Bu;
  const uint32_t sh = 34 - log2sb;  // top (log2sb - 2) bits
  return BtSeq{h1 >> sh, h2 >> sh, (1u << (log2sb - 2)) - 1};
}
// in-bin slot of probe position i (i < bt_probe_max: every slot is reached)
__host__ __device__ inline uint32_t bt_pos(const BtSeq &q, uint32_t i) {
  if (i < 4) return q.b1 * 4 + i;
  const uint32_t r = i - 4;
  return ((q.b2 + (r >> 2)) & q.nbmask) * 4 + (r & 3);
}
__host__ __device__ inline uint32_t bt_probe_max(uint32_t log2sb) { return (1u << log2sb) + 4; }
__host__ __device__ inline uint32_t bt_slot(uint64_t m, uint32_t log2sb, uint32_t i) {
  return ((uint32_t)(m >> kBinShift) << log2sb) | bt_pos(bt_seq(m, log2sb), i);
}
// Counter rows of the binned path: 32 B per key slot, the u64 ns sum then one
// u8 count per bucket (bytes 8 .. 8 + nbk), so two rows share a 64-B half
// line and the aggregate's row read-modify-write moves 32 B per touched key.
// A count that would pass 255 leaves the row: the aggregate adds the row's
// counts to the u64 spill array base64 [cap][nbk + 1] (atomics) and zeroes
// them; the scatter's direct path and overflow table add to base64 directly
// (its last cell is their ns sum).  A key's totals are row + base64.
constexpr uint32_t kRowBytes = 32;
constexpr uint32_t kRowMaxBk = kRowBytes - 8;
static_assert(kPartMaxBk <= kRowMaxBk, "binned rows hold every bucket count");
// Record duration word: the duration in ns (bits 0-58) and its histogram
// bucket (bits 59-63, from the scatter's bin table), so the aggregate needs no
// bucketing; a span of 2^59 ns or longer (18 years) takes the overflow path.
constexpr uint32_t kRecDurBits = 59;
constexpr uint64_t kRecDurMask = (1ULL << kRecDurBits) - 1;
constexpr uint32_t kBtStage = 4;     // records per bin stage: one 64-B chunk per flush
constexpr uint32_t kBtHq = 256;      // scatter deferred HLL raises
constexpr uint32_t kBtBlock = 1024;  // scatter workgroup
constexpr uint32_t kBtMaxWgSpans = 65520;  // u16 claim / overflow counters per scatter workgroup
// round-synchronous scatter (bt_scatter2_kernel): per bin a 4-record stage,
// a u16 claim count (pairs) and a u16 region fill; per wave a flush list of
// 128 bins; the overflow table; HLL queue; bin table; HLL bounds
constexpr uint32_t kBt2Hot = 240;
constexpr uint32_t kBt2HotErr = 128;  // (window slot, overflow entry) -> ERROR count
constexpr size_t kBt2ScatterLds = (size_t)kPartBins * (kBtStage * 16 + 2 + 2) + (kBtBlock / 64) * 128 * 2 +
                                  (size_t)kBt2Hot * (16 + 4 * kPartWords) + (size_t)kBtHq * 8 + 16 +
                                  (size_t)kBins * sizeof(BinEntry) + kLbMaxSub + kBt2HotErr * 8;
static_assert(kBt2ScatterLds <= 163840, "binned scatter2 LDS");

// Geometry of the counter rows and key table for the flush-time kernels
// (compact, gather, count-min fold): both table layouts, both row layouts.
struct RowGeom {
  uint32_t nbk;
  uint32_t row8;    // 1: 32-B u8-count rows + base64 (binned path), 0: u64 segment rows
  uint32_t binned;  // 1: binned key table
  uint32_t log2cap, log2sb, max_probe;
  uint64_t kmul, kinv;            // key <-> stored id (1, 1 unless binned)
  unsigned long long *base64;     // row8: u64 [cap][nbk + 1] spilled counts and sums
};

// Key-table layout: cap = 2^log2cap slots in buckets of 4 (log2cap in 4..31).
// A key's probe sequence is its first-choice bucket b1, then its second-choice
// bucket b2, then the buckets after b2 in order (every slot within cap + 4
// positions).  Inserts CAS into the first empty slot of the sequence and slots
// never empty again, so concurrent inserts of one key meet at the same slot.
// Two choices keep 97-99 % of a ~0.7-load table's keys in b1/b2, so the LDS
// lookup of the ingest kernel is two fixed 32-B bucket reads with no probe
// loop (ids are xxh64 outputs from the host; any bits are usable).
struct ProbeSeq {
  uint32_t b1, b2, nbmask;
};
__host__ __device__ inline ProbeSeq probe_seq(uint64_t key, uint32_t log2cap) {
  const uint32_t h1 = ((uint32_t)key ^ (uint32_t)(key >> 32)) * 0x9E3779B1u;
  // second choice from a 24-bit multiply (v_mul_u32_u24, full rate; a 32-bit
  // multiply is quarter rate): the top bits of its low word mix all 24 inputs
  const uint32_t h2 = ((h1 ^ (h1 >> 16)) & 0xFFFFFFu) * 0x85EBCAu;
  const uint32_t sh = 34 - log2cap;  // top (log2cap - 2) bits
  return ProbeSeq{h1 >> sh, h2 >> sh, (1u << (log2cap - 2)) - 1};
}
__host__ __device__ inline uint32_t seq_slot(const ProbeSeq &p, uint32_t i) {
  if (i < 4) return p.b1 * 4 + i;
  const uint32_t q = i - 4;
  return ((p.b2 + (q >> 2)) & p.nbmask) * 4 + (q & 3);
}
inline uint32_t max_probe_of(uint32_t log2cap) { return (1u << log2cap) + 4; }


// HBM-table path variants (spans per lane, prefetch; 256-thread blocks).  The
// small-table path has two: 0 = next-tile prefetch, 1 = none (1,024 threads,
// 4 spans per lane); the block field below is unused by it.
struct Variant {
  int spl;
  bool prefetch;
  uint32_t block;
};
constexpr int kNumVariants = 4;
constexpr Variant kVariants[kNumVariants] = {{4, false, 1024}, {2, true, 1024}, {4, true, 512},
                                             {2, false, 1024}};
constexpr uint32_t kHbmBlock = 256;
// small-table kernels: 0-3 ingest_lds_kernel {4,PF} {4,-} {2,PF} {2,-}, 4-7 the
// same with nt loads; 8-13 ingest_v2_kernel: 8 generic (nt tile loads), 9 three
// tiles in flight, 10 four spans per lane, 11 generic (default cache policy),
// 12 / 13 = 8 / 11 specialised for cap 2048, 17 buckets, HLL p 14; 14 = 12 with
// dynamic wave chunks; 15 = 14 generic; 16-18 = 14 with OPT 1 / 3 / 2; 19 = 16
// with the batched end-of-launch write-back (v2_epilogue); 20 = 19 LEAN; 21 =
// 20 with the TAG key lookup; 22 = 20 with the tail pool (POOL); 23 / 24 = 20
// with tile claims (OPT 3 / 2: NBUF claims of one wave tile per round); 25 =
// 15 with 512-thread workgroups; 26 = 25 with variant 20's options (OPT 1,
// EPI, LEAN): kLdsHalfBlockVariant, the product's choice for a table with a
// bin table whose LDS state fits a CU twice (two workgroups per CU).
constexpr int kNumLdsVariants = 27;
constexpr int kLdsSpl[kNumLdsVariants] = {4, 4, 2, 2, 4, 4, 2, 2, 2, 2, 4, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2};
constexpr int kLdsHalfBlockVariant = 26;
constexpr uint32_t lds_variant_block(int v) { return v == 25 || v == 26 ? 512u : 1024u; }
constexpr int kLdsPoolVariant = 22;
// v2 kernels keep u16 LDS counters for a whole launch: spans per workgroup per launch
constexpr uint32_t kMaxWgSpans = 65532;
// POOL launches: the static share per workgroup (whole 256-span chunks) leaves
// room for kPoolMaxSteal stolen blocks under kMaxWgSpans; a launch averages at
// most kPoolMaxWgSpans per workgroup, so the steal limits cover the pool
constexpr uint32_t kPoolMaxStatic = (kMaxWgSpans - kPoolMaxSteal * kPoolSpans) / 256 * 256;
constexpr uint32_t kPoolMaxWgSpans = kPoolMaxStatic + kPoolMaxSteal * kPoolSpans;
constexpr uint32_t kPoolMinStatic = 32 * 256;  // two fixed chunks per wave before any claim
constexpr uint32_t kDbgPerWg = 136;  // diagnostic stamps per workgroup: 8 + 16 waves x 8
// the exponential counting kernel's stamps in the same rows (slots the ingest
// kernel leaves free): start, prologue done, loop done, end at 4..7; its slab
// stores issued, its LDS zeroed and its entry selection done (thread 0) in
// the last slots of the wave rows
constexpr uint32_t kXcStamp = 4, kXcStampSlab = kDbgPerWg - 1, kXcStampZeroed = kDbgPerWg - 9,
                   kXcStampSelected = kDbgPerWg - 17, kXcStampTail = kDbgPerWg - 25;
constexpr uint32_t kHllQueue = 2048;  // deferred HLL raises per workgroup (8 B each)
constexpr uint32_t kErrTab = 1024;    // LDS (window, slot) -> ERROR count table per workgroup (4 B each)
// ingest_lds_kernel LDS beyond the table: HLL queue + its count + bin table
// (+ the ERROR table and HLL bounds of the v2 kernels; their TAG forms add
// cap u32 key tags, see kLdsTagBytes)
// (+ 64 B: the POOL kernels' map of stolen pool blocks)
constexpr size_t kLdsExtraBytes = kHllQueue * 8 + 32 + kBins * sizeof(BinEntry) + kErrTab * 4 + kLbMaxSub + 64;
constexpr size_t kLdsTagBytesPerSlot = 4;
constexpr int kLdsTagVariant = 21;  // the only small-table variant with LDS key tags

// launchers (spanagg_kernels.hip)
hipError_t launch_ingest_small(const IngestParams &P, uint32_t grid, size_t lds_bytes,
                               hipStream_t s, int variant);
hipError_t launch_ingest_hbm(const IngestParams &P, uint32_t grid, hipStream_t s, int variant);
hipError_t launch_ingest_part(const IngestParams &P, hipStream_t s);
hipError_t prepare_ingest_part();
hipError_t prepare_ingest_small(size_t lds_bytes);
void ingest_small_node(const IngestParams &P, uint32_t grid, size_t lds_bytes, int variant, void **args,
                       hipKernelNodeParams *np);
uint32_t ingest_small_block(bool bt, int variant, uint32_t log2cap, uint32_t nbk, uint32_t p);
uint32_t ingest_small_blocks_per_cu(bool bt, int variant, uint32_t log2cap, uint32_t nbk, uint32_t p,
                                    size_t lds_bytes);
// exponential-histogram engines with an LDS-sized key table: the small-table
// kernel in EXPO mode (header partials + per-span slots; spanagg_expo.hip
// reduces and counts)
hipError_t prepare_ingest_expo_small(size_t lds_bytes);
hipError_t launch_ingest_expo_small(const IngestParams &P, uint32_t grid, size_t lds_bytes, hipStream_t s);
uint32_t ingest_expo_blocks_per_cu(uint32_t log2cap, uint32_t p, size_t lds_bytes);
hipError_t launch_reduce_slabs(uint32_t *slab_cnt, unsigned long long *slab_sum,
                               unsigned long long *gcounts, uint32_t G, uint64_t cap,
                               uint32_t nbk, hipStream_t s);
hipError_t launch_compact(const unsigned long long *gkeys, unsigned long long *gcounts,
                          uint64_t cap, const RowGeom &g, unsigned long long *out_keys,
                          unsigned long long *out_rows, unsigned long long *out_n,
                          uint64_t out_cap, int reset, hipStream_t s);
hipError_t launch_gather_dense(const unsigned long long *gkeys, const unsigned long long *gcounts,
                               const RowGeom &g, const uint64_t *keys, uint64_t n, uint64_t *rows,
                               hipStream_t s);
hipError_t launch_fold_errcnt(const unsigned long long *gkeys, unsigned long long *errcnt,
                              uint64_t cap, unsigned long long *cms, uint32_t d, uint32_t w,
                              uint32_t shift, const uint64_t *seeds, uint64_t kinv, hipStream_t s);
// binned-table path (spanagg_binned.hip)
hipError_t prepare_ingest_bt(size_t agg_lds);
size_t bt_agg2_lds_bytes(uint32_t log2sb, uint32_t grid);
// the binned launch's two kernels (the engine runs the aggregate on its own
// stream, beside the next launch's scatter)
hipError_t launch_bt_scatter(const IngestParams &P, hipStream_t s);
hipError_t launch_bt_aggregate(const IngestParams &P, hipStream_t s);
hipError_t launch_reduce_errslab(uint32_t *errslab, uint32_t G, uint64_t per_wg, uint64_t ws,
                                 uint32_t log2cap, unsigned long long *errcnt_ws, hipStream_t s);
hipError_t launch_count_keys(const unsigned long long *gkeys, uint64_t cap,
                             unsigned long long *out, hipStream_t s);
// sorted union of series ids on the device (spanagg_union.hip): out = the
// distinct non-zero ids of in[0..n) ascending, *d_total (device u32) their
// count; scratch >= key_union_scratch_bytes(n); big_scratch / big_bytes: a
// grown-on-demand buffer for buckets the LDS sort cannot hold.  Synchronises
// `s` once (the largest bucket decides the sort's form).
size_t key_union_scratch_bytes(uint64_t n);
hipError_t key_union(const uint64_t *in, uint64_t n, uint64_t *out, uint32_t *d_total, void *scratch,
                     uint64_t **big_scratch, size_t *big_bytes, hipStream_t s);
// exponential histograms (spanagg_expo.hip)
hipError_t launch_expo_ingest(const ExpoParams &E, hipStream_t s);
hipError_t launch_expo_compact(const ExpoParams &E, unsigned long long *out_keys, ExpoRow *out_rows,
                               uint32_t *out_buckets, unsigned long long *out_n, hipStream_t s);
hipError_t launch_expo_init(ExpoHdr *hdr, int8_t *xscale, uint64_t cap, hipStream_t s);
size_t expo_count_lds_bytes(uint64_t cap, uint32_t max_size);
// LDS entries of the slab counting kernel for one workgroup's LDS budget, and its LDS bytes
uint32_t expo_slab_entries(uint64_t cap, uint32_t max_size, size_t budget);
size_t expo_slab_lds_bytes(uint64_t cap, uint32_t max_size, uint32_t ne);
hipError_t prepare_expo_slab(size_t lds_bytes);
hipError_t prepare_expo_count(size_t lds_bytes);
hipError_t launch_expo_fast_probe(const uint64_t *d, const int32_t *scale, uint64_t n, double div, int32_t *fast,
                                  int32_t *exact, hipStream_t s);
hipError_t launch_log2_err_probe(uint32_t i0, uint32_t n, double *block_max, uint32_t blocks, hipStream_t s);
hipError_t launch_expo_probe(const double *v, const int32_t *scale, int32_t *idx_out, double *log_out, uint64_t n,
                             hipStream_t s);

}  // namespace sa
