/*
 * spanagg.h -- C-ABI of libspanagg, the MI355X (gfx950) span-aggregation engine.
 *
 * Drop-in replacement for the per-span work of the otel-collector `spanmetrics`
 * connector that the reference demo wires into its traces pipeline
 * (/root/reference/src/otel-collector/otelcol-config.yml:115-116 declares it,
 * :118-127 makes it an exporter of `traces` and a receiver of `metrics`).
 * The connector itself is Go ([UPSTREAM] opentelemetry-collector-contrib
 * connector/spanmetricsconnector v0.125.0, image tag /root/reference/.env:14);
 * its source is not vendored, so the upstream entry points are cited by name.
 *
 *   upstream (Go)                                   replaced by
 *   ----------------------------------------------  -------------------------------
 *   createDefaultConfig / Config                    sa_config + sa_config_default
 *   createTracesToMetricsConnector, Start           sa_create
 *   ConsumeTraces -> aggregateMetrics (per span)    sa_ingest / sa_ingest_async / sa_ingest_device
 *   exportMetrics -> buildMetrics + resetState      sa_flush (+ host-side encoding)
 *   Shutdown                                        sa_destroy
 *   (new) per-service HLL + error count-min         sa_window_read / sa_window_advance
 *
 * Boundary rules (mirroring the connector's contracts):
 *  - Ownership: batches are borrowed for the duration of the call (page-locked
 *    columns passed to sa_ingest_async: until the next sa_ingest_async or
 *    sa_sync returns); results are owned by the library and released with
 *    sa_red_result_free / sa_sketch_result_free.
 *  - Errors: every call returns an sa_status (0 ok, <0 error); nothing throws
 *    or aborts across the ABI; sa_last_error() gives the message.
 *  - Threading: one engine is single-producer (the connector serialises
 *    ConsumeTraces and the export ticker on one mutex); callers serialise.
 *  - No torch / HIP types appear in signatures; device pointers and streams
 *    are passed as plain pointers.
 *
 * SoA v1 span batch (44 algorithmic bytes per span, one column per array):
 *   key_hash  u64  series id: hash of (resource identity, NUL-joined metric key);
 *                  computed by the host; 0 is reserved (counted as invalid)
 *   start_ns  u64  span.start_time_unix_nano
 *   end_ns    u64  span.end_time_unix_nano
 *   trace_w0  u64  trace_id bytes 0..7 read little-endian (memcpy of the wire bytes)
 *   trace_w1  u64  trace_id bytes 8..15 read little-endian
 *   meta      u32  bits 0-15 service_id, 16-18 span.kind, 19-20 status.code
 */
#ifndef SPANAGG_H
#define SPANAGG_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SA_ABI_VERSION 4
#define SA_MAX_BOUNDS 62

typedef enum {
    SA_OK = 0,
    SA_EINVAL = -1,   /* bad argument / config */
    SA_ENOMEM = -2,   /* host or device allocation failed */
    SA_EDEVICE = -3,  /* HIP runtime error or no usable gfx950 device */
    SA_EFULL = -4,    /* key table full: spans were dropped (see stats) */
    SA_ERANGE = -5,   /* window id outside the resident ring */
    SA_ESTATE = -6    /* call not valid in the engine's current state */
} sa_status;

typedef enum { SA_UNIT_MS = 0, SA_UNIT_S = 1 } sa_unit;

/* Test and profiling entry points (probes of single kernel stages, per-
 * workgroup timestamps) are not connector operations: they are declared in
 * spanagg_diag.h, which this header does not include.
 *
 * Diagnostic ablations (sa_config.flags), used only to attribute kernel time.
 * Only the laboratory build of the library accepts them (`make -C
 * opentelemetry-demo_amd ab` -> libspanagg_ab.so, used by tools/); the
 * product library returns SA_EINVAL for any flags != 0. */
#define SA_DIAG_NO_RED 1u     /* skip key lookup + counter updates */
#define SA_DIAG_NO_HLL 2u     /* skip HLL hashing + register updates */
#define SA_DIAG_NO_CMS 4u     /* skip count-min updates */
#define SA_DIAG_NO_FLUSH 8u   /* skip the LDS -> slab flush */
#define SA_DIAG_L2_INPUT 16u  /* every workgroup re-reads the batch's first 4 tiles
                                 (cache-resident input: prices the HBM stream) */

/* Path options (sa_config.options): each selects another kernel path (or
 * merge transport) that computes the SAME results -- the parity tests compare
 * the paths through them.  0 (the default) lets the engine pick by geometry. */
#define SA_OPT_NO_HLL_FILTER (1u << 0) /* every span gathers its HLL register (no lower-bound filter) */
#define SA_OPT_PARTITIONED   (1u << 1) /* large tables: the partitioned path instead of the binned one */
#define SA_OPT_ATOMIC_TABLE  (1u << 2) /* large tables: per-span HBM CAS + atomics (no partition) */
#define SA_OPT_EXPO_HBM      (1u << 3) /* exponential histograms on the HBM-table kernels at any size */
#define SA_OPT_EXPO_CACHED   (1u << 4) /* small exponential tables: the cached-probe counting kernel */
#define SA_OPT_IDENTITY_IDS  (1u << 5) /* binned table: stored id = series id (no random multiplier) */
#define SA_OPT_STAMPS        (1u << 6) /* per-workgroup timestamps for sa_debug_stamps */
#define SA_OPT_GROUP_COPY    (1u << 7) /* sa_group_create: merge through device copies, never RCCL */
#define SA_OPT_GROUP_RCCL    (1u << 8) /* sa_group_create: RCCL even for a group of one */
#define SA_OPT_ALL           0x1FFu

typedef struct {
    /* histogram.explicit.buckets (sorted ascending, finite) and histogram.unit */
    const double *bounds;
    uint32_t n_bounds;
    uint32_t unit;          /* sa_unit */
    /* build-owned sketches */
    uint32_t hll_p;         /* HLL precision, 4..18 (default 14) */
    uint32_t cms_d;         /* count-min rows, 1..8 (default 4) */
    uint32_t cms_w;         /* count-min columns, power of two (default 2048) */
    uint64_t window_ns;     /* sketch window length (default 10 s; < 2^56 ns) */
    uint32_t n_windows;     /* resident window ring, power of two (default 8) */
    uint32_t n_services;    /* service ids 0..n_services-1 get sketches */
    uint64_t key_capacity;  /* expected distinct series; table = next pow2 >= 1.25x */
    int32_t device;         /* HIP device ordinal (one engine per GPU / rank) */
    uint32_t flags;         /* 0 for production; SA_DIAG_* bits are profiling-only
                               ablations that skip work and make results WRONG
                               (laboratory build only) */
    /* histogram.exponential.max_size: 0 = explicit buckets (the default);
     * 2..4096 = exponential histograms (bounds unused; read with sa_flush_exp) */
    uint32_t exp_max_size;
    uint32_t options;       /* SA_OPT_* path options (0 = the engine's choice) */
} sa_config;

typedef struct {
    const uint64_t *key_hash, *start_ns, *end_ns, *trace_w0, *trace_w1;
    const uint32_t *meta;
    uint64_t n;
} sa_span_batch;

/* Delta RED state since the previous sa_flush, one row per series with any
 * span, sorted by key_hash ascending. */
typedef struct {
    uint64_t n_series;
    uint32_t n_buckets;            /* n_bounds + 1 */
    const uint64_t *key_hash;      /* [n_series] */
    const uint64_t *bucket_counts; /* [n_series][n_buckets] */
    const uint64_t *calls;         /* [n_series] == sum of bucket_counts (A8) */
    const uint64_t *sum_ns;        /* [n_series] exact sum of durations in ns */
    const double *sum;             /* [n_series] sum_ns / unit divisor (ms or s) */
} sa_red_result;

/* Exponential histograms (sa_config.exp_max_size > 0): the delta since the
 * previous sa_flush_exp, one row per series with any span, sorted by
 * key_hash.  Each row is go-expohisto's Histogram[float64] of the series'
 * durations (float64(end-start)/unit): positive bucket i at `scale` counts
 * values in (2^(i/2^scale), 2^((i+1)/2^scale)]; bucket_counts[r][j] is bucket
 * offset[r] + j for j < n_buckets[r]. */
typedef struct {
    uint64_t n_series;
    uint32_t max_size;             /* row stride of bucket_counts */
    uint32_t unit;                 /* sa_unit of sum/min/max */
    const uint64_t *key_hash;      /* [n_series] */
    const uint64_t *count;         /* [n_series] spans (== calls) */
    const uint64_t *zero_count;    /* [n_series] zero durations */
    const uint64_t *sum_ns;        /* [n_series] exact */
    const double *sum, *min, *max; /* [n_series] in the unit */
    const int32_t *scale, *offset; /* [n_series] */
    const uint32_t *n_buckets;     /* [n_series] */
    const uint64_t *bucket_counts; /* [n_series][max_size] */
} sa_exp_result;

typedef struct {
    uint64_t window_id;
    uint32_t n_services, hll_p;
    const uint8_t *hll;            /* [n_services][2^hll_p] registers */
    uint32_t cms_d, cms_w;
    const uint32_t *cms;           /* [cms_d][cms_w], saturating u32 */
} sa_sketch_result;

typedef struct {
    uint64_t spans;                /* spans accepted by sa_ingest* */
    uint64_t zero_key;             /* spans with key_hash == 0 (no RED update) */
    uint64_t invalid_service;      /* service_id >= n_services (no sketch update) */
    uint64_t window_out_of_range;  /* window outside the resident ring (no sketch update) */
    uint64_t dropped_table_full;   /* spans lost because the key table was full */
    uint64_t n_keys;               /* distinct series resident in the key table */
    uint64_t table_capacity;
    uint64_t window_base;          /* oldest resident window id */
    uint32_t small_table;          /* 1 = LDS-mirrored table path, 0 = HBM path */
    uint32_t pad;
    /* spans whose HLL update was skipped without reading their register: rho
     * at or below the lower bound of the register's sub-block, so it could not
     * raise it (the small-table and binned kernels; 0 on the other paths).
     * Diagnostic: shows how much of a window runs on the filtered path. */
    uint64_t hll_filtered;
} sa_stats;

typedef struct sa_engine sa_engine;

/* createDefaultConfig: default buckets {2,4,6,8,10,50,100,200,400,800,1000,1400,
 * 2000,5000,10000,15000} ms, HLL p=14, CMS 4x2048, 10 s windows, 8-window ring. */
void sa_config_default(sa_config *cfg);
int sa_abi_version(void);

int sa_create(const sa_config *cfg, sa_engine **out);
void sa_destroy(sa_engine *e);
const char *sa_last_error(const sa_engine *e);

/* Host-memory batch: packed into one of two pinned staging slots (chunks of
 * 2^18 spans or more: copied from the caller's pageable columns by the HIP
 * runtime, and waited for), copied to HBM and aggregated on the engine
 * stream.  Returns once the batch has been copied out of the caller's buffers
 * (they may be reused or freed at once); the
 * aggregation completes asynchronously -- every read (sa_flush*, sa_window_*,
 * sa_get_stats) and sa_sync wait for it, and a device error surfaces there. */
int sa_ingest(sa_engine *e, const sa_span_batch *batch);
/* sa_ingest for a host that alternates two page-locked column buffers (the
 * Node host's columnizer): when every column lies in sa_host_alloc memory the
 * DMA reads them after the call returns, and the call returns once the
 * columns of this engine's previous sa_ingest_async call have been read -- so
 * the caller may refill the other buffer while this one is copied, and must
 * leave this one alone until its next sa_ingest_async (or sa_sync /
 * sa_destroy) returns.  Any other columns, and any error return: as
 * sa_ingest (read before the call returns). */
int sa_ingest_async(sa_engine *e, const sa_span_batch *batch);
/* Page-locked host memory for batch columns a host builds itself (the Node
 * host's columnizer does): sa_ingest / sa_group_ingest copy columns that all
 * lie in such memory to HBM by DMA straight from the caller's arrays, with no
 * staging copy on the calling thread.  SA_ENOMEM when no GPU runtime can pin
 * memory (the caller then uses ordinary memory, which sa_ingest stages). */
int sa_host_alloc(size_t bytes, void **out);
void sa_host_free(void *p);
/* Device-resident batch (pointers into HBM of this engine's device).
 * `stream` is a hipStream_t (NULL = the engine's own stream). Asynchronous:
 * the batch must stay valid until the stream reaches this point. Ordered
 * after the engine's earlier non-ingest work (flush, window calls) and
 * before the caller's later work on `stream`; ingests on different streams
 * may run concurrently on the device (the engine orders them only where they
 * share state), which is how consecutive batches overlap. */
int sa_ingest_device(sa_engine *e, const sa_span_batch *batch, void *stream);
/* k device batches in order on `stream`: the same result as k
 * sa_ingest_device calls on it (same ordering rules, every batch valid until
 * the stream reaches the end of the k).  Small-table engines launch the k
 * ingests as one HIP graph, so consecutive launches carry no per-launch
 * dispatch gap; other engines (binned, exponential, laboratory options) and
 * batches that would need a split take the one-by-one path.  Replaces a loop
 * of ConsumeTraces calls over the batches a receiver queued (the connector's
 * aggregateMetrics per request, connector.go [UPSTREAM]). */
int sa_ingest_device_many(sa_engine *e, const sa_span_batch *batches, uint32_t k, void *stream);
/* Orders `stream` (NULL = the engine's stream) after every launch the engine
 * has enqueued so far, including work it runs on its own streams: the
 * high-cardinality (binned) path aggregates launch k on an engine stream
 * while launch k + 1 reads its batch, so the caller's stream passes an
 * ingest once the batch is consumed, not once it is aggregated.  Engine reads
 * (sa_flush*, sa_window_*, sa_get_stats) and sa_sync join by themselves; a
 * caller timing the aggregation with events on its own stream joins first. */
int sa_join(sa_engine *e, void *stream);
int sa_sync(sa_engine *e);

/* exportMetrics: delta since the last flush, then the engine's RED counters are
 * reset. Keys stay resident as a cache of the series seen, until more than half
 * the table is taken (35 % for the binned table of large key capacities): then
 * the flush empties it (sa_reclaim_keys), so series
 * that churn (new resources after evictions or restarts, delta purges) do not
 * fill it for good. Returns SA_EFULL (with the result still filled) if spans
 * were dropped since the previous flush: more distinct series within one flush
 * interval than key_capacity. */
int sa_flush(sa_engine *e, sa_red_result **out);
void sa_red_result_free(sa_red_result *r);
/* Key-table reclamation (what every flush does when the table is more than
 * half full, binned tables 35 %; force != 0: empty it now).  Only between a flush (or a resetting
 * sa_gather_dense) and the next ingest: SA_ESTATE otherwise.  Results do not
 * change: every row is zero then, and a series' next span re-inserts its key.
 * Replaces nothing in the reference (upstream keys live in a Go LRU map,
 * spanmetrics connector.go `resourceMetrics` / `dimensionsCache`). */
int sa_reclaim_keys(sa_engine *e, int force);
/* exportMetrics of an exponential-histogram engine (sa_flush returns
 * SA_ESTATE there, and sa_flush_exp does on an explicit-bucket engine). */
int sa_flush_exp(sa_engine *e, sa_exp_result **out);
void sa_exp_result_free(sa_exp_result *r);
/* Sketches of one resident window (not cleared). */
int sa_window_read(sa_engine *e, uint64_t window_id, sa_sketch_result **out);
/* Retire every window < new_base (clears their ring slots); spans whose window
 * is below the base or >= base + n_windows are counted in window_out_of_range. */
int sa_window_advance(sa_engine *e, uint64_t new_base);
void sa_sketch_result_free(sa_sketch_result *r);

int sa_get_stats(sa_engine *e, sa_stats *out);

/* ---- multi-GPU merge hooks (device pointers on this engine's device) ----
 * Used by the host's RCCL merge: gather the local key list, build the sorted
 * union across ranks, densify local counters against it, all-reduce. */
/* Folds pending partials into the HBM table and writes the resident keys that
 * have a non-zero delta into d_keys (capacity `cap`); *n_out = count (may exceed
 * cap, in which case nothing beyond cap is written). */
int sa_export_keys(sa_engine *e, uint64_t *d_keys, uint64_t cap, uint64_t *n_out, void *stream);
/* d_rows[i] = [bucket counts..., sum_ns] (n_buckets+1 u64) for d_keys[i]
 * (zeros if absent). reset != 0 clears the engine's delta counters afterwards. */
int sa_gather_dense(sa_engine *e, const uint64_t *d_keys, uint64_t n, uint64_t *d_rows,
                    int reset, void *stream);
/* Window sketches into device buffers: d_hll [n_services][2^p] u8 and
 * d_cms [d][w] u64 (unsaturated, for sum all-reduce). */
int sa_window_export(sa_engine *e, uint64_t window_id, uint8_t *d_hll, uint64_t *d_cms,
                     void *stream);

/* ---- engine groups: one engine per GPU behind one handle ----
 * The connector's single ConsumeTraces/exportMetrics pair over several GPUs.
 * Spans shard by trace id (engine = trace_w1 % n), so every trace's spans land
 * on one engine and the per-engine sketches stay exact partials; the group's
 * flush / window read return the merge:
 *   RED: key union across engines (a series seen on several engines is one
 *        row), bucket counts and ns sums added;
 *   HLL: registers max-merged (exact and idempotent);
 *   count-min: cells added, then saturated to u32.
 * Merge transport: when every member has its own device the group owns an
 * RCCL communicator over them (ncclAllGather of the key lists, ncclAllReduce
 * sum u64 of the dense rows and count-min cells, max u8 of the HLL
 * registers, over xGMI); members that share a device (or SA_OPT_GROUP_COPY)
 * merge through device-to-device copies onto member 0's device and a reduce
 * kernel there.  Results are identical either way (integer sums and maxima).
 * Threading: as an engine (single producer); sa_group_ingest fans the shards
 * out to one host thread per member. */
typedef struct sa_group sa_group;
/* devices[i] = HIP ordinal of member i (repeats allowed); cfg->device is ignored. */
int sa_group_create(const sa_config *cfg, const int32_t *devices, uint32_t n, sa_group **out);
void sa_group_destroy(sa_group *g);
const char *sa_group_last_error(const sa_group *g);
uint32_t sa_group_size(const sa_group *g);
/* 1 when the group merges over RCCL, 0 when through device copies */
int sa_group_uses_rccl(const sa_group *g);
/* Member engine i (for device-resident ingest of a shard the caller made). */
sa_engine *sa_group_member(sa_group *g, uint32_t i);
/* Host batch: split by trace_w1 % n, each shard ingested by its member.  The
 * split is one pass over trace_w1 (shard sizes) and one gather of each span
 * into its member's packed shard, both on worker threads; the call returns
 * once every member has copied its shard out of the caller's buffers. */
int sa_group_ingest(sa_group *g, const sa_span_batch *batch);
/* Device-resident batch in HBM of member `src`'s device (`stream`: a
 * hipStream_t of that device, NULL = the group's stream there).  A partition
 * kernel on that device counts the shards (trace_w1 % n; the call waits for
 * these counts, a few microseconds) and scatters every span into its member's
 * packed shard; shards of members on other devices are copied there
 * peer-to-peer (xGMI DMA), and every member ingests its shard on its own
 * stream.  Asynchronous otherwise: the batch must stay valid until `stream`
 * reaches this point (the partition has read it); sa_group_sync waits for the
 * members.  Same results as sa_group_ingest of the same spans. */
int sa_group_ingest_device(sa_group *g, const sa_span_batch *batch, uint32_t src, void *stream);
int sa_group_sync(sa_group *g);
/* Merged delta since the previous group flush (members reset); SA_EFULL as
 * sa_flush when any member dropped spans. Free with sa_red_result_free. */
int sa_group_flush(sa_group *g, sa_red_result **out);
/* exportMetrics of a group built with exp_max_size != 0: the members' delta
 * exponential histograms folded per series (the histogram one engine fed
 * every member's spans would hold). Free with sa_exp_result_free. */
int sa_group_flush_exp(sa_group *g, sa_exp_result **out);
/* Merged sketches of one resident window. Free with sa_sketch_result_free. */
int sa_group_window_read(sa_group *g, uint64_t window_id, sa_sketch_result **out);
int sa_group_window_advance(sa_group *g, uint64_t new_base);
/* Counters summed over members (n_keys and table_capacity too; window_base and
 * small_table from member 0). */
int sa_group_get_stats(sa_group *g, sa_stats *out);

/* ---- pure host helpers (no device needed) ---- */
/* Integer bucket thresholds: bucket(d_ns) = n_neg + #{i : d_ns > thr[i]} equals
 * sort.SearchFloat64s(bounds, float64(d_ns)/div) for every u64 d_ns. Returns
 * n_neg via *n_neg and fills thr[0 .. n_bounds-n_neg). */
int sa_bucket_thresholds(const double *bounds, uint32_t n_bounds, uint32_t unit,
                         uint64_t *thr, uint32_t *n_neg);
/* HLL estimate of one register array (standard estimator + linear counting). */
double sa_hll_estimate(const uint8_t *regs, uint32_t p);

#ifdef __cplusplus
}
#endif
#endif
