/*
 * spanmetrics_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference hot path (the otel-collector `spanmetrics`
 * connector wired at /root/reference/src/otel-collector/otelcol-config.yml:115-127)
 * plus the build-owned HLL / count-min sketch spec.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline -- never as the product.
 *
 * Parity status: the connector's Go source (opentelemetry-collector-contrib
 * connector/spanmetricsconnector v0.125.0, pulled in only as the image tag at
 * /root/reference/.env:14) is not in the container and Go is absent, so this
 * restatement is pinned by hand-derived known-answer vectors (tests/golden/) and
 * by the output-name contract in the reference's Grafana dashboards, not by
 * outputs of the reference itself: numeric parity is "unpinned" against the
 * real connector.
 *
 * Deliberately shares NO code with the product library: hashing, bucketing and
 * the sketch update are written out again here from the published algorithms,
 * and bucketing uses the Go-faithful float64 path (division then
 * sort.SearchFloat64s), not the product's integer thresholds.
 */
#ifndef SPANMETRICS_ORACLE_H
#define SPANMETRICS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_engine or_engine;

/* ---- primitives ------------------------------------------------------- */
/* xxHash64 (Yann Collet's published algorithm; cespare/xxhash/v2 in Go). */
uint64_t or_xxh64(const void *data, size_t len, uint64_t seed);
/* sort.SearchFloat64s: smallest i with a[i] >= x (a sorted ascending). */
uint32_t or_search_float64s(const double *a, uint32_t n, double x);
/* connector duration: end>start ? float64(end-start)/div : 0, div = 1e6 (ms) or 1e9 (s). */
double or_duration(uint64_t start_ns, uint64_t end_ns, uint32_t unit_seconds);
/* splitmix64 finalizer used for count-min columns. */
uint64_t or_splitmix64(uint64_t x);
/* HLL estimate (standard estimator with small-range linear counting). */
double or_hll_estimate(const uint8_t *regs, uint32_t p);

/* ---- aggregation over SoA v1 batches ---------------------------------- */
or_engine *or_create(const double *bounds, uint32_t n_bounds, uint32_t unit_seconds,
                     uint32_t hll_p, uint32_t cms_d, uint32_t cms_w,
                     uint64_t window_ns, uint32_t n_services);
void or_destroy(or_engine *e);
/* Per-span body of aggregateMetrics + sketch updates. */
void or_ingest(or_engine *e, const uint64_t *key_hash, const uint64_t *start_ns,
               const uint64_t *end_ns, const uint64_t *trace_w0, const uint64_t *trace_w1,
               const uint32_t *meta, uint64_t n);
/* RED-only variant (no sketches): the connector's own per-span work. */
void or_ingest_red(or_engine *e, const uint64_t *key_hash, const uint64_t *start_ns,
                   const uint64_t *end_ns, uint64_t n);
uint64_t or_n_series(const or_engine *e);
/* Series sorted by key_hash ascending. counts is [n][n_bounds+1]. */
void or_series(const or_engine *e, uint64_t *key_hash, uint64_t *counts, double *sum_go,
               uint64_t *sum_ns, uint64_t *calls);
/* Drop all RED state (resetState for delta temporality). */
void or_reset_red(or_engine *e);
uint64_t or_n_windows(const or_engine *e);
void or_window_ids(const or_engine *e, uint64_t *ids); /* ascending */
/* hll: [n_services][2^p] u8, cms: [cms_d][cms_w] u32. Returns 0, or -1 if unknown window. */
int or_window(const or_engine *e, uint64_t window_id, uint8_t *hll, uint32_t *cms);
/* counters: [0]=spans, [1]=invalid_service, [2]=zero_key */
void or_stats(const or_engine *e, uint64_t *out3);

/* ---- exponential histogram (histogram.exponential.max_size) ------------ */
/* Go's math.Log (src/math/log.go: Frexp reduction + the fdlibm polynomial),
 * operation for operation (build with -ffp-contract=off). */
double or_go_log(double x);
/* go-expohisto MapToIndex of a positive value at `scale` (logarithm mapping
 * for scale 1..20, exponent mapping for scale <= 0). */
int32_t or_expo_index(double v, int32_t scale);
/* One series' go-expohisto structure.Histogram[float64]: Update of each
 * duration float64(end-start)/div in arrival order (zeros -> zero_count,
 * downscale by changeScale when the positive range would reach max_size).
 * counts receives the positive buckets offset .. offset + *n_out - 1
 * (capacity max_size).  sum is float64 in arrival order. */
void or_expo_series(const uint64_t *start_ns, const uint64_t *end_ns, uint64_t n, uint32_t max_size,
                    uint32_t unit_seconds, uint64_t *count, uint64_t *zero_count, double *sum, double *min,
                    double *max, int32_t *scale, int32_t *offset, uint32_t *n_out, uint64_t *counts);

/* ---- reference-faithful string-keyed path (CPU baseline) ---------------- */
/* Spans given as (service string id, span name string id, kind, status) with
 * a string table; the key is built per span exactly as buildKey does
 * (svc \0 name \0 SpanKindStr \0 StatusCodeStr) and looked up in a hash map
 * keyed by the key bytes.  Returns number of distinct series. */
uint64_t or_aggregate_strings(const char *const *strings, const uint32_t *svc_id,
                              const uint32_t *name_id, const uint32_t *kind,
                              const uint32_t *status, const uint64_t *start_ns,
                              const uint64_t *end_ns, uint64_t n, const double *bounds,
                              uint32_t n_bounds, uint64_t *checksum_out);

#ifdef __cplusplus
}
#endif
#endif
