/*
 * spanmetrics_oracle.c -- TEST INFRASTRUCTURE ONLY (see spanmetrics_oracle.h).
 *
 * CPU restatement of the spanmetrics connector's per-span aggregation
 * ([UPSTREAM] connector/spanmetricsconnector v0.125.0 connector.go
 * `aggregateMetrics`, `buildKey`; internal/metrics/metrics.go
 * `explicitHistogram.Observe`, `Sum.Add` -- restated in SURVEY.md section 3A and
 * rows a5-a11), instantiated with the factory defaults the reference config
 * selects by declaring `spanmetrics:` with an empty body
 * (/root/reference/src/otel-collector/otelcol-config.yml:115-116), plus the
 * build-owned sketch spec.
 */
#include "spanmetrics_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* xxHash64, restated from the published specification (XXH64, seed variant). */
#define XP1 0x9E3779B185EBCA87ULL
#define XP2 0xC2B2AE3D27D4EB4FULL
#define XP3 0x165667B19E3779F9ULL
#define XP4 0x85EBCA77C2B2AE63ULL
#define XP5 0x27D4EB2F165667C5ULL

static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t rd64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i]; /* little-endian read */
    return v;
}
static inline uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t xround(uint64_t acc, uint64_t in) {
    acc += in * XP2;
    acc = rotl64(acc, 31);
    return acc * XP1;
}
static inline uint64_t xmerge(uint64_t acc, uint64_t v) {
    acc ^= xround(0, v);
    return acc * XP1 + XP4;
}

uint64_t or_xxh64(const void *data, size_t len, uint64_t seed) {
    const uint8_t *p = (const uint8_t *)data, *end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
        const uint8_t *limit = end - 32;
        do {
            v1 = xround(v1, rd64(p));
            v2 = xround(v2, rd64(p + 8));
            v3 = xround(v3, rd64(p + 16));
            v4 = xround(v4, rd64(p + 24));
            p += 32;
        } while (p <= limit);
        h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = seed + XP5;
    }
    h += (uint64_t)len;
    while (p + 8 <= end) {
        h ^= xround(0, rd64(p));
        h = rotl64(h, 27) * XP1 + XP4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)rd32(p) * XP1;
        h = rotl64(h, 23) * XP2 + XP3;
        p += 4;
    }
    while (p < end) {
        h ^= (uint64_t)(*p) * XP5;
        h = rotl64(h, 11) * XP1;
        ++p;
    }
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    return h;
}

/* Go sort.SearchFloat64s(a, x) = sort.Search(len(a), func(i) bool { return a[i] >= x }). */
uint32_t or_search_float64s(const double *a, uint32_t n, double x) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        uint32_t mid = lo + (hi - lo) / 2;
        if (!(a[mid] >= x)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

/* [UPSTREAM] connector.go: duration := 0.0; if end > start { duration =
 * float64(end-start) / unitDivider }  (unitDivider 1e6 for ms, 1e9 for s). */
double or_duration(uint64_t start_ns, uint64_t end_ns, uint32_t unit_seconds) {
    if (end_ns > start_ns) {
        double d = (double)(end_ns - start_ns);
        return d / (unit_seconds ? 1e9 : 1e6);
    }
    return 0.0;
}

uint64_t or_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static const uint64_t CMS_SEED[8] = {0x9E3779B97F4A7C15ULL, 0xBF58476D1CE4E5B9ULL,
                                     0x94D049BB133111EBULL, 0xD6E8FEB86659FD93ULL,
                                     0xA0761D6478BD642FULL, 0xE7037ED1A0B428DBULL,
                                     0x8EBC6AF09C88C6E3ULL, 0x589965CC75374CC3ULL};

double or_hll_estimate(const uint8_t *regs, uint32_t p) {
    const uint32_t m = 1u << p;
    double sum = 0.0;
    uint32_t zeros = 0;
    for (uint32_t j = 0; j < m; ++j) {
        sum += ldexp(1.0, -(int)regs[j]);
        zeros += regs[j] == 0;
    }
    const double alpha = m == 16 ? 0.673 : m == 32 ? 0.697 : m == 64 ? 0.709
                                                                    : 0.7213 / (1.0 + 1.079 / (double)m);
    double e = alpha * (double)m * (double)m / sum;
    if (e <= 2.5 * (double)m && zeros != 0) e = (double)m * log((double)m / (double)zeros);
    return e;
}

/* ------------------------------------------------------------------------ */
/* u64-keyed open-addressing map (index into dense arrays).                 */
typedef struct {
    uint64_t *keys; /* 0 = empty; callers never insert key 0 */
    uint32_t *idx;
    uint64_t cap, n;
} u64map;

static void map_init(u64map *m, uint64_t cap) {
    m->cap = cap;
    m->n = 0;
    m->keys = (uint64_t *)calloc(cap, sizeof(uint64_t));
    m->idx = (uint32_t *)calloc(cap, sizeof(uint32_t));
}
static void map_free(u64map *m) {
    free(m->keys);
    free(m->idx);
    memset(m, 0, sizeof *m);
}
static inline uint64_t map_slot(uint64_t key, uint64_t cap) { return or_splitmix64(key) & (cap - 1); }
/* returns index, inserting with value `fresh` when absent; *ins set when inserted */
static uint32_t map_get(u64map *m, uint64_t key, uint32_t fresh, int *ins) {
    if ((m->n + 1) * 2 > m->cap) {
        u64map g;
        map_init(&g, m->cap * 2);
        for (uint64_t i = 0; i < m->cap; ++i)
            if (m->keys[i]) {
                uint64_t s = map_slot(m->keys[i], g.cap);
                while (g.keys[s]) s = (s + 1) & (g.cap - 1);
                g.keys[s] = m->keys[i];
                g.idx[s] = m->idx[i];
            }
        g.n = m->n;
        map_free(m);
        *m = g;
    }
    uint64_t s = map_slot(key, m->cap);
    while (m->keys[s]) {
        if (m->keys[s] == key) {
            *ins = 0;
            return m->idx[s];
        }
        s = (s + 1) & (m->cap - 1);
    }
    m->keys[s] = key;
    m->idx[s] = fresh;
    m->n++;
    *ins = 1;
    return fresh;
}

typedef struct {
    uint64_t id;
    uint8_t *hll;  /* [S][m] */
    uint32_t *cms; /* [d][w] */
} or_window_t;

struct or_engine {
    double *bounds;
    uint32_t nb, nbk, unit_s;
    uint32_t hll_p, cms_d, cms_w, cms_shift, n_services;
    uint64_t window_ns;
    /* RED state, dense in first-seen order */
    u64map series_map;
    uint64_t n_series, series_cap;
    uint64_t *s_key, *s_counts, *s_sum_ns;
    double *s_sum_go;
    /* windows */
    u64map win_map;
    or_window_t *wins;
    uint64_t n_wins, wins_cap;
    uint64_t stats[3];
};

or_engine *or_create(const double *bounds, uint32_t n_bounds, uint32_t unit_seconds,
                     uint32_t hll_p, uint32_t cms_d, uint32_t cms_w, uint64_t window_ns,
                     uint32_t n_services) {
    if (hll_p < 4 || hll_p > 18 || cms_d == 0 || cms_d > 8 || cms_w < 2 ||
        (cms_w & (cms_w - 1)) || window_ns == 0)
        return NULL;
    or_engine *e = (or_engine *)calloc(1, sizeof *e);
    e->nb = n_bounds;
    e->nbk = n_bounds + 1;
    e->bounds = (double *)malloc(sizeof(double) * (n_bounds ? n_bounds : 1));
    memcpy(e->bounds, bounds, sizeof(double) * n_bounds);
    e->unit_s = unit_seconds;
    e->hll_p = hll_p;
    e->cms_d = cms_d;
    e->cms_w = cms_w;
    e->cms_shift = 64 - (uint32_t)__builtin_ctz(cms_w);
    e->window_ns = window_ns;
    e->n_services = n_services;
    map_init(&e->series_map, 1024);
    map_init(&e->win_map, 64);
    return e;
}

static void red_free(or_engine *e) {
    free(e->s_key);
    free(e->s_counts);
    free(e->s_sum_ns);
    free(e->s_sum_go);
    e->s_key = e->s_counts = e->s_sum_ns = NULL;
    e->s_sum_go = NULL;
    e->n_series = e->series_cap = 0;
}

void or_destroy(or_engine *e) {
    if (!e) return;
    red_free(e);
    map_free(&e->series_map);
    for (uint64_t i = 0; i < e->n_wins; ++i) {
        free(e->wins[i].hll);
        free(e->wins[i].cms);
    }
    free(e->wins);
    map_free(&e->win_map);
    free(e->bounds);
    free(e);
}

void or_reset_red(or_engine *e) {
    red_free(e);
    map_free(&e->series_map);
    map_init(&e->series_map, 1024);
}

static uint64_t series_index(or_engine *e, uint64_t key) {
    int ins;
    uint32_t i = map_get(&e->series_map, key, (uint32_t)e->n_series, &ins);
    if (ins) {
        if (e->n_series == e->series_cap) {
            uint64_t c = e->series_cap ? e->series_cap * 2 : 1024;
            e->s_key = (uint64_t *)realloc(e->s_key, c * sizeof(uint64_t));
            e->s_counts = (uint64_t *)realloc(e->s_counts, c * e->nbk * sizeof(uint64_t));
            e->s_sum_ns = (uint64_t *)realloc(e->s_sum_ns, c * sizeof(uint64_t));
            e->s_sum_go = (double *)realloc(e->s_sum_go, c * sizeof(double));
            e->series_cap = c;
        }
        e->s_key[i] = key;
        memset(e->s_counts + (uint64_t)i * e->nbk, 0, e->nbk * sizeof(uint64_t));
        e->s_sum_ns[i] = 0;
        e->s_sum_go[i] = 0.0;
        e->n_series++;
    }
    return i;
}

static or_window_t *window_get(or_engine *e, uint64_t wid) {
    int ins;
    /* window ids are stored +1 so id 0 is representable in the map */
    uint32_t i = map_get(&e->win_map, wid + 1, (uint32_t)e->n_wins, &ins);
    if (ins) {
        if (e->n_wins == e->wins_cap) {
            e->wins_cap = e->wins_cap ? e->wins_cap * 2 : 16;
            e->wins = (or_window_t *)realloc(e->wins, e->wins_cap * sizeof(or_window_t));
        }
        or_window_t *w = &e->wins[i];
        w->id = wid;
        w->hll = (uint8_t *)calloc((size_t)e->n_services << e->hll_p, 1);
        w->cms = (uint32_t *)calloc((size_t)e->cms_d * e->cms_w, sizeof(uint32_t));
        e->n_wins++;
    }
    return &e->wins[i];
}

/* explicitHistogram.Observe: sum += d; count++; bucketCounts[SearchFloat64s(bounds, d)]++
 * Sum.Add(1): calls += 1 (== histogram count; we keep the bucket vector only). */
static inline void red_observe(or_engine *e, uint64_t key, uint64_t s, uint64_t t) {
    uint64_t i = series_index(e, key);
    double d = or_duration(s, t, e->unit_s);
    uint32_t b = or_search_float64s(e->bounds, e->nb, d);
    e->s_counts[i * e->nbk + b] += 1;
    e->s_sum_go[i] += d;
    e->s_sum_ns[i] += t > s ? t - s : 0;
}

void or_ingest_red(or_engine *e, const uint64_t *key, const uint64_t *start,
                   const uint64_t *end, uint64_t n) {
    for (uint64_t k = 0; k < n; ++k) {
        e->stats[0]++;
        if (key[k] == 0) {
            e->stats[2]++;
            continue;
        }
        red_observe(e, key[k], start[k], end[k]);
    }
}

void or_ingest(or_engine *e, const uint64_t *key, const uint64_t *start, const uint64_t *end,
               const uint64_t *w0, const uint64_t *w1, const uint32_t *meta, uint64_t n) {
    const uint32_t p = e->hll_p;
    or_window_t *last = NULL;
    for (uint64_t k = 0; k < n; ++k) {
        e->stats[0]++;
        if (key[k] == 0) e->stats[2]++;
        else red_observe(e, key[k], start[k], end[k]);

        const uint32_t svc = meta[k] & 0xFFFFu;
        const uint32_t status = (meta[k] >> 19) & 3u;
        if (svc >= e->n_services) {
            e->stats[1]++;
            continue;
        }
        const uint64_t wid = end[k] / e->window_ns;
        or_window_t *w = (last && last->id == wid) ? last : window_get(e, wid);
        last = w;
        /* HLL: x = xxh64(trace_id[16], 0); idx = top p bits; rho = clz of the rest + 1 */
        uint8_t tid[16];
        for (int b = 0; b < 8; ++b) {
            tid[b] = (uint8_t)(w0[k] >> (8 * b));
            tid[8 + b] = (uint8_t)(w1[k] >> (8 * b));
        }
        const uint64_t x = or_xxh64(tid, 16, 0);
        const uint64_t idx = x >> (64 - p);
        const uint64_t rest = (x << p) | (1ULL << (p - 1));
        const uint8_t rho = (uint8_t)(__builtin_clzll(rest) + 1);
        uint8_t *reg = &w->hll[((uint64_t)svc << p) + idx];
        if (*reg < rho) *reg = rho;
        /* CMS over ERROR spans, keyed by the series key hash */
        if (status == 2) {
            for (uint32_t j = 0; j < e->cms_d; ++j) {
                const uint64_t col = or_splitmix64(key[k] ^ CMS_SEED[j]) >> e->cms_shift;
                uint32_t *c = &w->cms[(uint64_t)j * e->cms_w + col];
                if (*c != UINT32_MAX) ++*c;
            }
        }
    }
}

uint64_t or_n_series(const or_engine *e) { return e->n_series; }

static const uint64_t *g_sort_keys;
static int cmp_by_key(const void *a, const void *b) {
    uint64_t ka = g_sort_keys[*(const uint64_t *)a], kb = g_sort_keys[*(const uint64_t *)b];
    return ka < kb ? -1 : ka > kb;
}

void or_series(const or_engine *e, uint64_t *key, uint64_t *counts, double *sum_go,
               uint64_t *sum_ns, uint64_t *calls) {
    uint64_t n = e->n_series;
    uint64_t *ord = (uint64_t *)malloc(sizeof(uint64_t) * (n ? n : 1));
    for (uint64_t i = 0; i < n; ++i) ord[i] = i;
    g_sort_keys = e->s_key;
    qsort(ord, n, sizeof(uint64_t), cmp_by_key);
    for (uint64_t r = 0; r < n; ++r) {
        uint64_t i = ord[r];
        if (key) key[r] = e->s_key[i];
        uint64_t c = 0;
        for (uint32_t b = 0; b < e->nbk; ++b) {
            uint64_t v = e->s_counts[i * e->nbk + b];
            if (counts) counts[r * e->nbk + b] = v;
            c += v;
        }
        if (calls) calls[r] = c;
        if (sum_go) sum_go[r] = e->s_sum_go[i];
        if (sum_ns) sum_ns[r] = e->s_sum_ns[i];
    }
    free(ord);
}

uint64_t or_n_windows(const or_engine *e) { return e->n_wins; }

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

void or_window_ids(const or_engine *e, uint64_t *ids) {
    for (uint64_t i = 0; i < e->n_wins; ++i) ids[i] = e->wins[i].id;
    qsort(ids, e->n_wins, sizeof(uint64_t), cmp_u64);
}

int or_window(const or_engine *e, uint64_t wid, uint8_t *hll, uint32_t *cms) {
    for (uint64_t i = 0; i < e->n_wins; ++i)
        if (e->wins[i].id == wid) {
            if (hll) memcpy(hll, e->wins[i].hll, (size_t)e->n_services << e->hll_p);
            if (cms) memcpy(cms, e->wins[i].cms, sizeof(uint32_t) * e->cms_d * e->cms_w);
            return 0;
        }
    return -1;
}

void or_stats(const or_engine *e, uint64_t *out3) { memcpy(out3, e->stats, sizeof e->stats); }

/* ------------------------------------------------------------------------ */
/* Reference-faithful string-keyed aggregation: the CPU baseline.
 * [UPSTREAM] buildKey writes svc, then \0 + span.Name(), \0 + SpanKindStr,
 * \0 + StatusCodeStr (no extra dimensions with the default config); the key
 * is then looked up in the resource's metric maps.                          */
static const char *kind_str(uint32_t k) {
    static const char *s[6] = {"SPAN_KIND_UNSPECIFIED", "SPAN_KIND_INTERNAL", "SPAN_KIND_SERVER",
                               "SPAN_KIND_CLIENT",      "SPAN_KIND_PRODUCER", "SPAN_KIND_CONSUMER"};
    return k < 6 ? s[k] : "";
}
static const char *status_str(uint32_t c) {
    static const char *s[3] = {"STATUS_CODE_UNSET", "STATUS_CODE_OK", "STATUS_CODE_ERROR"};
    return c < 3 ? s[c] : "";
}

typedef struct {
    char *bytes;
    uint32_t len;
    uint64_t *counts;
    double sum;
} str_series;

uint64_t or_aggregate_strings(const char *const *strings, const uint32_t *svc_id,
                              const uint32_t *name_id, const uint32_t *kind,
                              const uint32_t *status, const uint64_t *start_ns,
                              const uint64_t *end_ns, uint64_t n, const double *bounds,
                              uint32_t n_bounds, uint64_t *checksum_out) {
    uint64_t cap = 1024, cnt = 0;
    str_series *tab = (str_series *)calloc(cap, sizeof(str_series));
    char buf[4096];
    for (uint64_t k = 0; k < n; ++k) {
        /* buildKey into a reused buffer */
        size_t len = 0;
        const char *parts[4] = {strings[svc_id[k]], strings[name_id[k]], kind_str(kind[k]),
                                status_str(status[k])};
        for (int q = 0; q < 4; ++q) {
            if (q) buf[len++] = '\0';
            size_t l = strlen(parts[q]);
            if (len + l >= sizeof buf) l = sizeof buf - len - 1;
            memcpy(buf + len, parts[q], l);
            len += l;
        }
        if ((cnt + 1) * 2 > cap) {
            uint64_t nc = cap * 2;
            str_series *nt = (str_series *)calloc(nc, sizeof(str_series));
            for (uint64_t i = 0; i < cap; ++i)
                if (tab[i].bytes) {
                    uint64_t s = or_xxh64(tab[i].bytes, tab[i].len, 0) & (nc - 1);
                    while (nt[s].bytes) s = (s + 1) & (nc - 1);
                    nt[s] = tab[i];
                }
            free(tab);
            tab = nt;
            cap = nc;
        }
        uint64_t s = or_xxh64(buf, len, 0) & (cap - 1);
        while (tab[s].bytes && !(tab[s].len == len && memcmp(tab[s].bytes, buf, len) == 0))
            s = (s + 1) & (cap - 1);
        if (!tab[s].bytes) {
            tab[s].bytes = (char *)malloc(len ? len : 1);
            memcpy(tab[s].bytes, buf, len);
            tab[s].len = (uint32_t)len;
            tab[s].counts = (uint64_t *)calloc(n_bounds + 1, sizeof(uint64_t));
            cnt++;
        }
        double d = or_duration(start_ns[k], end_ns[k], 0);
        tab[s].counts[or_search_float64s(bounds, n_bounds, d)]++;
        tab[s].sum += d;
    }
    uint64_t cs = 0;
    for (uint64_t i = 0; i < cap; ++i)
        if (tab[i].bytes) {
            for (uint32_t b = 0; b <= n_bounds; ++b) cs += tab[i].counts[b] * (b + 1);
            free(tab[i].bytes);
            free(tab[i].counts);
        }
    free(tab);
    if (checksum_out) *checksum_out = cs;
    return cnt;
}

/* ------------------------------------------------------------------------
 * Exponential histogram: [UPSTREAM] spanmetricsconnector internal/metrics
 * exponentialHistogram.Observe -> github.com/lightstep/go-expohisto
 * structure.Histogram[float64].Update, restated value by value.  The log is
 * Go's math.Log (src/math/log.go) with the same operations in the same order;
 * the Makefile builds this file with -ffp-contract=off so no multiply-add is
 * fused (Go does not fuse them on amd64).
 * ---------------------------------------------------------------------- */
double or_go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  int ki;
  double f1 = frexp(x, &ki);
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

int32_t or_expo_index(double v, int32_t scale) {
  uint64_t b;
  memcpy(&b, &v, 8);
  int64_t raw_exp = (int64_t)((b >> 52) & 0x7FF);
  const uint64_t sig = b & ((1ULL << 52) - 1);
  if (scale > 0) {
    if (v <= 0x1p-1022) return (int32_t)(-1022 * (1LL << scale));
    if (sig == 0) return (int32_t)((raw_exp - 1023) * (1LL << scale) - 1);
    const double x = floor(or_go_log(v) * ldexp(1.4426950408889634, scale));
    const int64_t max_index = (1024LL << scale) - 1;
    return x >= (double)max_index ? (int32_t)max_index : (int32_t)x;
  }
  if (raw_exp == 0) raw_exp -= (int64_t)__builtin_clzll(sig) - 12;
  const int32_t exp = (int32_t)(raw_exp - 1023);
  return (exp + (sig == 0 ? -1 : 0)) >> (-scale);
}

void or_expo_series(const uint64_t *start_ns, const uint64_t *end_ns, uint64_t n, uint32_t max_size,
                    uint32_t unit_seconds, uint64_t *count, uint64_t *zero_count, double *sum, double *min,
                    double *max, int32_t *scale, int32_t *offset, uint32_t *n_out, uint64_t *counts) {
  /* positive buckets: counts[i - start] for index i in [start, end] */
  uint64_t *tmp = (uint64_t *)calloc(max_size ? max_size : 1, 8);
  int32_t sc = 20, start = 0, end = -1;
  int have = 0;
  *count = *zero_count = 0;
  *sum = *min = *max = 0.0;
  memset(counts, 0, (size_t)max_size * 8);
  for (uint64_t j = 0; j < n; ++j) {
    const double v = or_duration(start_ns[j], end_ns[j], unit_seconds);
    if (*count == 0) *min = *max = v;
    else {
      if (v < *min) *min = v;
      if (v > *max) *max = v;
    }
    *count += 1;
    if (v == 0) {
      *zero_count += 1;
      continue;
    }
    *sum += v;
    for (int attempt = 0; attempt < 2; ++attempt) {
      const int32_t idx = or_expo_index(v, sc);
      int32_t hi = 0, lo = 0, fits = 1;
      if (!have) {
        start = end = idx;
        have = 1;
      } else if (idx < start) {
        if (end - idx >= (int32_t)max_size) {
          fits = 0, hi = end, lo = idx;
        } else {
          const int32_t shift = start - idx; /* make room below */
          memmove(counts + shift, counts, (size_t)(end - start + 1) * 8);
          memset(counts, 0, (size_t)shift * 8);
          start = idx;
        }
      } else if (idx > end) {
        if (idx - start >= (int32_t)max_size) fits = 0, hi = idx, lo = start;
        else end = idx;
      }
      if (fits) {
        counts[idx - start] += 1;
        break;
      }
      /* changeScale, then merge the buckets pairwise `change` times */
      int32_t change = 0;
      while (hi - lo >= (int32_t)max_size) {
        hi >>= 1;
        lo >>= 1;
        change++;
      }
      const int32_t ns = start >> change, ne = end >> change;
      memset(tmp, 0, (size_t)max_size * 8);
      for (int32_t i = start; i <= end; ++i) tmp[(i >> change) - ns] += counts[i - start];
      memcpy(counts, tmp, (size_t)max_size * 8);
      start = ns;
      end = ne;
      sc -= change;
    }
  }
  free(tmp);
  *scale = sc;
  *offset = have ? start : 0;
  *n_out = have ? (uint32_t)(end - start + 1) : 0;
}
