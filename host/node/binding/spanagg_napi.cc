// spanagg_napi.cc -- Node N-API addon over libspanagg's C-ABI (include/spanagg.h).
//
// This is the "TypeScript (Node N-API addon) calling a thin C-ABI HIP library"
// host of BASELINE.json's north_star: every export is a one-to-one wrapper of an
// sa_* entry point, with typed arrays as the column carriers (BigUint64Array for
// u64 columns, Uint32Array for meta) so a batch crosses into C++ without copies.
// The connector logic (key building, OTLP, temporality) lives in JS
// (lib/connector.js); nothing here aggregates.
//
// Error behaviour mirrors the ABI: a non-zero sa_status becomes a thrown JS
// Error with .code = the status and the engine's sa_last_error() text, except
// flush(), which returns SA_EFULL in .status (the result is still valid), as
// sa_flush does.
#include <algorithm>
#include <node_api.h>

#include <cstdint>
#include <array>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "otlp_columnizer.h"
#include "spanagg.h"

namespace {

napi_value throw_napi(napi_env env, const char *what) {
    const napi_extended_error_info *info = nullptr;
    napi_get_last_error_info(env, &info);
    bool pending = false;
    napi_is_exception_pending(env, &pending);
    if (!pending) {
        std::string msg = std::string("spanagg addon: ") + what;
        if (info && info->error_message) msg += std::string(": ") + info->error_message;
        napi_throw_error(env, nullptr, msg.c_str());
    }
    return nullptr;
}

napi_value throw_status(napi_env env, int rc, const std::string &msg) {
    napi_value m, err, code;
    napi_create_string_utf8(env, msg.c_str(), msg.size(), &m);
    napi_create_error(env, nullptr, m, &err);
    napi_create_int32(env, rc, &code);
    napi_set_named_property(env, err, "code", code);
    napi_throw(env, err);
    return nullptr;
}

napi_value throw_type(napi_env env, const std::string &msg) {
    napi_throw_type_error(env, nullptr, msg.c_str());
    return nullptr;
}

// Engine handle: a JS object wrapping one sa_engine* or one sa_group* (an
// engine per GPU behind the same calls), destroyed by destroy() or, failing
// that, by the GC finalizer.  The ops below dispatch on which one it holds.
struct Handle {
    sa_engine *e = nullptr;
    sa_group *g = nullptr;
    bool live() const { return e || g; }
    void destroy() {
        if (e) sa_destroy(e);
        if (g) sa_group_destroy(g);
        e = nullptr;
        g = nullptr;
    }
    const char *last_error() const { return g ? sa_group_last_error(g) : e ? sa_last_error(e) : ""; }
    int ingest(const sa_span_batch *b) { return g ? sa_group_ingest(g, b) : sa_ingest(e, b); }
    // the columnizer's buffers: an engine reads them by DMA after returning
    // (sa_ingest_async); a group copies them out before returning
    int ingest_async(const sa_span_batch *b) { return g ? sa_group_ingest(g, b) : sa_ingest_async(e, b); }
    int sync() { return g ? sa_group_sync(g) : sa_sync(e); }
    int flush(sa_red_result **r) { return g ? sa_group_flush(g, r) : sa_flush(e, r); }
    int window_read(uint64_t w, sa_sketch_result **r) {
        return g ? sa_group_window_read(g, w, r) : sa_window_read(e, w, r);
    }
    int window_advance(uint64_t b) { return g ? sa_group_window_advance(g, b) : sa_window_advance(e, b); }
    int stats(sa_stats *s) { return g ? sa_group_get_stats(g, s) : sa_get_stats(e, s); }
};

void finalize_handle(napi_env, void *data, void *) {
    auto *h = static_cast<Handle *>(data);
    h->destroy();
    delete h;
}

bool get_args(napi_env env, napi_callback_info info, size_t want, napi_value *argv) {
    size_t argc = want;
    if (napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr) != napi_ok) return false;
    for (size_t i = argc; i < want; ++i) napi_get_undefined(env, &argv[i]);
    return true;
}

Handle *get_handle(napi_env env, napi_value v) {
    void *p = nullptr;
    if (napi_unwrap(env, v, &p) != napi_ok || !p) {
        throw_type(env, "expected a spanagg engine handle");
        return nullptr;
    }
    auto *h = static_cast<Handle *>(p);
    if (!h->live()) {
        throw_status(env, SA_ESTATE, "engine already destroyed");
        return nullptr;
    }
    return h;
}

napi_value engine_error(napi_env env, Handle *h, int rc, const char *what) {
    std::string msg = std::string(what) + ": " + (h ? h->last_error() : "");
    return throw_status(env, rc, msg);
}

// ---- value helpers -------------------------------------------------------

bool is_undefined(napi_env env, napi_value v) {
    napi_valuetype t;
    return napi_typeof(env, v, &t) != napi_ok || t == napi_undefined || t == napi_null;
}

// Number or BigInt -> u64 (throws on other types, negatives and lossy values)
bool to_u64(napi_env env, napi_value v, uint64_t *out, const char *name) {
    napi_valuetype t;
    napi_typeof(env, v, &t);
    if (t == napi_bigint) {
        bool lossless = false;
        napi_get_value_bigint_uint64(env, v, out, &lossless);
        if (!lossless) {
            throw_type(env, std::string(name) + ": BigInt out of u64 range");
            return false;
        }
        return true;
    }
    if (t == napi_number) {
        double d;
        napi_get_value_double(env, v, &d);
        if (!(d >= 0) || d > 9007199254740991.0 ||
            d != static_cast<double>(static_cast<uint64_t>(d))) {
            throw_type(env, std::string(name) + ": expected a non-negative integer");
            return false;
        }
        *out = static_cast<uint64_t>(d);
        return true;
    }
    throw_type(env, std::string(name) + ": expected a number or BigInt");
    return false;
}

bool to_u32(napi_env env, napi_value v, uint32_t *out, const char *name) {
    uint64_t x;
    if (!to_u64(env, v, &x, name)) return false;
    if (x > 0xFFFFFFFFull) {
        throw_type(env, std::string(name) + ": out of u32 range");
        return false;
    }
    *out = static_cast<uint32_t>(x);
    return true;
}

napi_value num(napi_env env, double d) {
    napi_value v;
    napi_create_double(env, d, &v);
    return v;
}

napi_value big(napi_env env, uint64_t x) {
    napi_value v;
    napi_create_bigint_uint64(env, x, &v);
    return v;
}

void set(napi_env env, napi_value obj, const char *k, napi_value v) {
    napi_set_named_property(env, obj, k, v);
}

// Typed-array view of one element type; *len = element count.
bool typed(napi_env env, napi_value v, napi_typedarray_type want, void **data, size_t *len,
           const char *name) {
    static const char *names[] = {"Int8Array",    "Uint8Array",    "Uint8ClampedArray",
                                  "Int16Array",   "Uint16Array",   "Int32Array",
                                  "Uint32Array",  "Float32Array",  "Float64Array",
                                  "BigInt64Array", "BigUint64Array"};
    bool is = false;
    napi_is_typedarray(env, v, &is);
    napi_typedarray_type t;
    napi_value ab;
    size_t off;
    if (!is || napi_get_typedarray_info(env, v, &t, len, data, &ab, &off) != napi_ok || t != want) {
        throw_type(env, std::string(name) + ": expected a " + names[want]);
        return false;
    }
    return true;
}

// Fresh typed array holding a copy of n elements of src.
napi_value make_typed(napi_env env, napi_typedarray_type t, size_t elem, const void *src, size_t n) {
    void *dst = nullptr;
    napi_value ab, arr;
    if (napi_create_arraybuffer(env, n * elem, &dst, &ab) != napi_ok) return nullptr;
    if (n) std::memcpy(dst, src, n * elem);
    if (napi_create_typedarray(env, t, n, ab, 0, &arr) != napi_ok) return nullptr;
    return arr;
}

napi_value prop(napi_env env, napi_value obj, const char *k) {
    napi_value v = nullptr;
    bool has = false;
    if (is_undefined(env, obj) || napi_has_named_property(env, obj, k, &has) != napi_ok || !has) {
        napi_get_undefined(env, &v);
        return v;
    }
    napi_get_named_property(env, obj, k, &v);
    return v;
}

bool read_bounds(napi_env env, napi_value v, std::vector<double> *out) {
    bool is_arr = false;
    napi_is_array(env, v, &is_arr);
    if (is_arr) {
        uint32_t n;
        napi_get_array_length(env, v, &n);
        out->resize(n);
        for (uint32_t i = 0; i < n; ++i) {
            napi_value x;
            napi_get_element(env, v, i, &x);
            if (napi_get_value_double(env, x, &(*out)[i]) != napi_ok) {
                throw_type(env, "bounds: expected numbers");
                return false;
            }
        }
        return true;
    }
    void *d;
    size_t n;
    if (!typed(env, v, napi_float64_array, &d, &n, "bounds")) return false;
    out->assign(static_cast<double *>(d), static_cast<double *>(d) + n);
    return true;
}

bool read_unit(napi_env env, napi_value v, uint32_t *unit) {
    if (is_undefined(env, v)) {
        *unit = SA_UNIT_MS;
        return true;
    }
    char buf[8] = {0};
    size_t n = 0;
    if (napi_get_value_string_utf8(env, v, buf, sizeof buf, &n) != napi_ok ||
        (std::strcmp(buf, "ms") != 0 && std::strcmp(buf, "s") != 0)) {
        throw_type(env, "unit: expected 'ms' or 's'");
        return false;
    }
    *unit = buf[0] == 's' ? SA_UNIT_S : SA_UNIT_MS;
    return true;
}

// ---- exports -------------------------------------------------------------

napi_value AbiVersion(napi_env env, napi_callback_info) { return num(env, sa_abi_version()); }

// createDefaultConfig, as a plain object (bounds in the histogram unit)
napi_value ConfigDefault(napi_env env, napi_callback_info) {
    sa_config c;
    sa_config_default(&c);
    napi_value o, bounds, unit;
    if (napi_create_object(env, &o) != napi_ok ||
        napi_create_array_with_length(env, c.n_bounds, &bounds) != napi_ok)
        return throw_napi(env, "configDefault");
    for (uint32_t i = 0; i < c.n_bounds; ++i) napi_set_element(env, bounds, i, num(env, c.bounds[i]));
    set(env, o, "bounds", bounds);
    napi_create_string_utf8(env, c.unit == SA_UNIT_S ? "s" : "ms", NAPI_AUTO_LENGTH, &unit);
    set(env, o, "unit", unit);
    set(env, o, "hllP", num(env, c.hll_p));
    set(env, o, "cmsD", num(env, c.cms_d));
    set(env, o, "cmsW", num(env, c.cms_w));
    set(env, o, "windowNs", big(env, c.window_ns));
    set(env, o, "nWindows", num(env, c.n_windows));
    set(env, o, "nServices", num(env, c.n_services));
    set(env, o, "keyCapacity", num(env, static_cast<double>(c.key_capacity)));
    set(env, o, "device", num(env, c.device));
    set(env, o, "flags", num(env, c.flags));
    set(env, o, "options", num(env, c.options));
    return o;
}

// bucketThresholds(bounds, unit) -> {thresholds: BigUint64Array, nNeg}
napi_value BucketThresholds(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return throw_napi(env, "args");
    std::vector<double> b;
    uint32_t unit;
    if (!read_bounds(env, argv[0], &b) || !read_unit(env, argv[1], &unit)) return nullptr;
    std::vector<uint64_t> thr(b.size() + 1);
    uint32_t nneg = 0;
    int rc = sa_bucket_thresholds(b.data(), static_cast<uint32_t>(b.size()), unit, thr.data(), &nneg);
    if (rc != SA_OK) return throw_status(env, rc, "invalid histogram bounds");
    napi_value o;
    if (napi_create_object(env, &o) != napi_ok) return throw_napi(env, "bucketThresholds");
    set(env, o, "thresholds", make_typed(env, napi_biguint64_array, 8, thr.data(), b.size() - nneg));
    set(env, o, "nNeg", num(env, nneg));
    return o;
}

// hllEstimate(Uint8Array regs, p) -> number
napi_value HllEstimate(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return throw_napi(env, "args");
    void *d;
    size_t n;
    uint32_t p;
    if (!typed(env, argv[0], napi_uint8_array, &d, &n, "regs") || !to_u32(env, argv[1], &p, "p"))
        return nullptr;
    if (p < 4 || p > 18 || n != (size_t(1) << p))
        return throw_status(env, SA_EINVAL, "hllEstimate: regs.length must be 2^p, 4 <= p <= 18");
    return num(env, sa_hll_estimate(static_cast<const uint8_t *>(d), p));
}

// create(config) -> handle.  Missing fields take createDefaultConfig values.
napi_value Create(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_napi(env, "args");
    sa_config c;
    sa_config_default(&c);
    std::vector<double> bounds(c.bounds, c.bounds + c.n_bounds);
    napi_value cfg = argv[0], v;
    if (!is_undefined(env, v = prop(env, cfg, "bounds")) && !read_bounds(env, v, &bounds)) return nullptr;
    if (!read_unit(env, prop(env, cfg, "unit"), &c.unit)) return nullptr;
    struct U32Field {
        const char *k;
        uint32_t *dst;
    } u32s[] = {{"hllP", &c.hll_p},         {"cmsD", &c.cms_d},
                {"cmsW", &c.cms_w},         {"nWindows", &c.n_windows},
                {"nServices", &c.n_services}, {"flags", &c.flags},
                {"expMaxSize", &c.exp_max_size}, {"options", &c.options}};
    for (auto &f : u32s)
        if (!is_undefined(env, v = prop(env, cfg, f.k)) && !to_u32(env, v, f.dst, f.k)) return nullptr;
    if (!is_undefined(env, v = prop(env, cfg, "windowNs")) && !to_u64(env, v, &c.window_ns, "windowNs"))
        return nullptr;
    if (!is_undefined(env, v = prop(env, cfg, "keyCapacity")) &&
        !to_u64(env, v, &c.key_capacity, "keyCapacity"))
        return nullptr;
    if (!is_undefined(env, v = prop(env, cfg, "device"))) {
        uint32_t dev = 0;
        if (!to_u32(env, v, &dev, "device")) return nullptr;
        c.device = static_cast<int32_t>(dev);
    }
    c.bounds = bounds.data();
    c.n_bounds = static_cast<uint32_t>(bounds.size());
    // devices: [d0, d1, ...] -> an engine group (one engine per entry, spans
    // sharded by trace id, merged at flush / window read)
    std::vector<int32_t> devs;
    if (!is_undefined(env, v = prop(env, cfg, "devices"))) {
        bool arr = false;
        napi_is_array(env, v, &arr);
        uint32_t len = 0;
        if (!arr || napi_get_array_length(env, v, &len) != napi_ok || len == 0)
            return throw_type(env, "devices: expected a non-empty array of device ordinals");
        for (uint32_t i = 0; i < len; ++i) {
            napi_value x;
            uint32_t d = 0;
            napi_get_element(env, v, i, &x);
            if (!to_u32(env, x, &d, "devices[]")) return nullptr;
            devs.push_back(static_cast<int32_t>(d));
        }
    }
    auto *h = new Handle();
    int rc = devs.empty() ? sa_create(&c, &h->e)
                          : sa_group_create(&c, devs.data(), static_cast<uint32_t>(devs.size()), &h->g);
    if (rc != SA_OK || !h->live()) {
        delete h;
        return throw_status(env, rc ? rc : SA_EDEVICE,
                            devs.empty() ? "sa_create failed (invalid config, or no gfx950 GPU visible)"
                                         : "sa_group_create failed (invalid config, or no gfx950 GPU visible)");
    }
    napi_value obj;
    if (napi_create_object(env, &obj) != napi_ok ||
        napi_wrap(env, obj, h, finalize_handle, nullptr, nullptr) != napi_ok) {
        h->destroy();
        delete h;
        return throw_napi(env, "napi_wrap");
    }
    return obj;
}

napi_value Destroy(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_napi(env, "args");
    void *p = nullptr;
    if (napi_unwrap(env, argv[0], &p) == napi_ok && p) {
        static_cast<Handle *>(p)->destroy();
    }
    return nullptr;
}

napi_value LastError(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_napi(env, "args");
    Handle *h = get_handle(env, argv[0]);
    if (!h) return nullptr;
    napi_value s;
    napi_create_string_utf8(env, h->last_error(), NAPI_AUTO_LENGTH, &s);
    return s;
}

// ingest(h, {keyHash, startNs, endNs, traceW0, traceW1: BigUint64Array, meta: Uint32Array}):
// ConsumeTraces' per-span body for one columnar batch in host memory (the
// library stages it to HBM and launches the ingest kernel).
napi_value Ingest(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return throw_napi(env, "args");
    Handle *h = get_handle(env, argv[0]);
    if (!h) return nullptr;
    static const char *cols[] = {"keyHash", "startNs", "endNs", "traceW0", "traceW1"};
    const uint64_t *p64[5];
    size_t n = 0;
    for (int i = 0; i < 5; ++i) {
        void *d;
        size_t len;
        if (!typed(env, prop(env, argv[1], cols[i]), napi_biguint64_array, &d, &len, cols[i]))
            return nullptr;
        if (i == 0) n = len;
        else if (len != n) return throw_status(env, SA_EINVAL, "ingest: ragged SoA batch");
        p64[i] = static_cast<const uint64_t *>(d);
    }
    void *md;
    size_t mlen;
    if (!typed(env, prop(env, argv[1], "meta"), napi_uint32_array, &md, &mlen, "meta")) return nullptr;
    if (mlen != n) return throw_status(env, SA_EINVAL, "ingest: ragged SoA batch");
    sa_span_batch b{p64[0], p64[1], p64[2], p64[3], p64[4], static_cast<const uint32_t *>(md), n};
    int rc = h->ingest(&b);
    if (rc != SA_OK) return engine_error(env, h, rc, "sa_ingest");
    return nullptr;
}

napi_value Sync(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_napi(env, "args");
    Handle *h = get_handle(env, argv[0]);
    if (!h) return nullptr;
    int rc = h->sync();
    if (rc != SA_OK) return engine_error(env, h, rc, "sa_sync");
    return nullptr;
}

// flush(h) -> {status, nSeries, nBuckets, keyHash, bucketCounts [n*nb], calls, sumNs, sum}
napi_value Flush(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_napi(env, "args");
    Handle *h = get_handle(env, argv[0]);
    if (!h) return nullptr;
    sa_red_result *r = nullptr;
    int rc = h->flush(&r);
    if ((rc != SA_OK && rc != SA_EFULL) || !r) {
        if (r) sa_red_result_free(r);
        return engine_error(env, h, rc ? rc : SA_ESTATE, "sa_flush");
    }
    const size_t n = r->n_series, nb = r->n_buckets;
    napi_value o;
    if (napi_create_object(env, &o) != napi_ok) {
        sa_red_result_free(r);
        return throw_napi(env, "napi_create_object");
    }
    set(env, o, "status", num(env, rc));
    set(env, o, "nSeries", num(env, static_cast<double>(n)));
    set(env, o, "nBuckets", num(env, static_cast<double>(nb)));
    set(env, o, "keyHash", make_typed(env, napi_biguint64_array, 8, r->key_hash, n));
    set(env, o, "bucketCounts", make_typed(env, napi_biguint64_array, 8, r->bucket_counts, n * nb));
    set(env, o, "calls", make_typed(env, napi_biguint64_array, 8, r->calls, n));
    set(env, o, "sumNs", make_typed(env, napi_biguint64_array, 8, r->sum_ns, n));
    set(env, o, "sum", make_typed(env, napi_float64_array, 8, r->sum, n));
    sa_red_result_free(r);
    return o;
}

// flushExp(h) -> {status, nSeries, maxSize, keyHash, count, zeroCount, sumNs,
// sum, min, max, scale, offset, nBuckets, bucketCounts [n*maxSize]}
// (exponential-histogram engines; groups merge explicit buckets only)
napi_value FlushExp(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_napi(env, "args");
    Handle *h = get_handle(env, argv[0]);
    if (!h) return nullptr;
    sa_exp_result *r = nullptr;
    int rc = h->e ? sa_flush_exp(h->e, &r) : sa_group_flush_exp(h->g, &r);
    if ((rc != SA_OK && rc != SA_EFULL) || !r) {
        if (r) sa_exp_result_free(r);
        return engine_error(env, h, rc ? rc : SA_ESTATE, h->e ? "sa_flush_exp" : "sa_group_flush_exp");
    }
    const size_t n = r->n_series, m = r->max_size;
    napi_value o;
    napi_create_object(env, &o);
    set(env, o, "status", num(env, rc));
    set(env, o, "nSeries", num(env, static_cast<double>(n)));
    set(env, o, "maxSize", num(env, static_cast<double>(m)));
    set(env, o, "keyHash", make_typed(env, napi_biguint64_array, 8, r->key_hash, n));
    set(env, o, "count", make_typed(env, napi_biguint64_array, 8, r->count, n));
    set(env, o, "zeroCount", make_typed(env, napi_biguint64_array, 8, r->zero_count, n));
    set(env, o, "sumNs", make_typed(env, napi_biguint64_array, 8, r->sum_ns, n));
    set(env, o, "sum", make_typed(env, napi_float64_array, 8, r->sum, n));
    set(env, o, "min", make_typed(env, napi_float64_array, 8, r->min, n));
    set(env, o, "max", make_typed(env, napi_float64_array, 8, r->max, n));
    set(env, o, "scale", make_typed(env, napi_int32_array, 4, r->scale, n));
    set(env, o, "offset", make_typed(env, napi_int32_array, 4, r->offset, n));
    set(env, o, "nBuckets", make_typed(env, napi_uint32_array, 4, r->n_buckets, n));
    set(env, o, "bucketCounts", make_typed(env, napi_biguint64_array, 8, r->bucket_counts, n * m));
    sa_exp_result_free(r);
    return o;
}

// windowRead(h, windowId) -> {windowId, nServices, hllP, hll, cmsD, cmsW, cms}
napi_value WindowRead(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return throw_napi(env, "args");
    Handle *h = get_handle(env, argv[0]);
    uint64_t wid;
    if (!h || !to_u64(env, argv[1], &wid, "windowId")) return nullptr;
    sa_sketch_result *r = nullptr;
    int rc = h->window_read(wid, &r);
    if (rc != SA_OK || !r) {
        if (r) sa_sketch_result_free(r);
        return engine_error(env, h, rc ? rc : SA_ESTATE, "sa_window_read");
    }
    napi_value o;
    if (napi_create_object(env, &o) != napi_ok) {
        sa_sketch_result_free(r);
        return throw_napi(env, "napi_create_object");
    }
    set(env, o, "windowId", big(env, r->window_id));
    set(env, o, "nServices", num(env, r->n_services));
    set(env, o, "hllP", num(env, r->hll_p));
    set(env, o, "hll",
        make_typed(env, napi_uint8_array, 1, r->hll, size_t(r->n_services) << r->hll_p));
    set(env, o, "cmsD", num(env, r->cms_d));
    set(env, o, "cmsW", num(env, r->cms_w));
    set(env, o, "cms", make_typed(env, napi_uint32_array, 4, r->cms, size_t(r->cms_d) * r->cms_w));
    sa_sketch_result_free(r);
    return o;
}

napi_value WindowAdvance(napi_env env, napi_callback_info info) {
    napi_value argv[2];
    if (!get_args(env, info, 2, argv)) return throw_napi(env, "args");
    Handle *h = get_handle(env, argv[0]);
    uint64_t base;
    if (!h || !to_u64(env, argv[1], &base, "newBase")) return nullptr;
    int rc = h->window_advance(base);
    if (rc != SA_OK) return engine_error(env, h, rc, "sa_window_advance");
    return nullptr;
}

napi_value Stats(napi_env env, napi_callback_info info) {
    napi_value argv[1];
    if (!get_args(env, info, 1, argv)) return throw_napi(env, "args");
    Handle *h = get_handle(env, argv[0]);
    if (!h) return nullptr;
    sa_stats s;
    int rc = h->stats(&s);
    if (rc != SA_OK) return engine_error(env, h, rc, "sa_get_stats");
    napi_value o, b;
    if (napi_create_object(env, &o) != napi_ok) return throw_napi(env, "napi_create_object");
    set(env, o, "spans", big(env, s.spans));
    set(env, o, "zeroKey", big(env, s.zero_key));
    set(env, o, "invalidService", big(env, s.invalid_service));
    set(env, o, "windowOutOfRange", big(env, s.window_out_of_range));
    set(env, o, "droppedTableFull", big(env, s.dropped_table_full));
    set(env, o, "nKeys", big(env, s.n_keys));
    set(env, o, "tableCapacity", big(env, s.table_capacity));
    set(env, o, "windowBase", big(env, s.window_base));
    set(env, o, "hllFiltered", big(env, s.hll_filtered));
    napi_get_boolean(env, s.small_table != 0, &b);
    set(env, o, "smallTable", b);
    set(env, o, "engines", num(env, h->g ? sa_group_size(h->g) : 1));
    napi_get_boolean(env, h->g && sa_group_uses_rccl(h->g), &b);
    set(env, o, "rccl", b);
    return o;
}

// ---- native OTLP columnizer (otlp_columnizer.h) ----------------------------
//
// createColumnizer(engine, {dims, exclude, rules, keyAttributes}) -> columnizer
// columnize(c, Buffer) -> {status, error, spans, buffered, maxEnd, resources,
//                          newResources, newSeries, newServices}
// columnizerIngest(c)           sa_ingest of the buffered columns, then clear
// columnizerTake(c)             the buffered columns as typed arrays, then clear
// columnizerServiceId(c, name)  -> [id, isNew]
// columnizerForget(c, resHash)  drop a resource's key cache (LRU eviction)

struct ColHandle {
  otlpcol::Columnizer col;
  napi_ref engine_ref = nullptr;  // keeps the engine handle object alive
  Handle *engine = nullptr;
  explicit ColHandle(otlpcol::Options o) : col(std::move(o)) {}
};

void finalize_col(napi_env env, void *data, void *) {
  // (its pinned column buffers may still be read by an sa_ingest_async DMA:
  // sa_host_free -> hipHostFree synchronizes the device before freeing; the
  // engine handle itself may already be finalized here, so it is not used)
  auto *c = static_cast<ColHandle *>(data);
  if (c->engine_ref) napi_delete_reference(env, c->engine_ref);
  delete c;
}

ColHandle *get_col(napi_env env, napi_value v) {
  void *p = nullptr;
  napi_valuetype t;
  if (napi_typeof(env, v, &t) != napi_ok || t != napi_object || napi_unwrap(env, v, &p) != napi_ok || !p) {
    throw_type(env, "expected a columnizer");
    return nullptr;
  }
  return static_cast<ColHandle *>(p);
}

bool get_string(napi_env env, napi_value v, std::string *out, const char *name) {
  size_t n = 0;
  if (napi_get_value_string_utf8(env, v, nullptr, 0, &n) != napi_ok) {
    throw_type(env, std::string(name) + ": expected a string");
    return false;
  }
  out->resize(n);
  napi_get_value_string_utf8(env, v, &(*out)[0], n + 1, &n);
  return true;
}

bool array_items(napi_env env, napi_value v, std::vector<napi_value> *out, const char *name) {
  out->clear();
  if (is_undefined(env, v)) return true;
  bool is = false;
  napi_is_array(env, v, &is);
  if (!is) {
    throw_type(env, std::string(name) + ": expected an array");
    return false;
  }
  uint32_t n = 0;
  napi_get_array_length(env, v, &n);
  for (uint32_t i = 0; i < n; ++i) {
    napi_value x;
    napi_get_element(env, v, i, &x);
    out->push_back(x);
  }
  return true;
}

napi_value CreateColumnizer(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return throw_napi(env, "args");
  // engine: a handle from create(), or null for a columnizer that is only
  // drained with columnizerTake (tests, non-GPU consumers)
  void *hp = nullptr;
  const bool no_engine = is_undefined(env, argv[0]);
  if (!no_engine && (napi_unwrap(env, argv[0], &hp) != napi_ok || !hp))
    return throw_type(env, "expected a spanagg engine handle or null");
  otlpcol::Options o;
  std::vector<napi_value> items;
  if (!array_items(env, prop(env, argv[1], "dims"), &items, "dims")) return nullptr;
  for (napi_value d : items) {
    otlpcol::Dim dim;
    if (!get_string(env, prop(env, d, "name"), &dim.name, "dims[].name")) return nullptr;
    napi_value def = prop(env, d, "default");
    if (!is_undefined(env, def)) {
      dim.has_default = true;
      if (!get_string(env, def, &dim.def, "dims[].default")) return nullptr;
    }
    o.dims.push_back(std::move(dim));
  }
  if (!array_items(env, prop(env, argv[1], "exclude"), &items, "exclude")) return nullptr;
  for (napi_value x : items) {
    std::string k;
    if (!get_string(env, x, &k, "exclude[]")) return nullptr;
    if (k == "service.name") o.ex_service = true;
    else if (k == "span.name") o.ex_name = true;
    else if (k == "span.kind") o.ex_kind = true;
    else if (k == "status.code") o.ex_status = true;
  }
  if (!array_items(env, prop(env, argv[1], "rules"), &items, "rules")) return nullptr;
  for (napi_value x : items) {
    otlpcol::Rule r;
    std::string kind;
    if (!get_string(env, prop(env, x, "kind"), &kind, "rules[].kind")) return nullptr;
    if (kind == "strip_query") {
      r.kind = otlpcol::Rule::kStripQuery;
    } else if (kind == "glob") {
      r.kind = otlpcol::Rule::kGlob;
      if (!get_string(env, prop(env, x, "pattern"), &r.pattern, "rules[].pattern") ||
          !get_string(env, prop(env, x, "replacement"), &r.replacement, "rules[].replacement"))
        return nullptr;
      r.prepare();
    } else {
      return throw_status(env, SA_EINVAL, "rules[].kind must be strip_query or glob");
    }
    o.rules.push_back(std::move(r));
  }
  if (!array_items(env, prop(env, argv[1], "keyAttributes"), &items, "keyAttributes")) return nullptr;
  for (napi_value x : items) {
    std::string k;
    if (!get_string(env, x, &k, "keyAttributes[]")) return nullptr;
    o.key_attributes.push_back(std::move(k));
  }
  {
    napi_value tc = prop(env, argv[1], "testCollideSeed0");
    bool b = false;
    if (!is_undefined(env, tc)) napi_get_value_bool(env, tc, &b);
    o.test_collide_seed0 = b;
    napi_value tb = prop(env, argv[1], "testBatched");
    b = false;
    if (!is_undefined(env, tb)) napi_get_value_bool(env, tb, &b);
    o.test_batched = b;
  }
  {  // aggregation_cardinality_limit, exemplars, events (connector.js normalizeConfig)
    napi_value v = prop(env, argv[1], "cardinalityLimit");
    uint32_t u = 0;
    if (!is_undefined(env, v) && napi_get_value_uint32(env, v, &u) != napi_ok)
      return throw_type(env, "cardinalityLimit must be a number");
    o.card_limit = u;
    bool b = false;
    v = prop(env, argv[1], "exemplars");
    if (!is_undefined(env, v)) napi_get_value_bool(env, v, &b);
    o.exemplars = b;
    v = prop(env, argv[1], "exemplarsMax");
    u = 5;
    if (!is_undefined(env, v) && napi_get_value_uint32(env, v, &u) != napi_ok)
      return throw_type(env, "exemplarsMax must be a number");
    o.exemplars_max = u;
    b = false;
    v = prop(env, argv[1], "events");
    if (!is_undefined(env, v)) napi_get_value_bool(env, v, &b);
    o.events = b;
    v = prop(env, argv[1], "eventDims");
    if (!is_undefined(env, v)) {
      if (!array_items(env, v, &items, "eventDims")) return nullptr;
      for (napi_value d : items) {
        otlpcol::Dim dim;
        if (!get_string(env, prop(env, d, "name"), &dim.name, "eventDims[].name")) return nullptr;
        napi_value def = prop(env, d, "default");
        if (!is_undefined(env, def)) {
          dim.has_default = true;
          if (!get_string(env, def, &dim.def, "eventDims[].default")) return nullptr;
        }
        o.event_dims.push_back(std::move(dim));
      }
    }
  }
  {
    napi_value th = prop(env, argv[1], "threads");
    uint32_t t = 1;
    if (!is_undefined(env, th) && napi_get_value_uint32(env, th, &t) != napi_ok)
      return throw_type(env, "threads must be a number");
    o.threads = std::max(1u, std::min(t, 64u));
  }
  auto *c = new ColHandle(std::move(o));
  c->engine = static_cast<Handle *>(hp);
  napi_value obj;
  if (napi_create_object(env, &obj) != napi_ok ||
      (!no_engine && napi_create_reference(env, argv[0], 1, &c->engine_ref) != napi_ok) ||
      napi_wrap(env, obj, c, finalize_col, nullptr, nullptr) != napi_ok) {
    if (c->engine_ref) napi_delete_reference(env, c->engine_ref);
    delete c;
    return throw_napi(env, "createColumnizer");
  }
  return obj;
}

// one columnize result; `lean` (a batch's requests) leaves out empty reports
napi_value result_obj(napi_env env, const otlpcol::Result &r, bool lean) {
  napi_value o, arr, s;
  if (napi_create_object(env, &o) != napi_ok) return nullptr;
  const char *st = r.status == otlpcol::Result::kOk ? "ok" : r.status == otlpcol::Result::kFallback ? "fallback" : "error";
  napi_create_string_utf8(env, st, NAPI_AUTO_LENGTH, &s);
  set(env, o, "status", s);
  if (!lean || !r.error.empty()) {
    napi_create_string_utf8(env, r.error.c_str(), NAPI_AUTO_LENGTH, &s);
    set(env, o, "error", s);
  }
  set(env, o, "spans", num(env, (double)r.spans));
  set(env, o, "resources", make_typed(env, napi_biguint64_array, 8, r.resources.data(), r.resources.size()));
  if (!lean || !r.new_resources.empty()) {
    napi_create_array_with_length(env, r.new_resources.size(), &arr);
    for (size_t i = 0; i < r.new_resources.size(); ++i) {
      napi_value e;
      napi_create_object(env, &e);
      set(env, e, "hash", big(env, r.new_resources[i].hash));
      set(env, e, "off", num(env, (double)r.new_resources[i].off));
      set(env, e, "len", num(env, r.new_resources[i].len));
      napi_set_element(env, arr, (uint32_t)i, e);
    }
    set(env, o, "newResources", arr);
  }
  if (!lean || !r.new_series.empty()) {
    napi_create_array_with_length(env, r.new_series.size(), &arr);
    for (size_t i = 0; i < r.new_series.size(); ++i) {
      napi_value e;
      napi_create_object(env, &e);
      set(env, e, "sid", big(env, r.new_series[i].sid));
      set(env, e, "resHash", big(env, r.new_series[i].res_hash));
      set(env, e, "off", num(env, r.new_series[i].span_off));
      set(env, e, "len", num(env, r.new_series[i].span_len));
      set(env, e, "resOff", num(env, (double)r.new_series[i].res_off));
      set(env, e, "resLen", num(env, r.new_series[i].res_len));
      napi_set_element(env, arr, (uint32_t)i, e);
    }
    set(env, o, "newSeries", arr);
  }
  if (!lean || !r.exemplars.empty()) {
    napi_create_array_with_length(env, r.exemplars.size(), &arr);
    // the exemplars' ids as views of one buffer (the host keeps them as is)
    napi_value ab = nullptr;
    uint8_t *abd = nullptr;
    if (!r.exemplars.empty()) napi_create_arraybuffer(env, 24 * r.exemplars.size(), (void **)&abd, &ab);
    for (size_t i = 0; i < r.exemplars.size(); ++i) {
      const otlpcol::SpanRef &x = r.exemplars[i];
      napi_value e;
      napi_create_object(env, &e);
      set(env, e, "sid", big(env, x.sid));
      set(env, e, "off", num(env, x.span_off));
      set(env, e, "len", num(env, x.span_len));
      if (x.ids_ok && abd) {  // else the host decodes the span from off / len
        std::memcpy(abd + 24 * i, x.ids, 24);
        napi_value tv, sv;
        napi_create_typedarray(env, napi_uint8_array, 16, ab, 24 * i, &tv);
        napi_create_typedarray(env, napi_uint8_array, 8, ab, 24 * i + 16, &sv);
        set(env, e, "traceId", tv);
        set(env, e, "spanId", sv);
        set(env, e, "start", big(env, x.start));
        set(env, e, "end", big(env, x.end));
      }
      napi_set_element(env, arr, (uint32_t)i, e);
    }
    set(env, o, "exemplars", arr);
  }
  if (!lean || !r.new_event_series.empty()) {
    napi_create_array_with_length(env, r.new_event_series.size(), &arr);
    for (size_t i = 0; i < r.new_event_series.size(); ++i) {
      napi_value e;
      napi_create_object(env, &e);
      set(env, e, "sid", big(env, r.new_event_series[i].sid));
      set(env, e, "resHash", big(env, r.new_event_series[i].res_hash));
      set(env, e, "off", num(env, r.new_event_series[i].span_off));
      set(env, e, "len", num(env, r.new_event_series[i].span_len));
      set(env, e, "event", num(env, r.new_event_series[i].event));
      set(env, e, "resOff", num(env, (double)r.new_event_series[i].res_off));
      set(env, e, "resLen", num(env, r.new_event_series[i].res_len));
      napi_set_element(env, arr, (uint32_t)i, e);
    }
    set(env, o, "newEventSeries", arr);
  }
  if (!lean || r.event_records) set(env, o, "eventRecords", num(env, (double)r.event_records));
  if (!lean || !r.new_services.empty()) {
    napi_create_array_with_length(env, r.new_services.size(), &arr);
    for (size_t i = 0; i < r.new_services.size(); ++i) {
      napi_value e, nm;
      napi_create_array_with_length(env, 2, &e);
      napi_create_string_utf8(env, r.new_services[i].first.c_str(), r.new_services[i].first.size(), &nm);
      napi_set_element(env, e, 0, nm);
      napi_set_element(env, e, 1, num(env, r.new_services[i].second));
      napi_set_element(env, arr, (uint32_t)i, e);
    }
    set(env, o, "newServices", arr);
  }
  return o;
}

napi_value Columnize(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return throw_napi(env, "args");
  ColHandle *c = get_col(env, argv[0]);
  if (!c) return nullptr;
  void *data;
  size_t len;
  if (!typed(env, argv[1], napi_uint8_array, &data, &len, "request")) return nullptr;
  otlpcol::Result r = c->col.columnize(static_cast<const uint8_t *>(data), len);
  napi_value o = result_obj(env, r, false);
  if (!o) return throw_napi(env, "napi_create_object");
  set(env, o, "buffered", num(env, (double)c->col.buffered()));
  set(env, o, "maxEnd", big(env, c->col.max_end()));
  return o;
}

// columnizeBatch(c, [request bytes...]) -> {done, buffered, maxEnd, results}:
// the requests decoded on the columnizer's threads, committed in order; it
// stops after the first fallback (results[done - 1]), the caller passes the rest again
napi_value ColumnizeBatch(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return throw_napi(env, "args");
  ColHandle *c = get_col(env, argv[0]);
  if (!c) return nullptr;
  using clk = std::chrono::steady_clock;
  const auto t_in = clk::now();
  std::vector<napi_value> items;
  if (!array_items(env, argv[1], &items, "requests")) return nullptr;
  std::vector<const uint8_t *> bufs(items.size());
  std::vector<size_t> lens(items.size());
  for (size_t i = 0; i < items.size(); ++i) {
    void *data;
    if (!typed(env, items[i], napi_uint8_array, &data, &lens[i], "requests[]")) return nullptr;
    bufs[i] = static_cast<const uint8_t *>(data);
  }
  const auto t_cb = clk::now();
  otlpcol::BatchResult br = c->col.columnize_batch(bufs.data(), lens.data(), items.size());
  const auto t_out = clk::now();
  // Most requests of a steady stream bring nothing new: status ok, no new
  // services / resources / series, no exemplars or event series.  Those get
  // no result object; what the host must still see of them -- the resources
  // they touched, for its LRU -- comes as one list per gap between the
  // requests that do get one, each resource once, in order of last touch
  // (nothing is admitted to the LRU inside a gap, so that order is the one
  // request-at-a-time touches leave).
  //   results[i]: the request's result object, or undefined (a plain one)
  //   touch: resource hashes; touchEnd[k]: the end of the gap before the k-th
  //   result object (the last gap ends at touch.length)
  auto plain = [](const otlpcol::Result &r) {
    return r.status == otlpcol::Result::kOk && r.new_resources.empty() && r.new_series.empty() &&
           r.new_services.empty() && r.exemplars.empty() && r.new_event_series.empty();
  };
  std::vector<uint64_t> touch;
  std::vector<uint32_t> touch_end;
  size_t gap0 = 0;  // where the current gap starts in `touch`
  uint64_t spans = 0, plain_events = 0;
  for (const auto &r : br.results) {
    spans += r.spans;
    if (plain(r)) plain_events += r.event_records;
    if (!plain(r)) {
      touch_end.push_back((uint32_t)touch.size());
      gap0 = touch.size();
      continue;
    }
    for (uint64_t h : r.resources) {  // move to the back of the gap's list
      auto it = std::find(touch.begin() + gap0, touch.end(), h);
      if (it != touch.end()) touch.erase(it);
      touch.push_back(h);
    }
  }
  napi_value o, arr;
  if (napi_create_object(env, &o) != napi_ok) return throw_napi(env, "napi_create_object");
  set(env, o, "done", num(env, (double)br.done));
  set(env, o, "buffered", num(env, (double)c->col.buffered()));
  set(env, o, "maxEnd", big(env, c->col.max_end()));
  set(env, o, "spans", num(env, (double)spans));
  set(env, o, "plainEventRecords", num(env, (double)plain_events));  // event records of the plain requests
  // wall ns of columnize_batch's phases (threaded calls): decode, commit,
  // place; then this call's own argument unpacking and (so far) result building
  const auto ns = [](clk::duration d) { return (double)std::chrono::duration_cast<std::chrono::nanoseconds>(d).count(); };
  set(env, o, "phaseNs", make_typed(env, napi_float64_array, 8,
                                    std::array<double, 5>{(double)br.ns_decode, (double)br.ns_commit,
                                                          (double)br.ns_place, ns(t_cb - t_in),
                                                          ns(clk::now() - t_out)}.data(), 5));
  set(env, o, "touch", make_typed(env, napi_biguint64_array, 8, touch.data(), touch.size()));
  set(env, o, "touchEnd", make_typed(env, napi_uint32_array, 4, touch_end.data(), touch_end.size()));
  napi_create_array_with_length(env, br.results.size(), &arr);
  for (size_t i = 0; i < br.results.size(); ++i) {
    if (plain(br.results[i])) continue;
    napi_value e = result_obj(env, br.results[i], true);
    if (!e) return throw_napi(env, "napi_create_object");
    napi_set_element(env, arr, (uint32_t)i, e);
  }
  set(env, o, "results", arr);
  return o;
}

// columnizerDestroy(c): frees the columnizer now (its buffers, threads and
// dictionaries) instead of at garbage collection; later calls with `c` throw.
// Also keeps a finalizer from being pending at environment teardown, which
// this Node version does not survive.
napi_value ColumnizerDestroy(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return throw_napi(env, "args");
  void *p = nullptr;
  if (napi_remove_wrap(env, argv[0], &p) == napi_ok && p) {
    auto *c = static_cast<ColHandle *>(p);
    // its buffers may still be read by the engine's DMA (sa_ingest_async)
    if (c->engine && c->engine->live()) (void)c->engine->sync();
    if (c->engine_ref) napi_delete_reference(env, c->engine_ref);
    delete c;
  }
  return nullptr;
}

// columnizerResetExemplars(c): a new export interval (every series may take
// exemplars again)
napi_value ColumnizerResetExemplars(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return throw_napi(env, "args");
  ColHandle *c = get_col(env, argv[0]);
  if (!c) return nullptr;
  c->col.reset_exemplars();
  return nullptr;
}

napi_value ColumnizerIngest(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return throw_napi(env, "args");
  ColHandle *c = get_col(env, argv[0]);
  if (!c) return nullptr;
  if (!c->engine || !c->engine->live()) return throw_status(env, SA_ESTATE, "the columnizer has no live engine");
  const size_t n = c->col.buffered();
  if (n) {
    sa_span_batch b{c->col.key(), c->col.start(), c->col.end(), c->col.w0(), c->col.w1(), c->col.meta(), n};
    const int rc = c->engine->ingest_async(&b);
    if (rc != SA_OK) {
      // a failed ingest rejects these columns' requests (the host reports them
      // to their senders): drop the columns too, so a retry counts nothing
      // twice (an error return has read the columns, as sa_ingest does)
      c->col.clear_buffer();
      return engine_error(env, c->engine, rc, "sa_ingest_async");
    }
    // the engine's DMA may still read this buffer: columnize into the other
    // one (the next ingest returns once this one has been read)
    c->col.swap_buffers();
    return num(env, (double)n);
  }
  c->col.clear_buffer();
  return num(env, (double)n);
}

// columnizerTake(c) -> the buffered SoA columns (copies), then clear
napi_value ColumnizerTake(napi_env env, napi_callback_info info) {
  napi_value argv[1];
  if (!get_args(env, info, 1, argv)) return throw_napi(env, "args");
  ColHandle *c = get_col(env, argv[0]);
  if (!c) return nullptr;
  const size_t n = c->col.buffered();
  napi_value o;
  napi_create_object(env, &o);
  set(env, o, "keyHash", make_typed(env, napi_biguint64_array, 8, c->col.key(), n));
  set(env, o, "startNs", make_typed(env, napi_biguint64_array, 8, c->col.start(), n));
  set(env, o, "endNs", make_typed(env, napi_biguint64_array, 8, c->col.end(), n));
  set(env, o, "traceW0", make_typed(env, napi_biguint64_array, 8, c->col.w0(), n));
  set(env, o, "traceW1", make_typed(env, napi_biguint64_array, 8, c->col.w1(), n));
  set(env, o, "meta", make_typed(env, napi_uint32_array, 4, c->col.meta(), n));
  c->col.clear_buffer();
  return o;
}

napi_value ColumnizerServiceId(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return throw_napi(env, "args");
  ColHandle *c = get_col(env, argv[0]);
  std::string name;
  if (!c || !get_string(env, argv[1], &name, "name")) return nullptr;
  bool is_new = false;
  const uint32_t id = c->col.service_id(name, &is_new);
  napi_value arr, b;
  napi_create_array_with_length(env, 2, &arr);
  napi_set_element(env, arr, 0, num(env, id));
  napi_get_boolean(env, is_new, &b);
  napi_set_element(env, arr, 1, b);
  return arr;
}

// columnizerLearn(c, resHash, keyBytes, sid): a series the host interned itself
napi_value ColumnizerLearn(napi_env env, napi_callback_info info) {
  napi_value argv[4];
  if (!get_args(env, info, 4, argv)) return throw_napi(env, "args");
  ColHandle *c = get_col(env, argv[0]);
  uint64_t rh, sid;
  void *d;
  size_t n;
  if (!c || !to_u64(env, argv[1], &rh, "resHash") || !typed(env, argv[2], napi_uint8_array, &d, &n, "key") ||
      !to_u64(env, argv[3], &sid, "sid"))
    return nullptr;
  c->col.learn(rh, std::string(static_cast<const char *>(d), n), sid);
  return nullptr;
}

// columnizerRemap(c, from, to): the host's id for a reported series differs
napi_value ColumnizerRemap(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return throw_napi(env, "args");
  ColHandle *c = get_col(env, argv[0]);
  uint64_t from, to;
  if (!c || !to_u64(env, argv[1], &from, "from") || !to_u64(env, argv[2], &to, "to")) return nullptr;
  c->col.remap(from, to);
  return nullptr;
}

napi_value ColumnizerForget(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return throw_napi(env, "args");
  ColHandle *c = get_col(env, argv[0]);
  uint64_t h;
  if (!c || !to_u64(env, argv[1], &h, "resHash")) return nullptr;
  c->col.forget_resource(h);
  return nullptr;
}

// building blocks, for tests: {xxh64(hex, seed) -> BigInt, formatFloat(x), applyRules(rules, name)}
napi_value ColumnizerSelfTest(napi_env env, napi_callback_info info) {
  napi_value argv[3];
  if (!get_args(env, info, 3, argv)) return throw_napi(env, "args");
  std::string what;
  if (!get_string(env, argv[0], &what, "what")) return nullptr;
  if (what == "xxh64") {
    void *d;
    size_t n;
    uint64_t seed;
    if (!typed(env, argv[1], napi_uint8_array, &d, &n, "data") || !to_u64(env, argv[2], &seed, "seed")) return nullptr;
    return big(env, otlpcol::xxh64(d, n, seed));
  }
  if (what == "formatFloat") {
    double x;
    if (napi_get_value_double(env, argv[1], &x) != napi_ok) return throw_type(env, "x: expected a number");
    const std::string s = otlpcol::format_float(x);
    napi_value out;
    napi_create_string_utf8(env, s.c_str(), s.size(), &out);
    return out;
  }
  return throw_status(env, SA_EINVAL, "unknown self-test");
}

// xxh64(bytes, seed) -> BigInt: the host's series and resource ids (keys.js
// uses it once the addon is loaded; its BigInt restatement costs tens of
// microseconds per key, which made the discovery of new series the host's
// main JavaScript cost)
napi_value Xxh64(napi_env env, napi_callback_info info) {
  napi_value argv[2];
  if (!get_args(env, info, 2, argv)) return throw_napi(env, "args");
  void *d;
  size_t n;
  uint64_t seed;
  if (!typed(env, argv[0], napi_uint8_array, &d, &n, "data") || !to_u64(env, argv[1], &seed, "seed")) return nullptr;
  return big(env, otlpcol::xxh64(d, n, seed));
}

// page-locked column buffers for the native columnizer (sa_ingest then DMAs
// them without a staging copy); nullptr -> the columnizer uses the heap
void *host_alloc_hook(size_t bytes) {
  void *p = nullptr;
  return sa_host_alloc(bytes, &p) == SA_OK ? p : nullptr;
}

napi_value Init(napi_env env, napi_value exports) {
  otlpcol::set_host_allocator(&host_alloc_hook, &sa_host_free);
    struct Fn {
        const char *name;
        napi_callback cb;
    } fns[] = {{"abiVersion", AbiVersion},
               {"configDefault", ConfigDefault},
               {"bucketThresholds", BucketThresholds},
               {"hllEstimate", HllEstimate},
               {"create", Create},
               {"destroy", Destroy},
               {"lastError", LastError},
               {"ingest", Ingest},
               {"sync", Sync},
               {"flush", Flush},
               {"flushExp", FlushExp},
               {"windowRead", WindowRead},
               {"windowAdvance", WindowAdvance},
               {"stats", Stats},
               {"createColumnizer", CreateColumnizer},
               {"columnize", Columnize},
               {"columnizeBatch", ColumnizeBatch},
               {"columnizerResetExemplars", ColumnizerResetExemplars},
               {"columnizerDestroy", ColumnizerDestroy},
               {"columnizerIngest", ColumnizerIngest},
               {"columnizerTake", ColumnizerTake},
               {"columnizerServiceId", ColumnizerServiceId},
               {"columnizerForget", ColumnizerForget},
               {"columnizerLearn", ColumnizerLearn},
               {"columnizerRemap", ColumnizerRemap},
               {"columnizerSelfTest", ColumnizerSelfTest},
               {"xxh64", Xxh64}};
    for (auto &f : fns) {
        napi_value v;
        if (napi_create_function(env, f.name, NAPI_AUTO_LENGTH, f.cb, nullptr, &v) != napi_ok ||
            napi_set_named_property(env, exports, f.name, v) != napi_ok)
            return throw_napi(env, f.name);
    }
    napi_value st;
    napi_create_object(env, &st);
    struct Code {
        const char *k;
        int v;
    } codes[] = {{"OK", SA_OK},         {"EINVAL", SA_EINVAL}, {"ENOMEM", SA_ENOMEM},
                 {"EDEVICE", SA_EDEVICE}, {"EFULL", SA_EFULL},   {"ERANGE", SA_ERANGE},
                 {"ESTATE", SA_ESTATE}};
    for (auto &c : codes) set(env, st, c.k, num(env, c.v));
    set(env, exports, "status", st);
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
