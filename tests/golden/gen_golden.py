#!/usr/bin/env python3
"""Generates tests/golden/spanmetrics_kat.json -- TEST INFRASTRUCTURE.

An independent pure-Python restatement of the spanmetrics connector's
per-span aggregation ([UPSTREAM] connector/spanmetricsconnector v0.125.0,
restated in SURVEY.md 3A / rows a5-a11 / Appendix A) and of the build-owned
sketch spec (Appendix C).  IEEE-754 double arithmetic in CPython equals Go's
float64; bisect.bisect_left equals sort.SearchFloat64s; int -> float
conversion is correctly rounded in both.  Hashes use the third-party
`xxhash` package (3.8.1, the reference algorithm of cespare/xxhash/v2) so the
C oracle's own xxHash64 is checked against an independent implementation.

The reference's Go source is not in the container and Go is absent, so these
vectors are hand-derived known answers (Appendix A: A2, A3, A4, A8, A9, A10
at the series-id level), not outputs of the reference itself.

Run:  python tests/golden/gen_golden.py  (rewrites the JSON deterministically)
"""
from __future__ import annotations

import bisect
import json
import os
import random

import xxhash

DEFAULT_BOUNDS = [2, 4, 6, 8, 10, 50, 100, 200, 400, 800, 1000, 1400, 2000, 5000, 10000, 15000]
CMS_SEED = [0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB, 0xD6E8FEB86659FD93,
            0xA0761D6478BD642F, 0xE7037ED1A0B428DB, 0x8EBC6AF09C88C6E3, 0x589965CC75374CC3]
M64 = (1 << 64) - 1
T0 = 1_767_225_600 * 1_000_000_000


def splitmix64(x):
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def clz64(x):
    return 64 - x.bit_length()


def restate(spans, bounds, unit_div, hll_p, cms_d, cms_w, window_ns, n_services):
    """spans: list of (key, start, end, w0, w1, meta)."""
    series = {}
    windows = {}
    stats = dict(spans=0, invalid_service=0, zero_key=0)
    shift = 64 - (cms_w.bit_length() - 1)
    for key, s, e, w0, w1, meta in spans:
        stats["spans"] += 1
        if key == 0:
            stats["zero_key"] += 1
        else:
            d = float(e - s) / unit_div if e > s else 0.0
            b = bisect.bisect_left(bounds, d)
            st = series.setdefault(key, dict(counts=[0] * (len(bounds) + 1), sum_go=0.0, sum_ns=0))
            st["counts"][b] += 1
            st["sum_go"] += d
            st["sum_ns"] = (st["sum_ns"] + (e - s if e > s else 0)) & M64
        svc, status = meta & 0xFFFF, (meta >> 19) & 3
        if svc >= n_services:
            stats["invalid_service"] += 1
            continue
        wid = e // window_ns
        w = windows.setdefault(wid, dict(hll={}, cms={}))
        x = xxhash.xxh64_intdigest(w0.to_bytes(8, "little") + w1.to_bytes(8, "little"), seed=0)
        idx = x >> (64 - hll_p)
        rho = clz64(((x << hll_p) & M64) | (1 << (hll_p - 1))) + 1
        k = (svc, idx)
        if w["hll"].get(k, 0) < rho:
            w["hll"][k] = rho
        if status == 2:
            for j in range(cms_d):
                col = splitmix64(key ^ CMS_SEED[j]) >> shift
                w["cms"][(j, col)] = min(w["cms"].get((j, col), 0) + 1, 0xFFFFFFFF)
    out_series = [dict(key=k, counts=v["counts"], sum_go=v["sum_go"].hex(), sum_ns=v["sum_ns"])
                  for k, v in sorted(series.items())]
    out_windows = [dict(window=wid,
                        hll=sorted([s, i, r] for (s, i), r in w["hll"].items()),
                        cms=sorted([j, c, v] for (j, c), v in w["cms"].items()))
                   for wid, w in sorted(windows.items())]
    return out_series, out_windows, stats


def thresholds(bounds, unit_div):
    """Independent restatement of A4: T = max{d : float(d)/div <= b}."""
    neg = sum(1 for b in bounds if b < 0)
    out = []
    for b in bounds[neg:]:
        if float(M64) / unit_div <= b:
            out.append(M64)
            continue
        lo, hi = 0, M64
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if float(mid) / unit_div <= b:
                lo = mid
            else:
                hi = mid
        out.append(lo)
    return neg, out


def meta(svc, kind, status):
    return svc | (kind << 16) | (status << 19)


def case_kat_basic():
    """Hand-built: A2 (end<=start), A3 (bound equality, +1 ns, +Inf bucket),
    A8/A9, HLL duplicates, CMS on ERROR, invalid service, zero key."""
    k1, k2, k3 = 0x1111111111111111, 0x2222222222222222, 0xFFFFFFFFFFFFFFFF
    tA = (0x0123456789ABCDEF, 0xFEDCBA9876543210)
    tB = (0x0000000000000001, 0x0000000000000000)
    s = T0 + 5_000_000_000
    spans = [
        (k1, s, s + 2_000_000, *tA, meta(0, 2, 0)),           # exactly 2 ms -> bucket 0
        (k1, s, s + 2_000_001, *tA, meta(0, 2, 0)),           # 2 ms + 1 ns -> bucket 1
        (k1, s, s, *tA, meta(0, 2, 0)),                       # zero duration -> bucket 0
        (k1, s + 10, s, *tB, meta(0, 2, 0)),                  # end < start -> 0 (A2)
        (k1, s, s + 15_000_000_000, *tB, meta(0, 2, 0)),      # exactly 15 s -> bucket 15
        (k1, s, s + 15_000_000_001, *tB, meta(0, 2, 0)),      # -> +Inf bucket 16
        (k2, s, s + 50_000_000, *tA, meta(1, 3, 2)),          # ERROR -> CMS
        (k2, s, s + 49_999_999, *tA, meta(1, 3, 2)),
        (k2, s + 10_000_000_000, s + 10_000_000_000 + 7_123_456, *tB, meta(1, 3, 2)),  # next window
        (k3, s, s + 1, *tB, meta(2, 1, 1)),
        (k3, s, s + (1 << 62), *tB, meta(2, 1, 1)),           # huge duration
        (0, s, s + 5, *tA, meta(0, 2, 0)),                    # zero key: no RED, sketches yes
        (k1, s, s + 3_000_000, *tA, meta(70, 2, 2)),          # invalid service (n_services=64)
    ]
    return dict(name="kat_basic", bounds=DEFAULT_BOUNDS, unit="ms", hll_p=14, cms_d=4, cms_w=2048,
                window_ns=10_000_000_000, n_services=64, spans=spans)


def case_random(name, n, seed, n_keys, n_services, bounds=DEFAULT_BOUNDS, unit="ms", hll_p=14,
                cms_d=4, cms_w=2048):
    rng = random.Random(seed)
    keys = [rng.getrandbits(64) | 1 for _ in range(n_keys)]
    traces = [(rng.getrandbits(64), rng.getrandbits(64)) for _ in range(max(1, n // 5))]
    div = 1e9 if unit == "s" else 1e6
    spans = []
    for _ in range(n):
        k = keys[min(int(rng.paretovariate(1.2)) - 1, n_keys - 1)]
        st = T0 + rng.randrange(0, 40_000_000_000)
        r = rng.random()
        if r < 0.05:
            d = -rng.randrange(0, 1000)
        elif r < 0.15:
            d = int(bounds[rng.randrange(len(bounds))] * div) + rng.choice((-1, 0, 1))
        else:
            d = int(rng.lognormvariate(15.4, 1.6))
        e = max(0, st + d)
        tw = traces[rng.randrange(len(traces))]
        sv = rng.randrange(n_services + 1)  # one past the end -> invalid service
        stt = rng.choices((0, 1, 2, 3), (80, 10, 8, 2))[0]
        spans.append((k, st, e, tw[0], tw[1], meta(sv, rng.randrange(8), stt)))
    return dict(name=name, bounds=list(bounds), unit=unit, hll_p=hll_p, cms_d=cms_d, cms_w=cms_w,
                window_ns=10_000_000_000, n_services=n_services, spans=spans)


def case_custom_bounds(unit):
    bounds = [-1.5, -0.0, 0.1, 0.3, 1.0000001, 3.3, 7.77, 1e3, 2.5e6]
    div = 1e9 if unit == "s" else 1e6
    neg, thr = thresholds(bounds, div)
    spans = []
    key = 0xABCDEF0123456789
    s = T0 + 1_000_000_000
    for t in thr:
        if t == M64:
            continue
        for dd in (-1, 0, 1):
            d = t + dd
            if d < 0:
                continue
            spans.append((key, s, s + d, 1, 2, meta(3, 2, 0)))
    return dict(name=f"custom_bounds_{unit}", bounds=bounds, unit=unit, hll_p=10, cms_d=2, cms_w=64,
                window_ns=10_000_000_000, n_services=8, spans=spans,
                thresholds=dict(n_neg=neg, thr=thr))


def build_case(c):
    div = 1e9 if c["unit"] == "s" else 1e6
    series, windows, stats = restate(c["spans"], c["bounds"], div, c["hll_p"], c["cms_d"],
                                     c["cms_w"], c["window_ns"], c["n_services"])
    neg, thr = thresholds(c["bounds"], div)
    c = dict(c)
    c["spans"] = [list(x) for x in c["spans"]]
    c["expected"] = dict(series=series, windows=windows, stats=stats,
                         thresholds=dict(n_neg=neg, thr=thr))
    c.pop("thresholds", None)
    return c


def hash_vectors():
    rng = random.Random(99)
    vec = []
    for n in (0, 1, 3, 4, 7, 8, 15, 16, 17, 31, 32, 33, 63, 64, 100):
        data = bytes(rng.getrandbits(8) for _ in range(n))
        for seed in (0, 1, 0x9E3779B97F4A7C15):
            vec.append(dict(data=data.hex(), seed=seed, xxh64=xxhash.xxh64_intdigest(data, seed=seed)))
    sm = [dict(x=x, splitmix64=splitmix64(x)) for x in (0, 1, 42, M64, 0x123456789ABCDEF0)]
    return vec, sm


# ---- connector-level options (host logic of the Node connector) -----------
# Restated from [UPSTREAM] spanmetricsconnector config.go / connector.go
# v0.125.0 (confidence M: the Go source is not in the container): resetState
# drops, after an export, the cumulative resources whose lastSeen is at least
# metrics_expiration old; calls_dimensions / histogram.dimensions add
# dimensions to one metric's key only (separate sums / histograms maps).


def restate_expiration(ops, exp_ns):
    res, out = {}, []
    for op in ops:
        t = op["t"]
        if "consume" in op:
            for svc, n in op["consume"]:
                r = res.setdefault(svc, dict(calls=0, start=t, last=t))
                r["calls"] += n
                r["last"] = t
        else:  # an export (cumulative): every resource, then the expired ones go
            out.append({svc: [r["calls"], r["start"]] for svc, r in sorted(res.items())})
            for svc in [k for k, r in res.items() if t - r["last"] >= exp_ns]:
                del res[svc]
    return out


def case_expiration():
    s = 1_000_000_000
    ops = [dict(t=0, consume=[["a", 1], ["b", 2]]), dict(t=1 * s, export=True),
           dict(t=2 * s, consume=[["a", 1]]), dict(t=4 * s, export=True),
           dict(t=6 * s, export=True),                      # b (last seen 0) expires after this one
           dict(t=7 * s, consume=[["b", 5]]), dict(t=8 * s, export=True),   # b back, fresh start
           dict(t=9 * s, export=True),                      # a (last seen 2 s) expires after this one
           dict(t=10 * s, export=True)]
    return dict(name="metrics_expiration", config={"metrics_expiration": "5s"}, ops=ops,
                expected=restate_expiration(ops, 5 * s))


KIND = ["SPAN_KIND_UNSPECIFIED", "SPAN_KIND_INTERNAL", "SPAN_KIND_SERVER", "SPAN_KIND_CLIENT",
        "SPAN_KIND_PRODUCER", "SPAN_KIND_CONSUMER"]


def restate_split(spans, dims, calls_dims, hist_dims):
    """spans: (service, name, kind, status, {attr: str}); dims: [(name, default)].
    Returns the calls and histogram data points as [[attrs...], count]."""
    def point(svc, name, kind, st, attrs, ds):
        key = [svc, name, KIND[kind], ["STATUS_CODE_UNSET", "STATUS_CODE_OK", "STATUS_CODE_ERROR"][st]]
        at = [["service.name", svc], ["span.name", name], ["span.kind", KIND[kind]], ["status.code", key[3]]]
        for dn, dd in ds:
            v = attrs.get(dn, dd)
            if v is None:
                continue          # a missing dimension without a default adds nothing (A5)
            key.append(v)
            at.append([dn, v])
        return "\0".join(key), at
    calls, hist = {}, {}
    for svc, name, kind, st, attrs in spans:
        for table, ds in ((calls, dims + calls_dims), (hist, dims + hist_dims)):
            k, at = point(svc, name, kind, st, attrs, ds)
            e = table.setdefault(k, [at, 0])
            e[1] += 1
    return [v for _, v in sorted(calls.items())], [v for _, v in sorted(hist.items())]


def case_split_dims():
    spans = [("a", "GET /x", 2, 0, {"http.method": "GET", "http.route": "/x"}),
             ("a", "GET /x", 2, 0, {"http.method": "GET", "http.route": "/y"}),
             ("a", "GET /x", 2, 0, {"http.method": "POST"}),
             ("a", "GET /x", 2, 2, {"http.route": "/x"}),
             ("a", "op", 1, 0, {}),
             ("b", "op", 3, 1, {"http.method": "GET", "region": "us"}),
             ("b", "op", 3, 2, {"http.method": "GET", "region": "us"}),
             ("b", "op", 3, 2, {"http.method": "PUT", "region": "us"})]
    dims, cd, hd = [["region", None]], [["http.method", None]], [["http.route", "none"]]
    calls, hist = restate_split(spans, dims, cd, hd)
    cfg = {"dimensions": [{"name": "region"}], "calls_dimensions": [{"name": "http.method"}],
           "histogram": {"dimensions": [{"name": "http.route", "default": "none"}]}}
    # the window's sketches see every span once (connector.go keeps one
    # sums and one histograms map, but the sketches are this engine's own:
    # one ERROR count per ERROR span, under its histogram-series key): each
    # count-min row holds the window's ERROR spans exactly once
    errors = sum(1 for s in spans if s[3] == 2)
    err_points = sorted([at, n] for at, n in hist if ["status.code", "STATUS_CODE_ERROR"] in at)
    return dict(name="calls_and_histogram_dimensions", config=cfg,
                spans=[[a, b, c, d, e] for a, b, c, d, e in spans],
                expected=dict(calls=calls, histogram=hist, window_error_spans=errors, top_errors=err_points))


def case_histogram_disable():
    spans = [("a", "op", 2, 0, {}), ("a", "op", 2, 0, {}), ("b", "op", 2, 2, {})]
    calls, _ = restate_split(spans, [], [], [])
    return dict(name="histogram_disable", config={"histogram": {"disable": True}},
                spans=[[a, b, c, d, e] for a, b, c, d, e in spans], expected=dict(calls=calls, histogram=[]))


def restate_scope(spans, dims, scopes):
    """include_instrumentation_scope ([UPSTREAM] connector.go buildKey /
    buildAttributes, confidence L): a span whose scope name is listed is keyed
    with the scope's name and version after the dimensions, and its data point
    carries span.instrumentation.scope.name / .version.  spans: (service, name,
    kind, status, {attr: str}, scope name, scope version).  Returns the calls
    data points as [[attrs...], count]."""
    table = {}
    for svc, name, kind, st, attrs, sn, sv in spans:
        stc = ["STATUS_CODE_UNSET", "STATUS_CODE_OK", "STATUS_CODE_ERROR"][st]
        key = [svc, name, KIND[kind], stc]
        at = [["service.name", svc], ["span.name", name], ["span.kind", KIND[kind]], ["status.code", stc]]
        for dn, dd in dims:
            v = attrs.get(dn, dd)
            if v is None:
                continue
            key.append(v)
            at.append([dn, v])
        if sn in scopes:
            key += [sn, sv]
            at += [["span.instrumentation.scope.name", sn], ["span.instrumentation.scope.version", sv]]
        e = table.setdefault("\0".join(key), [at, 0])
        e[1] += 1
    return [v for _, v in sorted(table.items())]


def case_scope():
    spans = [("a", "GET", 2, 0, {"region": "eu"}, "io.opentelemetry.http", "1.2.0"),
             ("a", "GET", 2, 0, {"region": "eu"}, "io.opentelemetry.http", "1.3.0"),
             ("a", "GET", 2, 0, {"region": "eu"}, "io.opentelemetry.http", "1.3.0"),
             ("a", "GET", 2, 0, {"region": "eu"}, "io.opentelemetry.grpc", "1.3.0"),   # not listed
             ("a", "GET", 2, 0, {"region": "eu"}, "", ""),                             # no scope
             ("a", "GET", 2, 0, {}, "io.opentelemetry.http", ""),                     # empty version
             ("b", "op", 1, 2, {"region": "us"}, "manual", "0.1"),
             ("b", "op", 1, 2, {"region": "us"}, "manual", "0.1")]
    scopes = ["io.opentelemetry.http", "manual"]
    return dict(name="include_instrumentation_scope",
                config={"dimensions": [{"name": "region"}], "include_instrumentation_scope": scopes},
                spans=[list(s[:5]) + [s[5], s[6]] for s in spans],
                expected=dict(calls=restate_scope(spans, [["region", None]], set(scopes))))


def main():
    cases = [
        build_case(case_kat_basic()),
        build_case(case_random("random_default", 4000, 1234, 40, 6)),
        build_case(case_random("random_wide", 3000, 77, 300, 12, hll_p=8, cms_d=3, cms_w=256)),
        build_case(case_custom_bounds("ms")),
        build_case(case_custom_bounds("s")),
    ]
    xv, sm = hash_vectors()
    out = dict(generator="tests/golden/gen_golden.py", xxhash_version=xxhash.VERSION, cases=cases,
               xxh64_vectors=xv, splitmix64_vectors=sm,
               connector_cases=[case_expiration(), case_split_dims(), case_histogram_disable(),
                                case_scope()])
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "spanmetrics_kat.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
        f.write("\n")
    print(f"wrote {path}: {sum(len(c['spans']) for c in cases)} spans in {len(cases)} cases")


if __name__ == "__main__":
    main()
