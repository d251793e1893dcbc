"""Synthetic span streams for the BASELINE.json configs.

Vocabulary comes from the reference demo: the 20 OTEL_SERVICE_NAMEs of
/root/reference/docker-compose.yml (:39,73,106,148,192,219,250,287,290,349,388,
421,456,489,520,552,584,613,643,677) and span names from its trace-based tests
and manual spans.  Everything is seeded (PCG64).

C2: n spans over 20 services x 25 span names (kind fixed per name), Zipf(1.1)
over the (service, name) pairs, status per span UNSET/OK/ERROR = 88/10/2 %
(so up to 1,500 series), lognormal(ln 5 ms, 1.5) durations in integer ns
clipped to [0, 60 s], 0.5 % with end <= start, 0.5 % exactly on a bucket
bound, ~10 spans per trace, start times spread over 60 s.
C4: the same with 1,000,000 distinct keys (2,000 http.route x 500
k8s.pod.name dimension values).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .engine import DEFAULT_BOUNDS_MS, SpanBatch, pack_meta
from .keys import build_key, resource_hash, series_hash

SERVICES = (
    "accounting", "ad", "cart", "checkout", "currency", "email", "fraud-detection", "frontend",
    "frontend-web", "frontend-proxy", "image-provider", "load-generator", "payment",
    "product-catalog", "quote", "recommendation", "shipping", "flagd", "flagd-ui", "kafka",
)

SPAN_NAMES = (
    ("oteldemo.AdService/GetAds", 2), ("POST /oteldemo.CartService/AddItem", 3), ("HMSET", 3),
    ("EXPIRE", 3), ("oteldemo.CheckoutService/PlaceOrder", 2), ("orders publish", 4),
    ("grpc.oteldemo.PaymentService/Charge", 2), ("Currency/Convert", 2),
    ("Currency/GetSupportedCurrencies", 2), ("oteldemo.ShippingService/GetQuote", 2),
    ("oteldemo.ShippingService/ShipOrder", 2), ("/oteldemo.RecommendationService/ListRecommendations", 2),
    ("oteldemo.ProductCatalogService/GetProduct", 2), ("oteldemo.ProductCatalogService/ListProducts", 2),
    ("oteldemo.ProductCatalogService/SearchProducts", 2), ("POST /send_order_confirmation", 2),
    ("sinatra.render_template", 1), ("send_email", 1), ("charge", 1), ("getRandomAds", 1),
    ("get_product_list", 1), ("calculate-quote", 1), ("prepareOrderItemsAndShippingQuoteFromCart", 1),
    ("GET /api/products/{productId}", 2), ("orders receive", 5),
)

T0_NS = 1_767_225_600 * 1_000_000_000  # 2026-01-01T00:00:00Z


@dataclass
class Workload:
    batch: SpanBatch
    key_strings: list          # per series index: (service, name, kind, status)
    key_hashes: np.ndarray     # [n_keys] u64
    key_index: np.ndarray      # [n] per-span series index
    service_id: np.ndarray     # [n] u32
    name_id: np.ndarray        # [n] u32 (index into SPAN_NAMES)
    kind: np.ndarray
    status: np.ndarray
    first_window: int
    n_windows: int
    n_services: int


def _durations(rng, n, bounds_ms):
    d = np.exp(rng.normal(np.log(5e6), 1.5, n))
    d = np.clip(d, 0, 60e9).astype(np.uint64)
    on_bound = rng.random(n) < 0.005
    b = np.asarray(bounds_ms, dtype=np.float64)
    d[on_bound] = (b[rng.integers(0, len(b), on_bound.sum())] * 1e6).astype(np.uint64)
    return d


def generate_c2(n: int, seed: int = 42, n_services: int = 20, names_per_service: int = 25,
                zipf_s: float = 1.1, spans_per_trace: int = 10, spread_s: int = 60,
                err: float = 0.02, ok: float = 0.10, bounds_ms=DEFAULT_BOUNDS_MS) -> Workload:
    rng = np.random.Generator(np.random.PCG64(seed))
    K = n_services * names_per_service
    w = 1.0 / np.arange(1, K + 1, dtype=np.float64) ** zipf_s
    w /= w.sum()
    perm = rng.permutation(K)
    pair = perm[np.searchsorted(np.cumsum(w), rng.random(n), side="right").clip(0, K - 1)]
    svc = (pair // names_per_service).astype(np.uint32)
    name = (pair % names_per_service).astype(np.uint32)
    kinds = np.array([k for _, k in SPAN_NAMES], dtype=np.uint32)
    kind = kinds[name % len(SPAN_NAMES)]
    u = rng.random(n)
    status = np.where(u < err, 2, np.where(u < err + ok, 1, 0)).astype(np.uint32)

    # series table: (pair, status) -> id
    key_strings, key_hashes = [], np.zeros(K * 3, dtype=np.uint64)
    for p in range(K):
        s, nm = p // names_per_service, p % names_per_service
        sname = SERVICES[s % len(SERVICES)] if s < len(SERVICES) else f"service-{s}"
        nname, kd = SPAN_NAMES[nm % len(SPAN_NAMES)]
        if nm >= len(SPAN_NAMES):
            nname = f"{nname}#{nm}"
        rh = resource_hash({"service.name": sname})
        for st in range(3):
            key_strings.append((sname, nname, kd, st))
            key_hashes[p * 3 + st] = series_hash(rh, build_key(sname, nname, kd, st))
    key_index = (pair.astype(np.int64) * 3 + status).astype(np.int64)

    start = (T0_NS + rng.integers(0, spread_s * 1_000_000_000, n, dtype=np.int64)).astype(np.uint64)
    dur = _durations(rng, n, bounds_ms)
    end = start + dur
    back = rng.random(n) < 0.005
    end[back] = start[back] - rng.integers(0, 1_000_000, back.sum(), dtype=np.int64).astype(np.uint64)

    n_traces = max(1, n // spans_per_trace)
    tw0 = rng.integers(0, 2**63, n_traces, dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        rng.integers(0, 2, n_traces, dtype=np.int64).astype(np.uint64)
    tw1 = rng.integers(0, 2**63, n_traces, dtype=np.int64).astype(np.uint64) * np.uint64(2) + \
        rng.integers(0, 2, n_traces, dtype=np.int64).astype(np.uint64)
    tr = rng.integers(0, n_traces, n)
    batch = SpanBatch(key_hashes[key_index], start, end, tw0[tr], tw1[tr],
                      pack_meta(svc, kind, status))
    # spans with end < start near T0 fall in the window before T0's
    first_window = int(end.min()) // 10_000_000_000 if n else T0_NS // 10_000_000_000
    n_win = int(end.max()) // 10_000_000_000 - first_window + 1 if n else 1
    return Workload(batch, key_strings, key_hashes, key_index, svc, name, kind, status,
                    int(first_window), int(n_win), n_services)


def generate_highcard(n: int, seed: int = 7, routes: int = 2000, pods: int = 500,
                      zipf_s: float = 0.0, spans_per_trace: int = 10, spread_s: int = 60,
                      bounds_ms=DEFAULT_BOUNDS_MS):
    """C4: 1M keys = http.route x k8s.pod.name; uniform (zipf_s=0) or Zipf."""
    rng = np.random.Generator(np.random.PCG64(seed))
    K = routes * pods
    if zipf_s > 0:
        w = 1.0 / np.arange(1, K + 1, dtype=np.float64) ** zipf_s
        w /= w.sum()
        kidx = np.searchsorted(np.cumsum(w), rng.random(n), side="right").clip(0, K - 1)
        kidx = rng.permutation(K)[kidx]
    else:
        kidx = rng.integers(0, K, n)
    # key ids: xxh64 of the NUL-joined key with dimension values (vectorised via
    # a per-key hash table computed once)
    import xxhash
    rh = resource_hash({"service.name": "frontend"})
    prefix = rh.to_bytes(8, "little") + build_key("frontend", "GET", 2, 0)
    khash = np.fromiter(
        (xxhash.xxh64_intdigest(prefix + f"\x00/api/route/{k // pods}\x00frontend-pod-{k % pods}".encode())
         or 1 for k in range(K)), dtype=np.uint64, count=K)
    svc = np.zeros(n, dtype=np.uint32)
    status = np.where(rng.random(n) < 0.02, 2, 0).astype(np.uint32)
    start = (T0_NS + rng.integers(0, spread_s * 1_000_000_000, n, dtype=np.int64)).astype(np.uint64)
    end = start + _durations(rng, n, bounds_ms)
    n_traces = max(1, n // spans_per_trace)
    tw0 = rng.integers(0, 2**63, n_traces, dtype=np.int64).astype(np.uint64)
    tw1 = rng.integers(0, 2**63, n_traces, dtype=np.int64).astype(np.uint64)
    tr = rng.integers(0, n_traces, n)
    batch = SpanBatch(khash[kidx], start, end, tw0[tr], tw1[tr], pack_meta(svc, 2, status))
    return batch, khash, int(end.min()) // 10_000_000_000


@dataclass
class C5Workload:
    """C5 stream: spans in end-time order over `duration_s`, plus the anomaly spec."""
    base: Workload            # C2-shaped spans, re-timed (batch sorted by end_ns)
    window_ns: int
    first_window: int
    n_windows: int
    error_service: int        # service id whose error rate is multiplied
    error_windows: tuple      # window offsets [lo, hi] of the error anomaly
    burst_service: int        # service id with the distinct-trace burst
    burst_windows: tuple      # window offsets [lo, hi] of the burst


def generate_c5(n: int, seed: int = 5, duration_s: int = 600, window_s: int = 10,
                error_factor: float = 20.0, error_windows=(30, 35), burst_factor: float = 4.0,
                burst_windows=(40, 42)) -> C5Workload:
    """C5: C2 traffic re-timed uniformly over 600 s (60 windows
    of 10 s), sorted by end time as a collector receives it.  Injected
    anomalies: the `payment` service's error rate x20 in windows 30-35 (the
    demo's paymentFailure flag, demo.flagd.json:67-80) and a burst of new
    traces at `frontend` in windows 40-42 (x4 its spans, each extra span in a
    fresh trace).  The stream holds n spans plus the burst's extra spans."""
    wl = generate_c2(n, seed=seed)
    rng = np.random.Generator(np.random.PCG64(seed + 1000))
    W = window_s * 1_000_000_000
    t0 = (T0_NS // W) * W
    b = wl.batch
    dur = np.where(b.end_ns > b.start_ns, b.end_ns - b.start_ns, 0).astype(np.uint64)
    dur = np.minimum(dur, np.uint64(W // 2))  # keep each span inside its own window or the next
    end = (t0 + rng.integers(0, duration_s * 1_000_000_000, n, dtype=np.int64)).astype(np.uint64)
    start = end - dur
    win = ((end - np.uint64(t0)) // np.uint64(W)).astype(np.int64)
    pay = SERVICES.index("payment")
    fe = SERVICES.index("frontend")
    status = wl.status.copy()
    key_index = wl.key_index.copy()
    # error anomaly: flip OK/UNSET payment spans to ERROR with the extra probability
    in_err = (wl.service_id == pay) & (win >= error_windows[0]) & (win <= error_windows[1])
    flip = in_err & (status != 2) & (rng.random(n) < min(1.0, 0.02 * (error_factor - 1)))
    status[flip] = 2
    key_index[flip] = key_index[flip] - (key_index[flip] % 3) + 2
    # distinct-trace burst: (burst_factor - 1) extra copies of every frontend span
    # in the burst windows, each in a fresh trace
    in_burst = np.nonzero((wl.service_id == fe) & (win >= burst_windows[0]) & (win <= burst_windows[1]))[0]
    extra = np.tile(in_burst, int(burst_factor) - 1)
    m = len(extra)
    idx = np.concatenate([np.arange(n), extra])
    w0 = np.concatenate([b.trace_w0, rng.integers(0, 2**63, m, dtype=np.int64).astype(np.uint64)])
    w1 = np.concatenate([b.trace_w1, rng.integers(0, 2**63, m, dtype=np.int64).astype(np.uint64)])
    order = np.argsort(end[idx], kind="stable")
    sel = idx[order]
    batch = SpanBatch(wl.key_hashes[key_index][sel], start[sel], end[sel], w0[order], w1[order],
                      pack_meta(wl.service_id[sel], wl.kind[sel], status[sel]))
    base = Workload(batch, wl.key_strings, wl.key_hashes, key_index[sel], wl.service_id[sel],
                    wl.name_id[sel], wl.kind[sel], status[sel], int(t0 // W),
                    duration_s // window_s, wl.n_services)
    return C5Workload(base, W, int(t0 // W), duration_s // window_s, pay, tuple(error_windows), fe,
                      tuple(burst_windows))
