"""The Node N-API host (host/node): north_star's TypeScript/Node side of the
C-ABI.  CPU tests check the JS pieces against independent Python code
(protobuf from descriptor_pb2, keys.py, xxhash, re); the GPU test runs OTLP
bytes through the real addon and checks every stage against the C oracle."""
import base64
import json
import os
import re
import shutil
import subprocess

import numpy as np
import pytest
import xxhash

from otlp_pb import M
from spanagg import keys as pykeys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE_DIR = os.path.join(ROOT, "host", "node")
NODE = shutil.which("node")

pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def node(script, payload, timeout=120, env=None):
    p = subprocess.run([NODE, os.path.join(NODE_DIR, "test", script)], input=json.dumps(payload),
                       capture_output=True, text=True, timeout=timeout, env=env)
    assert p.returncode == 0, p.stderr[-4000:]
    return json.loads(p.stdout)


# ---- typed attribute values: python value <-> [type, payload] --------------------

def typed(v):
    if isinstance(v, bool):
        return ["bool", v]
    if isinstance(v, int):
        return ["int", str(v)]
    if isinstance(v, float):
        return ["double", v]
    if isinstance(v, bytes):
        return ["bytes", v.hex()]
    if isinstance(v, list):
        return ["array", [typed(x) for x in v]]
    if isinstance(v, dict):
        return ["kvlist", [[k, typed(x)] for k, x in v.items()]]
    if v is None:
        return ["empty", None]
    return ["string", v]


def untyped(tv):
    t, v = tv
    return {"bool": lambda: v, "int": lambda: int(v), "double": lambda: float(v),
            "bytes": lambda: bytes.fromhex(v), "array": lambda: [untyped(x) for x in v],
            "kvlist": lambda: {k: untyped(x) for k, x in v}, "empty": lambda: None,
            "string": lambda: v}[t]()


def set_any(av, v):
    if isinstance(v, bool):
        av.bool_value = v
    elif isinstance(v, int):
        av.int_value = v
    elif isinstance(v, float):
        av.double_value = v
    elif isinstance(v, bytes):
        av.bytes_value = v
    elif isinstance(v, list):
        av.array_value.SetInParent()
        for x in v:
            set_any(av.array_value.values.add(), x)
    elif isinstance(v, dict):
        av.kvlist_value.SetInParent()
        for k, x in v.items():
            kv = av.kvlist_value.values.add(key=k)
            set_any(kv.value, x)
    else:
        av.string_value = v


def get_any(av):
    which = av.WhichOneof("value")
    if which is None:
        return None
    if which == "array_value":
        return [get_any(x) for x in av.array_value.values]
    if which == "kvlist_value":
        return {kv.key: get_any(kv.value) for kv in av.kvlist_value.values}
    return getattr(av, which)


def add_attrs(repeated, attrs):
    for k, v in attrs.items():
        set_any(repeated.add(key=k).value, v)


# ---- CPU: unit suite, hashes, keys, transform, codec ---------------------------

def test_node_unit_suite():
    p = subprocess.run([NODE, os.path.join(NODE_DIR, "test", "run.js")], capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
    assert "passed" in p.stdout


def test_xxh64_matches_python_xxhash():
    rng = np.random.default_rng(3)
    cases = [(rng.integers(0, 256, n, dtype=np.uint8).tobytes().hex(), seed)
             for n in list(range(0, 70)) + [100, 255, 1024] for seed in (0, 1)]
    got = node("cli.js", {"cmd": "xxh64", "cases": cases})
    exp = ["%016x" % xxhash.xxh64_intdigest(bytes.fromhex(h), seed=s) for h, s in cases]
    assert got == exp


KEY_VECTORS = [
    dict(service="frontend", span_name="GET /api/cart", kind=2, status=0),
    dict(service="checkout", span_name="oteldemo.CheckoutService/PlaceOrder", kind=3, status=2,
         resource_attrs={"service.name": "checkout", "k8s.pod.name": "checkout-7d9f", "pid": 41,
                         "ratio": 0.5, "debug": False, "tags": ["a", 1, 2.5, True]}),
    dict(service="svc", span_name="op", kind=9, status=7),  # A7 out-of-range enums
    dict(service="svc", span_name="op", kind=1, status=1,
         dims=[{"name": "http.status_code"}, {"name": "region", "default": "eu-west"},
               {"name": "absent"}],
         span_attrs={"http.status_code": 200}),
    dict(service="svc", span_name="op", kind=1, status=1,
         dims=[{"name": "http.status_code"}, {"name": "region", "default": "eu-west"},
               {"name": "absent"}],
         span_attrs={"http.status_code": "200"}),  # A6
    dict(service="svc", span_name="op", kind=5, status=0, exclude=["span.kind", "status.code"],
         dims=[{"name": "k8s.pod.name"}, {"name": "f"}, {"name": "m"}, {"name": "raw"}],
         span_attrs={"f": 1e21, "m": {"x": "y", "n": 2}, "raw": b"\x00\xff"},
         resource_attrs={"k8s.pod.name": "pod-1", "b": b"\x01"}),
    dict(service="", span_name="", kind=0, status=0, resource_attrs={}),
    dict(service="ünïcode", span_name="ΣΠΑΝ", kind=4, status=2, resource_attrs={"service.name": "ünïcode"}),
    dict(service="svc", span_name="op", kind=1, status=1, dims=[{"name": "x"}],
         span_attrs={"x": 1.5e-7}),
]


def test_keys_match_python_keys_module():
    vecs = []
    for v in KEY_VECTORS:
        w = dict(v)
        w["span_attrs"] = [[k, typed(x)] for k, x in v.get("span_attrs", {}).items()]
        w["resource_attrs"] = [[k, typed(x)] for k, x in v.get("resource_attrs", {}).items()]
        vecs.append(w)
    got = node("cli.js", {"cmd": "keys", "vectors": vecs})
    for v, g in zip(KEY_VECTORS, got):
        dims = [(d["name"], d.get("default")) for d in v.get("dims", [])]
        key = pykeys.build_key(v["service"], v["span_name"], v["kind"], v["status"], dims,
                               v.get("span_attrs", {}), v.get("resource_attrs", {}),
                               v.get("exclude", ()))
        rh = pykeys.resource_hash(v.get("resource_attrs", {}))
        assert bytes.fromhex(g["key"]) == key, (v, key)
        assert int(g["resource_hash"], 16) == rh, v
        assert int(g["series"], 16) == pykeys.series_hash(rh, key), v
    # datapoint attributes keep the first-seen type (A6): int stays int, string stays string
    assert got[3]["attrs"][4] == ["http.status_code", ["int", "200"]]
    assert got[3]["attrs"][5] == ["region", ["string", "eu-west"]]
    assert got[4]["attrs"][4] == ["http.status_code", ["string", "200"]]
    assert got[3]["key"] == got[4]["key"]


def demo_transform(name: str) -> str:
    """Python statement of otelcol-config.yml:106-113 (regexp + whole-value glob)."""
    name = re.sub(r"\?.*", "", name)
    if re.fullmatch(r"GET /api/products/.*", name, flags=re.S):
        name = "GET /api/products/{productId}"
    return name


def test_transform_rules_match_python_statement():
    names = ["GET /api/products/0PUK6V6EV0", "GET /api/products/0PUK6V6EV0?currencyCode=USD",
             "GET /api/cart?sessionId=abc", "POST /api/products/1", "GET /api/products",
             "GET /api/products/", "?", "a?b?c", "GET /api/recommendations?productIds=1,2",
             "oteldemo.CartService/GetCart", ""]
    assert node("cli.js", {"cmd": "transform", "names": names}) == [demo_transform(n) for n in names]


def _py_traces_request(spec):
    req = M["ExportTraceServiceRequest"]()
    for res_attrs, spans in spec:
        rs = req.resource_spans.add()
        add_attrs(rs.resource.attributes, res_attrs)
        ss = rs.scope_spans.add()
        ss.scope.name = "test-scope"
        for s in spans:
            sp = ss.spans.add(trace_id=s["trace_id"], span_id=s.get("span_id", b"\x01" * 8),
                              name=s["name"], kind=s["kind"], start_time_unix_nano=s["start"],
                              end_time_unix_nano=s["end"])
            add_attrs(sp.attributes, s.get("attrs", {}))
            if s.get("status"):
                sp.status.code = s["status"]
                sp.status.message = s.get("message", "")
            # fields the connector ignores must be skipped cleanly
            ev = sp.events.add(time_unix_nano=1, name="ev")
            add_attrs(ev.attributes, {"k": "v"})
            sp.flags = 0x101
    return req


SPEC = [
    ({"service.name": "frontend", "k8s.pod.name": "fe-1", "pid": 7, "w": 0.25},
     [dict(trace_id=bytes(range(16)), name="GET /api/products/X?y=1", kind=2, start=10, end=2_000_010,
           attrs={"http.route": "/api/products/{id}", "n": -3, "big": 2 ** 63 - 1, "neg": -(2 ** 63),
                  "ok": True, "arr": ["a", 2, 0.5], "kv": {"x": "y"}, "raw": b"\x00\x01\xff"},
           status=2, message="boom"),
      dict(trace_id=b"\xff" * 16, name="", kind=0, start=2 ** 64 - 2, end=2 ** 64 - 1)]),
    ({"host.name": "no-service"}, [dict(trace_id=b"\x01" * 16, name="x", kind=1, start=1, end=2)]),
]


def test_decode_python_protobuf_bytes():
    raw = _py_traces_request(SPEC).SerializeToString()
    got = node("cli.js", {"cmd": "decode_traces", "b64": base64.b64encode(raw).decode()})
    assert len(got["resource_spans"]) == 2
    for (res_attrs, spans), rs in zip(SPEC, got["resource_spans"]):
        assert {k: untyped(v) for k, v in rs["resource"]} == res_attrs
        assert rs["scope_spans"][0]["scope"] == "test-scope"
        for s, g in zip(spans, rs["scope_spans"][0]["spans"]):
            assert bytes.fromhex(g["trace_id"]) == s["trace_id"]
            assert g["name"] == s["name"] and g["kind"] == s["kind"]
            assert (int(g["start"]), int(g["end"])) == (s["start"], s["end"])
            assert g["status"] == s.get("status", 0) and g["message"] == s.get("message", "")
            assert {k: untyped(v) for k, v in g["attributes"]} == s.get("attrs", {})


def test_encode_traces_parsed_by_python_protobuf():
    req = {"resource_spans": [{"resource": [[k, typed(v)] for k, v in SPEC[0][0].items()],
                               "scope_spans": [{"scope": "s", "spans": [
                                   {"trace_id": s["trace_id"].hex(), "span_id": "0102030405060708",
                                    "name": s["name"], "kind": s["kind"], "start": str(s["start"]),
                                    "end": str(s["end"]), "status": s.get("status", 0),
                                    "message": s.get("message", ""),
                                    "attributes": [[k, typed(v)] for k, v in s.get("attrs", {}).items()]}
                                   for s in SPEC[0][1]]}]}]}
    out = node("cli.js", {"cmd": "encode_traces", "req": req})
    msg = M["ExportTraceServiceRequest"].FromString(base64.b64decode(out["b64"]))
    rs = msg.resource_spans[0]
    assert {kv.key: get_any(kv.value) for kv in rs.resource.attributes} == SPEC[0][0]
    for s, sp in zip(SPEC[0][1], rs.scope_spans[0].spans):
        assert sp.trace_id == s["trace_id"] and sp.name == s["name"] and sp.kind == s["kind"]
        assert (sp.start_time_unix_nano, sp.end_time_unix_nano) == (s["start"], s["end"])
        assert sp.status.code == s.get("status", 0)
        assert {kv.key: get_any(kv.value) for kv in sp.attributes} == s.get("attrs", {})
    # and the Python encoding of the same request decodes to the same bytes' meaning
    assert msg.SerializeToString() == M["ExportTraceServiceRequest"].FromString(
        msg.SerializeToString()).SerializeToString()


def test_encode_metrics_parsed_by_python_protobuf():
    attrs = [["service.name", ["string", "frontend"]], ["http.status_code", ["int", "200"]]]
    req = {"resource_metrics": [{"resource": [["service.name", ["string", "frontend"]]],
                                 "scope": "spanmetricsconnector", "metrics": [
        {"name": "traces.span.metrics.calls", "kind": "sum", "temporality": 2, "monotonic": True,
         "points": [{"attributes": attrs, "start": "5", "time": "1700000000000000000", "as_int": "42"}]},
        {"name": "traces.span.metrics.duration", "unit": "ms", "kind": "histogram", "temporality": 1,
         "points": [{"attributes": attrs, "start": "5", "time": "9", "count": "3", "sum": 0.0,
                     "bucket_counts": ["1", "0", "2"], "explicit_bounds": [2, 4]}]},
        {"name": "g", "kind": "gauge", "points": [{"attributes": [], "time": "9", "as_double": 2.5}]}]}]}
    out = node("cli.js", {"cmd": "encode_metrics", "req": req})
    msg = M["ExportMetricsServiceRequest"].FromString(base64.b64decode(out["b64"]))
    sm = msg.resource_metrics[0].scope_metrics[0]
    assert sm.scope.name == "spanmetricsconnector"
    calls, dur, g = sm.metrics
    assert calls.name == "traces.span.metrics.calls" and calls.WhichOneof("data") == "sum"
    assert calls.sum.is_monotonic and calls.sum.aggregation_temporality == 2
    dp = calls.sum.data_points[0]
    assert dp.as_int == 42 and dp.time_unix_nano == 1700000000000000000 and dp.start_time_unix_nano == 5
    assert {kv.key: get_any(kv.value) for kv in dp.attributes} == {"service.name": "frontend",
                                                                    "http.status_code": 200}
    h = dur.histogram.data_points[0]
    assert dur.unit == "ms" and dur.histogram.aggregation_temporality == 1
    assert h.count == 3 and h.HasField("sum") and h.sum == 0.0
    assert list(h.bucket_counts) == [1, 0, 2] and list(h.explicit_bounds) == [2.0, 4.0]
    assert g.WhichOneof("data") == "gauge" and g.gauge.data_points[0].as_double == 2.5


# ---- GPU: OTLP bytes -> Node host -> N-API -> libspanagg, vs the oracle --------

SERVICES = ["frontend", "cart", "checkout", "payment", "product-catalog", "recommendation"]
NAMES = ["GET /api/products/{}?currencyCode=USD", "GET /api/cart", "POST /api/checkout",
         "oteldemo.PaymentService/Charge", "GET /api/products/{}", "GET /api/recommendations?ids={}"]
T0 = 1_700_000_000_000_000_000 - (1_700_000_000_000_000_000 % 10_000_000_000)


def synth_requests(seed, n_requests=12, per_request=2500):
    """Python-built OTLP requests plus the per-span facts the checks need."""
    rng = np.random.default_rng(seed)
    bounds_ns = np.array([2, 4, 6, 8, 10, 50, 100, 200, 400, 800, 1000, 1400, 2000, 5000, 10000,
                          15000], dtype=np.uint64) * 1_000_000
    requests, facts = [], []
    for _ in range(n_requests):
        req = M["ExportTraceServiceRequest"]()
        n_res = int(rng.integers(1, 5))
        for _ in range(n_res):
            svc = SERVICES[int(rng.integers(len(SERVICES)))]
            pod = f"{svc}-{int(rng.integers(2))}"
            res_attrs = {"service.name": svc, "k8s.pod.name": pod}
            skip = rng.random() < 0.05
            if skip:
                res_attrs = {"host.name": pod}  # A1: contributes nothing
            rs = req.resource_spans.add()
            add_attrs(rs.resource.attributes, res_attrs)
            ss = rs.scope_spans.add()
            for _ in range(per_request // n_res):
                name = NAMES[int(rng.integers(len(NAMES)))].format(int(rng.integers(50)))
                kind = int(rng.integers(0, 6))
                status = int(rng.choice([0, 1, 2], p=[0.8, 0.1, 0.1]))
                start = T0 + int(rng.integers(0, 35_000_000_000))
                r = rng.random()
                if r < 0.02:
                    dur = -int(rng.integers(0, 1000))           # A2: end <= start
                elif r < 0.05:
                    dur = int(bounds_ns[int(rng.integers(len(bounds_ns)))]) + int(rng.integers(-1, 2))  # A3
                else:
                    dur = int(np.clip(rng.lognormal(np.log(5e6), 1.5), 0, 15e9))  # keeps every window in the ring
                end = start + dur
                tid = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
                sp = ss.spans.add(trace_id=tid, span_id=b"\x02" * 8, name=name, kind=kind,
                                  start_time_unix_nano=start, end_time_unix_nano=end)
                if status:
                    sp.status.code = status
                if not skip:
                    facts.append((res_attrs, demo_transform(name), kind, status, start, end, tid))
        requests.append(base64.b64encode(req.SerializeToString()).decode())
    return requests, facts


@pytest.mark.gpu
@pytest.mark.parametrize("native,devices", [(True, None), (False, None), (True, [0, 0]), (False, [0, 0])],
                         ids=["native-columnizer", "js-columnizer", "native-group2", "js-group2"])
def test_node_host_end_to_end_matches_oracle(native, devices):
    """devices=[0, 0]: the connector drives an engine group (two engines on the
    lease's one GPU, spans sharded by trace id, merged through device copies
    at every flush and window read) through the same N-API calls."""
    import pyoracle
    from spanagg.engine import SpanBatch

    requests, facts = synth_requests(seed=11)
    env = dict(os.environ, SPANAGG_NODE_GPU="1")
    config = {"batch_size": 4096, "key_capacity": 4096}
    if devices:
        config["devices"] = devices
    out = node("e2e.js", {"requests": requests, "config": config,
                          "exports_after": [3, 7], "native": native}, timeout=300, env=env)
    n = len(facts)

    # 1. the SoA v1 columns independent Python code derives from the spans
    svc_ids = out["services"]
    exp = {
        "keyHash": np.array([pykeys.series_hash(pykeys.resource_hash(ra), pykeys.build_key(
            ra["service.name"], nm, k, st)) for ra, nm, k, st, *_ in facts], dtype=np.uint64),
        "startNs": np.array([f[4] for f in facts], dtype=np.uint64),
        "endNs": np.array([f[5] for f in facts], dtype=np.uint64),
        "meta": np.array([svc_ids[f[0]["service.name"]] | (f[2] << 16) | (f[3] << 19) for f in facts],
                         dtype=np.uint32),
    }
    tids = np.frombuffer(b"".join(f[6] for f in facts), dtype="<u8").reshape(-1, 2)
    exp["traceW0"], exp["traceW1"] = tids[:, 0].copy(), tids[:, 1].copy()
    if not native:  # the JS path's columns were captured at the N-API boundary
        cols = {k: np.frombuffer(base64.b64decode(v), dtype=np.uint32 if k == "meta" else np.uint64)
                for k, v in out["columns"].items()}
        for k in exp:
            assert np.array_equal(cols[k], exp[k]), k

    # 2. the engine's deltas, summed over the three flushes, equal the oracle bit-exactly
    batch = SpanBatch(exp["keyHash"], exp["startNs"], exp["endNs"], exp["traceW0"],
                      exp["traceW1"], exp["meta"])
    o = pyoracle.Oracle(n_services=64)
    o.ingest(batch)
    ref = o.series()
    assert len(out["flushes"]) == 3 and all(f["status"] == 0 for f in out["flushes"])
    nb = 17
    tot_counts, tot_ns = {}, {}
    for f in out["flushes"]:
        keys_ = np.frombuffer(base64.b64decode(f["key_hash"]), np.uint64)
        cnt = np.frombuffer(base64.b64decode(f["bucket_counts"]), np.uint64).reshape(-1, nb)
        sns = np.frombuffer(base64.b64decode(f["sum_ns"]), np.uint64)
        for k, c, s in zip(keys_, cnt, sns):
            tot_counts[int(k)] = tot_counts.get(int(k), 0) + c.astype(np.uint64)
            tot_ns[int(k)] = tot_ns.get(int(k), 0) + int(s)
    assert sorted(tot_counts) == [int(k) for k in ref["key_hash"]]
    for i, k in enumerate(ref["key_hash"]):
        assert np.array_equal(tot_counts[int(k)], ref["bucket_counts"][i])
        assert tot_ns[int(k)] == int(ref["sum_ns"][i])

    # 3. the final cumulative OTLP metrics (parsed by python protobuf) carry the totals
    msg = M["ExportMetricsServiceRequest"].FromString(base64.b64decode(out["metrics"][-1]))
    ref_ix = {int(k): i for i, k in enumerate(ref["key_hash"])}
    seen = 0
    for rm in msg.resource_metrics:
        res_attrs = {kv.key: get_any(kv.value) for kv in rm.resource.attributes}
        calls, dur = rm.scope_metrics[0].metrics
        assert rm.scope_metrics[0].scope.name == "spanmetricsconnector"
        assert (calls.name, dur.name, dur.unit) == ("traces.span.metrics.calls",
                                                    "traces.span.metrics.duration", "ms")
        for cdp, hdp in zip(calls.sum.data_points, dur.histogram.data_points):
            a = {kv.key: get_any(kv.value) for kv in hdp.attributes}
            kind = pykeys.SPAN_KIND_STR.index(a["span.kind"])
            st = pykeys.STATUS_CODE_STR.index(a["status.code"])
            sid = pykeys.series_hash(pykeys.resource_hash(res_attrs), pykeys.build_key(
                a["service.name"], a["span.name"], kind, st))
            i = ref_ix[sid]
            assert list(hdp.bucket_counts) == [int(x) for x in ref["bucket_counts"][i]]
            assert hdp.count == int(ref["calls"][i]) == cdp.as_int
            assert abs(hdp.sum - ref["sum_go"][i]) <= 1e-9 * max(abs(ref["sum_go"][i]), 1e-300)
            assert list(hdp.explicit_bounds) == [2, 4, 6, 8, 10, 50, 100, 200, 400, 800, 1000, 1400,
                                                 2000, 5000, 10000, 15000]
            assert hdp.start_time_unix_nano < hdp.time_unix_nano
            assert calls.sum.aggregation_temporality == 2 and calls.sum.is_monotonic
            seen += 1
    assert seen == len(ref["key_hash"])
    assert not any("{productId}" not in f[1] and f[1].startswith("GET /api/products/") for f in facts)

    # 4. window sketches: HLL registers and count-min cells bit-exact
    oracle_windows = set(o.window_ids())
    assert oracle_windows and oracle_windows <= {int(w["window_id"]) for w in out["windows"]}
    for w in out["windows"]:
        wid = int(w["window_id"])
        hll = np.frombuffer(base64.b64decode(w["hll"]), np.uint8).reshape(64, 1 << 14)
        cms = np.frombuffer(base64.b64decode(w["cms"]), np.uint32).reshape(4, 2048)
        if wid in oracle_windows:
            rh, rc = o.window(wid)
            assert np.array_equal(hll, rh) and np.array_equal(cms, rc), wid
        else:
            assert not hll.any() and not cms.any()
    st = out["stats"]
    assert int(st["spans"]) == n and int(st["windowOutOfRange"]) == 0 and int(st["droppedTableFull"]) == 0
    assert int(st["engines"]) == (len(devices) if devices else 1)


def test_receiver_interoperates_with_grpcio_and_http_clients():
    """A real gRPC stack (grpcio, HTTP/2) and a plain HTTP client talk to the
    Node receiver; the bytes are Python-protobuf encoded."""
    grpc = pytest.importorskip("grpc")
    import urllib.request

    p = subprocess.Popen([NODE, os.path.join(NODE_DIR, "test", "serve.js")], stdin=subprocess.PIPE,
                         stdout=subprocess.PIPE, text=True)
    try:
        ports = json.loads(p.stdout.readline())
        raw = _py_traces_request(SPEC).SerializeToString()
        with grpc.insecure_channel(f"127.0.0.1:{ports['grpc']}") as ch:
            export = ch.unary_unary("/opentelemetry.proto.collector.trace.v1.TraceService/Export",
                                    request_serializer=None, response_deserializer=None)
            assert export(raw, timeout=10) == b""  # empty ExportTraceServiceResponse
            with pytest.raises(grpc.RpcError) as ei:
                ch.unary_unary("/opentelemetry.proto.collector.trace.v1.TraceService/Nope")(raw, timeout=10)
            assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED
        req = urllib.request.Request(f"http://127.0.0.1:{ports['http']}/v1/traces", data=raw,
                                     headers={"Content-Type": "application/x-protobuf"}, method="POST")
        with urllib.request.urlopen(req, timeout=10) as r:
            assert r.status == 200
        out, _ = p.communicate(timeout=30)
    finally:
        if p.poll() is None:
            p.kill()
    summary = json.loads(out.strip().splitlines()[-1])
    assert summary["requests"] == 2
    assert summary["spans"] == 2 * sum(len(spans) for _, spans in SPEC)
    assert summary["names"][:2] == [s["name"] for s in SPEC[0][1]]


def test_exponential_histograms_through_the_node_connector():
    """`histogram.exponential` in the Node connector (over the test stand-in
    engine, host logic only): the OTLP ExponentialHistogram it encodes, parsed
    by Python protobuf, equals an independent go-expohisto restatement
    (tests/golden/gen_expo.py) of each series' durations -- scale, offset,
    buckets, zero count, count, min, max, sum."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_expo", os.path.join(os.path.dirname(__file__), "golden",
                                                                           "gen_expo.py"))
    gen_expo = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen_expo)
    rng = np.random.default_rng(5)
    req = M["ExportTraceServiceRequest"]()
    per_series = {}
    for svc in ("frontend", "cart"):
        rs = req.resource_spans.add()
        add_attrs(rs.resource.attributes, {"service.name": svc})
        ss = rs.scope_spans.add()
        for i in range(400):
            name = f"op-{i % 3}"
            start = T0 + int(rng.integers(0, 5_000_000_000))
            dur = 0 if i % 37 == 0 else int(np.exp(rng.uniform(8, 24)))
            ss.spans.add(trace_id=rng.integers(0, 256, 16, dtype=np.uint8).tobytes(), span_id=b"\x01" * 8,
                         name=name, kind=2, start_time_unix_nano=start, end_time_unix_nano=start + dur)
            per_series.setdefault((svc, name), []).append(dur)
    out = node("cli.js", {"cmd": "connector_export", "requests": [base64.b64encode(req.SerializeToString()).decode()],
                          "spanmetrics": {"histogram": {"exponential": {"max_size": 24}}}})
    msg = M["ExportMetricsServiceRequest"].FromString(base64.b64decode(out["b64"]))
    seen = 0
    for rm in msg.resource_metrics:
        svc = {kv.key: get_any(kv.value) for kv in rm.resource.attributes}["service.name"]
        calls, dur = rm.scope_metrics[0].metrics
        assert dur.WhichOneof("data") == "exponential_histogram" and dur.unit == "ms"
        assert dur.exponential_histogram.aggregation_temporality == 2
        for dp in dur.exponential_histogram.data_points:
            name = {kv.key: get_any(kv.value) for kv in dp.attributes}["span.name"]
            h = gen_expo.Histogram(24)
            for d in per_series[(svc, name)]:
                h.update(d / 1e6)
            e = h.result()
            assert (dp.count, dp.zero_count, dp.scale, dp.positive.offset) == \
                (e["count"], e["zero_count"], e["scale"], e["offset"])
            assert list(dp.positive.bucket_counts) == e["counts"]
            assert dp.min == float.fromhex(e["min"]) and dp.max == float.fromhex(e["max"])
            assert abs(dp.sum - float.fromhex(e["sum"])) <= 1e-9 * float.fromhex(e["sum"])
            assert not dp.negative.bucket_counts
            seen += 1
    assert seen == len(per_series)


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [None, [0, 0]], ids=["engine", "group2"])
def test_node_host_exponential_end_to_end(devices):
    """histogram.exponential through the real addon: OTLP bytes -> native
    columnizer (consumeTracesBatch on worker threads) -> GPU exponential
    histograms (sa_flush_exp / sa_group_flush_exp) -> host fold of the deltas
    into cumulative histograms -> OTLP.  The last cumulative export, parsed by
    Python protobuf, equals the go-expohisto restatement of every series'
    durations (tests/golden/gen_expo.py); the window sketches stay bit-exact."""
    import importlib.util
    import pyoracle
    from spanagg.engine import SpanBatch
    spec = importlib.util.spec_from_file_location("gen_expo", os.path.join(os.path.dirname(__file__), "golden",
                                                                           "gen_expo.py"))
    gen_expo = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen_expo)
    requests, facts = synth_requests(seed=23)
    env = dict(os.environ, SPANAGG_NODE_GPU="1")
    config = {"batch_size": 4096, "key_capacity": 4096, "columnizer_threads": 4,
              "histogram": {"exponential": {"max_size": 40}}}
    if devices:
        config["devices"] = devices
    out = node("e2e.js", {"requests": requests, "config": config, "exports_after": [3, 7], "native": True,
                          "batch": True}, timeout=300, env=env)
    series = {}
    for ra, nm, k, st, start, end, _ in facts:
        sid = pykeys.series_hash(pykeys.resource_hash(ra), pykeys.build_key(ra["service.name"], nm, k, st))
        series.setdefault(sid, []).append(end - start if end > start else 0)
    msg = M["ExportMetricsServiceRequest"].FromString(base64.b64decode(out["metrics"][-1]))
    seen = 0
    for rm in msg.resource_metrics:
        res_attrs = {kv.key: get_any(kv.value) for kv in rm.resource.attributes}
        calls, dur = rm.scope_metrics[0].metrics
        assert dur.WhichOneof("data") == "exponential_histogram"
        for cdp, dp in zip(calls.sum.data_points, dur.exponential_histogram.data_points):
            a = {kv.key: get_any(kv.value) for kv in dp.attributes}
            sid = pykeys.series_hash(pykeys.resource_hash(res_attrs), pykeys.build_key(
                a["service.name"], a["span.name"], pykeys.SPAN_KIND_STR.index(a["span.kind"]),
                pykeys.STATUS_CODE_STR.index(a["status.code"])))
            h = gen_expo.Histogram(40)
            for d in series[sid]:
                h.update(d / 1e6)
            e = h.result()
            assert (dp.count, dp.zero_count, dp.scale, dp.positive.offset) == \
                (e["count"], e["zero_count"], e["scale"], e["offset"]), sid
            assert list(dp.positive.bucket_counts) == e["counts"], sid
            assert dp.min == float.fromhex(e["min"]) and dp.max == float.fromhex(e["max"])
            assert cdp.as_int == e["count"]
            seen += 1
    assert seen == len(series)
    tids = np.frombuffer(b"".join(f[6] for f in facts), dtype="<u8").reshape(-1, 2)
    svc_ids = out["services"]
    sids = [pykeys.series_hash(pykeys.resource_hash(f[0]), pykeys.build_key(f[0]["service.name"], f[1], f[2], f[3]))
            for f in facts]
    batch = SpanBatch(np.array(sids, dtype=np.uint64),
        np.array([f[4] for f in facts], dtype=np.uint64), np.array([f[5] for f in facts], dtype=np.uint64),
        tids[:, 0].copy(), tids[:, 1].copy(),
        np.array([svc_ids[f[0]["service.name"]] | (f[2] << 16) | (f[3] << 19) for f in facts], dtype=np.uint32))
    o = pyoracle.Oracle(n_services=64)
    o.ingest(batch)
    for w in out["windows"]:
        wid = int(w["window_id"])
        if wid in set(o.window_ids()):
            rh, rc = o.window(wid)
            assert np.array_equal(np.frombuffer(base64.b64decode(w["hll"]), np.uint8).reshape(64, 1 << 14), rh)
            assert np.array_equal(np.frombuffer(base64.b64decode(w["cms"]), np.uint32).reshape(4, 2048), rc)
    assert int(out["stats"]["engines"]) == (len(devices) if devices else 1)
    assert int(out["stats"]["nativeRequests"]) == len(requests)
