"""What the reference itself pins on this path, checked on CPU:

* the output-name contract: the Grafana dashboards query
  traces_span_metrics_calls_total / traces_span_metrics_duration_milliseconds_*
  with labels service_name, span_name, status_code and the value
  STATUS_CODE_ERROR (tests/golden/dashboard_contract.json, extracted from
  src/grafana/provisioning/dashboards/demo/*.json by
  tests/golden/extract_dashboard_contract.py).  The Node host's OTLP metrics
  output, translated the way Prometheus' OTLP receiver does it, must yield
  exactly those series names and labels;
* the collector config: the host reads the demo's own
  otelcol-config.yml (+ extras) and derives the connector config, the
  transform rules and the pipeline wiring from it.

The reference files are read only when /root/reference is present (this
container); the GPU box runs none of this.
"""
import base64
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
from test_node_host import NODE, add_attrs, demo_transform, get_any, node  # noqa: E402
from otlp_pb import M  # noqa: E402

REF = "/root/reference"
CONTRACT = os.path.join(HERE, "golden", "dashboard_contract.json")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")
need_ref = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")), reason="reference absent")

# Prometheus 3.3.1 (.env:21) OTLP receiver, default translation strategy
# (UnderscoreEscapingWithSuffixes), restated: metric names are split on
# characters outside [A-Za-z0-9], the unit's full word is appended unless
# already a token, monotonic sums get `_total`; histograms expose _bucket
# (label `le`), _sum and _count; attribute keys map every character outside
# [A-Za-z0-9_] to `_` (a leading digit gets a `key_` prefix).
UNIT_WORDS = {"ms": "milliseconds", "s": "seconds", "us": "microseconds", "ns": "nanoseconds",
              "By": "bytes", "1": ""}


def prom_metric_name(name, unit, monotonic_sum):
    tokens = [t for t in re.split(r"[^A-Za-z0-9]+", name) if t]
    word = UNIT_WORDS.get(unit, unit)
    if word and word not in tokens:
        tokens.append(word)
    if monotonic_sum and tokens[-1] != "total":
        tokens.append("total")
    return "_".join(tokens)


def prom_label(key):
    k = re.sub(r"[^A-Za-z0-9_]", "_", key)
    return "key_" + k if k[:1].isdigit() else k


def prom_series(msg):
    """ExportMetricsServiceRequest -> {series name: [label dicts]}."""
    out = {}
    for rm in msg.resource_metrics:
        for sm in rm.scope_metrics:
            for m in sm.metrics:
                kind = m.WhichOneof("data")
                if kind == "sum":
                    base = prom_metric_name(m.name, m.unit, m.sum.is_monotonic)
                    for dp in m.sum.data_points:
                        out.setdefault(base, []).append(
                            {prom_label(kv.key): str(get_any(kv.value)) for kv in dp.attributes})
                elif kind == "histogram":
                    base = prom_metric_name(m.name, m.unit, False)
                    for dp in m.histogram.data_points:
                        lab = {prom_label(kv.key): str(get_any(kv.value)) for kv in dp.attributes}
                        out.setdefault(base + "_sum", []).append(lab)
                        out.setdefault(base + "_count", []).append(lab)
                        for le in list(dp.explicit_bounds) + ["+Inf"]:
                            out.setdefault(base + "_bucket", []).append(dict(lab, le=str(le)))
    return out


def traces_request():
    """Three services, every span kind and status code, query strings and a
    product-id path the demo's transform rules rewrite."""
    req = M["ExportTraceServiceRequest"]()
    t0 = 1_700_000_000_000_000_000
    for si, svc in enumerate(["frontend", "payment", "product-catalog"]):
        rs = req.resource_spans.add()
        add_attrs(rs.resource.attributes, {"service.name": svc})
        ss = rs.scope_spans.add()
        for i in range(12):
            sp = ss.spans.add()
            sp.trace_id = bytes([si, i]) + bytes(14)
            sp.span_id = bytes([i]) * 8
            sp.name = ["GET /api/products/0PUK6V6EV0?currencyCode=USD", "oteldemo.PaymentService/Charge",
                       "GET /api/cart?sessionId=1"][i % 3]
            sp.kind = i % 6
            sp.start_time_unix_nano = t0 + i
            sp.end_time_unix_nano = t0 + i + (i + 1) * 1_500_000
            sp.status.code = i % 3
    return req.SerializeToString()


def contract():
    with open(CONTRACT) as f:
        return json.load(f)


@need_ref
def test_dashboard_contract_fixture_is_current():
    p = subprocess.run([sys.executable, os.path.join(HERE, "golden", "extract_dashboard_contract.py"), "--check"])
    assert p.returncode == 0, "tests/golden/dashboard_contract.json is stale: re-run the extractor"


def test_host_output_yields_the_dashboards_series():
    out = node("cli.js", {"cmd": "connector_export",
                          "requests": [base64.b64encode(traces_request()).decode()]})
    series = prom_series(M["ExportMetricsServiceRequest"].FromString(base64.b64decode(out["b64"])))
    c = contract()
    # every series name the dashboards query exists, and the host emits no other spanmetrics series
    assert set(c["metrics"]) <= set(series), sorted(series)
    assert {s for s in series if s.startswith("traces_span_metrics")} == set(c["metrics"])
    for name in c["metrics"]:
        keys = set().union(*(set(lab) for lab in series[name]))
        wanted = set(c["label_keys"]) - ({"le"} if not name.endswith("_bucket") else set())
        assert wanted <= keys, (name, sorted(keys))
    for key, values in c["label_values"].items():
        seen = {lab.get(key) for lab in series["traces_span_metrics_calls_total"]}
        assert set(values) <= seen, (key, seen)
    # the four datapoint attributes and nothing else (no dimensions configured)
    labs = series["traces_span_metrics_calls_total"][0]
    assert set(labs) == {"service_name", "span_name", "span_kind", "status_code"}
    assert {lab["span_kind"] for lab in series["traces_span_metrics_calls_total"]} >= {
        "SPAN_KIND_SERVER", "SPAN_KIND_CLIENT", "SPAN_KIND_INTERNAL"}


@need_ref
def test_collector_config_read_from_the_reference_files():
    texts = []
    for f in ("otelcol-config.yml", "otelcol-config-extras.yml"):
        with open(os.path.join(REF, "src", "otel-collector", f)) as fh:
            texts.append(fh.read())
    names = ["GET /api/products/0PUK6V6EV0", "GET /api/products/0PUK6V6EV0?currencyCode=USD",
             "GET /api/cart?sessionId=abc", "POST /api/products/1", "GET /api/products", "?", "a?b?c",
             "oteldemo.CartService/GetCart", ""]
    got = node("cli.js", {"cmd": "collector_config", "texts": texts,
                          "env": {"OTEL_COLLECTOR_HOST": "otel-collector", "OTEL_COLLECTOR_PORT_HTTP": "4318"},
                          "names": names})
    assert got["spanmetrics"] == {}  # `spanmetrics:` with an empty body: createDefaultConfig
    assert got["memory_limiter"] == {"check_interval": "5s", "limit_percentage": 80,
                                     "spike_limit_percentage": 25}
    assert got["wiring"]["traces"]["processors"] == ["memory_limiter", "transform", "batch"]
    assert got["wiring"]["metrics"]["exporters"][0] == "otlphttp/prometheus"
    assert got["n_rules"] == 2 and got["error_mode"] == "ignore"
    assert got["names"] == [demo_transform(n) for n in names]


@need_ref
def test_host_output_under_the_reference_config_matches_the_contract():
    """The pipeline built from the reference's own config file: the transform
    rules collapse the product ids and strip the query strings before keying."""
    texts = []
    for f in ("otelcol-config.yml", "otelcol-config-extras.yml"):
        with open(os.path.join(REF, "src", "otel-collector", f)) as fh:
            texts.append(fh.read())
    out = node("cli.js", {"cmd": "connector_export", "texts": texts,
                          "requests": [base64.b64encode(traces_request()).decode()]})
    series = prom_series(M["ExportMetricsServiceRequest"].FromString(base64.b64decode(out["b64"])))
    assert set(contract()["metrics"]) <= set(series)
    span_names = {lab["span_name"] for lab in series["traces_span_metrics_calls_total"]}
    assert span_names == {"GET /api/products/{productId}", "oteldemo.PaymentService/Charge", "GET /api/cart"}


def test_prometheus_name_translation_restatement():
    assert prom_metric_name("traces.span.metrics.calls", "", True) == "traces_span_metrics_calls_total"
    assert prom_metric_name("traces.span.metrics.duration", "ms", False) == \
        "traces_span_metrics_duration_milliseconds"
    assert prom_label("service.name") == "service_name"
    assert prom_label("1abc") == "key_1abc"
