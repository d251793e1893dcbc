#!/usr/bin/env python3
"""Extracts the spanmetrics output contract that the reference's Grafana
dashboards pin into tests/golden/dashboard_contract.json.

Reads every PromQL expression of
/root/reference/src/grafana/provisioning/dashboards/demo/*.json that queries a
`traces_span_metrics_*` series and records:
  * the metric names it queries,
  * the label keys it matches on or groups by (`le` included),
  * the label values it matches literally (e.g. status_code="STATUS_CODE_ERROR"),
  * per dashboard file, how many expressions and which metrics.
The JSON is data only (names, keys, values, counts); no dashboard text is kept.

Run in this container (the reference is absent on the GPU box):
    python tests/golden/extract_dashboard_contract.py [--check]
--check exits 1 when the committed fixture differs from a fresh extraction.
"""
import glob
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/src/grafana/provisioning/dashboards/demo"
OUT = os.path.join(HERE, "dashboard_contract.json")
METRIC_RE = re.compile(r"\b(traces_span_metrics_[a-z_]+)")
MATCHER_RE = re.compile(r"([A-Za-z_][A-Za-z0-9_]*)\s*(=~|!~|!=|=)\s*\"([^\"]*)\"")
BY_RE = re.compile(r"\bby\s*\(([^)]*)\)")


def exprs_of(obj, out):
    if isinstance(obj, dict):
        for k, v in obj.items():
            if k in ("expr", "query") and isinstance(v, str):
                out.append(v)
            exprs_of(v, out)
    elif isinstance(obj, list):
        for x in obj:
            exprs_of(x, out)
    return out


def extract(ref_dir=REF):
    metrics, label_keys, literal = set(), set(), {}
    files = {}
    for path in sorted(glob.glob(os.path.join(ref_dir, "*.json"))):
        with open(path) as f:
            doc = json.load(f)
        found = [e for e in exprs_of(doc, []) if "traces_span_metrics" in e]
        if not found:
            continue
        fm = set()
        for e in found:
            names = set(METRIC_RE.findall(e))
            fm |= names
            metrics |= names
            for key, op, val in MATCHER_RE.findall(e):
                if key == "__name__":
                    continue
                label_keys.add(key)
                if op == "=" and not val.startswith("$"):
                    literal.setdefault(key, set()).add(val)
            for grp in BY_RE.findall(e):
                label_keys |= {g.strip() for g in grp.split(",") if g.strip()}
        files[os.path.basename(path)] = {"expressions": len(found), "metrics": sorted(fm)}
    return {
        "source": "src/grafana/provisioning/dashboards/demo/*.json (PromQL over Prometheus' OTLP translation)",
        "metrics": sorted(metrics),
        "label_keys": sorted(label_keys),
        "label_values": {k: sorted(v) for k, v in sorted(literal.items())},
        "files": files,
    }


def main():
    got = extract()
    if "--check" in sys.argv:
        with open(OUT) as f:
            sys.exit(0 if json.load(f) == got else 1)
    with open(OUT, "w") as f:
        json.dump(got, f, indent=1, sort_keys=True)
        f.write("\n")
    print(json.dumps(got, indent=1))


if __name__ == "__main__":
    main()
