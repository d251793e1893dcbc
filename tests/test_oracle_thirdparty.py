"""The golden RED answers against a third-party histogram implementation.

The golden vectors (tests/golden/gen_golden.py) and the C oracle are both this
repository's restatements of the connector's per-span body ([UPSTREAM]
spanmetricsconnector connector.go aggregateMetrics -> internal/metrics
explicitHistogram.Observe: `sort.SearchFloat64s(bounds, value)`, a float64
sum in arrival order).  Here the same spans go through prometheus_client
(0.26, importable in this image; the demo's metrics end in Prometheus), whose
Histogram.observe adds the value to a float sum and counts it in the first
bucket with value <= bound (+Inf last) -- the "le" semantics SearchFloat64s
implements.  Per series (zero keys skipped, as the connector skips spans it
cannot key), every bucket count and the float sum must equal the golden
answer exactly, which pins the bucket boundary rule (a value on a bound falls
in that bound's bucket), the +Inf bucket, the float64 ns -> unit conversion,
a negative duration's 0 and the summation order against code this repository
did not write.  (This pins the RED semantics, not the Go connector itself:
its source is not in the container)
"""
import collections

import pytest

prometheus_client = pytest.importorskip("prometheus_client")


def _prom_series(case):
    div = 1e6 if case["unit"] == "ms" else 1e9
    hists = collections.OrderedDict()
    reg = prometheus_client.CollectorRegistry()
    for i, (key, start, end, _w0, _w1, _meta) in enumerate(case["spans"]):
        if key == 0:
            continue
        if key not in hists:
            hists[key] = prometheus_client.Histogram(f"h{len(hists)}", "golden", buckets=list(case["bounds"]),
                                                     registry=reg)
        d = end - start if end > start else 0
        hists[key].observe(float(d) / div)
    out = {}
    for key, h in hists.items():
        # cumulative "le" buckets in bound order, +Inf last
        cum = [s.value for s in h.collect()[0].samples if s.name.endswith("_bucket")]
        counts = [int(cum[0])] + [int(cum[i] - cum[i - 1]) for i in range(1, len(cum))]
        # (the exposition omits _sum when a bound is negative; the float the
        # histogram accumulated is read from the histogram itself)
        out[key] = (counts, float(h._sum.get()))
    return out


@pytest.mark.parametrize("idx", range(5))
def test_golden_red_matches_prometheus_client(golden, idx):
    case = golden["cases"][idx]
    got = _prom_series(case)
    exp = case["expected"]["series"]
    assert sorted(got) == sorted(s["key"] for s in exp)
    for s in exp:
        counts, total = got[s["key"]]
        assert counts == s["counts"], (case["name"], s["key"])
        assert total.hex() == s["sum_go"], (case["name"], s["key"])
