"""The CPU oracle (oracle/) against the committed golden vectors.

The vectors come from tests/golden/gen_golden.py, an independent pure-Python
restatement of the connector semantics that hashes with
the third-party xxhash package.  Numeric parity against the real Go connector
is unpinned (its source is not available); see DESIGN.md section 3.
"""
import numpy as np
import pytest

import pyoracle
from spanagg import SpanBatch


def _batch(spans):
    a = np.array(spans, dtype=object) if spans else np.zeros((0, 6), dtype=object)
    col = lambda i, dt: np.array([int(x) for x in a[:, i]], dtype=dt) if len(a) else np.zeros(0, dt)
    return SpanBatch(col(0, np.uint64), col(1, np.uint64), col(2, np.uint64), col(3, np.uint64),
                     col(4, np.uint64), col(5, np.uint32))


def _oracle_for(case):
    return pyoracle.Oracle(bounds=case["bounds"], unit=case["unit"], hll_p=case["hll_p"],
                           cms_d=case["cms_d"], cms_w=case["cms_w"], window_ns=case["window_ns"],
                           n_services=case["n_services"])


def test_xxh64_vectors(golden):
    for v in golden["xxh64_vectors"]:
        assert pyoracle.xxh64(bytes.fromhex(v["data"]), v["seed"]) == v["xxh64"]


def test_splitmix64_vectors(golden):
    for v in golden["splitmix64_vectors"]:
        assert pyoracle.splitmix64(v["x"]) == v["splitmix64"]


@pytest.mark.parametrize("idx", range(5))
def test_oracle_reproduces_golden(golden, idx):
    case = golden["cases"][idx]
    o = _oracle_for(case)
    o.ingest(_batch(case["spans"]))
    exp = case["expected"]
    got = o.series()
    assert [int(k) for k in got["key_hash"]] == [s["key"] for s in exp["series"]]
    for i, s in enumerate(exp["series"]):
        assert [int(c) for c in got["bucket_counts"][i]] == s["counts"]
        assert int(got["calls"][i]) == sum(s["counts"])           # A8
        assert float(got["sum_go"][i]).hex() == s["sum_go"]       # A9, bit-exact Go order
        assert int(got["sum_ns"][i]) == s["sum_ns"]
    assert o.window_ids() == [w["window"] for w in exp["windows"]]
    for w in exp["windows"]:
        hll, cms = o.window(w["window"])
        nz = np.argwhere(hll)
        assert sorted([int(a), int(b), int(hll[a, b])] for a, b in nz) == w["hll"]
        nz = np.argwhere(cms)
        assert sorted([int(a), int(b), int(cms[a, b])] for a, b in nz) == w["cms"]
    assert o.stats() == exp["stats"]


def test_known_answers_kat_basic(golden):
    """Spot-check the hand-built case against the Appendix A statements."""
    case = golden["cases"][0]
    assert case["name"] == "kat_basic"
    s = {x["key"]: x for x in case["expected"]["series"]}
    k1 = s[0x1111111111111111]["counts"]
    assert k1[0] == 3          # exactly 2 ms, zero duration, end < start (A2, A3)
    assert k1[1] == 2          # 2 ms + 1 ns (A3), and 3 ms from the invalid-service span
                               # (RED still counts it; only sketches skip it)
    assert k1[15] == 1         # exactly 15 s
    assert k1[16] == 1         # +Inf bucket
    assert case["expected"]["stats"] == dict(spans=13, invalid_service=1, zero_key=1)


def test_search_float64s_matches_bisect():
    import bisect
    rng = np.random.default_rng(3)
    bounds = sorted(rng.uniform(-5, 100, 20).tolist())
    for x in np.concatenate([rng.uniform(-10, 110, 500), np.array(bounds)]):
        assert pyoracle.search_float64s(bounds, x) == bisect.bisect_left(bounds, x)


def test_hll_estimate_small_range():
    p = 10
    regs = np.zeros(1 << p, np.uint8)
    assert pyoracle.hll_estimate(regs, p) == 0.0
    regs[:100] = 1
    m = 1 << p
    assert abs(pyoracle.hll_estimate(regs, p) - m * np.log(m / (m - 100))) < 1e-9
