"""Exponential-histogram oracle (oracle/spanmetrics_oracle.c) against the
pure-Python restatement's known answers (tests/golden/expo_kat.json, made by
tests/golden/gen_expo.py): Go's math.Log bit for bit, go-expohisto's index
mapping, and whole histograms with their downscales."""
import json
import os

import numpy as np
import pytest

import pyoracle

KAT = os.path.join(os.path.dirname(__file__), "golden", "expo_kat.json")


@pytest.fixture(scope="module")
def kat():
    with open(KAT) as f:
        return json.load(f)


def test_go_log_bit_exact(kat):
    for x, y in kat["go_log"]:
        assert pyoracle.go_log(float.fromhex(x)).hex() == y, x


def test_index_mapping(kat):
    for d, s, idx in kat["map_to_index_ms"]:
        assert pyoracle.expo_index(float(d) / 1e6, s) == idx, (d, s)


def test_histograms(kat):
    for c in kat["cases"]:
        ds = np.array(c["durations_ns"], dtype=np.uint64)
        r = pyoracle.expo_series(np.zeros_like(ds), ds, c["max_size"], c["unit"] == "s")
        e = c["expected"]
        assert (r["count"], r["zero_count"]) == (e["count"], e["zero_count"]), c["name"]
        assert (r["scale"], r["offset"]) == (e["scale"], e["offset"]), c["name"]
        assert [int(x) for x in r["counts"]] == e["counts"], c["name"]
        assert r["sum"].hex() == e["sum"] and r["min"].hex() == e["min"] and r["max"].hex() == e["max"], c["name"]
