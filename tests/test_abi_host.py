"""libspanagg C-ABI: loads, exports every declared symbol, host-only helpers are
exact, and the product path fails loudly without a gfx950 GPU (no CPU fallback)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import pyoracle
from spanagg import _lib, bucket_thresholds, hll_estimate
from spanagg.engine import Config, Engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(headers=("spanagg.h", "spanagg_diag.h")):
    text = "".join(open(os.path.join(ROOT, "include", h)).read() for h in headers)
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sa_[a-z_]+)\s*\(", text)))


def test_diagnostic_entry_points_live_outside_the_product_header():
    """Verdict r4: the probes and the stamp reader are declared in
    spanagg_diag.h, which the drop-in header does not include."""
    product, diag = declared_symbols(("spanagg.h",)), declared_symbols(("spanagg_diag.h",))
    probes = {"sa_expo_probe", "sa_expo_fast_probe", "sa_key_union_probe", "sa_debug_stamps"}
    assert probes <= set(diag)
    assert not probes & set(product)
    assert '#include "spanagg_diag.h"' not in open(os.path.join(ROOT, "include", "spanagg.h")).read()


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 19
    for s in syms:
        assert hasattr(lib, s), s
    # the ctypes signature table covers the whole header
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == syms


def test_abi_version():
    assert _lib.load().sa_abi_version() == 4


def test_product_library_has_no_laboratory():
    """Verdict r3: the product libspanagg.so reads no environment (no getenv
    import at all) and carries one kernel per path; the A/B variants and the
    ablation kernels live in the laboratory build (libspanagg_ab.so, tools/)."""
    import subprocess
    so = os.path.join(os.path.dirname(_lib.__file__), "libspanagg.so")
    dyn = subprocess.run(["nm", "-D", "--undefined-only", so], capture_output=True, text=True, check=True).stdout
    assert "getenv" not in dyn
    strings = subprocess.run(["strings", so], capture_output=True, text=True, check=True).stdout
    for lab in ("bt_aggregate2_kernel", "ingest_lds_kernelILi1E", "SPANAGG_VARIANT", "SPANAGG_BT_AGG",
                "SPANAGG_XT", "SPANAGG_FAIL_AGG", "SPANAGG_NO_SETEV", "SPANAGG_XREC", "SPANAGG_XSTREAM", "SPANAGG_XIDX_OFF"):
        assert lab not in strings, lab


def test_diagnostic_flags_rejected_by_product_library():
    """SA_DIAG_* ablations need the laboratory build: the product library
    refuses them (before touching a device) instead of running wrong kernels."""
    with pytest.raises(_lib.SpanAggError) as ei:
        Engine(Config(flags=1))
    assert ei.value.code == _lib.SA_EINVAL
    with pytest.raises(_lib.SpanAggError) as ei:
        Engine(Config(options=1 << 20))  # unknown option bit
    assert ei.value.code == _lib.SA_EINVAL


def test_config_default_matches_connector_defaults():
    lib = _lib.load()
    c = _lib.sa_config()
    lib.sa_config_default(C.byref(c))
    assert [c.bounds[i] for i in range(c.n_bounds)] == [
        2, 4, 6, 8, 10, 50, 100, 200, 400, 800, 1000, 1400, 2000, 5000, 10000, 15000]
    assert c.unit == _lib.SA_UNIT_MS
    assert (c.hll_p, c.cms_d, c.cms_w, c.window_ns) == (14, 4, 2048, 10_000_000_000)


def test_thresholds_default_are_exact_ms():
    thr, nneg = bucket_thresholds([2, 4, 6, 8, 10, 50, 100, 200, 400, 800, 1000, 1400, 2000, 5000,
                                   10000, 15000])
    assert nneg == 0
    assert [int(t) for t in thr] == [int(b * 1_000_000) for b in
                                     (2, 4, 6, 8, 10, 50, 100, 200, 400, 800, 1000, 1400, 2000,
                                      5000, 10000, 15000)]


def test_thresholds_match_golden(golden):
    for case in golden["cases"]:
        thr, nneg = bucket_thresholds(case["bounds"], case["unit"])
        exp = case["expected"]["thresholds"]
        assert nneg == exp["n_neg"], case["name"]
        assert [int(t) for t in thr] == exp["thr"], case["name"]


@pytest.mark.parametrize("unit", ["ms", "s"])
def test_threshold_bucketing_equals_search_float64s(unit):
    """A4: n_neg + #{d > T_i} == SearchFloat64s(bounds, float64(d)/div) for all d."""
    rng = np.random.default_rng(11)
    bounds = np.sort(np.concatenate([rng.uniform(0, 20, 10), rng.uniform(-1, 0, 2),
                                     [1e-7, 0.333, 1e15]]))
    thr, nneg = bucket_thresholds(bounds, unit)
    div = 1e9 if unit == "s" else 1e6
    ds = ([int(x) for x in rng.integers(0, 30 * int(div), 3000)]
          + [int(t) + k for t in thr if 0 < int(t) < 2**62 for k in (-1, 0, 1)]
          + [0, 1, 2**53 - 1, 2**53, 2**53 + 1, 2**63, 2**64 - 1])
    for d in ds:
        mine = nneg + sum(1 for t in thr if d > int(t))
        ref = pyoracle.search_float64s(bounds, pyoracle.duration(0, d, unit == "s"))
        assert mine == ref, d


def test_thresholds_reject_unsorted_and_nan():
    with pytest.raises(Exception):
        bucket_thresholds([3, 2, 1])
    with pytest.raises(Exception):
        bucket_thresholds([1, float("nan")])


def test_hll_estimate_matches_oracle():
    rng = np.random.default_rng(5)
    for p in (4, 8, 14):
        for fill in (0.0, 0.01, 0.3, 1.0):
            regs = np.where(rng.random(1 << p) < fill, rng.integers(1, 20, 1 << p), 0).astype(np.uint8)
            a, b = hll_estimate(regs, p), pyoracle.hll_estimate(regs, p)
            assert a == pytest.approx(b, rel=1e-12, abs=0)


def test_engine_fails_loudly_without_gpu(has_gpu):
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(_lib.SpanAggError) as ei:
        Engine(Config())
    assert ei.value.code == _lib.SA_EDEVICE


def test_engine_rejects_bad_config():
    with pytest.raises(_lib.SpanAggError) as ei:
        Engine(Config(cms_w=1000))
    assert ei.value.code == _lib.SA_EINVAL
    with pytest.raises(_lib.SpanAggError):
        Engine(Config(bounds=(5, 1)))


def test_group_fails_loudly_without_gpu(has_gpu):
    from spanagg import Group
    if has_gpu:
        pytest.skip("GPU present")
    with pytest.raises(_lib.SpanAggError) as ei:
        Group([0, 0], Config())
    assert ei.value.code == _lib.SA_EDEVICE
    with pytest.raises(_lib.SpanAggError) as ei:
        Group([], Config())
    assert ei.value.code == _lib.SA_EINVAL
