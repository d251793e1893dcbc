"""Shared comparison helpers: product (GPU) results vs the CPU oracle."""
import numpy as np

SUM_RTOL = 1e-9  # north_star: duration sums within 1e-9 relative


def assert_red_equal(res, ora, unit_div=1e6):
    """res: spanagg.RedResult; ora: pyoracle.Oracle.series() dict."""
    assert len(res.key_hash) == len(ora["key_hash"]), (len(res.key_hash), len(ora["key_hash"]))
    assert np.array_equal(res.key_hash, ora["key_hash"])
    assert np.array_equal(res.bucket_counts, ora["bucket_counts"])       # bit-exact
    assert np.array_equal(res.calls, ora["calls"])                       # A8
    assert np.array_equal(res.sum_ns, ora["sum_ns"])                     # exact ns
    ref = ora["sum_go"]
    denom = np.maximum(np.abs(ref), 1e-300)
    rel = np.abs(res.sum - ref) / denom
    ok = (rel <= SUM_RTOL) | ((ref == 0) & (res.sum == 0))
    assert ok.all(), f"sum rel err max {rel.max()}"


def assert_red_golden(res, exp_series):
    assert [int(k) for k in res.key_hash] == [s["key"] for s in exp_series]
    for i, s in enumerate(exp_series):
        assert [int(c) for c in res.bucket_counts[i]] == s["counts"]
        assert int(res.calls[i]) == sum(s["counts"])
        assert int(res.sum_ns[i]) == s["sum_ns"]
        ref = float.fromhex(s["sum_go"])
        if ref == 0:
            assert res.sum[i] == 0
        else:
            assert abs(res.sum[i] - ref) / abs(ref) <= SUM_RTOL


def sketch_sparse(hll, cms):
    nz = np.argwhere(hll)
    h = sorted([int(a), int(b), int(hll[a, b])] for a, b in nz)
    nz = np.argwhere(cms)
    c = sorted([int(a), int(b), int(cms[a, b])] for a, b in nz)
    return h, c
