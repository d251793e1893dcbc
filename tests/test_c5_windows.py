"""Config C5: sliding 10 s windows over a 600 s stream with
injected anomalies -- the per-service HLL distinct-trace and count-min ERROR
sketches, streamed through a resident ring of 8 windows that advances with the
data.  CPU tests check the workload and the detection on the oracle's
sketches; the GPU test streams the same spans through libspanagg and requires
every window's registers and cells to be bit-exact with the oracle."""
import numpy as np
import pytest

import pyoracle
from spanagg.sketch import anomalous, cms_query, distinct_traces, heavy_hitters
from spanagg.synth import generate_c5

N = 300_000
RING = 8


@pytest.fixture(scope="module")
def c5():
    return generate_c5(N)


@pytest.fixture(scope="module")
def oracle_windows(c5):
    o = pyoracle.Oracle(n_services=c5.base.n_services)
    o.ingest(c5.base.batch)
    return {w: o.window(w) for w in o.window_ids()}


def error_keys(c5):
    """Series ids of the payment service's ERROR keys (status code 2)."""
    ks = c5.base.key_strings
    return [int(c5.base.key_hashes[i]) for i, (svc, _, _, st) in enumerate(ks)
            if st == 2 and svc == "payment"]


def detect(c5, windows):
    """(payment ERROR estimate, frontend distinct traces) per window offset."""
    pay_err, fe_distinct = [], []
    ekeys = error_keys(c5)
    for off in range(c5.n_windows):
        hll, cms = windows[c5.first_window + off]
        pay_err.append(sum(cms_query(cms, k) for k in ekeys))
        fe_distinct.append(distinct_traces(hll[c5.burst_service:c5.burst_service + 1], 14)[0])
    return pay_err, fe_distinct


def test_c5_stream_is_time_ordered_and_spans_sixty_windows(c5):
    end = c5.base.batch.end_ns
    assert np.all(np.diff(end.astype(np.int64)) >= 0)
    wins = end // np.uint64(c5.window_ns)
    assert int(wins.min()) == c5.first_window
    assert int(wins.max()) == c5.first_window + c5.n_windows - 1


def test_cms_point_query_bounds_the_exact_error_count(c5, oracle_windows):
    b = c5.base.batch
    wins = (b.end_ns // np.uint64(c5.window_ns)).astype(np.int64)
    err = ((b.meta >> 19) & 3) == 2
    for off in (0, 31, 59):
        w = c5.first_window + off
        _, cms = oracle_windows[w]
        keys, counts = np.unique(b.key_hash[err & (wins == w)], return_counts=True)
        for k, c in zip(keys, counts):
            assert cms_query(cms, int(k)) >= int(c)
        assert int(cms.sum(axis=1)[0]) == int(counts.sum())  # each row counts every ERROR span once


def test_oracle_sketches_flag_exactly_the_injected_windows(c5, oracle_windows):
    pay_err, fe = detect(c5, oracle_windows)
    lo, hi = c5.error_windows
    assert anomalous(pay_err, factor=5.0) == list(range(lo, hi + 1))
    blo, bhi = c5.burst_windows
    assert anomalous(fe, factor=2.0, min_base=10.0) == list(range(blo, bhi + 1))
    # heavy hitters inside an anomalous window are payment ERROR series
    hh = heavy_hitters(oracle_windows[c5.first_window + lo][1], error_keys(c5), k=3)
    assert hh and all(c > 0 for _, c in hh)


@pytest.mark.gpu
def test_c5_streamed_through_a_ring_of_8_windows_is_bit_exact(c5, oracle_windows):
    from spanagg import Config, Engine

    b = c5.base.batch
    wins = (b.end_ns // np.uint64(c5.window_ns)).astype(np.int64)
    cuts = np.searchsorted(wins, np.arange(c5.first_window, c5.first_window + c5.n_windows + 1))
    got = {}
    with Engine(Config(n_services=c5.base.n_services, n_windows=RING, key_capacity=1000)) as e:
        base = c5.first_window
        e.window_advance(base)
        for off in range(c5.n_windows):
            w = c5.first_window + off
            if w >= base + RING:  # the ring moves with the data: close the oldest window
                sk = e.window_read(base)
                got[base] = (sk.hll, sk.cms)
                base += 1
                e.window_advance(base)
            e.ingest(b.slice(int(cuts[off]), int(cuts[off + 1])))
        for w in range(base, c5.first_window + c5.n_windows):
            sk = e.window_read(w)
            got[w] = (sk.hll, sk.cms)
        st = e.stats()
        red = e.flush()
    assert st["window_out_of_range"] == 0 and st["dropped_table_full"] == 0
    assert int(red.calls.sum()) == len(b)
    for w, (hll, cms) in oracle_windows.items():
        assert np.array_equal(got[w][0], hll), w
        assert np.array_equal(got[w][1], cms), w
    assert detect(c5, got) == detect(c5, oracle_windows)
