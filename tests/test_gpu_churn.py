"""Key-table churn (sa_reclaim_keys; ADVICE r1 "reclaim key slots").

A long-running collector keeps meeting new series (new pods, restarts, delta
purges), many more over its life than key_capacity.  Each flush leaves every
row at zero, and once the table is more than half full (binned tables: 35 %)
the flush empties it, so only the series of ONE flush interval have to fit.  Checked against the
oracle interval by interval (RED bit-exact, no drops) and, for the window
sketches, over all intervals at once (the per-slot error counts are folded
into the count-min before the keys go)."""
import numpy as np
import pytest

import pyoracle
from parity_util import assert_red_equal
from spanagg import Config, Engine, SpanBatch, pack_meta
from spanagg import _lib

pytestmark = pytest.mark.gpu
W = 10_000_000_000
BASE = 176_722_560


def _interval(rng, n_keys, spans_per_key, n_services=8):
    keys = rng.integers(1, 2**63, n_keys, dtype=np.int64).astype(np.uint64)
    n = n_keys * spans_per_key
    k = np.repeat(keys, spans_per_key)
    rng.shuffle(k)
    end = (BASE * W + rng.integers(0, 4 * W, n)).astype(np.uint64)
    dur = rng.integers(0, 3_000_000_000, n).astype(np.uint64)
    svc = rng.integers(0, n_services, n)
    status = np.where(rng.random(n) < 0.1, 2, 0)
    return SpanBatch(k, end - dur, end, rng.integers(0, 2**63, n, dtype=np.int64).astype(np.uint64),
                     rng.integers(0, 2**63, n, dtype=np.int64).astype(np.uint64), pack_meta(svc, 2, status))


# LDS-mirrored (small) table, partitioned HBM table, binned table
@pytest.mark.parametrize("key_capacity,per_interval", [(1000, 700), (100_000, 70_000), (300_000, 200_000)])
def test_churn_beyond_capacity_no_drops(key_capacity, per_interval):
    rng = np.random.default_rng(key_capacity)
    batches = [_interval(rng, per_interval, 2) for _ in range(5)]  # 5 x the series of one interval
    with Engine(Config(n_services=8, n_windows=8, key_capacity=key_capacity)) as e:
        e.window_advance(BASE)
        for b in batches:
            e.ingest(b)
            res = e.flush()  # raises SA_EFULL on any drop
            o = pyoracle.Oracle(n_services=8)
            o.ingest_red(b)
            assert_red_equal(res, o.series())
            assert 2 * e.stats()["n_keys"] <= e.stats()["table_capacity"]  # reclaimed when over half
        assert e.stats()["dropped_table_full"] == 0
        o = pyoracle.Oracle(n_services=8)
        for b in batches:
            o.ingest(b)
        for wid in o.window_ids():
            sk = e.window_read(wid)
            hll, cms = o.window(wid)
            assert np.array_equal(sk.hll, hll), wid
            assert np.array_equal(sk.cms, cms), wid


@pytest.mark.parametrize("n_keys,kept", [(150_000, True), (200_000, False)])
def test_binned_reclaim_threshold(n_keys, kept):
    # key_capacity 300,000: the binned table of 2^19 slots in 2,048 bins of
    # 256; the flush keeps up to 35 % (183,500 keys) resident, so a fully
    # churned next interval stays near 70 % and fills no bin
    rng = np.random.default_rng(n_keys)
    with Engine(Config(n_services=8, n_windows=8, key_capacity=300_000)) as e:
        e.window_advance(BASE)
        e.ingest(_interval(rng, n_keys, 1))
        e.flush()
        st = e.stats()
        assert st["table_capacity"] == 1 << 19 and st["small_table"] == 0
        assert st["n_keys"] == (n_keys if kept else 0)


def test_forced_reclaim_changes_nothing_and_needs_a_flush():
    rng = np.random.default_rng(5)
    a, b = _interval(rng, 500, 3), _interval(rng, 500, 3)
    outs = []
    for force in (False, True):
        with Engine(Config(n_services=8, n_windows=8, key_capacity=4000)) as e:
            e.window_advance(BASE)
            e.ingest(a)
            with pytest.raises(_lib.SpanAggError) as ei:
                e.reclaim_keys(force=True)  # unflushed spans: their rows live in the slots
            assert ei.value.code == _lib.SA_ESTATE
            first = e.flush()
            if force:
                e.reclaim_keys(force=True)
                assert e.stats()["n_keys"] == 0
            else:
                e.reclaim_keys()  # policy: 500 of 8192 slots resident, kept
                assert e.stats()["n_keys"] == 500
            e.ingest(b)
            second = e.flush()
            sk = [e.window_read(w) for w in range(BASE, BASE + 4)]
            outs.append((first, second, sk))
    (f0, s0, k0), (f1, s1, k1) = outs
    for x, y in ((f0, f1), (s0, s1)):
        assert np.array_equal(x.key_hash, y.key_hash) and np.array_equal(x.bucket_counts, y.bucket_counts)
        assert np.array_equal(x.sum_ns, y.sum_ns)
    for x, y in zip(k0, k1):
        assert np.array_equal(x.hll, y.hll) and np.array_equal(x.cms, y.cms)


def test_expo_churn_beyond_capacity():
    rng = np.random.default_rng(9)
    with Engine(Config(n_services=8, n_windows=8, key_capacity=1000, exp_max_size=20)) as e:
        e.window_advance(BASE)
        for _ in range(4):
            b = _interval(rng, 700, 2)
            e.ingest(b)
            res = e.flush_exp()
            ora = pyoracle.expo_aggregate(b, 20)
            assert [int(k) for k in res.key_hash] == sorted(ora)
            for i, k in enumerate(res.key_hash):
                o = ora[int(k)]
                assert (int(res.count[i]), int(res.scale[i]), int(res.offset[i])) == (o["count"], o["scale"], o["offset"])
                assert [int(x) for x in res.buckets[i]] == [int(x) for x in o["counts"]]
        assert e.stats()["dropped_table_full"] == 0
