"""Engine groups (include/spanagg.h sa_group_*): several engines behind one
handle, spans sharded by trace id, merged at flush / window read.  On the
one-GPU lease both transports run: two members on device 0 merge through
device copies + a reduce kernel, a group of one with SA_OPT_GROUP_RCCL
merges over a one-rank RCCL communicator.  Bar: the merge equals the CPU
oracle fed the whole stream (bucket counts, calls, ns sums, HLL registers and
count-min cells bit-exact; duration sums within 1e-9 relative)."""
import numpy as np
import pytest

import pyoracle
from parity_util import assert_red_equal
from spanagg._lib import OPT_GROUP_COPY, OPT_GROUP_RCCL
from spanagg import Config, Engine, Group
from spanagg.synth import generate_c2, generate_highcard

pytestmark = pytest.mark.gpu


def _check_windows(g, o):
    for wid in o.window_ids():
        sk = g.window_read(wid)
        hll, cms = o.window(wid)
        assert np.array_equal(sk.hll, hll), wid
        assert np.array_equal(sk.cms, cms), wid


@pytest.mark.parametrize("devices,rccl", [([0, 0], False), ([0, 0, 0], False), ([0], True)])
def test_group_matches_oracle_c2(devices, rccl):
    wl = generate_c2(400_003, seed=21)
    opt = OPT_GROUP_RCCL if rccl else OPT_GROUP_COPY
    with Group(devices, Config(n_services=wl.n_services, n_windows=16, options=opt)) as g:
        assert g.size == len(devices)
        assert g.uses_rccl == rccl
        g.window_advance(wl.first_window)
        g.ingest(wl.batch)
        res = g.flush()
        o = pyoracle.Oracle(n_services=wl.n_services)
        o.ingest(wl.batch)
        assert_red_equal(res, o.series())
        _check_windows(g, o)
        st = g.stats()
        assert st["spans"] == len(wl.batch)
        # members keep their keys, or the flush emptied their more than half
        # full tables (sa_reclaim_keys; 2,048 slots each here)
        assert st["n_keys"] == 0 or st["n_keys"] >= len(res.key_hash)


def test_group_delta_flushes_and_equals_one_engine():
    wl = generate_c2(300_000, seed=5)
    a, b = wl.batch.slice(0, 170_000), wl.batch.slice(170_000, 300_000)
    cfg = Config(n_services=wl.n_services, n_windows=16, options=OPT_GROUP_COPY)
    with Group([0, 0], cfg) as g, Engine(cfg) as e:
        for x in (g, e):
            x.window_advance(wl.first_window)
        for part in (a, b):
            g.ingest(part)
            e.ingest(part)
            rg, re_ = g.flush(), e.flush()
            assert np.array_equal(rg.key_hash, re_.key_hash)
            assert np.array_equal(rg.bucket_counts, re_.bucket_counts)
            assert np.array_equal(rg.sum_ns, re_.sum_ns)
        empty = g.flush()  # nothing since the last flush
        assert len(empty.key_hash) == 0


def test_group_high_cardinality_binned_members():
    """Members on the binned HBM-table path (1 M keys): the key union spans
    series seen by one member only and by both."""
    batch, _, first = generate_highcard(1_500_000, seed=3)
    with Group([0, 0], Config(n_services=1, n_windows=16, key_capacity=1_200_000, options=OPT_GROUP_COPY)) as g:
        g.window_advance(first)
        g.ingest(batch)
        res = g.flush()
        o = pyoracle.Oracle(n_services=1)
        o.ingest(batch)
        assert_red_equal(res, o.series())
        _check_windows(g, o)


def test_group_rejects_bad_arguments():
    with pytest.raises(Exception):
        Group([], Config())


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
def test_group_exponential_histograms_fold_to_one_engine(devices):
    """sa_group_flush_exp: each member's delta exponential histograms (its own
    trace-id shard, so its own scales) folded per series on the host must be
    the histogram of the whole stream, bit-exact against the go-expohisto
    restatement, over two flush intervals."""
    wl = generate_c2(300_000, seed=31)
    parts = [wl.batch.slice(0, 120_000), wl.batch.slice(120_000, 300_000)]
    with Group(devices, Config(n_services=wl.n_services, n_windows=16, exp_max_size=12)) as g:
        g.window_advance(wl.first_window)
        for part in parts:
            g.ingest(part)
            res = g.flush_exp()
            ora = pyoracle.expo_aggregate(part, 12)
            assert [int(k) for k in res.key_hash] == sorted(ora)
            for i, k in enumerate(res.key_hash):
                o = ora[int(k)]
                assert (int(res.count[i]), int(res.zero_count[i]), int(res.scale[i]), int(res.offset[i])) == \
                    (o["count"], o["zero_count"], o["scale"], o["offset"]), k
                assert [int(x) for x in res.buckets[i]] == [int(x) for x in o["counts"]], k
                assert res.min[i] == o["min"] and res.max[i] == o["max"]
        with pytest.raises(Exception):
            g.flush()  # explicit-bucket flush of an exponential group: SA_ESTATE
        o = pyoracle.Oracle(n_services=wl.n_services)
        o.ingest(wl.batch)
        _check_windows(g, o)
