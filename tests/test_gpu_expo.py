"""Exponential histograms on the GPU (sa_config.exp_max_size, the
spanmetrics `histogram.exponential` option) against the oracle's
value-by-value go-expohisto restatement (oracle/spanmetrics_oracle.c,
itself pinned to tests/golden/expo_kat.json).  Bar: count, zero count,
scale, offset and every bucket bit-exact; min/max exact; sum within 1e-9
relative (exact ns on the GPU, arrival-order float64 in the oracle); the
kernel's Go math.Log bit-exact with the oracle's."""
import json
import os

import numpy as np
import pytest

import pyoracle
from spanagg._lib import OPT_EXPO_CACHED, OPT_EXPO_HBM
from spanagg import Config, Engine, SpanBatch, pack_meta
from spanagg import _lib
from spanagg.synth import generate_c2

pytestmark = pytest.mark.gpu
KAT = os.path.join(os.path.dirname(__file__), "golden", "expo_kat.json")


def _check(res, batch, max_size, unit_s=False):
    ora = pyoracle.expo_aggregate(batch, max_size, unit_s)
    assert [int(k) for k in res.key_hash] == sorted(ora)
    for i, k in enumerate(res.key_hash):
        o = ora[int(k)]
        assert (int(res.count[i]), int(res.zero_count[i])) == (o["count"], o["zero_count"]), k
        assert (int(res.scale[i]), int(res.offset[i])) == (o["scale"], o["offset"]), k
        assert [int(x) for x in res.buckets[i]] == [int(x) for x in o["counts"]], k
        assert res.min[i] == o["min"] and res.max[i] == o["max"], k
        assert abs(res.sum[i] - o["sum"]) <= 1e-9 * max(abs(o["sum"]), 1e-300), k


def _engine(wl, **kw):
    e = Engine(Config(n_services=wl.n_services, n_windows=16, **kw))
    e.window_advance(wl.first_window)
    return e


def test_gpu_log_and_index_bit_exact():
    kat = json.load(open(KAT))
    rng = np.random.default_rng(3)
    vals = np.concatenate([[float.fromhex(x) for x, _ in kat["go_log"] if float.fromhex(x) > 2.0 ** -1000],
                           np.exp(rng.uniform(-14, 14, 20000)),
                           rng.integers(1, 10**11, 20000) / 1e6])
    scales = rng.integers(-6, 21, len(vals)).astype(np.int32)
    with Engine(Config(exp_max_size=160)) as e:
        idx, logs = e.expo_probe(vals, scales)
    for v, s, i, lg in zip(vals, scales, idx, logs):
        assert lg.hex() == pyoracle.go_log(v).hex(), v
        assert int(i) == pyoracle.expo_index(v, int(s)), (v, s)
    for d, s, i in kat["map_to_index_ms"]:
        with Engine(Config(exp_max_size=160)) as e:
            gi, _ = e.expo_probe([d / 1e6], [s])
        assert int(gi[0]) == i


def test_fast_log2_error_bound():
    """The fast bucket index (expo_index_fast, sa_device.h) assumes
    |v_log_f32(m) - log2(m)| <= 2^-20 over every float m in [1, 2) (its
    kFastFxErr adds the duration's rounding to a float and the fixed-point
    conversions): measured here exhaustively on the device, so a part whose
    hardware log2 were less accurate fails this test instead of mis-bucketing
    near bucket boundaries."""
    with Engine(Config(exp_max_size=160)) as e:
        _, _, err = e.expo_fast_probe([], [])
    assert 0 < err <= 2.0 ** -20, err


@pytest.mark.parametrize("unit", ["ms", "s"])
def test_fast_index_agrees_with_exact_path(unit):
    """Wherever the fast path answers it gives the exact (Go math.Log) index;
    near bucket boundaries and powers of two it defers.  Durations: random over
    1 ns .. ~1 day, every power of two, and values straddling bucket
    boundaries at each scale."""
    rng = np.random.default_rng(11)
    div = 1e9 if unit == "s" else 1e6
    d = np.concatenate([
        np.exp(rng.uniform(0, np.log(8.64e13), 300000)).astype(np.uint64) + 1,
        2 ** np.arange(0, 47, dtype=np.uint64),
        rng.integers(1, 2**20, 50000, dtype=np.uint64)])
    # boundary straddlers: d near div * 2^(k / 2^s) for a few scales
    b = []
    for s in (1, 3, 5, 8, 12):
        for k in rng.integers(-20 * 2**s, 30 * 2**s, 400):
            c = div * 2.0 ** (float(k) / 2**s)
            if 2 <= c < 2**62:
                b += [int(c) - 1, int(c), int(c) + 1]
    d = np.concatenate([d, np.array(b, dtype=np.uint64)])
    scales = rng.integers(-4, 21, len(d)).astype(np.int32)
    with Engine(Config(exp_max_size=160, unit="s" if unit == "s" else "ms")) as e:
        fast, exact, _ = e.expo_fast_probe(d, scales, log2_err=False)
    taken = fast != np.iinfo(np.int32).min
    assert np.array_equal(fast[taken], exact[taken])
    # spot-check the exact column against the oracle's restatement
    for i in rng.integers(0, len(d), 3000):
        assert int(exact[i]) == pyoracle.expo_index(float(d[i]) / div, int(scales[i])), (int(d[i]), int(scales[i]))
    low = scales <= 8
    assert taken[low].mean() > 0.99, taken[low].mean()  # the fast path carries the common case


@pytest.mark.parametrize("path", ["small", "small_cached", "hbm"])
@pytest.mark.parametrize("max_size,unit", [(160, "ms"), (8, "ms"), (20, "s"), (2, "ms")])
def test_expo_histograms_match_oracle(max_size, unit, path):
    """small: the small-table kernel in EXPO mode (LDS header partials, slab
    reduce, LDS slab counts for the selected series); small_cached: the same
    with the cached-probe counting kernel (SA_OPT_EXPO_CACHED); hbm: the
    pass-1 global-atomic path (SA_OPT_EXPO_HBM)."""
    opt = {"small": 0, "small_cached": OPT_EXPO_CACHED, "hbm": OPT_EXPO_HBM}[path]
    wl = generate_c2(200_003, seed=13)
    with _engine(wl, exp_max_size=max_size, unit=unit, options=opt) as e:
        assert e.stats()["small_table"] == (0 if path == "hbm" else 1)
        e.ingest(wl.batch)
        res = e.flush_exp()
        _check(res, wl.batch, max_size, unit == "s")


@pytest.mark.slow
def test_expo_small_table_full_size_device_launches():
    """C2 at its full 10 M spans through sa_ingest_device in two launches
    (the second one a fresh trace-id variant), the bench's c2expo shape."""
    import torch

    import bench
    wl = generate_c2(10_000_000, seed=42)
    dev = torch.device("cuda", 0)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
            for c in wl.batch.columns()]
    var = bench.trace_variants(cols[3], cols[4], 2, seed=5)
    with _engine(wl, exp_max_size=160, key_capacity=1500) as e:
        assert e.stats()["small_table"] == 1
        for w0, w1 in var:
            e.ingest_device(cols[0], cols[1], cols[2], w0, w1, cols[5])
        res = e.flush_exp()
        both = SpanBatch(*[np.concatenate([c, c]) for c in wl.batch.columns()])
        _check(res, both, 160)
        assert int(res.count.sum()) == 2 * len(wl.batch) - 2 * int((wl.batch.key_hash == 0).sum())


def test_expo_entry_selection_from_a_different_mix():
    """Each counting launch uses the LDS entries the previous launch selected
    from its own counts (the first launch selects its own).  A launch whose
    series are all new to that selection (keys disjoint from the previous
    launch's) counts everything through the tail and its overflow; then the
    first mix again.  Every bucket as the oracle's."""
    a = generate_c2(300_000, seed=21, names_per_service=10).batch
    cols = a.columns()
    b = SpanBatch(*[c ^ np.uint64(0x5DEECE66D12345) if i == 0 else c for i, c in enumerate(cols)])
    b.key_hash[a.key_hash == 0] = 0  # (keep the zero keys zero)
    wl = generate_c2(10, seed=21, names_per_service=10)
    with _engine(wl, exp_max_size=160, key_capacity=1300) as e:
        assert e.stats()["small_table"] == 1
        for x in (a, b, a):
            e.ingest(x)
        both = SpanBatch(*[np.concatenate([p, q, r]) for p, q, r in zip(a.columns(), b.columns(), a.columns())])
        _check(e.flush_exp(), both, 160)


def test_expo_state_across_launches_and_delta_flushes():
    """Several ingests before one flush (kept buckets merged down when a later
    batch widens the range), then a second interval from scratch."""
    wl = generate_c2(240_000, seed=17)
    parts = [wl.batch.slice(0, 50_000), wl.batch.slice(50_000, 140_000), wl.batch.slice(140_000, 240_000)]
    with _engine(wl, exp_max_size=12) as e:
        e.ingest(parts[0])
        e.ingest(parts[1])
        first = SpanBatch(*[np.concatenate([a, b]) for a, b in zip(parts[0].columns(), parts[1].columns())])
        _check(e.flush_exp(), first, 12)
        e.ingest(parts[2])
        _check(e.flush_exp(), parts[2], 12)
        assert len(e.flush_exp().key_hash) == 0


def test_expo_edges_zero_pow2_and_huge():
    ds = [0, 0, 1, 999_999, 1_000_000, 1_000_001, 2_000_000, 4_000_000, 500_000, 60_000_000_000,
          3_600_000_000_000, 7]
    n = len(ds)
    start = np.full(n, 10**18, dtype=np.uint64)
    end = start + np.array(ds, dtype=np.uint64)
    end[1] = start[1] - 5  # end <= start: duration 0 (A2)
    batch = SpanBatch(np.array([11, 11, 11, 11, 11, 11, 22, 22, 22, 22, 22, 22], dtype=np.uint64), start, end,
                      np.arange(n, dtype=np.uint64), np.arange(n, dtype=np.uint64), pack_meta([0] * n, 2, 0))
    with Engine(Config(n_services=1, n_windows=16, exp_max_size=4)) as e:
        e.window_advance(10**18 // 10**10)
        e.ingest(batch)
        _check(e.flush_exp(), batch, 4)


@pytest.mark.parametrize("path", ["small", "hbm"])
def test_expo_huge_durations(path):
    """Durations around 2^52 ns and up to 9e17 ns (weeks to decades) on both
    table paths: the fast log2 index path, the exact Go math.Log path and the
    rescale by shifted scale-20 indices all agree with the oracle."""
    ds = [2**52 - 3, 2**52 - 2, 2**52 - 1, 2**52, 2**52 + 1, 3 * 2**52, 9 * 10**17, 5_000_000, 2**40, 1]
    n = len(ds)
    end = np.full(n, 10**18, dtype=np.uint64)
    start = end - np.array(ds, dtype=np.uint64)
    batch = SpanBatch(np.array([11, 22] * (n // 2), dtype=np.uint64), start, end,
                      np.arange(n, dtype=np.uint64), np.arange(n, dtype=np.uint64), pack_meta([0] * n, 2, 0))
    for max_size in (4, 160):
        with Engine(Config(n_services=1, n_windows=16, exp_max_size=max_size,
                           options=0 if path == "small" else OPT_EXPO_HBM)) as e:
            assert e.stats()["small_table"] == (1 if path == "small" else 0)
            e.window_advance(10**18 // 10**10)
            e.ingest(batch)
            _check(e.flush_exp(), batch, max_size)


@pytest.mark.parametrize("max_size", [160, 8])
def test_expo_huge_durations_in_a_mix(max_size):
    """The slab path's span records hold a duration below 2^52 - 1 ns and
    send longer ones back to the span's times (span_rec_of, sa_internal.h):
    every 97th span of a C2 mix (~1.4 k series, so both the LDS entries and
    the tail records see them) gets a duration of 2^52 - 1 + k ns, k = 0 .. 4,
    and a few get exactly 2^52 - 2."""
    wl = generate_c2(200_003, seed=29)
    b = wl.batch
    start = b.start_ns.copy()
    idx = np.arange(0, len(b), 97)
    start[idx] = b.end_ns[idx] - (np.uint64(2**52 - 1) + (idx % 5).astype(np.uint64))
    start[idx[::7] + 1] = b.end_ns[idx[::7] + 1] - np.uint64(2**52 - 2)
    batch = SpanBatch(b.key_hash, start, b.end_ns, b.trace_w0, b.trace_w1, b.meta)
    with _engine(wl, exp_max_size=max_size) as e:
        assert e.stats()["small_table"] == 1
        e.ingest(batch)
        _check(e.flush_exp(), batch, max_size)


def test_expo_launches_over_two_streams_pipelined():
    """Small-table exponential engines run launch k + 1's ingest kernel beside
    launch k's reduce / count / fold (two sets of header partials and span
    slots; launch k + 1's reduce waits for launch k's fold).  Six
    device-resident launches alternate over two streams, each batch's times
    overwritten on its stream right after the call; launches 3 and 5
    stretch their durations (x 40, x 0.02) so the scales move under the
    pipeline; a delta flush after the fourth launch."""
    import torch
    dev = torch.device("cuda", 0)
    wl = generate_c2(600_000, seed=37)
    parts = []
    for i in range(6):
        b = wl.batch.slice(i * 100_000, (i + 1) * 100_000)
        f = {2: 40.0, 4: 0.02}.get(i)
        start = b.start_ns.copy()
        if f is not None:  # (spans with end > start; the others keep their zero duration)
            pos = b.end_ns > b.start_ns
            d = ((b.end_ns[pos] - b.start_ns[pos]).astype(np.float64) * f).astype(np.uint64)
            start[pos] = b.end_ns[pos] - d
        parts.append(SpanBatch(b.key_hash, start, b.end_ns, b.trace_w0, b.trace_w1, b.meta))
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream(dev))
    dcols = [[torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
              for c in p.columns()] for p in parts]
    torch.cuda.synchronize(dev)
    with _engine(wl, exp_max_size=160) as e:
        assert e.stats()["small_table"] == 1
        for i, cols in enumerate(dcols):
            st = streams[i % 2]
            e.ingest_device(*cols, stream=st.cuda_stream)
            # the columns are the caller's again once its stream passes the
            # call: overwritten there at once (the histogram kernels must
            # read the engine's span records, not these)
            with torch.cuda.stream(st):
                cols[1].fill_(7)
                cols[2].fill_(3)
            if i == 3:
                first = SpanBatch(*[np.concatenate(c) for c in zip(*[q.columns() for q in parts[:4]])])
                _check(e.flush_exp(), first, 160)
        second = SpanBatch(*[np.concatenate(c) for c in zip(*[q.columns() for q in parts[4:]])])
        _check(e.flush_exp(), second, 160)


def test_expo_sketches_unchanged():
    wl = generate_c2(150_000, seed=23)
    with _engine(wl, exp_max_size=160) as e:
        e.ingest(wl.batch)
        o = pyoracle.Oracle(n_services=wl.n_services)
        o.ingest(wl.batch)
        for wid in o.window_ids():
            sk = e.window_read(wid)
            hll, cms = o.window(wid)
            assert np.array_equal(sk.hll, hll) and np.array_equal(sk.cms, cms), wid
        with pytest.raises(_lib.SpanAggError) as ei:
            e.flush()
        assert ei.value.code == _lib.SA_ESTATE
