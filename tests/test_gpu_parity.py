"""GPU parity: libspanagg's HIP path vs the golden vectors and the CPU oracle.

Bar (north_star): bucket counts, calls, HLL registers and CMS cells bit-exact;
duration sums within 1e-9 relative (the engine sums exact u64 ns; the oracle
sums float64 ms in Go's arrival order).
"""
import numpy as np
import pytest

import pyoracle
from parity_util import assert_red_equal, assert_red_golden, sketch_sparse
from spanagg._lib import OPT_ATOMIC_TABLE, OPT_PARTITIONED
from spanagg import Config, Engine, SpanBatch, pack_meta
from spanagg import _lib
from spanagg.synth import generate_c2, generate_highcard

pytestmark = pytest.mark.gpu


def _batch(spans):
    cols = list(zip(*spans)) if spans else [[]] * 6
    mk = lambda i, dt: np.array([int(x) for x in cols[i]], dtype=dt)
    return SpanBatch(mk(0, np.uint64), mk(1, np.uint64), mk(2, np.uint64), mk(3, np.uint64),
                     mk(4, np.uint64), mk(5, np.uint32))


def _pow2_at_least(x):
    p = 1
    while p < x:
        p <<= 1
    return p


RING = 16


def engine_for_case(case, key_capacity=1000, **kw):
    """Ring of RING windows from the case's first window; windows beyond it
    (e.g. the 2^62 ns span of kat_basic) are counted out of range."""
    wins = [w["window"] for w in case["expected"]["windows"]]
    lo = min(wins) if wins else 0
    e = Engine(Config(bounds=case["bounds"], unit=case["unit"], hll_p=case["hll_p"],
                      cms_d=case["cms_d"], cms_w=case["cms_w"], window_ns=case["window_ns"],
                      n_windows=RING, n_services=case["n_services"], key_capacity=key_capacity,
                      **kw))
    e.window_advance(lo)
    return e, lo


def expected_oor(case, lo):
    n = 0
    for _, _, end, _, _, meta in case["spans"]:
        if (meta & 0xFFFF) < case["n_services"]:
            w = end // case["window_ns"]
            n += not (lo <= w < lo + RING)
    return n


@pytest.mark.parametrize("idx", range(5))
# LDS-mirrored (small) table, partitioned HBM table (2^17 slots), binned table (2^19)
@pytest.mark.parametrize("key_capacity", [1000, 100_000, 300_000])
def test_golden_cases(golden, idx, key_capacity):
    case = golden["cases"][idx]
    e, lo = engine_for_case(case, key_capacity=key_capacity)
    with e:
        assert e.stats()["small_table"] == (1 if key_capacity == 1000 else 0)
        e.ingest(_batch(case["spans"]))
        res = e.flush()
        assert_red_golden(res, case["expected"]["series"])
        for w in case["expected"]["windows"]:
            if not lo <= w["window"] < lo + RING:
                continue
            sk = e.window_read(w["window"])
            h, c = sketch_sparse(sk.hll, sk.cms)
            assert h == w["hll"], case["name"]
            assert c == w["cms"], case["name"]
        st = e.stats()
        exp = case["expected"]["stats"]
        assert st["spans"] == exp["spans"]
        assert st["zero_key"] == exp["zero_key"]
        assert st["invalid_service"] == exp["invalid_service"]
        assert st["window_out_of_range"] == expected_oor(case, lo)
        assert st["dropped_table_full"] == 0


def _oracle_run(wl_batch, n_services, **kw):
    o = pyoracle.Oracle(n_services=n_services, **kw)
    o.ingest(wl_batch)
    return o


def _check_windows(e, o, first_window, n_services):
    ids = o.window_ids()
    assert ids, "no windows"
    for wid in ids:
        sk = e.window_read(wid)
        hll, cms = o.window(wid)
        assert np.array_equal(sk.hll, hll), wid
        assert np.array_equal(sk.cms, cms), wid
        for s in range(n_services):
            assert sk.distinct_traces(s) == pytest.approx(pyoracle.hll_estimate(hll[s], 14),
                                                          rel=1e-12)


@pytest.mark.parametrize("n", [1, 2, 3, 1023, 2049, 100_003])
def test_c2_small_sizes_vs_oracle(n):
    wl = generate_c2(n, seed=n)
    with Engine(Config(n_services=wl.n_services, n_windows=16)) as e:
        e.window_advance(wl.first_window)
        e.ingest(wl.batch)
        res = e.flush()
        o = _oracle_run(wl.batch, wl.n_services)
        assert_red_equal(res, o.series())
        _check_windows(e, o, wl.first_window, wl.n_services)


def test_empty_batch():
    with Engine(Config()) as e:
        e.ingest(SpanBatch(*(np.zeros(0, np.uint64) for _ in range(5)), np.zeros(0, np.uint32)))
        res = e.flush()
        assert len(res.key_hash) == 0
        assert e.stats()["spans"] == 0


def test_ragged_batch_rejected():
    with pytest.raises(ValueError):
        SpanBatch(np.zeros(3, np.uint64), np.zeros(2, np.uint64), np.zeros(3, np.uint64),
                  np.zeros(3, np.uint64), np.zeros(3, np.uint64), np.zeros(3, np.uint32))


def test_c2_full_size_bit_exact():
    """BASELINE config 2 at full size: 10M spans, default buckets."""
    wl = generate_c2(10_000_000, seed=42)
    with Engine(Config(n_services=wl.n_services, n_windows=16)) as e:
        e.window_advance(wl.first_window)
        e.ingest(wl.batch)
        res = e.flush()
        o = _oracle_run(wl.batch, wl.n_services)
        assert_red_equal(res, o.series())
        _check_windows(e, o, wl.first_window, wl.n_services)
        # size-independent properties
        assert int(res.calls.sum()) == 10_000_000 - e.stats()["zero_key"]
        assert e.stats()["dropped_table_full"] == 0


def test_device_ingest_matches_host_ingest():
    import torch
    wl = generate_c2(500_000, seed=5)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).cuda()
            for c in wl.batch.columns()]
    with Engine(Config(n_services=wl.n_services, n_windows=16)) as e1, \
            Engine(Config(n_services=wl.n_services, n_windows=16)) as e2:
        e1.window_advance(wl.first_window)
        e2.window_advance(wl.first_window)
        e1.ingest(wl.batch)
        s = torch.cuda.Stream()
        keep = []
        with torch.cuda.stream(s):
            # several device batches on a torch stream, split at odd offsets;
            # odd offsets are re-materialised to keep 16-B alignment
            cuts = [0, 1, 77_777, 300_001, 500_000]
            for a, b in zip(cuts, cuts[1:]):
                sl = [c[a:b].clone() for c in cols]
                keep.append(sl)
                e2.ingest_device(*sl, n=b - a, stream=s.cuda_stream)
        torch.cuda.synchronize()
        r1, r2 = e1.flush(), e2.flush()
        for f in ("key_hash", "bucket_counts", "calls", "sum_ns"):
            assert np.array_equal(getattr(r1, f), getattr(r2, f))
        for wid in range(wl.first_window, wl.first_window + 10):
            a, b = e1.window_read(wid), e2.window_read(wid)
            assert np.array_equal(a.hll, b.hll) and np.array_equal(a.cms, b.cms)


def test_device_ingest_two_streams_overlap():
    """Batches alternating over two streams (the pipelined ingest bench.py
    times): the launches may overlap on the device, each into its own slab set.
    A flush between them and a null-stream batch check the joins."""
    import torch
    wl = generate_c2(1_200_000, seed=11)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).cuda()
            for c in wl.batch.columns()]
    cuts = [0, 150_000, 300_000, 450_000, 600_000, 750_000, 900_000, 1_050_000, 1_200_000]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    with Engine(Config(n_services=wl.n_services, n_windows=16)) as e:
        e.window_advance(wl.first_window)
        parts = [[c[a:b] for c in cols] for a, b in zip(cuts, cuts[1:])]  # offsets are 16-B aligned
        for i in range(4):
            e.ingest_device(*parts[i], n=cuts[i + 1] - cuts[i], stream=streams[i % 2].cuda_stream)
        r1 = e.flush()
        for i in range(4, 8):
            st = None if i == 6 else streams[i % 2].cuda_stream
            e.ingest_device(*parts[i], n=cuts[i + 1] - cuts[i], stream=st)
        r2 = e.flush()
        torch.cuda.synchronize()
        assert_red_equal(r1, _oracle_run(wl.batch.slice(0, cuts[4]), wl.n_services).series())
        assert_red_equal(r2, _oracle_run(wl.batch.slice(cuts[4], cuts[8]), wl.n_services).series())
        _check_windows(e, _oracle_run(wl.batch, wl.n_services), wl.first_window, wl.n_services)


@pytest.mark.parametrize("zipf", [0.0, 1.1])
def test_binned_two_streams_overlap(zipf):
    """The binned path fed from two streams: launches on alternating streams,
    each inserting keys first seen in it (CAS write-back; a slot another launch
    took sends its counts down the probe sequence), and the Zipf mix's hot rows
    spilling into the u64 array while other launches add to it."""
    import torch
    batch, _, w0 = generate_highcard(3_000_000, routes=2000, pods=500, seed=21, zipf_s=zipf)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).cuda()
            for c in batch.columns()]
    cuts = [0, 500_000, 1_000_000, 1_500_000, 2_000_000, 2_500_000, 3_000_000]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    torch.cuda.synchronize()
    with Engine(Config(n_services=1, n_windows=16, key_capacity=1_000_000)) as e:
        assert e.stats()["small_table"] == 0
        e.window_advance(w0)
        for i in range(len(cuts) - 1):
            e.ingest_device(*[c[cuts[i]:cuts[i + 1]] for c in cols], n=cuts[i + 1] - cuts[i],
                            stream=streams[i % 2].cuda_stream)
        res = e.flush()
        torch.cuda.synchronize()
        o = _oracle_run(batch, 1)
        assert_red_equal(res, o.series())
        assert e.stats()["dropped_table_full"] == 0
        for wid in o.window_ids():
            sk = e.window_read(wid)
            hll, cms = o.window(wid)
            assert np.array_equal(sk.hll, hll) and np.array_equal(sk.cms, cms), wid


def test_device_ingest_null_stream_orders_with_torch():
    """stream=NULL runs on the engine's stream, which is blocking: batches made
    on torch's legacy default stream and freed right after the call are safe."""
    import torch
    wl = generate_c2(300_000, seed=6)
    with Engine(Config(n_services=wl.n_services, n_windows=16)) as e:
        e.window_advance(wl.first_window)
        for a, b in ((0, 100_000), (100_000, 300_000)):
            cols = [torch.from_numpy(c[a:b].view(np.int64) if c.dtype == np.uint64
                                     else c[a:b].view(np.int32)).cuda() for c in wl.batch.columns()]
            e.ingest_device(*cols, n=b - a)
            del cols
            junk = torch.full((4_000_000,), -1, dtype=torch.int64, device="cuda")  # reuse memory
            del junk
        res = e.flush()
        o = _oracle_run(wl.batch, wl.n_services)
        assert_red_equal(res, o.series())


def test_flush_is_delta_and_resets():
    wl = generate_c2(200_000, seed=9)
    half = 100_000
    with Engine(Config(n_services=wl.n_services, n_windows=16)) as e:
        e.window_advance(wl.first_window)
        e.ingest(wl.batch.slice(0, half))
        r1 = e.flush()
        e.ingest(wl.batch.slice(half, len(wl.batch)))
        r2 = e.flush()
        r3 = e.flush()
        assert len(r3.key_hash) == 0
        o1 = _oracle_run(wl.batch.slice(0, half), wl.n_services)
        o2 = _oracle_run(wl.batch.slice(half, len(wl.batch)), wl.n_services)
        assert_red_equal(r1, o1.series())
        assert_red_equal(r2, o2.series())


def test_epoch_flush_u16_counters():
    """> 65,535 spans of one (key, bucket) per workgroup: exercises the LDS
    u16 epoch flush into the workgroup slabs."""
    import torch
    n = 40_000_000
    dev = "cuda"
    key = torch.full((n,), 12345, dtype=torch.int64, device=dev)
    start = torch.full((n,), 10**18, dtype=torch.int64, device=dev)
    end = start + 1_000_000
    w0 = torch.arange(n, dtype=torch.int64, device=dev)
    w1 = torch.zeros(n, dtype=torch.int64, device=dev)
    meta = torch.zeros(n, dtype=torch.int32, device=dev)
    with Engine(Config(n_windows=8)) as e:
        e.window_advance(10**18 // 10**10)
        e.ingest_device(key, start, end, w0, w1, meta, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        res = e.flush()
        assert res.key_hash.tolist() == [12345]
        assert int(res.bucket_counts[0, 0]) == n
        assert int(res.bucket_counts[0].sum()) == n
        assert int(res.sum_ns[0]) == n * 1_000_000


def test_table_full_reports_drops():
    rng = np.random.default_rng(1)
    n = 5000
    keys = rng.integers(1, 2**63, 200, dtype=np.int64).astype(np.uint64)
    b = SpanBatch(keys[rng.integers(0, 200, n)], np.full(n, 10**18, np.uint64),
                  np.full(n, 10**18 + 5, np.uint64), rng.integers(0, 2**62, n).astype(np.uint64),
                  np.zeros(n, np.uint64), np.zeros(n, np.uint32))
    with Engine(Config(key_capacity=8)) as e:  # 16 slots
        e.window_advance(10**18 // 10**10)
        e.ingest(b)
        with pytest.raises(_lib.SpanAggError) as ei:
            e.flush()
        assert ei.value.code == _lib.SA_EFULL
        st = e.stats()
        assert st["n_keys"] == 0  # the full table was reclaimed by the flush
        assert st["dropped_table_full"] > 0
    with Engine(Config(key_capacity=8)) as e:
        e.ingest(b)
        res = e.flush(allow_drops=True)
        assert int(res.calls.sum()) + e.stats()["dropped_table_full"] == n


def test_window_ring_out_of_range_and_advance():
    base = 176_722_560
    w = 10_000_000_000
    ends = np.array([(base + k) * w + 5 for k in (-1, 0, 1, 3, 4, 9)], dtype=np.uint64)
    n = len(ends)
    b = SpanBatch(np.arange(1, n + 1, dtype=np.uint64), ends - 1, ends, np.arange(n, dtype=np.uint64),
                  np.ones(n, np.uint64), pack_meta(np.zeros(n), 2, 2))
    with Engine(Config(n_windows=4)) as e:
        e.window_advance(base)
        e.ingest(b)
        assert e.stats()["window_out_of_range"] == 3   # base-1, base+4, base+9
        s0 = e.window_read(base)
        assert s0.hll.sum() > 0 and s0.cms.sum() == 4  # one ERROR span x 4 rows
        with pytest.raises(_lib.SpanAggError):
            e.window_read(base + 4)
        e.window_advance(base + 2)
        with pytest.raises(_lib.SpanAggError):
            e.window_read(base)
        s3 = e.window_read(base + 3)
        assert s3.cms.sum() == 4
        s5 = e.window_read(base + 5)                   # recycled slot starts clean
        assert s5.hll.sum() == 0 and s5.cms.sum() == 0


@pytest.mark.parametrize("window_ns,n_windows,kcap", [
    (10_000_000_000, 16, 1000),        # C2 geometry, LDS-mirrored table
    (10_000_000_000, 16, 1_200_000),   # binned table (C4's scatter)
    (3, 1024, 1000),                   # odd 3-ns windows, the largest small-path ring
])
def test_window_boundaries_vs_oracle(window_ns, n_windows, kcap):
    """Ends on and next to every window boundary of the ring (the first and
    last nanosecond of each window, and the ring's own edges): the kernels'
    window slot takes a float estimate whose floor is exact away from the
    boundaries and an integer correction near them (sa_device.h,
    window_slot_lean).  Half the spans are ERROR, so each window's count-min
    cells and HLL registers pin the window every span went to."""
    rng = np.random.default_rng(window_ns + n_windows)
    w0 = 176_722_560 if window_ns > 1000 else 5_000_000_011
    ks = np.arange(n_windows, dtype=np.uint64)
    if n_windows > 64:
        ks = np.unique(np.concatenate([ks[:8], ks[-8:], rng.choice(ks, 48, replace=False)]))
    offs = np.array(sorted({0, 1, 2, window_ns // 2, window_ns - 2, window_ns - 1}), dtype=np.uint64)
    offs = offs[offs < window_ns]
    ends = ((w0 + ks[:, None]) * np.uint64(window_ns) + offs[None, :]).ravel()
    ends = np.concatenate([ends, (w0 + rng.integers(0, n_windows, 4000, dtype=np.uint64)) * np.uint64(window_ns)
                           + rng.integers(0, window_ns, 4000, dtype=np.uint64)])
    ends = np.repeat(ends, 3)  # three spans per end time: distinct series and traces
    n = len(ends)
    dur = rng.integers(0, 50_000_000, n, dtype=np.uint64)
    starts = np.where(ends > dur, ends - dur, 0).astype(np.uint64)
    b = SpanBatch(rng.integers(1, 41, n, dtype=np.uint64), starts, ends,
                  rng.integers(1, 2**63, n, dtype=np.uint64), rng.integers(1, 2**63, n, dtype=np.uint64),
                  pack_meta(np.zeros(n), 2, np.where(rng.random(n) < 0.5, 2, 1)))
    with Engine(Config(n_services=1, n_windows=n_windows, window_ns=window_ns, key_capacity=kcap)) as e:
        if n_windows == 16:
            assert e.stats()["small_table"] == (1 if kcap == 1000 else 0)
        e.window_advance(w0)
        e.ingest(b)
        assert e.stats()["window_out_of_range"] == 0
        res = e.flush()
        o = _oracle_run(b, 1, window_ns=window_ns)
        assert_red_equal(res, o.series())
        _check_windows(e, o, w0, 1)
        # the ring's edges: the nanosecond before its first window and its
        # end are out of range (sketches skip them; RED counts every span),
        # the first and last nanoseconds inside are not
        first, last = e.window_read(w0).cms.sum(), e.window_read(w0 + n_windows - 1).cms.sum()
        edge = np.array([w0 * window_ns - 1, w0 * window_ns, (w0 + n_windows) * window_ns - 1,
                         (w0 + n_windows) * window_ns], dtype=np.uint64)
        e.ingest(SpanBatch(np.full(4, 7, np.uint64), edge - 1, edge, np.arange(1, 5, dtype=np.uint64),
                           np.ones(4, np.uint64), pack_meta(np.zeros(4), 2, 2)))
        assert e.stats()["window_out_of_range"] == 2
        assert int(e.flush().calls.sum()) == 4
        assert e.window_read(w0).cms.sum() == first + 4  # one ERROR span x cms_d rows
        assert e.window_read(w0 + n_windows - 1).cms.sum() == last + 4


def test_high_cardinality_hbm_table_vs_oracle():
    """Config 4 shape at reduced size: HBM key-table path with many keys."""
    batch, khash, w0 = generate_highcard(1_000_000, routes=400, pods=250)
    with Engine(Config(n_services=1, n_windows=16, key_capacity=200_000)) as e:
        assert e.stats()["small_table"] == 0
        e.window_advance(w0)
        e.ingest(batch)
        res = e.flush()
        o = _oracle_run(batch, 1)
        assert_red_equal(res, o.series())
        for wid in o.window_ids():
            sk = e.window_read(wid)
            hll, cms = o.window(wid)
            assert np.array_equal(sk.hll, hll) and np.array_equal(sk.cms, cms)


@pytest.mark.parametrize("shape", ["zipf_bins_spill", "lds_tables_spill"])
def test_partitioned_hbm_path_spills_vs_oracle(shape):
    """The partitioned HBM-table path (part_scatter + part_aggregate) where it
    falls back to the direct path: a Zipf key mix overfills the hot keys' bins,
    and ~2.9 M distinct keys (~1,400 per bin) overfill the 1,024-slot LDS
    tables.  Two ingests (two launches, bin counters reset between) and the
    per-span atomic path (SA_OPT_ATOMIC_TABLE) on the same input must agree.
    (SA_OPT_PARTITIONED keeps tables the binned path would take on this one.)"""
    if shape == "zipf_bins_spill":
        batch, _, w0 = generate_highcard(2_000_000, seed=3, routes=400, pods=250, zipf_s=1.2)
        kcap = 200_000
    else:
        batch, _, w0 = generate_highcard(4_000_000, seed=4, routes=3000, pods=1000)
        kcap = 3_500_000
    half = len(batch) // 2 // 16 * 16
    results = []
    for opt in (OPT_PARTITIONED, OPT_ATOMIC_TABLE):
        with Engine(Config(n_services=1, n_windows=16, key_capacity=kcap, options=opt)) as e:
            assert e.stats()["small_table"] == 0
            e.window_advance(w0)
            e.ingest(batch.slice(0, half))
            e.ingest(batch.slice(half, len(batch)))
            res = e.flush()
            wins = {}
            for wid in range(w0, w0 + 16):
                sk = e.window_read(wid)
                wins[wid] = (sk.hll.copy(), sk.cms.copy())
            results.append((res, wins, e.stats()))
    o = _oracle_run(batch, 1)
    for res, wins, st in results:
        assert st["dropped_table_full"] == 0
        assert_red_equal(res, o.series())
        for wid in o.window_ids():
            hll, cms = o.window(wid)
            assert np.array_equal(wins[wid][0], hll) and np.array_equal(wins[wid][1], cms)


def _check_highcard(e, batch, n):
    res = e.flush()
    o = _oracle_run(batch, 1)
    assert_red_equal(res, o.series())
    for wid in o.window_ids():
        sk = e.window_read(wid)
        hll, cms = o.window(wid)
        assert np.array_equal(sk.hll, hll) and np.array_equal(sk.cms, cms), wid
    st = e.stats()
    assert st["dropped_table_full"] == 0
    # size-independent: every non-zero-key span is one call, in one series
    assert int(res.calls.sum()) == n - st["zero_key"]
    assert len(np.unique(res.key_hash)) == len(res.key_hash)


def test_c4_full_size_bit_exact():
    """BASELINE config 4 at full size: 1 M keys (2,000 routes x 500 pods),
    10 M spans in one launch of the partitioned path (the bench workload)."""
    n = 10_000_000
    batch, _, w0 = generate_highcard(n)
    with Engine(Config(n_services=1, n_windows=16, key_capacity=1_200_000)) as e:
        assert e.stats()["small_table"] == 0
        e.window_advance(w0)
        e.ingest(batch)
        _check_highcard(e, batch, n)


def test_partitioned_batch_above_launch_limit_is_split():
    """One sa_ingest of 2^24 + 1,001 spans: more than one partitioned launch
    takes (kPartMaxSpans), so the engine splits it into two launches whose
    bin counters and record runs must not leak into each other."""
    n = (1 << 24) + 1001
    batch, _, w0 = generate_highcard(n, seed=9, routes=400, pods=250)
    with Engine(Config(n_services=1, n_windows=16, key_capacity=200_000)) as e:
        assert e.stats()["small_table"] == 0
        e.window_advance(w0)
        e.ingest(batch)
        _check_highcard(e, batch, n)


def test_partitioned_one_bin_overflow_table_full_vs_oracle():
    """Every key in one bin (top 11 bits fixed), 60,000 distinct keys: the bin
    run overflows at once, each scatter workgroup's LDS overflow table fills
    (> 512 distinct spilling keys) and the rest takes the direct path; the
    one bin's aggregate sees more keys than its LDS table holds."""
    n = 2_000_000
    batch, _, w0 = generate_highcard(n, seed=11, routes=400, pods=250)
    cols = batch.columns()
    rng = np.random.Generator(np.random.PCG64(11))
    ids = rng.integers(0, 60_000, n).astype(np.uint64)
    with np.errstate(over="ignore"):
        low = (ids + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
    keys = (np.uint64(0x2AB) << np.uint64(53)) | (low >> np.uint64(11)) | np.uint64(1)
    one_bin = SpanBatch(keys, *cols[1:])
    with Engine(Config(n_services=1, n_windows=16, key_capacity=200_000)) as e:
        assert e.stats()["small_table"] == 0
        e.window_advance(w0)
        e.ingest(one_bin)
        _check_highcard(e, one_bin, n)


def test_repeat_runs_identical():
    wl = generate_c2(1_000_000, seed=77)
    outs = []
    for _ in range(2):
        with Engine(Config(n_services=wl.n_services, n_windows=16)) as e:
            e.window_advance(wl.first_window)
            e.ingest(wl.batch)
            outs.append(e.flush())
    for f in ("key_hash", "bucket_counts", "sum_ns"):
        assert np.array_equal(getattr(outs[0], f), getattr(outs[1], f))
