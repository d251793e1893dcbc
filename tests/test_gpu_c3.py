"""BASELINE config 3 on what one GPU can prove.

C3 is 1 B spans sharded by trace id over 8 MI355X (rank =
trace_w1 % 8, 125 M spans per GPU), standing in for the reference's single
collector instance (/root/reference/docker-compose.yml:748-756, the
spanmetrics connector at src/otel-collector/otelcol-config.yml:116).  The
8-GPU hardware leg is the driver's; here:
  * one engine ingests a full C3 rank shard (125 M spans, every trace_w1 % 8
    == 3) as device-resident 10 M-span launches, checked against the oracle;
  * an 8-member engine group on device 0 takes 80 M device-resident spans
    through sa_group_ingest_device (the partition kernel shards them by trace
    id into the members' buffers) and merges at flush / window read;
  * sa_group_ingest (host batches) splits in one pass and copies out before
    returning: overwriting the caller's columns right after it changes
    nothing.
Bar: bucket counts, calls, ns sums, HLL registers and count-min cells
bit-exact with the oracle fed the same spans; duration sums within 1e-9."""
import ctypes as C

import numpy as np
import pytest

import bench
import pyoracle
from parity_util import assert_red_equal
from spanagg import Config, Engine, Group, SpanBatch
from spanagg.dist import shard_of
from spanagg.synth import generate_c2, generate_highcard

pytestmark = pytest.mark.gpu


def _device_cols(batch, dev):
    import torch
    return [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
            for c in batch.columns()]


def _check(x, o):
    assert_red_equal(x.flush(), o.series())
    for wid in o.window_ids():
        sk = x.window_read(wid)
        hll, cms = o.window(wid)
        assert np.array_equal(sk.hll, hll), wid
        assert np.array_equal(sk.cms, cms), wid


@pytest.mark.slow
def test_c3_rank_shard_125m_one_engine():
    import torch
    dev = torch.device("cuda", 0)
    n, rank, world = 10_000_000, 3, 8
    sizes = [n] * 12 + [5_000_000]  # 125 M spans
    wl = generate_c2(n, seed=42 + rank)
    cols = _device_cols(wl.batch, dev)
    variants = bench.trace_variants(cols[3], cols[4], len(sizes), seed=1000 + rank, rank=rank, world=world)
    o = pyoracle.Oracle(n_services=wl.n_services)
    with Engine(Config(n_services=wl.n_services, n_windows=16, key_capacity=1500)) as e:
        e.window_advance(wl.first_window)
        for (w0, w1), m in zip(variants, sizes):
            e.ingest_device(cols[0], cols[1], cols[2], w0, w1, cols[5], n=m)
            hw1 = w1[:m].cpu().numpy().view(np.uint64)
            assert (shard_of(hw1, world) == rank).all()
            b = wl.batch.slice(0, m)
            o.ingest(SpanBatch(b.key_hash, b.start_ns, b.end_ns, w0[:m].cpu().numpy().view(np.uint64), hw1,
                               b.meta))
        torch.cuda.synchronize(dev)
        assert e.stats()["spans"] == sum(sizes) == 125_000_000
        _check(e, o)


@pytest.mark.slow
def test_group_device_ingest_8_members_80m():
    """8 members on device 0 (device-copy merge transport), 8 launches of 10 M
    spans each partitioned on the device by sa_group_ingest_device."""
    import torch
    dev = torch.device("cuda", 0)
    n = 10_000_000
    wl = generate_c2(n, seed=77)
    cols = _device_cols(wl.batch, dev)
    variants = bench.trace_variants(cols[3], cols[4], 8, seed=3000)
    o = pyoracle.Oracle(n_services=wl.n_services)
    with Group([0] * 8, Config(n_services=wl.n_services, n_windows=16, key_capacity=1500)) as g:
        assert g.size == 8 and not g.uses_rccl
        g.window_advance(wl.first_window)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        for w0, w1 in variants:
            g.ingest_device(cols[0], cols[1], cols[2], w0, w1, cols[5], n=n, src=0, stream=s.cuda_stream)
            o.ingest(SpanBatch(wl.batch.key_hash, wl.batch.start_ns, wl.batch.end_ns,
                               w0.cpu().numpy().view(np.uint64), w1.cpu().numpy().view(np.uint64), wl.batch.meta))
        g.sync()
        st = g.stats()
        assert st["spans"] == 8 * n
        _check(g, o)


@pytest.mark.parametrize("members,n", [(3, 100_003), (5, 1_234_567), (2, 1)])
def test_group_device_ingest_matches_oracle(members, n):
    """Ragged sizes, an odd member count (trace_w1 % n from 32-bit halves),
    zero keys and invalid services ride along."""
    import torch
    dev = torch.device("cuda", 0)
    wl = generate_c2(max(n, 2), seed=members)
    b = wl.batch.slice(0, n)
    key = b.key_hash.copy()
    meta = b.meta.copy()
    if n > 100:
        key[::97] = 0
        meta[5::89] = (meta[5::89] & ~np.uint32(0xFFFF)) | np.uint32(70)  # service 70 >= n_services
    b = SpanBatch(key, b.start_ns, b.end_ns, b.trace_w0, b.trace_w1, meta)
    cols = _device_cols(b, dev)
    with Group([0] * members, Config(n_services=wl.n_services, n_windows=16)) as g:
        g.window_advance(wl.first_window)
        for _ in range(2):  # both staging sets
            g.ingest_device(*cols, n=n)
        g.sync()
        o = pyoracle.Oracle(n_services=wl.n_services)
        o.ingest(b)
        o.ingest(b)
        _check(g, o)
        st = g.stats()
        assert st["spans"] == 2 * n
        assert st["zero_key"] == 2 * int((key == 0).sum())


def test_group_device_ingest_alternating_streams():
    """Advisor r3: consecutive sa_group_ingest_device calls on two different
    caller streams.  Each staging set has its own shard counters and cursors,
    so a call's count/scan never rewrites the cursors the previous call's
    partition kernel (on the other stream) may still be reading."""
    import torch
    dev = torch.device("cuda", 0)
    n = 2_000_003
    wl = generate_c2(n, seed=21)
    cols = _device_cols(wl.batch, dev)
    variants = bench.trace_variants(cols[3], cols[4], 6, seed=4000)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream(dev))
    o = pyoracle.Oracle(n_services=wl.n_services)
    with Group([0] * 4, Config(n_services=wl.n_services, n_windows=16, key_capacity=1500)) as g:
        g.window_advance(wl.first_window)
        for i, (w0, w1) in enumerate(variants):
            g.ingest_device(cols[0], cols[1], cols[2], w0, w1, cols[5], n=n, src=0,
                            stream=streams[i % 2].cuda_stream)
            o.ingest(SpanBatch(wl.batch.key_hash, wl.batch.start_ns, wl.batch.end_ns,
                               w0.cpu().numpy().view(np.uint64), w1.cpu().numpy().view(np.uint64), wl.batch.meta))
        g.sync()
        torch.cuda.synchronize(dev)
        assert g.stats()["spans"] == 6 * n
        _check(g, o)


def test_group_device_ingest_cross_device_matches_host_split():
    """Advisor r3: the cross-device branch of sa_group_ingest_device (peer
    staging buffers, hipMemcpyPeerAsync of each packed shard, cross-device
    event waits) against the host split (sa_group_ingest) of the same spans.
    Needs two GPUs: the round's GPU boxes have one, so this runs only where a
    multi-GPU box is available (unverified until then)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU: the cross-device branch needs two devices")
    devs = list(range(min(4, torch.cuda.device_count())))
    n = 3_000_001
    wl = generate_c2(n, seed=31)
    cols = _device_cols(wl.batch, torch.device("cuda", 0))
    cfg = Config(n_services=wl.n_services, n_windows=16, key_capacity=1500)
    with Group(devs, cfg) as gd, Group(devs, cfg) as gh:
        gd.window_advance(wl.first_window)
        gh.window_advance(wl.first_window)
        for _ in range(3):  # both staging sets, then the first again
            gd.ingest_device(*cols, n=n, src=0)
            gh.ingest(wl.batch)
        gd.sync()
        a, b = gd.flush(), gh.flush()
        assert np.array_equal(a.key_hash, b.key_hash)
        assert np.array_equal(a.bucket_counts, b.bucket_counts)
        assert np.array_equal(a.sum_ns, b.sum_ns)
        o = pyoracle.Oracle(n_services=wl.n_services)
        for _ in range(3):
            o.ingest(wl.batch)
        assert_red_equal(a, o.series())


@pytest.mark.slow
def test_group_c4_8_members_device_flush():
    """Verdict r3: an 8-member group on device 0 at C4 cardinality (1 M series
    over 2,000 routes x 500 pods, 10 M spans per launch, two launches) through
    sa_group_ingest_device, flushed against the oracle.  Each member holds
    ~0.75 M of the series, so the flush unions ~6 M ids on the device (the
    engine's own bucket sort + per-bucket bitonic sort and unique,
    spanagg_union.hip), densifies 8 x 1 M rows, sums them on the device and
    builds the result's columns there (no host sort, no host row loop)."""
    import time
    import torch
    dev = torch.device("cuda", 0)
    n = 10_000_000
    batch, _, first = generate_highcard(n, seed=29)
    cols = _device_cols(batch, dev)
    variants = bench.trace_variants(cols[3], cols[4], 2, seed=5000)
    o = pyoracle.Oracle(n_services=1)
    with Group([0] * 8, Config(n_services=1, n_windows=16, key_capacity=1_200_000)) as g:
        g.window_advance(first)
        for w0, w1 in variants:
            g.ingest_device(cols[0], cols[1], cols[2], w0, w1, cols[5], n=n, src=0)
            o.ingest(SpanBatch(batch.key_hash, batch.start_ns, batch.end_ns, w0.cpu().numpy().view(np.uint64),
                               w1.cpu().numpy().view(np.uint64), batch.meta))
        g.sync()
        t0 = time.perf_counter()
        res = g.flush()
        flush_ms = (time.perf_counter() - t0) * 1e3
        ref = o.series()
        assert len(res.key_hash) == len(ref["key_hash"]) >= 990_000
        assert_red_equal(res, ref)
        for wid in o.window_ids():
            sk = g.window_read(wid)
            hll, cms = o.window(wid)
            assert np.array_equal(sk.hll, hll) and np.array_equal(sk.cms, cms), wid
        print(f"C4 x 8 group flush: {len(res.key_hash):,} series in {flush_ms:.1f} ms")


def test_group_device_ingest_binned_members():
    import torch
    dev = torch.device("cuda", 0)
    batch, _, first = generate_highcard(2_000_000, seed=11)
    cols = _device_cols(batch, dev)
    with Group([0, 0, 0], Config(n_services=1, n_windows=16, key_capacity=1_200_000)) as g:
        g.window_advance(first)
        g.ingest_device(*cols)
        g.sync()
        o = pyoracle.Oracle(n_services=1)
        o.ingest(batch)
        _check(g, o)


@pytest.mark.parametrize("n", [100_000, 900_001])
def test_group_host_ingest_columns_reusable_at_return(n):
    """sa_group_ingest copies every shard out before it returns (one shard of
    the larger batch exceeds the 2^18-span pageable-copy threshold)."""
    wl = generate_c2(n, seed=9)
    b = wl.batch
    keep = SpanBatch(*[c.copy() for c in b.columns()])
    with Group([0, 0], Config(n_services=wl.n_services, n_windows=16)) as g:
        g.window_advance(wl.first_window)
        g.ingest(b)
        for c in b.columns():  # the caller reuses its buffers at once
            c[:] = 0
        o = pyoracle.Oracle(n_services=wl.n_services)
        o.ingest(keep)
        _check(g, o)


@pytest.mark.parametrize("n", [100_000, 300_000, 2_500_000])
def test_ingest_columns_reusable_at_return(n):
    """Advisor r2: sa_ingest returns once the caller's columns are copied --
    chunks below 2^18 spans through the pinned slots, larger ones through the
    runtime's pageable copy, which the engine now waits for."""
    wl = generate_c2(n, seed=13)
    b = wl.batch
    keep = SpanBatch(*[c.copy() for c in b.columns()])
    with Engine(Config(n_services=wl.n_services, n_windows=16)) as e:
        e.window_advance(wl.first_window)
        e.ingest(b)
        for c in b.columns():
            c[:] = 0xAB
        del b
        o = pyoracle.Oracle(n_services=wl.n_services)
        o.ingest(keep)
        _check(e, o)


def _pinned_batch(lib, n):
    """A SpanBatch whose columns lie in sa_host_alloc (page-locked) memory."""
    p = C.c_void_p()
    assert lib.sa_host_alloc(n * 44 + 64, C.byref(p)) == 0
    raw = (C.c_uint8 * (n * 44 + 64)).from_address(p.value)
    buf = np.frombuffer(raw, dtype=np.uint8)
    cols = [buf[i * n * 8:(i + 1) * n * 8].view(np.uint64) for i in range(5)]
    meta = buf[5 * n * 8:5 * n * 8 + n * 4].view(np.uint32)
    return p, cols, meta


def test_ingest_async_double_buffered_pinned_columns():
    """sa_ingest_async (the Node host's columnizer path): two page-locked
    column buffers alternate; after each call the previous buffer is
    overwritten with the next chunk at once, and the buffer just passed is
    left alone until the following call returns.  Any early reuse would
    count garbage."""
    wl = generate_c2(2_400_000, seed=29)
    b = wl.batch
    chunks = [slice(i, min(i + 300_000, len(b))) for i in range(0, len(b), 300_000)]
    with Engine(Config(n_services=wl.n_services, n_windows=16)) as e:
        e.window_advance(wl.first_window)
        bufs = [_pinned_batch(e.lib, 300_000) for _ in range(2)]
        try:
            for i, sl in enumerate(chunks):
                p, cols, meta = bufs[i % 2]
                m = sl.stop - sl.start
                for c, src in zip(cols, b.columns()[:5]):
                    c[:m] = src[sl]
                meta[:m] = b.meta[sl]
                e.ingest_async(SpanBatch(*[c[:m] for c in cols], meta[:m]))
                # the other buffer (the previous call's) is free now: poison it
                pp, pcols, pmeta = bufs[(i + 1) % 2]
                for c in pcols:
                    c[:] = 0xAB
            e.sync()
        finally:
            for p, _, _ in bufs:
                e.lib.sa_host_free(p)
        o = pyoracle.Oracle(n_services=wl.n_services)
        o.ingest(b)
        _check(e, o)


def test_ingest_async_pageable_columns_read_before_return():
    """sa_ingest_async with ordinary (pageable) columns behaves as sa_ingest:
    the columns are read before the call returns, so overwriting them at
    once changes nothing."""
    wl = generate_c2(600_000, seed=31)
    b = wl.batch
    keep = SpanBatch(*[c.copy() for c in b.columns()])
    with Engine(Config(n_services=wl.n_services, n_windows=16)) as e:
        e.window_advance(wl.first_window)
        e.ingest_async(b)
        for c in b.columns():
            c[:] = 0xAB
        o = pyoracle.Oracle(n_services=wl.n_services)
        o.ingest(keep)
        _check(e, o)
