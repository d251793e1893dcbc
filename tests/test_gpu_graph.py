"""sa_ingest_device_many: k device batches launched as one HIP graph.

The graph path must give exactly what k sa_ingest_device calls give: RED,
every window's HLL registers and count-min cells bit-exact with the oracle fed
the same spans.  The batches are ragged slices of one C2 workload; the calls
exercise both of the engine's graphs being built, each being re-pointed at new
batches (kernel-node parameter updates), single-batch calls between them on a
second stream, and the one-by-one fallback (k = 1, and a binned engine).

Reference: the per-span aggregation the connector declared at
/root/reference/src/otel-collector/otelcol-config.yml:115-116 runs per
ConsumeTraces call ([UPSTREAM] connector.go aggregateMetrics); this entry takes
a receiver's queued requests in one call.
"""
import numpy as np
import pytest

import pyoracle
from parity_util import assert_red_equal
from spanagg import Config, Engine, SpanBatch
from spanagg.synth import generate_c2, generate_highcard

pytestmark = pytest.mark.gpu


def _device_cols(batch, dev):
    import torch
    return [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
            for c in batch.columns()]


def _slices(n, parts, rng):
    cuts = np.sort(rng.choice(np.arange(2, n, 2), size=parts - 1, replace=False))  # even: 16-B aligned columns
    return list(zip(np.concatenate([[0], cuts]), np.concatenate([cuts, [n]])))


def _check(e, o):
    assert_red_equal(e.flush(), o.series())
    for wid in o.window_ids():
        sk = e.window_read(wid)
        hll, cms = o.window(wid)
        assert np.array_equal(sk.hll, hll) and np.array_equal(sk.cms, cms)


def test_graph_ingest_matches_oracle():
    import torch
    dev = torch.device("cuda", 0)
    wl = generate_c2(1_200_000, seed=11)
    cols = _device_cols(wl.batch, dev)
    rng = np.random.default_rng(5)
    sl = _slices(len(wl.batch), 14, rng)
    bts = [tuple(c[a:b] for c in cols) for a, b in sl]
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    for s in (s1, s2):
        s.wait_stream(torch.cuda.current_stream(dev))  # (the columns' copies)
    with Engine(Config(n_services=wl.n_services, n_windows=16, device=0)) as e:
        e.window_advance(wl.first_window)
        e.ingest_device_many(bts[0:3], stream=s1.cuda_stream)     # graph 0 built
        e.ingest_device_many(bts[3:6], stream=s1.cuda_stream)     # graph 1 built
        e.ingest_device(*bts[6], stream=s2.cuda_stream)           # one launch, another stream
        e.ingest_device_many(bts[7:10], stream=s2.cuda_stream)    # graph 0 re-pointed
        e.ingest_device_many(bts[10:13], stream=s1.cuda_stream)   # graph 1 re-pointed
        e.ingest_device_many(bts[13:14], stream=s1.cuda_stream)   # k = 1: one-by-one path
        e.join(s1.cuda_stream)
        e.join(s2.cuda_stream)
        torch.cuda.synchronize(dev)
        assert e.stats()["spans"] == len(wl.batch)
        o = pyoracle.Oracle(n_services=wl.n_services)
        o.ingest(wl.batch)
        _check(e, o)


def test_graph_ingest_fresh_variants_many_calls():
    """The bench's regime: every batch a fresh trace-id variant of the C2
    batch, 8 calls of k = 5 alternating the two graphs (each re-pointed three
    times), checked against the oracle fed the same 40 variants."""
    import torch

    import bench
    dev = torch.device("cuda", 0)
    wl = generate_c2(400_000, seed=3)
    cols = _device_cols(wl.batch, dev)
    var = bench.trace_variants(cols[3], cols[4], 40, seed=77)
    torch.cuda.synchronize(dev)
    o = pyoracle.Oracle(n_services=wl.n_services)
    with Engine(Config(n_services=wl.n_services, n_windows=16, device=0)) as e:
        e.window_advance(wl.first_window)
        for c in range(8):
            e.ingest_device_many([(cols[0], cols[1], cols[2], w0, w1, cols[5]) for w0, w1 in var[5 * c:5 * c + 5]])
        torch.cuda.synchronize(dev)
        b = wl.batch
        for w0, w1 in var:
            o.ingest(SpanBatch(b.key_hash, b.start_ns, b.end_ns, w0.cpu().numpy().view(np.uint64),
                               w1.cpu().numpy().view(np.uint64), b.meta))
        _check(e, o)


def test_binned_engine_takes_the_one_by_one_path():
    import torch
    dev = torch.device("cuda", 0)
    batch, _, first_window = generate_highcard(300_000, seed=9)
    cols = _device_cols(batch, dev)
    sl = _slices(len(batch), 3, np.random.default_rng(1))
    torch.cuda.synchronize(dev)
    with Engine(Config(n_services=1, n_windows=16, key_capacity=1_200_000, device=0)) as e:
        e.window_advance(first_window)
        e.ingest_device_many([tuple(c[a:b] for c in cols) for a, b in sl])
        torch.cuda.synchronize(dev)
        o = pyoracle.Oracle(n_services=1)
        o.ingest(batch)
        _check(e, o)
