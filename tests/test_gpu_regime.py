"""The regime bench.py times, checked against the oracle.

bench.py's `value` comes from launches 31-50 of one window: by then every
launch is a fresh trace-id variant of the batch (bench.trace_variants) and the
HLL lower-bound filter (spanagg_kernels.hip ingest_v2_kernel step 1,
spanagg_binned.hip bt_scatter2_kernel) skips the register gather of most
spans.  These tests drive 40 launches of distinct variants into one window
ring exactly as bench.py does (two alternating launch streams, device-resident
columns) and compare RED, every window's HLL registers and count-min cells
bit-exactly with the oracle fed the same 40 variants; the engine's
`hll_filtered` counter proves that the filtered path carried the late
launches (>= 50 % of their spans), so a bound that were ever too high would
show as a lost HLL raise here.

Reference: the sketches stand beside the connector declared at
/root/reference/src/otel-collector/otelcol-config.yml:116 (SURVEY.md
Appendix C spec)."""
import numpy as np
import pytest

import bench
import pyoracle
from parity_util import assert_red_equal
from spanagg import Config, Engine, SpanBatch
from spanagg.synth import generate_c2, generate_highcard

pytestmark = pytest.mark.gpu

LAUNCHES = 40
LATE = 10  # the last launches: the settled regime bench.py times


def _device_cols(batch, dev):
    import torch
    return [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
            for c in batch.columns()]


def _drive(eng, batch, n_launch, seed):
    """LAUNCHES launches of distinct trace-id variants over two streams (the
    bench's step()); returns the oracle inputs and hll_filtered before the
    late launches."""
    import torch
    dev = torch.device("cuda", 0)
    cols = _device_cols(batch, dev)
    variants = bench.trace_variants(cols[3], cols[4], LAUNCHES, seed=seed)
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    host = []
    filt_before_late = None
    for i, (w0, w1) in enumerate(variants):
        if i == LAUNCHES - LATE:
            torch.cuda.synchronize(dev)
            filt_before_late = eng.stats()["hll_filtered"]
        s = streams[i % 2]
        s.wait_stream(torch.cuda.current_stream(dev))
        eng.ingest_device(cols[0], cols[1], cols[2], w0, w1, cols[5], n=n_launch, stream=s.cuda_stream)
        host.append((w0[:n_launch].cpu().numpy().view(np.uint64), w1[:n_launch].cpu().numpy().view(np.uint64)))
    torch.cuda.synchronize(dev)
    return host, filt_before_late


def _oracle(batch, host, n_launch, n_services):
    o = pyoracle.Oracle(n_services=n_services)
    b = batch.slice(0, n_launch)
    for w0, w1 in host:
        o.ingest(SpanBatch(b.key_hash, b.start_ns, b.end_ns, w0, w1, b.meta))
    return o


def _check(eng, o, filt_late, n_launch):
    assert_red_equal(eng.flush(), o.series())
    for wid in o.window_ids():
        sk = eng.window_read(wid)
        hll, cms = o.window(wid)
        assert np.array_equal(sk.hll, hll), f"window {wid}: HLL registers differ"
        assert np.array_equal(sk.cms, cms), f"window {wid}: count-min cells differ"
    assert filt_late >= 0.5 * LATE * n_launch, (filt_late, LATE * n_launch)


@pytest.mark.slow
def test_c2_bench_regime_40_variants_bit_exact():
    n = 10_000_000
    wl = generate_c2(n, seed=42)
    with Engine(Config(n_services=wl.n_services, n_windows=16, key_capacity=1500)) as e:
        assert e.stats()["small_table"] == 1
        e.window_advance(wl.first_window)
        host, f0 = _drive(e, wl.batch, n, seed=1000)
        filt_late = e.stats()["hll_filtered"] - f0
        o = _oracle(wl.batch, host, n, wl.n_services)
        _check(e, o, filt_late, n)


@pytest.mark.slow
def test_c4_binned_bench_regime_40_variants_bit_exact():
    # the size bench.py times C4 at: the record regions are sized per launch
    # (engine bt_region_for), so the benched size is the one to pin
    n = 10_000_000
    batch, _, first = generate_highcard(n, seed=7)
    with Engine(Config(n_services=1, n_windows=16, key_capacity=1_200_000)) as e:
        assert e.stats()["small_table"] == 0
        e.window_advance(first)
        host, f0 = _drive(e, batch, n, seed=2000)
        filt_late = e.stats()["hll_filtered"] - f0
        o = _oracle(batch, host, n, 1)
        _check(e, o, filt_late, n)
