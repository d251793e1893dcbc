"""GPU parity of the binned-table high-cardinality path (spanagg_binned.hip:
bt_scatter2_kernel + bt_aggregate3_kernel; tables of 2^19..2^22 slots)
against the CPU oracle, including the spill paths (stage/region overflow
table, the direct path), the u8 rows' spill array, full bins and launch
splitting.

Bar (north_star): bucket counts, calls, HLL registers and count-min cells
bit-exact; duration sums within 1e-9 relative (parity_util.SUM_RTOL).
"""
import numpy as np
import pytest

import pyoracle
from parity_util import assert_red_equal
from spanagg._lib import OPT_IDENTITY_IDS, OPT_PARTITIONED
from spanagg import Config, Engine, SpanBatch
from spanagg.synth import generate_highcard

pytestmark = pytest.mark.gpu


def _oracle(batch):
    o = pyoracle.Oracle(n_services=1)
    o.ingest(batch)
    return o


def _check(e, batch, o=None, n_dropped=0, o_windows=None):
    """RED of `batch` since the last flush vs the oracle; sketch windows
    (cumulative, not reset by flush) vs o_windows (default: the same oracle)."""
    o = o or _oracle(batch)
    res = e.flush()
    assert_red_equal(res, o.series())
    ow = o_windows or o
    for wid in ow.window_ids():
        sk = e.window_read(wid)
        hll, cms = ow.window(wid)
        assert np.array_equal(sk.hll, hll), wid
        assert np.array_equal(sk.cms, cms), wid
    st = e.stats()
    assert st["dropped_table_full"] == n_dropped
    assert int(res.calls.sum()) == len(batch) - st["zero_key"]  # zero_key: 0 in these workloads
    return res


def _engine(kcap, **kw):
    e = Engine(Config(n_services=1, n_windows=16, key_capacity=kcap, **kw))
    assert e.stats()["small_table"] == 0
    return e


def test_c4zipf_full_size_bit_exact():
    """BASELINE config 4, Zipf(1.1) over the 1 M keys, 10 M spans in one
    binned launch (the bench's c4zipf workload): the hottest keys overfill
    their stages and regions, so the overflow table and the direct path run."""
    n = 10_000_000
    batch, _, w0 = generate_highcard(n, zipf_s=1.1)
    with _engine(1_200_000) as e:
        e.window_advance(w0)
        e.ingest(batch)
        _check(e, batch)


@pytest.mark.parametrize("zipf", [0.0, 1.3])
def test_binned_matches_partitioned_path(zipf):
    """Same input through the binned path and the round-1 partitioned path
    (SA_OPT_PARTITIONED), two ingests each: both equal the oracle."""
    batch, _, w0 = generate_highcard(3_000_000, seed=13, routes=1000, pods=300, zipf_s=zipf)
    half = len(batch) // 2
    o = _oracle(batch)
    for opt in (0, OPT_PARTITIONED):
        with _engine(600_000, options=opt) as e:
            e.window_advance(w0)
            e.ingest(batch.slice(0, half))
            e.ingest(batch.slice(half, len(batch)))
            _check(e, batch, o)


@pytest.mark.parametrize("zipf", [0.0, 1.2])
def test_binned_pipeline_new_keys_every_launch(zipf):
    """The launch pipeline (spanagg_engine.cpp sa_engine::bt_rec): launch k's
    aggregate runs on the engine's stream beside launch k + 1's scatter.  Every
    launch brings a key set no launch had (the series ids XORed with a
    per-launch constant), so launch k's aggregate inserts its keys into the
    HBM sub-tables while launch k + 1's scatter inserts the hot keys of its
    own mix (overflow table, direct path) into the same bins: the write-back
    must find-or-insert and relocate, never duplicate or overwrite a key.
    Launches alternate over two caller streams, device-resident."""
    import torch
    dev = torch.device("cuda", 0)
    n = 2_000_000
    # 150 k keys per launch, 0.9 M over the six (the table holds 1.2 M)
    batch, _, w0 = generate_highcard(n, seed=41, routes=500, pods=300, zipf_s=zipf)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
            for c in batch.columns()]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream(dev))
    o = pyoracle.Oracle(n_services=1)
    rng = np.random.Generator(np.random.PCG64(43))
    with _engine(1_200_000) as e:
        e.window_advance(w0)
        keep = []
        for i in range(6):
            c = int(rng.integers(1, 2**63 - 1))
            kx = cols[0] ^ c
            keep.append(kx)
            e.ingest_device(kx, cols[1], cols[2], cols[3], cols[4], cols[5], n=n, stream=streams[i % 2].cuda_stream)
            o.ingest(SpanBatch(batch.key_hash ^ np.uint64(c), batch.start_ns, batch.end_ns, batch.trace_w0,
                               batch.trace_w1, batch.meta))
        torch.cuda.synchronize(dev)
        res = e.flush()
        assert_red_equal(res, o.series())
        assert len(np.unique(res.key_hash)) == len(res.key_hash)
        for wid in o.window_ids():
            sk = e.window_read(wid)
            hll, cms = o.window(wid)
            assert np.array_equal(sk.hll, hll) and np.array_equal(sk.cms, cms), wid
        assert e.stats()["dropped_table_full"] == 0


def test_binned_paired_aggregates_with_reads_between():
    """Launches are aggregated in pairs (sa_engine::bt_pend): a launch's
    records wait for the next launch's, unless something reads first.  Five
    launches over two streams with a flush and a window read after the first
    (a pending set aggregated alone), a stats read after the fourth (a pair
    just done), a window advance after the third, and a flush at the end
    (the fifth launch pending): every flush and window equal to the oracle
    fed the same spans."""
    import torch
    dev = torch.device("cuda", 0)
    n = 1_500_000
    batch, _, w0 = generate_highcard(n, seed=47, routes=800, pods=400, zipf_s=1.1)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
            for c in batch.columns()]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    for st in streams:
        st.wait_stream(torch.cuda.current_stream(dev))
    o_all = pyoracle.Oracle(n_services=1)  # the sketches: every launch
    o_red = pyoracle.Oracle(n_services=1)  # RED since the last flush
    with _engine(1_200_000) as e:
        e.window_advance(w0)
        for i in range(5):
            c = np.uint64(0x9E3779B97F4A7C15 * (i + 1) & (2**64 - 1))
            tw = cols[4] ^ int(c.view(np.int64))
            e.ingest_device(cols[0], cols[1], cols[2], cols[3], tw, cols[5], n=n, stream=streams[i % 2].cuda_stream)
            b = SpanBatch(batch.key_hash, batch.start_ns, batch.end_ns, batch.trace_w0, batch.trace_w1 ^ c, batch.meta)
            o_all.ingest(b)
            o_red.ingest(b)
            if i == 0:  # the first launch's records are pending here
                assert_red_equal(e.flush(), o_red.series())
                o_red = pyoracle.Oracle(n_services=1)
                wid = o_all.window_ids()[0]
                sk = e.window_read(wid)
                hll, cms = o_all.window(wid)
                assert np.array_equal(sk.hll, hll) and np.array_equal(sk.cms, cms)
            if i == 2:  # pending again (launch 2): a window advance joins it
                e.window_advance(w0)
            if i == 3:
                assert e.stats()["dropped_table_full"] == 0
        torch.cuda.synchronize(dev)
        assert_red_equal(e.flush(), o_red.series())
        for wid in o_all.window_ids():
            sk = e.window_read(wid)
            hll, cms = o_all.window(wid)
            assert np.array_equal(sk.hll, hll) and np.array_equal(sk.cms, cms), wid


def test_binned_pairing_across_host_and_device_ingest():
    """Host-buffer and device-resident ingests interleaved on the binned path:
    a device launch leaves its records pending, the host sa_ingest that
    follows joins first (the pending set is aggregated alone) and leaves its
    own launch pending, and the next device launch pairs with it.  The window
    equals the oracle fed all three batches."""
    import torch
    dev = torch.device("cuda", 0)
    n = 1_000_000
    batch, _, w0 = generate_highcard(n, seed=53, routes=600, pods=300)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
            for c in batch.columns()]
    o = pyoracle.Oracle(n_services=1)
    with _engine(1_200_000) as e:
        e.window_advance(w0)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        for i in range(3):
            c = np.uint64((0xD1B54A32D192ED03 * (i + 1)) & (2**64 - 1))
            b = SpanBatch(batch.key_hash, batch.start_ns, batch.end_ns, batch.trace_w0, batch.trace_w1 ^ c, batch.meta)
            if i == 1:
                e.ingest(b)  # host buffers
            else:
                tw = cols[4] ^ int(c.view(np.int64))
                e.ingest_device(cols[0], cols[1], cols[2], cols[3], tw, cols[5], n=n, stream=s.cuda_stream)
            o.ingest(b)
        torch.cuda.synchronize(dev)
        assert_red_equal(e.flush(), o.series())
        for wid in o.window_ids():
            sk = e.window_read(wid)
            hll, cms = o.window(wid)
            assert np.array_equal(sk.hll, hll) and np.array_equal(sk.cms, cms), wid


def test_binned_u8_rows_spill():
    """Row counts are u8 (32-B rows): a bucket count that would pass 255 moves
    the row's counts into the u64 spill array -- within one launch for the hot
    keys of a Zipf mix, over several launches for the others.  Totals stay
    exact across launches, and the spill array resets with the rows at flush."""
    batch, _, w0 = generate_highcard(200_000, seed=17, routes=50, pods=40, zipf_s=1.1)
    with _engine(600_000) as e:
        e.window_advance(w0)
        for rounds in (4, 2):  # the second interval starts from rows and spills reset by the flush
            o = pyoracle.Oracle(n_services=1)
            for _ in range(rounds):
                e.ingest(batch)
                o.ingest(batch)
            res = e.flush()
            assert_red_equal(res, o.series())
            assert int(res.calls.sum()) == rounds * len(batch)
            assert int(res.bucket_counts.max()) > 255 * rounds  # the spill path ran
        assert e.stats()["dropped_table_full"] == 0


def test_binned_full_bin_reports_drops():
    """With the identity id map (SA_OPT_IDENTITY_IDS) 1,000 keys that share their
    top 11 bits all land in one bin of 256 slots: the bin fills, the spans of
    the keys that found no slot are dropped and reported, every kept series
    is exact (a key is kept or dropped as a whole: slots never empty)."""
    n = 200_000
    batch, _, w0 = generate_highcard(n, seed=19, routes=100, pods=100)
    rng = np.random.Generator(np.random.PCG64(19))
    ids = rng.integers(0, 1000, n).astype(np.uint64)
    with np.errstate(over="ignore"):
        low = (ids + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
    keys = (np.uint64(0x155) << np.uint64(53)) | (low >> np.uint64(11)) | np.uint64(1)
    one_bin = SpanBatch(keys, *batch.columns()[1:])
    ref = _oracle(one_bin).series()
    with _engine(400_000, options=OPT_IDENTITY_IDS) as e:  # cap 2^19: 2,048 bins of 256 slots
        e.window_advance(w0)
        e.ingest(one_bin)
        res = e.flush(allow_drops=True)
        st = e.stats()
        assert len(res.key_hash) == 256
        assert int(res.calls.sum()) + st["dropped_table_full"] == n
        pos = np.searchsorted(ref["key_hash"], res.key_hash)
        assert np.array_equal(ref["key_hash"][pos], res.key_hash)
        assert np.array_equal(ref["bucket_counts"][pos], res.bucket_counts)
        assert np.array_equal(ref["sum_ns"][pos], res.sum_ns)


def test_binned_batch_above_launch_limit_is_split():
    """17 M spans in one sa_ingest: more than one binned launch takes (one
    scatter workgroup per CU x 65,520 spans), so it is split in two."""
    n = 17_000_000
    batch, _, w0 = generate_highcard(n, seed=23, routes=400, pods=250)
    with _engine(600_000) as e:
        e.window_advance(w0)
        e.ingest(batch)
        _check(e, batch)


def test_binned_repeat_runs_identical():
    """Placement (the per-engine random id multiplier, atomics order) never
    changes results."""
    batch, _, w0 = generate_highcard(1_000_000, seed=29, routes=500, pods=200, zipf_s=1.1)
    outs = []
    for _ in range(2):
        with _engine(600_000) as e:
            e.window_advance(w0)
            e.ingest(batch)
            outs.append(e.flush())
    for f in ("key_hash", "bucket_counts", "sum_ns"):
        assert np.array_equal(getattr(outs[0], f), getattr(outs[1], f))


_FAIL_SCRIPT = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from spanagg import Config, Engine, _lib
from spanagg.synth import generate_highcard
batch, _, first = generate_highcard(200_000, seed=5)
dev = torch.device("cuda", 0)
cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
        for c in batch.columns()]
e = Engine(Config(n_services=1, n_windows=16, key_capacity=1_200_000))
e.window_advance(first)
e.ingest_device(*cols, n=len(batch))              # pending: aggregated with the next launch
codes = []
for call in (lambda: e.ingest_device(*cols, n=len(batch)),   # its paired aggregate fails (injected)
             lambda: e.ingest(batch),                        # the host path reports it
             lambda: e.flush(),                              # and every read
             lambda: e.window_read(first)):
    try:
        call()
        codes.append(0)
    except _lib.SpanAggError as x:
        codes.append(x.code)
print("CODES", codes)
"""


def test_failed_pending_aggregate_is_reported_by_every_later_call():
    """Advisor r4: a pending binned record set belongs to an ingest that
    already returned SA_OK; when the aggregate that takes it fails to launch,
    the failure sticks -- the ingest that launched it, later host ingests,
    flushes and window reads all return SA_EDEVICE instead of results without
    those records.  The launch failure is injected in the laboratory build
    (SPANAGG_FAIL_AGG=1: the process's first aggregate launch fails), run in a
    child process so the product library of this process stays untouched."""
    import os
    import subprocess
    import sys
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "opentelemetry-demo_amd")
    lab = os.path.join(pkg, "spanagg", "libspanagg_ab.so")
    if not os.path.exists(lab):
        pytest.skip("laboratory build (make -C opentelemetry-demo_amd ab) not present")
    env = dict(os.environ, SPANAGG_LIB=lab, SPANAGG_FAIL_AGG="1")
    p = subprocess.run([sys.executable, "-c", _FAIL_SCRIPT, pkg], env=env, capture_output=True, text=True,
                       timeout=240)
    line = [l for l in p.stdout.splitlines() if l.startswith("CODES")]
    assert line, p.stdout + p.stderr
    import ast
    codes = ast.literal_eval(line[0][len("CODES "):])
    assert codes == [-3, -3, -3, -3], codes
