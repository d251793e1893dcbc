"""Multi-rank merge (spanagg/dist.py) on CPU with the gloo backend.

Each rank aggregates its trace-id shard (here with the CPU oracle standing in
for a GPU engine -- the oracle is only the test's data source) and the ranks
merge through the same key-union + all_reduce code the GPUs run over RCCL.
The merged result must equal a single-rank aggregation of the whole batch:
counts / ns sums bit-exact, HLL registers exact (max-merge), CMS exact (sum).
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


class OraclePartial:
    """LocalPartial backed by oracle arrays (test adapter)."""

    def __init__(self, oracle):
        self.o = oracle
        self.s = oracle.series()
        self.n_buckets = oracle.nbk
        self.device = torch.device("cpu")

    def export_keys(self):
        nz = self.s["calls"] > 0
        return torch.from_numpy(self.s["key_hash"][nz].view(np.int64).copy())

    def gather_dense(self, keys, reset):
        k = keys.numpy().view(np.uint64)
        rows = np.zeros((len(k), self.n_buckets + 1), np.uint64)
        idx = {int(x): i for i, x in enumerate(self.s["key_hash"])}
        for r, key in enumerate(k):
            i = idx.get(int(key))
            if i is not None:
                rows[r, : self.n_buckets] = self.s["bucket_counts"][i]
                rows[r, self.n_buckets] = self.s["sum_ns"][i]
        return torch.from_numpy(rows.view(np.int64))

    def window(self, wid):
        try:
            hll, cms = self.o.window(wid)
        except KeyError:
            hll = np.zeros((self.o.n_services, 1 << self.o.hll_p), np.uint8)
            cms = np.zeros((self.o.cms_d, self.o.cms_w), np.uint32)
        return torch.from_numpy(hll.copy()), torch.from_numpy(cms.astype(np.int64))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, errq):
    try:
        for p in (os.path.join(ROOT, "opentelemetry-demo_amd"), os.path.join(ROOT, "oracle"), HERE):
            sys.path.insert(0, p)
        import pyoracle
        from spanagg.dist import merge_red, merge_window, shard_of
        from spanagg.synth import generate_c2

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        wl = generate_c2(n, seed=123)
        mine = shard_of(wl.batch.trace_w1, world) == rank
        idx = np.nonzero(mine)[0]
        sub = wl.batch.slice(0, 0)
        from spanagg import SpanBatch
        sub = SpanBatch(*(c[idx] for c in wl.batch.columns()))
        o = pyoracle.Oracle(n_services=wl.n_services)
        o.ingest(sub)
        part = OraclePartial(o)
        red = merge_red(part)
        full = pyoracle.Oracle(n_services=wl.n_services)
        full.ingest(wl.batch)
        ref = full.series()
        assert np.array_equal(red.key_hash, ref["key_hash"])
        assert np.array_equal(red.bucket_counts, ref["bucket_counts"])
        assert np.array_equal(red.calls, ref["calls"])
        assert np.array_equal(red.sum_ns, ref["sum_ns"])
        rel = np.abs(red.sum - ref["sum_go"]) / np.maximum(np.abs(ref["sum_go"]), 1e-300)
        assert rel.max() <= 1e-9
        for wid in full.window_ids():
            hll, cms = merge_window(part, wid)
            rh, rc = full.window(wid)
            assert np.array_equal(hll, rh), wid
            assert np.array_equal(cms, rc), wid
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as ex:  # report to the parent
        import traceback
        errq.put(f"rank {rank}: {ex!r}\n{traceback.format_exc()}")
        raise


@pytest.mark.parametrize("world", [2, 3])
def test_merge_matches_single_rank(world):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 60_000, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_shard_of_keeps_traces_together():
    sys.path.insert(0, os.path.join(ROOT, "opentelemetry-demo_amd"))
    from spanagg.dist import shard_of
    w1 = np.array([5, 5, 6, 2**64 - 1], dtype=np.uint64)
    s = shard_of(w1, 4)
    assert s[0] == s[1]
    assert list(s) == [1, 1, 2, 3]


def _gpu_worker(rank, world, port, n, errq, kcap=1500):
    """The real GPU merge hooks (sa_export_keys / sa_gather_dense /
    sa_window_export through EnginePartial) with two ranks sharing cuda:0 over
    gloo (RCCL refuses two ranks on one device; the merge code is the same)."""
    try:
        for p in (os.path.join(ROOT, "opentelemetry-demo_amd"), os.path.join(ROOT, "oracle"), HERE):
            sys.path.insert(0, p)
        import pyoracle
        from spanagg import Config, Engine, SpanBatch
        from spanagg.dist import EnginePartial, merge_red, merge_window, shard_of
        from spanagg.synth import generate_c2

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        wl = generate_c2(n, seed=321)
        idx = np.nonzero(shard_of(wl.batch.trace_w1, world) == rank)[0]
        sub = SpanBatch(*(c[idx] for c in wl.batch.columns()))
        full = pyoracle.Oracle(n_services=wl.n_services)
        full.ingest(wl.batch)
        ref = full.series()
        with Engine(Config(n_services=wl.n_services, n_windows=16, key_capacity=kcap, device=0)) as e:
            e.window_advance(wl.first_window)
            e.ingest(sub)
            part = EnginePartial(e, torch.device("cuda", 0))
            red = merge_red(part)
            assert np.array_equal(red.key_hash, ref["key_hash"])
            assert np.array_equal(red.bucket_counts, ref["bucket_counts"])
            assert np.array_equal(red.sum_ns, ref["sum_ns"])
            for wid in full.window_ids():
                hll, cms = merge_window(part, wid)
                rh, rc = full.window(wid)
                assert np.array_equal(hll, rh), wid
                assert np.array_equal(cms, rc), wid
            # merge_red reset the engine's deltas: a second merge is empty
            assert len(merge_red(part).key_hash) == 0
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as ex:
        import traceback
        errq.put(f"rank {rank}: {ex!r}\n{traceback.format_exc()}")
        raise


@pytest.mark.gpu
@pytest.mark.parametrize("kcap", [1500, 600_000])  # LDS-mirrored table, binned HBM table
def test_gpu_merge_hooks_two_ranks_match_single_aggregation(kcap):
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, 200_000, errq, kcap)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=200)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
