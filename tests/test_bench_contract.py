"""bench.py host logic on CPU: traffic summaries are picked by workload, and the
CPU-baseline worker (the oracle port, bench.py's cpu_baseline leg) reports a
rate.  The timed GPU steps themselves run only on the GPU box."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("workload,fname", [("c2", "traffic.json"), ("c4", "traffic_c4.json")])
def test_traffic_summary_matches_workload(workload, fname):
    path = os.path.join(ROOT, "profiles", fname)
    traffic, src = bench.load_traffic(path, workload)
    assert src == os.path.join("profiles", fname)
    assert traffic > 44 * 10_000_000 * 0.9  # at least the algorithmic bytes (minus noise)


def test_traffic_summary_of_another_workload_is_not_used():
    path = os.path.join(ROOT, "profiles", "traffic_c4.json")
    assert bench.load_traffic(path, "c4zipf") == (None, None)
    assert bench.load_traffic(os.path.join(ROOT, "profiles", "missing.json"), "c2") == (None, None)


def test_cpu_worker_reports_a_rate():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-worker", "1",
                        "--cpu-seconds", "0.2"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["spans"] >= 2_000_000 and r["seconds"] > 0


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bench_batches_sit_in_their_trace_id_shard(world):
    """bench.py at N ranks: every span of a rank's batch and of each of its
    trace-id variants is owned by that rank under spanagg.dist.shard_of, and
    spans of one trace stay together (equal ids map to equal ids)."""
    import torch
    from spanagg.dist import shard_of
    rng = np.random.default_rng(world)
    w0 = torch.from_numpy(rng.integers(0, 2**63, 20000, dtype=np.int64))
    w1 = torch.from_numpy(rng.integers(0, 2**64 - 1, 20000, dtype=np.uint64).view(np.int64))
    w1[1000:1010] = w1[0]  # one trace with several spans
    for rank in range(world):
        for v0, v1 in bench.trace_variants(w0, w1, 3, seed=5, rank=rank, world=world):
            u = v1.numpy().view(np.uint64)
            assert (shard_of(u, world) == rank).all()
            assert (u[1000:1010] == u[0]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_bench_trace_id_shards_on_device(world):
    """The same sharding on device-resident columns (bench.py applies it to
    cuda tensors): every span of each variant lands on its rank."""
    import torch
    from spanagg.dist import shard_of
    rng = np.random.default_rng(world)
    w0 = torch.from_numpy(rng.integers(0, 2**63, 50000, dtype=np.int64)).cuda()
    w1 = torch.from_numpy(rng.integers(0, 2**64 - 1, 50000, dtype=np.uint64).view(np.int64)).cuda()
    for rank in range(world):
        for _, v1 in bench.trace_variants(w0, w1, 3, seed=9, rank=rank, world=world):
            assert v1.is_cuda
            assert (shard_of(v1.cpu().numpy().view(np.uint64), world) == rank).all()
