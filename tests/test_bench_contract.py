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


_RANK_SCRIPT = r'''
import json, os, sys, time
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
with open(os.path.join(sys.argv[1], f"rank{rank}.json"), "w") as f:
    json.dump({k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                                          "SPANAGG_BENCH_LAUNCHER")}, f)
fail = int(sys.argv[2])
if fail >= 0:
    if rank == fail:
        sys.exit(3)
    time.sleep(120)      # the others wait, as in a collective the failed rank never joins
if rank == 0:
    print(json.dumps({"n_gpus": world}))
'''


@pytest.mark.parametrize("n", [2, 4])
def test_launch_ranks_spawns_n_rank_processes(tmp_path, n, capfd):
    """bench.py --gpus N without torch.distributed.run: launch_ranks starts N
    children with the torch.distributed.run environment (distinct RANK /
    LOCAL_RANK, one WORLD_SIZE, one loopback rendezvous), and rank 0's stdout
    is what the parent prints."""
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    rc = bench.launch_ranks(n, [str(tmp_path), "-1"], script=str(script), timeout=120)
    assert rc == 0
    envs = [json.loads((tmp_path / f"rank{i}.json").read_text()) for i in range(n)]
    assert sorted(int(e["RANK"]) for e in envs) == list(range(n))
    assert all(e["RANK"] == e["LOCAL_RANK"] and e["WORLD_SIZE"] == str(n) for e in envs)
    assert len({e["MASTER_PORT"] for e in envs}) == 1 and envs[0]["MASTER_ADDR"] == "127.0.0.1"
    assert all(e["SPANAGG_BENCH_LAUNCHER"].startswith("bench.py") for e in envs)
    out = capfd.readouterr().out.strip().splitlines()
    assert json.loads(out[-1]) == {"n_gpus": n}


def test_launch_ranks_propagates_a_rank_failure(tmp_path):
    """A rank that fails ends the job with its exit code, and the ranks left
    waiting for it are stopped (not left to hang until a time limit)."""
    script = tmp_path / "rank.py"
    script.write_text(_RANK_SCRIPT)
    t0 = __import__("time").monotonic()
    rc = bench.launch_ranks(3, [str(tmp_path), "1"], script=str(script), timeout=100)
    assert rc == 3
    assert __import__("time").monotonic() - t0 < 60


def test_bench_self_launch_without_gpu_fails_loudly():
    """`bench.py --gpus 2` on a box without a GPU: both rank children fail and
    the parent returns non-zero (it neither hangs nor prints a line)."""
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--spans", "1000",
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode != 0
    assert not p.stdout.strip()


@pytest.mark.gpu
def test_bench_self_launch_two_ranks_one_device():
    """The scaling line's launch path on a one-GPU box: a bare `bench.py
    --gpus 2` (no outer launcher) starts two ranks on cuda:0 over gloo; the
    line reports n_gpus 2, the backend, a world size of 2 and both ranks."""
    env = dict(os.environ, SPANAGG_BENCH_ONE_DEVICE="1")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--spans", "1000000",
                        "--steps", "4", "--warmup", "1", "--settle", "1", "--soak-s", "0", "--sub", "",
                        "--no-cpu-baseline", "--host-otlp-spans", "0", "--h2d-reps", "0"],
                       capture_output=True, text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["n_gpus"] == 2 and r["calls_check"]
    d = r["distributed"]
    assert d["world_size"] == 2 and d["backend"] == "gloo" and d["launcher"].startswith("bench.py")
    assert sorted(x["rank"] for x in d["per_rank"]) == [0, 1]
