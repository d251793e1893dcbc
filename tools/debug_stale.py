#!/usr/bin/env python3
"""Does a freshly created engine see stale key-table contents left in a
recycled allocation by a previous engine?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opentelemetry-demo_amd"))

import numpy as np  # noqa: E402

from spanagg import Config, Engine, SpanBatch  # noqa: E402
from spanagg.synth import generate_c2  # noqa: E402


def random_batch(n, n_keys, seed):
    rng = np.random.default_rng(seed)
    keys = rng.integers(1, 2**63, n_keys, dtype=np.int64).astype(np.uint64)
    t = np.full(n, 10**18, np.uint64)
    return SpanBatch(keys[rng.integers(0, n_keys, n)], t, t + 1000, np.arange(n, dtype=np.uint64),
                     np.zeros(n, np.uint64), np.zeros(n, np.uint32))


def run(tag, cfg, batch, base=10**8):
    e = Engine(cfg)
    pre = e.stats()["n_keys"]
    e.window_advance(base)
    e.ingest(batch)
    st = e.stats()
    r = e.flush(allow_drops=True)
    uniq = len(np.unique(batch.key_hash))
    print(f"{tag}: pre n_keys={pre} post n_keys={st['n_keys']} uniq={uniq} series={len(r.key_hash)} "
          f"dropped={st['dropped_table_full']} calls={int(r.calls.sum())}/{len(batch)}", flush=True)
    e.close()


for i in range(3):
    run(f"small-A{i}", Config(), random_batch(300_000, 1400, 100 + i))
for i in range(3):
    run(f"hbm-{i}", Config(key_capacity=300_000), random_batch(300_000, 50_000, 200 + i))
    run(f"small-after-hbm-{i}", Config(), random_batch(300_000, 1400, 300 + i))
wl = generate_c2(500_000, seed=5)
run("c2-500k", Config(n_services=20, n_windows=16), wl.batch, wl.first_window)
