#!/usr/bin/env python3
"""Diagnose unexpected key-table drops: host vs device ingest of one batch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opentelemetry-demo_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spanagg import Config, Engine  # noqa: E402
from spanagg.synth import generate_c2  # noqa: E402


def report(tag, e, wl):
    st = e.stats()
    r = e.flush(allow_drops=True)
    ks = set(int(k) for k in r.key_hash)
    exp = set(int(k) for k in np.unique(wl.batch.key_hash))
    print(tag, "n_keys", st["n_keys"], "dropped", st["dropped_table_full"], "series", len(r.key_hash),
          "calls", int(r.calls.sum()), "missing", len(exp - ks), "extra", len(ks - exp), flush=True)


for n, seed in ((500_000, 5), (10_000_000, 42), (1_000_000, 77)):
    wl = generate_c2(n, seed=seed)
    print("distinct keys in batch", len(np.unique(wl.batch.key_hash)), "n", n, flush=True)
    for rep in range(2):
        with Engine(Config(n_services=wl.n_services, n_windows=16)) as e:
            e.window_advance(wl.first_window)
            e.ingest(wl.batch)
            report(f"host rep{rep}", e, wl)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).cuda()
            for c in wl.batch.columns()]
    for rep in range(2):
        with Engine(Config(n_services=wl.n_services, n_windows=16)) as e:
            e.window_advance(wl.first_window)
            e.ingest_device(*cols, n=n, stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            report(f"dev rep{rep}", e, wl)
    with Engine(Config(n_services=wl.n_services, n_windows=16, flags=6)) as e:  # no sketches
        e.window_advance(wl.first_window)
        e.ingest(wl.batch)
        report("host nosketch", e, wl)
