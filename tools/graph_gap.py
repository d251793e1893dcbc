"""Probe: the per-launch cost of C2 ingests issued as stream launches against
the same launches captured once into a HIP graph and replayed.

The rocprofv3 traces put ~6 us between one C2 kernel's end and the next one's
start on a stream (launch period 99.0 us against a 92.8 us kernel median), and
the MI355X guide measures ~1.2 us per kernel boundary inside a hipGraph.  This
probe prices that difference on the product library: K back-to-back
`ingest_device` calls on one stream (HIP events around them) against the same
next K calls captured into a graph (torch.cuda.CUDAGraph, relaxed capture)
and replayed once, R interleaved rounds.  Every launch reads its own trace-id
variant.  The check at the end: calls in the flush = spans of every launch
executed (the captures themselves run nothing) minus zero keys.

  python tools/graph_gap.py [--spans N] [--k K] [--rounds R]
Prints one JSON line.  Measurement only: the product path launches on streams.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "opentelemetry-demo_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spans", type=int, default=10_000_000)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from spanagg import Config, Engine
    from spanagg.synth import generate_c2

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n, k = a.spans, a.k
    wl = generate_c2(n, seed=42, names_per_service=25)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
            for c in wl.batch.columns()]
    nvar = 16 + 2 * a.rounds * k
    var = bench.trace_variants(cols[3], cols[4], nvar, seed=1000)
    eng = Engine(Config(n_services=wl.n_services, n_windows=16, key_capacity=1500, device=0))
    eng.window_advance(wl.first_window)
    s = torch.cuda.Stream(dev)
    used = [0]

    def step(vi):
        w0, w1 = var[vi % nvar]
        eng.ingest_device(cols[0], cols[1], cols[2], w0, w1, cols[5], n=n, stream=s.cuda_stream)
        used[0] += 1

    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    out = {"spans": n, "k": k, "rounds": a.rounds, "stream_us_per_launch": [], "graph_us_per_launch": []}
    nxt = [16]

    def fresh():
        nxt[0] += 1
        return nxt[0] - 1

    with torch.cuda.stream(s):
        for i in range(16):  # cold + settling launches
            step(i)
        torch.cuda.synchronize()
        # interleaved rounds, every launch on a fresh variant: K stream
        # launches, then K launches captured into a graph and replayed once
        for _ in range(a.rounds):
            e0, e1 = ev(), ev()
            e0.record(s)
            for i in range(k):
                step(fresh())
            e1.record(s)
            torch.cuda.synchronize()
            out["stream_us_per_launch"].append(round(e0.elapsed_time(e1) * 1e3 / k, 2))
            g = torch.cuda.CUDAGraph()
            before = used[0]
            try:
                with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
                    for i in range(k):
                        step(fresh())
            except Exception as e:  # noqa: BLE001 -- the capture itself is what is probed
                out["capture_error"] = repr(e)[:400]
                print(json.dumps(out), flush=True)
                return 1
            captured, used[0] = used[0] - before, before  # (the capture ran nothing)
            torch.cuda.synchronize()
            e0, e1 = ev(), ev()
            e0.record(s)
            g.replay()
            e1.record(s)
            torch.cuda.synchronize()
            used[0] += captured
            out["graph_us_per_launch"].append(round(e0.elapsed_time(e1) * 1e3 / k, 2))
            del g
    st = eng.stats()
    red = eng.flush()
    calls = int(red.calls.sum())
    out["launches_executed"] = used[0]
    out["calls_ok"] = calls == used[0] * n - st["zero_key"]
    out["calls"], out["zero_key"] = calls, int(st["zero_key"])
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
