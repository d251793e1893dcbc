#!/usr/bin/env python3
"""bench.py -- spans/sec aggregated (RED + HLL + CMS) on N x MI355X.

A "step" is one pass of the hot path over one device-resident batch: one
sa_ingest_device launch aggregating `--spans` synthetic SoA v1 spans (BASELINE
config 2 shape: 10M spans, ~500 (service, span) pairs -> <=1,500 series,
default buckets, per-service HLL p=14 + count-min 4x2048 over 10 s windows).
With N ranks every rank aggregates its own trace-id shard (weak scaling; no
collective on the data path); after the timed region the ranks merge their
partials once over RCCL (reported as merge_ms, outside `value`).  Under
torch.distributed.run (WORLD_SIZE set) each process is one rank; a bare
`python3 bench.py --gpus N` starts the N rank processes itself (launch_ranks:
child processes, before this one imports torch) and passes rank 0's line on.
The line's `distributed` object records the backend, the process group's
world size (checked equal to N) and every rank's own figures.

Steps alternate over `--streams` (default 2) launch streams: the engine keeps
two sets of per-workgroup slabs, so a launch waits only for the launch two
back and consecutive batches overlap (the next batch's workgroups start on the
CUs the current batch's workgroups leave).  `value` and `ms_per_step` are the
wall clock of the timed steps.

Every launch aggregates a distinct trace-id variant of the batch (trace ids
XORed with a per-variant constant), so HLL registers keep rising as on a live
stream; the cold first launch on a fresh engine is reported on its own, and
the next `--settle` launches (default 16), while the window's HLL registers
and their lower bounds settle, are timed one by one as `settle_ms` and kept
out of `value` and `kernel_ms` (a 10 s window at these rates spans ~10^5
launches, so the settled launch is the one a collector runs).  After the
timed steps, `--soak-s` seconds (default 2) of back-to-back launches give the
`sustained` rate (trace-id variants repeat there, so it is the rate of a
saturated window, never a kernel figure).  `value_incl_settle` prices the
whole window from its cold start: spans of the cold, settling and timed
launches over their time (HIP events for the first two, wall clock for the
timed steps).  `hll_filter_off` is the C2 kernel time of the same launches
with the HLL lower-bound filter off (every span gathers its register).  At
N=1 the line also carries `c4` and `c4zipf` sub-objects (BASELINE config 4,
uniform and Zipf(1.1) over 1 M series) with their own roofline.

Prints ONE JSON line on rank 0. `roofline` prices the ingest kernel against
HBM (44 algorithmic bytes per span / 8 TB/s).  Its `kernel_ms` is the kernel
alone: HIP events around a block of back-to-back serial launches on one
stream, divided by their number (`kernel_ms_bracketed`: events around each
launch on its own), inside the run (overlapping launches would double-count,
so these are not taken from the timed steps); `roofline.pipelined` prices the timed steps'
device time per step (one start event all streams wait on, to the last
stream's end event).
`cpu_baseline` times the CPU oracle port (oracle/, RED+HLL+CMS, 1 thread) on
rank 0 at N=1 over a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "opentelemetry-demo_amd"))

METRIC = "spans/sec aggregated (RED+HLL+CMS) at 1/8 GPU; % of HBM roofline"
BYTES_PER_SPAN = 44
HBM_PEAK_GBS = 8000.0


def cpu_baseline(wl, seconds: float):
    """Oracle port (RED + HLL + CMS over SoA v1, one thread) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle

    sample = wl.batch.slice(0, min(len(wl.batch), 2_000_000))
    o = pyoracle.Oracle(n_services=wl.n_services)
    reps, t0 = 0, time.perf_counter()
    while True:
        o.ingest(sample)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    o.close()
    port = {"value": reps * len(sample) / el, "unit": "spans/s", "cores": 1, "kind": "port",
            "sample": f"first {len(sample):,} spans of the rank-0 batch ingested {reps}x "
                      f"({reps * len(sample):,} spans, {el:.1f} s) by oracle/ or_ingest "
                      "(RED + HLL + CMS, Go-faithful float64 bucketing)"}
    # Connector-faithful RED only: NUL-joined string key built per span and
    # looked up in a string-keyed map (what aggregateMetrics does per span).
    from spanagg.synth import SERVICES, SPAN_NAMES
    strings = list(SERVICES) + [n for n, _ in SPAN_NAMES]
    m = len(sample)
    n_series, _, dt = pyoracle.aggregate_strings(
        strings, wl.service_id[:m], len(SERVICES) + wl.name_id[:m] % len(SPAN_NAMES), wl.kind[:m],
        wl.status[:m], wl.batch.start_ns[:m], wl.batch.end_ns[:m])
    conn = {"value": m / dt, "unit": "spans/s", "cores": 1, "kind": "port",
            "sample": f"first {m:,} spans, string-keyed buildKey + map lookup + "
                      f"SearchFloat64s (RED only, {n_series} series, {dt:.2f} s)"}
    return port, conn


def cpu_worker(seed: int, seconds: float) -> None:
    """One process of the multi-core CPU baseline: the oracle port over its own
    2 M-span C2 sample (sharded across the host cores)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from spanagg.synth import generate_c2

    wl = generate_c2(2_000_000, seed=seed)
    o = pyoracle.Oracle(n_services=wl.n_services)
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.ingest(wl.batch)
        reps += 1
    el = time.perf_counter() - t0
    print(json.dumps({"spans": reps * len(wl.batch), "seconds": el}), flush=True)


def cpu_baseline_multicore(workers: int, seconds: float):
    """`workers` oracle processes at once (each its own shard, no sharing), the
    way a sharded CPU collector would use the box; rate = sum of their rates."""
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--cpu-worker", str(100 + i),
                               "--cpu-seconds", str(seconds)], stdout=subprocess.PIPE, text=True)
             for i in range(workers)]
    total = 0.0
    for p in procs:
        out, _ = p.communicate(timeout=seconds + 120)
        r = json.loads(out.strip().splitlines()[-1])
        total += r["spans"] / r["seconds"]
    return {"value": total, "unit": "spans/s", "cores": workers, "kind": "port",
            "sample": f"{workers} processes, each the oracle port (RED + HLL + CMS) over its own "
                      f"2,000,000-span C2 shard for {seconds:.0f} s"}


def load_traffic(path, workload):
    try:
        with open(path) as f:
            t = json.load(f)
        if t.get("workload") == workload:
            return t.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    except (OSError, ValueError):
        pass
    return None, None


def host_otlp_rate(spans: int, threads: int = 8, batch: int = 128, extra=()):
    """the OTLP decode+aggregate rate from protobuf bytes -- the
    Node host (native columnizer in the N-API addon, `threads` decode threads
    with the JavaScript thread one of them, `batch` requests per
    consumeTracesBatch as the pipeline queue hands them over) feeding this GPU
    through sa_ingest (host memory, PCIe included).  Not `value`."""
    node = shutil.which("node")
    script = os.path.join(ROOT, "host", "node", "test", "host_rate.js")
    if node is None or not os.path.exists(os.path.join(ROOT, "host", "node", "build", "spanagg.node")):
        return None
    try:
        p = subprocess.run([node, "--max-old-space-size=16000", script, str(spans), "--gpu", "--threads",
                            str(threads), "--batch", str(batch), *extra], capture_output=True, text=True, timeout=240)
        r = json.loads(p.stdout.strip().splitlines()[-1])
    except Exception as e:  # reported, never fatal for the bench line
        return {"error": str(e)[:200]}
    hc = "--highcard" in extra
    vocab = ("500 pods (k8s.pod.name) x 2,000 routes (http.route dimension) = 1 M possible series, "
             f"{r.get('series', 0):,} distinct in the sample, binned engine table, every series known (a whole "
             "warm-up pass first)" if hc else "20 services x 25 names")
    return {"value": r["spans_per_s"], "unit": "spans/s", "cores": r["cores"], "mb_per_s": r["mb_per_s"],
            "calls_check": r["calls_check"], "columnizer": r["columnizer"],
            "seconds_in": r.get("seconds_in"), "options": list(extra),
            **({"series": r.get("series")} if hc else {}),
            **({"exemplars": r["exemplars"], "event_records": r["event_records"]}
               if "--exemplars" in extra else {}),
            "sample": f"{r['spans']:,} spans in {r['requests']} OTLP requests of 512 spans, "
                      f"{batch} requests per batch, {vocab}, decode + transform rules + "
                      "keying + columnise + sa_ingest_async (two pinned column buffers, H2D + kernel)"}


def box_cores():
    """Host cores this job may use: nproc, the CPU affinity set and the cgroup
    CPU quota (a GPU box's job gets a share of a larger machine)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
            if path.endswith("cpu.max") and parts[0] != "max":
                quota = int(parts[0]) / int(parts[1])
            elif not path.endswith("cpu.max") and int(parts[0]) > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    quota = int(parts[0]) / int(f.read().split()[0])
            break
        except (OSError, ValueError, IndexError):
            continue
    usable = min(nproc, aff, int(quota) if quota else nproc)
    return {"nproc": nproc, "affinity": aff, "cgroup_quota_cpus": quota, "usable": max(1, usable)}


def to_shard(w1, rank, world):
    """Trace-id word 1 moved into this rank's shard: w1 - w1 % world + rank, so
    spanagg.dist.shard_of (trace_w1 % world) sends every span of the batch to
    this rank, as a collector sharding one stream by trace id would (traces
    stay distinct up to 64-bit collisions).  w1: int64 tensor (u64 bits)."""
    if world == 1:
        return w1
    import torch
    u = w1.view(torch.uint64) if hasattr(torch, "uint64") else None
    if u is not None:
        try:
            return (u - u % world + rank).view(torch.int64)
        except (RuntimeError, TypeError):
            pass
    # unsigned remainder from signed int64 arithmetic: 2^64 = q * world + r
    r64 = (1 << 64) % world
    rem = torch.remainder(w1, world)                     # (w1 as signed) mod world
    rem = torch.where(w1 < 0, torch.remainder(rem + r64, world), rem)
    return w1 - rem + rank


def trace_variants(w0, w1, k, seed, rank=0, world=1):
    """k distinct trace-id column pairs from one batch's: every trace id XORed
    with a per-variant random 128-bit constant (a bijection, so the traces of
    a variant stay distinct and keep their span counts), then kept in this
    rank's trace-id shard (to_shard).  Each step of the bench aggregates a
    variant no launch has seen, so HLL registers keep rising as they would on
    a live stream."""
    import numpy as np
    rng = np.random.Generator(np.random.PCG64(seed))
    out = [(w0, to_shard(w1, rank, world))]
    for _ in range(k - 1):
        c0, c1 = (int(x) for x in rng.integers(-2**63, 2**63 - 1, 2, dtype=np.int64))
        out.append((w0 ^ c0, to_shard(w1 ^ c1, rank, world)))
    return out


def n_variants(args, launches, device):
    """Trace-id variants to build: one per launch before the soak (--variants 0,
    the default), so every launch `value`, `kernel_ms` and a rocprofv3 trace of
    the run see is a fresh trace-id set; an explicit --variants caps it.  Each
    variant is 16 B/span of device memory; the count is bounded by what fits in
    half the free HBM (a 400-step trace of 10 M-span batches needs ~93 GB)."""
    want = launches if args.variants <= 0 else min(args.variants, launches)
    import torch
    free, _ = torch.cuda.mem_get_info(device)
    per_span = 44 if getattr(args, "fresh_cols", False) else 16  # (--fresh-cols: every column per variant)
    fit = max(2, int(free // 2 // (per_span * args.spans)))
    if want > fit:
        print(f"bench: {want} trace-id variants do not fit; using {fit} (variants repeat)", file=sys.stderr)
    return min(want, fit)


WORKLOADS = {
    "c2": ("C2: synthetic SoA v1 spans, 20 services x 25 span names (Zipf 1.1) x 3 status codes -> "
           "<=1,500 series, default spanmetrics buckets, lognormal durations, ~10 spans/trace, "
           "per-service HLL p=14 + error count-min 4x2048, 10 s windows; a fresh trace-id set every step"),
    "c4": ("C4: 1,000,000 series (2,000 http.route x 500 k8s.pod.name), uniform over keys, binned HBM "
           "key table, HLL + count-min; a fresh trace-id set every step"),
    "c4zipf": ("C4 Zipf: 1,000,000 series (2,000 http.route x 500 k8s.pod.name), Zipf(s=1.1) over keys, "
               "binned HBM key table, HLL + count-min; a fresh trace-id set every step"),
    "c2expo": ("C2 with histogram.exponential (max_size 160): the C2 spans, per-series go-expohisto "
               "histograms (small-table kernel in EXPO mode + slab reduce/rescale + LDS-cached bucket "
               "counts), HLL + count-min; a fresh trace-id set every step"),
}


def run_workload(name, n, args, device, rank, world, barrier):
    """One workload on this rank: a fresh engine, device-resident columns,
    cold first launch, warm-up, the kernel alone (serial launches, HIP events
    on the launch stream), then the timed steps over the streams.  Every
    launch aggregates a distinct trace-id variant of the batch."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from spanagg import Config, Engine
    from spanagg.synth import generate_c2, generate_highcard

    exp_max = 160 if name == "c2expo" else 0
    if name in ("c2", "c2expo"):
        nps = getattr(args, "names_per_service", 25)
        wl = generate_c2(n, seed=42 + rank, names_per_service=nps)
        # (20 services x nps names x 3 status codes: 1,500 series at the default 25)
        batch, first_window, n_services, key_capacity = wl.batch, wl.first_window, wl.n_services, 60 * nps
    else:
        batch, _, first_window = generate_highcard(n, seed=7 + rank, zipf_s=1.1 if name == "c4zipf" else 0.0)
        wl, n_services, key_capacity = None, 1, 1_200_000
    cols = []
    for c in batch.columns():
        cols.append(torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(device))
    n_iso = max(3, args.steps // 5)
    gk = getattr(args, "graph_k", 0) if (name == "c2" and world == 1) else 0
    g_calls = max(1, args.steps // gk) if gk > 0 else 0
    n_var = n_variants(args, 1 + args.settle + args.warmup + 2 * n_iso + args.steps + (2 + g_calls) * gk, device)
    variants = trace_variants(cols[3], cols[4], n_var, seed=1000 + rank, rank=rank, world=world)
    # every variant's own copy of the other columns too (--fresh-cols): no
    # launch re-reads an address an earlier launch read, so no column can be
    # served from the last-level cache across launches
    full = [(cols[0].clone(), cols[1].clone(), cols[2].clone(), w0, w1, cols[5].clone())
            if getattr(args, "fresh_cols", False) else (cols[0], cols[1], cols[2], w0, w1, cols[5])
            for w0, w1 in variants]
    if world > 1:  # every span of every variant belongs to this rank's trace-id shard
        from spanagg.dist import shard_of
        for _, vw1 in variants[:2]:
            assert (shard_of(vw1[:4096].cpu().numpy().view(np.uint64), world) == rank).all()
    eng = Engine(Config(n_services=max(n_services, 1), n_windows=16, key_capacity=key_capacity,
                        device=device.index, exp_max_size=exp_max))
    eng.window_advance(first_window)
    streams = [torch.cuda.Stream(device) for _ in range(max(1, args.streams))]
    stream = streams[0]
    torch.cuda.set_stream(stream)
    launches = [0]

    def step(i, s=None):
        s = s or streams[i % len(streams)]
        v = full[launches[0] % len(full)]
        launches[0] += 1
        eng.ingest_device(v[0], v[1], v[2], v[3], v[4], v[5], n=n, stream=s.cuda_stream)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    torch.cuda.synchronize(device)
    # 0) the cold first launch on a fresh engine (empty key table and sketches)
    c0, c1 = ev(), ev()
    c0.record(stream)
    step(0, stream)
    eng.join(stream.cuda_stream)
    c1.record(stream)
    # settling launches: the first launches into a window raise many HLL
    # registers and its lower bounds are still low, so they run longer (a 10 s
    # window at this rate is ~10^5 launches, all but the first few settled);
    # timed one by one and reported as settle_ms, never part of value
    st = [(ev(), ev()) for _ in range(args.settle)]
    for a, b in st:
        eng.join(stream.cuda_stream)
        a.record(stream)
        step(0, stream)
        eng.join(stream.cuda_stream)
        b.record(stream)
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(device)
    cold_ms = c0.elapsed_time(c1)
    settle_ms = [round(a.elapsed_time(b), 4) for a, b in st]
    # 1) the kernel alone: serial launches on one stream.  kernel_ms: HIP events
    #    around n_iso back-to-back launches, divided by n_iso (each launch's
    #    duration plus the gap to the next); kernel_ms_bracketed: HIP events
    #    around each launch on its own (adds the events' own cost per launch)
    iso = [(ev(), ev()) for _ in range(n_iso)]
    for a, b in iso:
        eng.join(stream.cuda_stream)
        a.record(stream)
        step(0, stream)
        eng.join(stream.cuda_stream)
        b.record(stream)
    k0, k1 = ev(), ev()
    eng.join(stream.cuda_stream)
    k0.record(stream)
    for _ in range(n_iso):
        step(0, stream)
    eng.join(stream.cuda_stream)  # (the binned path aggregates on an engine stream)
    k1.record(stream)
    torch.cuda.synchronize(device)
    kernel_ms_bracketed = sum(a.elapsed_time(b) for a, b in iso) / len(iso)
    kernel_ms = k0.elapsed_time(k1) / n_iso
    # 2) the timed steps, alternating over the streams
    start = ev()
    ends = [ev() for _ in streams]
    barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    start.record(stream)
    for s in streams[1:]:
        s.wait_event(start)
    for i in range(args.steps):
        step(i)
    enqueue_s = time.perf_counter() - t0
    for s, e_ in zip(streams, ends):
        eng.join(s.cuda_stream)
        e_.record(s)
    torch.cuda.synchronize(device)
    elapsed = time.perf_counter() - t0
    barrier()
    device_ms = max(start.elapsed_time(e_) for e_ in ends) / max(1, args.steps)
    # 2b) the same launches as groups of K through sa_ingest_device_many (one
    #     HIP graph per call on small-table engines, so no dispatch gap between
    #     the K kernels); both of the engine's graphs are instantiated by two
    #     untimed calls, the timed calls re-point them at fresh variants
    graph = None
    if gk > 0:
        def many(s):
            bs = []
            for _ in range(gk):
                v = full[launches[0] % len(full)]
                launches[0] += 1
                bs.append((v[0], v[1], v[2], v[3], v[4], v[5], n))
            eng.ingest_device_many(bs, stream=s.cuda_stream)

        for _ in range(2):
            many(stream)
        eng.join(stream.cuda_stream)
        torch.cuda.synchronize(device)
        g0, g1 = ev(), ev()
        tg = time.perf_counter()
        g0.record(stream)
        for _ in range(g_calls):
            many(stream)
        eng.join(stream.cuda_stream)
        g1.record(stream)
        torch.cuda.synchronize(device)
        g_el = time.perf_counter() - tg
        graph = {"k": gk, "steps": g_calls * gk, "ms_per_step": g_el * 1e3 / (g_calls * gk),
                 "device_ms_per_step": g0.elapsed_time(g1) / (g_calls * gk)}
    # 3) sustained: back-to-back launches over the streams for --soak-s seconds
    #    (after the timed steps, never part of value; trace-id variants repeat
    #    here, so later HLL reads raise little) -- the rate a collector holds
    soak = None
    if args.soak_s > 0:
        per = max(1, int(args.soak_s / max(device_ms * 1e-3, 1e-5)) // 8)  # launches per host check
        n_soak, ts = 0, time.perf_counter()
        while True:
            for i in range(per):
                step(i)
            n_soak += per
            torch.cuda.synchronize(device)
            if time.perf_counter() - ts >= args.soak_s:
                break
        soak_s = time.perf_counter() - ts
        soak = {"value": n * n_soak / soak_s, "unit": "spans/s", "launches": n_soak, "seconds": soak_s,
                "note": f"trace-id variants repeat every {len(variants)} launches here, so the window's HLL "
                        "registers saturate and their raises idle: the rate of a saturated window, not a "
                        "figure of the kernel on fresh traces (value's timed steps are all fresh variants)"}
    own = {"rank": rank, "device": str(device), "ms_per_step": elapsed * 1e3 / max(1, args.steps),
           "kernel_ms": kernel_ms, "device_ms_per_step": device_ms}
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms, kernel_ms_bracketed, device_ms, cold_ms], dtype=torch.float64,
                         device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms, kernel_ms_bracketed, device_ms, cold_ms = (float(x) for x in t)
    # one flush (+ RCCL merge across ranks) after the timed region
    torch.cuda.synchronize(device)
    tm = time.perf_counter()
    if world > 1:
        from spanagg.dist import EnginePartial, merge_red, merge_window
        part = EnginePartial(eng, device)
        red = merge_red(part, reset=True)
        merge_window(part, first_window + 1)
    else:
        red = eng.flush_exp() if exp_max else eng.flush()
    torch.cuda.synchronize(device)
    merge_ms = (time.perf_counter() - tm) * 1e3
    own["merge_ms"] = merge_ms
    per_rank = [own]
    if world > 1:  # every rank's own figures (value uses the max over ranks)
        per_rank = [None] * world
        dist.all_gather_object(per_rank, own)
    st = eng.stats()
    calls = int(red.count.sum()) if exp_max else int(red.calls.sum())
    calls_ok = calls == launches[0] * n * world - st["zero_key"] * (1 if world == 1 else world)
    # the whole window from its cold start: cold + settling launches (HIP
    # events, one by one) + the timed steps (wall clock); the warm-up and the
    # isolated kernel-time launches in between are left out
    incl_s = (cold_ms + sum(settle_ms)) * 1e-3 + elapsed
    out = {"value_incl_settle": world * n * (1 + args.settle + args.steps) / incl_s,
           "wl": wl, "batch": batch, "eng": eng, "first_window": first_window, "elapsed": elapsed,
           "kernel_ms": kernel_ms, "kernel_ms_bracketed": kernel_ms_bracketed, "device_ms": device_ms,
           "cold_ms": cold_ms, "settle_ms": settle_ms, "sustained": soak, "graph": graph,
           "merge_ms": merge_ms, "per_rank": per_rank,
           "calls_ok": calls_ok, "enqueue_s": enqueue_s, "streams": len(streams), "variants": n_var,
           "launches": launches[0], "hll_p": 14,
           "hll_filtered_frac": st["hll_filtered"] / max(1, launches[0] * n)}
    del variants, cols
    return out


def kernel_ms_filter_off(n, args, device):
    """C2 kernel time with the HLL lower-bound filter off (SA_OPT_NO_HLL_FILTER
    at engine creation): every span reads its HLL register.  Same launches as the
    main run's kernel time (fresh variants, after cold + settle + warm-up), so
    the filter's share of the kernel time is visible beside `value`."""
    import numpy as np
    import torch

    from spanagg import Config, Engine
    from spanagg.synth import generate_c2

    wl = generate_c2(n, seed=42)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(device)
            for c in wl.batch.columns()]
    n_iso = max(3, args.steps // 5)
    k = 1 + args.settle + args.warmup + n_iso
    variants = trace_variants(cols[3], cols[4], k, seed=1000)
    from spanagg._lib import OPT_NO_HLL_FILTER
    eng = Engine(Config(n_services=wl.n_services, n_windows=16, key_capacity=1500, device=device.index,
                        options=OPT_NO_HLL_FILTER))
    eng.window_advance(wl.first_window)
    s = torch.cuda.current_stream(device)
    for w0, w1 in variants[: k - n_iso]:
        eng.ingest_device(cols[0], cols[1], cols[2], w0, w1, cols[5], n=n, stream=s.cuda_stream)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for w0, w1 in variants[k - n_iso:]:
        eng.ingest_device(cols[0], cols[1], cols[2], w0, w1, cols[5], n=n, stream=s.cuda_stream)
    b.record(s)
    torch.cuda.synchronize(device)
    ms = a.elapsed_time(b) / n_iso
    filt = eng.stats()["hll_filtered"]
    eng.close()
    return {"kernel_ms": ms, "hll_filtered": filt,
            "note": "C2 kernel alone (serial launches after cold + settle + warm-up, fresh trace-id variants) "
                    "with SA_OPT_NO_HLL_FILTER: every span gathers its HLL register"}


def run_group(n, members, args, device):
    """--group N: N engines of one group on this one device, fed through
    sa_group_ingest_device (the partition kernel shards each batch by trace id
    into the members' buffers), then one group flush (device key union, dense
    rows summed on the device).  Measures the group's overhead on one GPU
    (partition + N smaller launches) and the flush at the workload's
    cardinality (--workload c4: ~1 M series, every member holding most of
    them), not multi-GPU scaling."""
    import numpy as np
    import torch

    from spanagg import Config, Group
    from spanagg.synth import generate_c2, generate_highcard

    if args.workload in ("c4", "c4zipf"):
        batch, _, first = generate_highcard(n, seed=7, zipf_s=1.1 if args.workload == "c4zipf" else 0.0)
        n_services, kcap = 1, 1_200_000
    else:
        wl = generate_c2(n, seed=42)
        batch, first, n_services, kcap = wl.batch, wl.first_window, wl.n_services, 1500
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(device)
            for c in batch.columns()]
    k = args.warmup + args.steps
    variants = trace_variants(cols[3], cols[4], n_variants(args, k, device), seed=1000)
    g = Group([device.index] * members, Config(n_services=n_services, n_windows=16, key_capacity=kcap))
    g.window_advance(first)
    s = torch.cuda.current_stream(device)
    for i in range(args.warmup):
        w0, w1 = variants[i % len(variants)]
        g.ingest_device(cols[0], cols[1], cols[2], w0, w1, cols[5], n=n, stream=s.cuda_stream)
    g.sync()
    torch.cuda.synchronize(device)
    # the first flush (after the warmup launches) sets up the page-locked
    # result buffers; a collector flushes every interval, so the timed flush
    # is the second one, after the timed launches
    tf = time.perf_counter()
    red = g.flush()
    first_flush_ms = (time.perf_counter() - tf) * 1e3
    calls = int(red.calls.sum())
    del red
    t0 = time.perf_counter()
    for i in range(args.warmup, k):
        w0, w1 = variants[i % len(variants)]
        g.ingest_device(cols[0], cols[1], cols[2], w0, w1, cols[5], n=n, stream=s.cuda_stream)
    g.sync()
    torch.cuda.synchronize(device)
    el = time.perf_counter() - t0
    tf = time.perf_counter()
    red = g.flush()
    flush_ms = (time.perf_counter() - tf) * 1e3
    calls += int(red.calls.sum())
    st = g.stats()
    g.close()
    return {"members": members, "workload": args.workload, "value": n * args.steps / el, "unit": "spans/s",
            "ms_per_step": el * 1e3 / args.steps, "flush_ms": flush_ms, "first_flush_ms": first_flush_ms,
            "flush_series": len(red.key_hash), "calls_check": calls == n * k - st["zero_key"],
            "note": f"{members} engines of one group on this device, sa_group_ingest_device of {n:,}-span "
                    "device batches (partition kernel + one launch per member); flush_ms: the second "
                    "sa_group_flush (device key union, dense rows summed on the device, one D2H into reused "
                    "page-locked buffers), first_flush_ms: the first, which allocates them; overhead on one "
                    "GPU, not scaling"}


def roofline(name, n, r, traffic_path=None):
    achieved = BYTES_PER_SPAN * n / (r["kernel_ms"] * 1e-3) / 1e9
    tpath = traffic_path or os.path.join(ROOT, "profiles", "traffic.json" if name == "c2" else f"traffic_{name}.json")
    traffic, tsrc = load_traffic(tpath, name)
    piped = BYTES_PER_SPAN * n / (r["device_ms"] * 1e-3) / 1e9
    kern = {"c2": "ingest_v2_kernel (spanagg_kernels.hip)",
            "c2expo": "ingest_v2_kernel EXPO mode + expo_reduce_rescale_kernel + expo_count_slab_kernel + "
                      "expo_fold_kernel (spanagg_kernels.hip, spanagg_expo.hip)",
            "c4": "bt_scatter2_kernel + bt_aggregate3_kernel (spanagg_binned.hip)",
            "c4zipf": "bt_scatter2_kernel + bt_aggregate3_kernel (spanagg_binned.hip)"}[name]
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kern, "kernel_ms": r["kernel_ms"],
            "kernel_ms_bracketed": r["kernel_ms_bracketed"],
            "bytes_per_span": BYTES_PER_SPAN, "traffic_source": tsrc,
            "pipelined": {"streams": r["streams"], "device_ms_per_step": r["device_ms"], "achieved": piped,
                          "frac": piped / HBM_PEAK_GBS}}
    if traffic:
        # what the kernel really moves (PMC bytes / kernel time), beside the
        # algorithmic-byte fraction above
        roof["measured_gbs"] = traffic / (r["kernel_ms"] * 1e-3) / 1e9
        roof["measured_frac"] = roof["measured_gbs"] / HBM_PEAK_GBS
        roof["traffic_over_algorithmic"] = traffic / (BYTES_PER_SPAN * n)
    return roof


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv, script=None, timeout=None, env=None) -> int:
    """`bench.py --gpus N` without an outer launcher: start N rank processes of
    `script` (default this file) with `argv`, one per GPU (RANK = LOCAL_RANK =
    i, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free port), as
    torch.distributed.run would.  This parent never imports torch or touches a
    GPU (it only spawns and waits), so no process that initialised the GPU is
    ever replaced.  Rank 0's stdout passes through to ours (its one JSON
    line); the other ranks' stdout goes to our stderr.  Returns 0 when every
    rank exits 0; otherwise the first failing rank's code (or 1), after
    terminating the ranks still running, so a rank that dies while the others
    wait in a collective cannot hang the job."""
    script = script or os.path.abspath(__file__)
    base = dict(os.environ if env is None else env)
    base.update({"WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                 "MASTER_PORT": str(free_port()), "GROUP_RANK": "0", "NODE_RANK": "0"})
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    base["SPANAGG_BENCH_LAUNCHER"] = "bench.py (one child process per rank)"
    procs = []
    for i in range(n):
        e = dict(base, RANK=str(i), LOCAL_RANK=str(i))
        procs.append(subprocess.Popen([sys.executable, "-u", script, *argv], env=e,
                                      stdout=None if i == 0 else sys.stderr, start_new_session=True))
    def signal_live(sig):
        for j in live:
            try:
                os.killpg(procs[j].pid, sig)
            except ProcessLookupError:
                pass

    t0, rc, kill_at = time.monotonic(), 0, None
    live = list(range(n))
    while live:
        for i in list(live):
            code = procs[i].poll()
            if code is None:
                continue
            live.remove(i)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench: rank {i} exited with {code}; stopping the other ranks", file=sys.stderr)
                signal_live(15)
                kill_at = time.monotonic() + 20  # SIGKILL what SIGTERM did not end
        now = time.monotonic()
        if timeout is not None and live and now - t0 > timeout and rc == 0:
            print(f"bench: ranks {live} still running after {timeout} s; stopping them", file=sys.stderr)
            rc, kill_at = 124, now
        if kill_at is not None and live and now >= kill_at:
            signal_live(9)
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--fresh-cols", dest="fresh_cols", action="store_true",
                    help="every launch reads its own copy of every column (not only of the trace ids)")
    ap.add_argument("--spans", type=int, default=10_000_000, help="spans per step per GPU")
    ap.add_argument("--workload", choices=list(WORKLOADS), default="c2")
    ap.add_argument("--names-per-service", dest="names_per_service", type=int, default=25,
                    help="span names per service of the C2 vocabulary (probe runs only; the C2 config is 25)")
    ap.add_argument("--streams", type=int, default=2,
                    help="launch streams the steps alternate over (the engine's two slab sets "
                         "let consecutive launches overlap); 1 = strictly serial launches")
    ap.add_argument("--soak-s", type=float, default=2.0,
                    help="seconds of back-to-back launches after the timed steps (reported as sustained)")
    ap.add_argument("--settle", type=int, default=16,
                    help="untimed launches after the cold one, before the warm-up (HLL registers settle)")
    ap.add_argument("--variants", type=int, default=0,
                    help="distinct trace-id variants of the batch (0 = one per launch before the soak; "
                         "N = at most N, repeating after that)")
    ap.add_argument("--sub", default="c4,c4zipf,c2expo",
                    help="extra workloads reported as sub-objects of the line at N=1 ('' = none)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--h2d-reps", type=int, default=5,
                    help="host-buffer sa_ingest repetitions (PCIe-inclusive rate; 0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=None,
                    help="PMC traffic summary of the main workload (default profiles/traffic[_<wl>].json)")
    ap.add_argument("--host-otlp-spans", type=int, default=2_000_000,
                    help="spans for the Node host's OTLP->GPU rate (0 = skip)")
    ap.add_argument("--cpu-workers", type=int, default=None,
                    help="processes for the multi-core CPU baseline (default: every usable host core; 0 = skip)")
    ap.add_argument("--group", type=int, default=0,
                    help="also time an N-member engine group on this one device (sa_group_ingest_device)")
    ap.add_argument("--graph-k", dest="graph_k", type=int, default=10,
                    help="C2 at N=1: also time the steps as groups of K through sa_ingest_device_many "
                         "(one HIP graph per call; reported as the c2_graph sub-object; 0 = skip)")
    ap.add_argument("--no-filter-off", action="store_true",
                    help="skip the C2 kernel time with the HLL lower-bound filter off")
    ap.add_argument("--cpu-worker", type=int, default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.cpu_worker is not None:  # child of cpu_baseline_multicore (no GPU use)
        cpu_worker(args.cpu_worker, args.cpu_seconds)
        return 0
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no outer launcher: start the N rank processes ourselves (before any
        # torch import or GPU call in this process) and pass rank 0's line on
        return launch_ranks(args.gpus, sys.argv[1:])

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: WORLD_SIZE {world} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    # SPANAGG_BENCH_ONE_DEVICE=1 rehearses the N-rank path on a one-GPU box:
    # every rank on cuda:0, gloo collectives (never for a reported number)
    one_dev = os.environ.get("SPANAGG_BENCH_ONE_DEVICE") == "1"
    torch.cuda.set_device(0 if one_dev else local_rank)
    device = torch.device("cuda", 0 if one_dev else local_rank)
    backend = None
    if world > 1:
        if one_dev:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)
        backend = dist.get_backend()
        if dist.get_world_size() != args.gpus:
            print(f"bench: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}", file=sys.stderr)
            return 2

    def barrier():
        if world > 1:
            dist.barrier()

    n = args.spans
    main_r = run_workload(args.workload, n, args, device, rank, world, barrier)
    eng, batch = main_r["eng"], main_r["batch"]

    # the host-buffer boundary (sa_ingest: the batch starts in pageable host
    # memory, PCIe H2D included), timed after the device-resident steps; it
    # is reported beside `value`, never as it
    h2d = None
    if world == 1 and args.h2d_reps > 0:
        eng.ingest(batch)  # warm the staging buffers
        torch.cuda.synchronize(device)
        th = time.perf_counter()
        for _ in range(args.h2d_reps):
            eng.ingest(batch)
        torch.cuda.synchronize(device)
        h2d_s = time.perf_counter() - th
        h2d_calls = int(eng.flush().calls.sum())
        h2d = {"value": args.h2d_reps * n / h2d_s, "unit": "spans/s",
               "ms_per_batch": h2d_s * 1e3 / args.h2d_reps,
               "gb_per_s": BYTES_PER_SPAN * n * args.h2d_reps / h2d_s / 1e9,
               "calls_check": h2d_calls == (args.h2d_reps + 1) * n,
               "sample": f"{args.h2d_reps} x sa_ingest of the {n:,}-span batch from pageable "
                         "host numpy columns (H2D + kernel), after one warm-up ingest"}
    eng.close()

    subs = {}
    if world == 1:
        for sub in [w for w in args.sub.split(",") if w and w != args.workload]:
            r = run_workload(sub, n, args, device, rank, world, barrier)
            r["eng"].close()
            subs[sub] = {"workload": WORKLOADS[sub], "value": n * args.steps / r["elapsed"], "unit": "spans/s",
                         "value_incl_settle": r["value_incl_settle"],
                         "ms_per_step": r["elapsed"] * 1e3 / args.steps, "steps": args.steps,
                         "warmup": args.warmup, "cold_launch_ms": r["cold_ms"], "settle_ms": r["settle_ms"],
                         "sustained": r["sustained"],
                         "roofline": roofline(sub, n, r), "calls_check": r["calls_ok"],
                         "trace_variants": r["variants"]}
            torch.cuda.empty_cache()

    extra = {}
    g = main_r.get("graph")
    if g is not None:
        # K steps per sa_ingest_device_many call (one HIP graph of K launches),
        # fresh trace-id variants, one stream; wall clock around the calls
        ach = BYTES_PER_SPAN * n / (g["ms_per_step"] * 1e-3) / 1e9
        extra["c2_graph"] = {
            "workload": WORKLOADS["c2"] + f"; K = {g['k']} batches per sa_ingest_device_many call (one HIP graph)",
            "value": n / (g["ms_per_step"] * 1e-3), "unit": "spans/s", "ms_per_step": g["ms_per_step"],
            "device_ms_per_step": g["device_ms_per_step"], "steps": g["steps"], "k": g["k"],
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "per": "wall-clock step (launch gaps included)"},
            "calls_check": main_r["calls_ok"]}
    if world == 1 and args.workload == "c2" and not args.no_filter_off:
        extra["hll_filter_off"] = kernel_ms_filter_off(n, args, device)
        torch.cuda.empty_cache()
    if world == 1 and args.group > 1:
        extra["group"] = run_group(n, args.group, args, device)
        torch.cuda.empty_cache()

    result = None
    ok = main_r["calls_ok"] and all(v["calls_check"] for v in subs.values()) and \
        all(v.get("calls_check", True) for v in extra.values())
    if rank == 0:
        elapsed = main_r["elapsed"]
        result = {
            "metric": METRIC, "value": world * n * args.steps / elapsed, "unit": "spans/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (seeded PCG64 generator, spanagg/synth.py; each rank's batch in its trace-id shard "
                    "(trace_w1 % N == rank); every launch "
                    "a distinct trace-id variant of the rank's batch)",
            "config": {"workload": WORKLOADS[args.workload], "spans_per_step_per_gpu": n,
                       **({"rehearsal": "all ranks on one device, gloo"} if one_dev else {}),
                       "global_spans_per_step": n * world,
                       "parallelism": f"trace-id shards x{world}, RCCL merge at flush"},
            "roofline": roofline(args.workload, n, main_r, args.traffic),
            "value_incl_settle": main_r["value_incl_settle"],
            "cold_launch_ms": main_r["cold_ms"], "settle_ms": main_r["settle_ms"],
            "sustained": main_r["sustained"],
            "trace_variants": main_r["variants"],
            "hll_filtered_frac": main_r["hll_filtered_frac"],
            "merge_ms": main_r["merge_ms"], "calls_check": main_r["calls_ok"],
            "distributed": {"world_size": world, "backend": backend,
                            "launcher": os.environ.get("SPANAGG_BENCH_LAUNCHER", "external" if world > 1 else None),
                            "per_rank": main_r["per_rank"]},
            "host_enqueue_us_per_step": main_r["enqueue_s"] * 1e6 / max(1, args.steps),
        }
        result.update(subs)
        result.update(extra)
        if "c2_graph" in extra:
            # the same kernel launched K at a time from a HIP graph (no dispatch
            # gap between launches): device time per launch, HIP events around
            # the calls on their stream; `frac` above stays the serial launches'
            gd = extra["c2_graph"]["device_ms_per_step"]
            result["roofline"]["graph_ms_per_launch"] = gd
            result["roofline"]["frac_graph_launches"] = BYTES_PER_SPAN * n / (gd * 1e-3) / 1e9 / HBM_PEAK_GBS
        if h2d is not None:
            result["host_buffer_ingest"] = h2d
        wl = main_r["wl"]
        if world == 1 and not args.no_cpu_baseline and wl is not None:
            port, conn = cpu_baseline(wl, args.cpu_seconds)
            result["cpu_baseline"] = port
            result["cpu_baseline_connector"] = conn
            cores = box_cores()
            workers = cores["usable"] if args.cpu_workers is None else args.cpu_workers
            if workers > 1:
                mc = cpu_baseline_multicore(workers, args.cpu_seconds / 2)
                mc.update({"nproc": cores["nproc"], "affinity_cpus": cores["affinity"],
                           "cgroup_quota_cpus": cores["cgroup_quota_cpus"]})
                result["cpu_baseline_multicore"] = mc
        if world == 1 and args.host_otlp_spans > 0:
            # the box's usable cores (its cgroup CPU share), at most 16 decode threads
            hthreads = max(1, min(16, box_cores()["usable"]))
            result["host_otlp"] = host_otlp_rate(args.host_otlp_spans, threads=hthreads)
            # the same with exemplars (5 per data point) and span events (exception.type) on
            result["host_otlp_exemplars_events"] = host_otlp_rate(args.host_otlp_spans, threads=hthreads,
                                                                  extra=("--exemplars", "--events"))
            # SURVEY 8(d) also asks for the decode + aggregate rate on one core
            result["host_otlp_1core"] = host_otlp_rate(args.host_otlp_spans, threads=1)
            # BASELINE config 4's 1 M-series vocabulary through the Node host (binned engine table)
            result["host_otlp_c4"] = host_otlp_rate(args.host_otlp_spans, threads=hthreads, extra=("--highcard",))
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
