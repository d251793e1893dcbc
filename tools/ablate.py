#!/usr/bin/env python3
"""Attribute ingest-kernel time by ablation (cdna_hip_programming.md section 7,
diagnostic loop step 2): the same C2 batch through engines built with
SA_DIAG_* bits, timed in interleaved rounds in ONE process (HIP events on the
launch stream), median per variant.  Results of ablated variants are wrong by
design; only their time matters."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opentelemetry-demo_amd"))
# the laboratory build (variants, ablation flags): make -C opentelemetry-demo_amd ab
os.environ.setdefault("SPANAGG_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "opentelemetry-demo_amd", "spanagg", "libspanagg_ab.so"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spanagg import Config, Engine  # noqa: E402
from spanagg.synth import generate_c2  # noqa: E402

NO_RED, NO_HLL, NO_CMS, NO_FLUSH, L2_INPUT = 1, 2, 4, 8, 16
NO_BIN, NO_WIN, NO_STAT, NO_LOOP = 32, 64, 128, 256
LO = NO_RED | NO_HLL | NO_CMS | NO_FLUSH
VARIANTS_FINE = {
    "prologue_only": NO_LOOP | NO_FLUSH,
    "prologue_flush": NO_LOOP,
    "lo_nobin": LO | NO_BIN,
    "lo_nowin": LO | NO_WIN,
    "lo_nostat": LO | NO_STAT,
    "lo_bare": LO | NO_BIN | NO_WIN | NO_STAT,
    "lo_bare_l2": LO | NO_BIN | NO_WIN | NO_STAT | L2_INPUT,
    "hll_store": 512,
    "hll_noread": 1024,
    "lds_spread": 4096,
    "cheap_hash": 16384,
    "diag_baseline": 65536,  # an unused bit: the diagnostic build with full work
}
VARIANTS_C4 = {
    "lookup_only": 2048,  # HBM path: key-table lookups, no counter atomics
    "lookup_only_no_sketch": 2048 | NO_HLL | NO_CMS,
    "wg_scope_atomics": 8192,
}
VARIANTS = {
    "l2_input": L2_INPUT,
    "l2_input_no_hll": L2_INPUT | NO_HLL,
    "l2_input_loads_only": L2_INPUT | NO_RED | NO_HLL | NO_CMS | NO_FLUSH,
    "full": 0,
    "no_cms": NO_CMS,
    "no_hll": NO_HLL,
    "no_sketch": NO_HLL | NO_CMS,
    "no_flush": NO_FLUSH,
    "no_red": NO_RED | NO_FLUSH,
    "loads_only": NO_RED | NO_HLL | NO_CMS | NO_FLUSH,
}


def main():
    n = int(os.environ.get("ABL_SPANS", 10_000_000))
    rounds = int(os.environ.get("ABL_ROUNDS", 7))
    reps = int(os.environ.get("ABL_REPS", 10))
    c4 = os.environ.get("ABL_WORKLOAD") in ("c4", "c4zipf")
    if c4:  # high-cardinality HBM-table path (1 M keys, one service)
        from spanagg.synth import generate_highcard
        hb, _, hfirst = generate_highcard(n, seed=7, routes=int(os.environ.get("ABL_ROUTES", 2000)),
                                          zipf_s=1.1 if os.environ.get("ABL_WORKLOAD") == "c4zipf" else 0.0)

        class _W:
            batch, first_window, n_services = hb, hfirst, 1
        wl = _W()
    else:
        wl = generate_c2(n, seed=42)
    kcap = int(os.environ.get("ABL_KCAP", 1_200_000 if c4 else 1000))
    dev = torch.device("cuda", 0)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
            for c in wl.batch.columns()]
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    engines = {}
    base_variant = os.environ.get("SPANAGG_VARIANT", "0")
    os.environ["SPANAGG_VARIANT"] = os.environ.get("ABL_BASE", base_variant)
    if os.environ.get("ABL_NO_DIAG"):  # structure variants only
        VARIANTS.clear()
    if os.environ.get("ABL_FLAGS"):  # explicit set: "name:flags,name:flags"
        VARIANTS.clear()
        VARIANTS.update({k: int(v) for k, v in (x.split(":") for x in os.environ["ABL_FLAGS"].split(","))})
    if c4 and not os.environ.get("ABL_FLAGS"):
        VARIANTS.update(VARIANTS_C4)
    if os.environ.get("ABL_FINE"):
        VARIANTS.update(VARIANTS_FINE)
    for name, fl in VARIANTS.items():
        e = Engine(Config(n_services=wl.n_services, n_windows=16, flags=fl, key_capacity=kcap))
        e.window_advance(wl.first_window)
        engines[name] = e
    # kernel-structure variants (sa_internal.h kVariants), full work
    for v in [int(x) for x in os.environ.get("ABL_VARS", "0,8,11,12").split(",") if x]:
        os.environ["SPANAGG_VARIANT"] = str(v)
        e = Engine(Config(n_services=wl.n_services, n_windows=16, key_capacity=kcap))
        e.window_advance(wl.first_window)
        engines[f"variant{v}"] = e
    os.environ["SPANAGG_VARIANT"] = base_variant
    # engine-creation environment variants: "name:VAR=v;VAR2=v,name2:VAR=v"
    for spec in [x for x in os.environ.get("ABL_ENVS", "").split(",") if x]:
        name, kv = spec.split(":", 1)
        saved = {}
        for item in [y for y in kv.split(";") if y]:
            k, v = item.split("=", 1)
            saved[k] = os.environ.get(k)
            os.environ[k] = v
        e = Engine(Config(n_services=wl.n_services, n_windows=16, key_capacity=kcap))
        e.window_advance(wl.first_window)
        engines[name] = e
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for kc in [int(x) for x in os.environ.get("ABL_KCAPS", "").split(",") if x]:
        e = Engine(Config(n_services=wl.n_services, n_windows=16, key_capacity=kc))
        e.window_advance(wl.first_window)
        engines[f"key_capacity{kc}"] = e
    times = {k: [] for k in engines}
    for r in range(rounds):
        for name, e in engines.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e.ingest_device(*cols, n=n, stream=stream.cuda_stream)  # warm
            a.record(stream)
            for _ in range(reps):
                e.ingest_device(*cols, n=n, stream=stream.cuda_stream)
            b.record(stream)
            b.synchronize()
            times[name].append(a.elapsed_time(b) / reps * 1e3)  # us per launch
    # pure-read reference: torch reductions over the same 44 B/span
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        a.record(stream)
        for _ in range(reps):
            s = sum(c.sum() for c in cols)
        b.record(stream)
        b.synchronize()
    torch_read_us = a.elapsed_time(b) / reps * 1e3
    out = {"spans": n, "bytes": 44 * n, "rounds": rounds, "reps": reps, "variants": {}}
    for k, v in times.items():
        med = statistics.median(v)
        out["variants"][k] = {"median_us": med, "min_us": min(v),
                              "gbs": 44 * n / (med * 1e-6) / 1e9,
                              "spans_per_s": n / (med * 1e-6)}
    out["torch_sum_read_us"] = torch_read_us
    out["torch_sum_read_gbs"] = 44 * n / (torch_read_us * 1e-6) / 1e9
    print(json.dumps(out, indent=1))
    for e in engines.values():
        e.close()


if __name__ == "__main__":
    main()
