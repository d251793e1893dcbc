#!/usr/bin/env python3
"""Per-workgroup timeline of the small-table ingest kernel from in-kernel
s_memrealtime stamps (diagnostic build path, SA_OPT_STAMPS)."""
import ctypes as C
import json
import os
import sys

# the laboratory build (variants, ablation flags): make -C opentelemetry-demo_amd ab
os.environ.setdefault("SPANAGG_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                  "opentelemetry-demo_amd", "spanagg", "libspanagg_ab.so"))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opentelemetry-demo_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spanagg import Config, Engine, _lib  # noqa: E402
from spanagg.synth import generate_c2  # noqa: E402


def timeline(e):
    n = C.c_uint64(0)
    e.lib.sa_debug_stamps(e._h, None, 0, C.byref(n))
    buf = np.zeros(n.value, np.uint64)
    e.lib.sa_debug_stamps(e._h, buf.ctypes.data_as(_lib.u64p), n.value, C.byref(n))
    full = buf.reshape(-1, 136).astype(np.int64)
    t = full[:, :4]
    keep = t[:, 0] > 0
    t = t[keep]
    w = full[keep, 8:].reshape(-1, 16, 8)
    segs = w[:, :, :6].sum(axis=(0, 1)).astype(float)
    wend = w[:, :, 6] - t[:, :1]  # per-wave loop end relative to the WG start
    us = lambda x: x / 100.0  # 100 MHz
    t0 = t[:, 0].min()
    q = lambda a: {"min": float(us(a.min())), "med": float(us(np.median(a))), "max": float(us(a.max()))}
    return {"wgs": int(len(t)), "start_skew": q(t[:, 0] - t0), "init": q(t[:, 1] - t[:, 0]),
            "loop": q(t[:, 2] - t[:, 1]), "flush": q(t[:, 3] - t[:, 2]),
            "end": q(t[:, 3] - t0),
            "seg_share": [round(x / max(segs.sum(), 1), 3) for x in segs],
            "wave_loop_end": q(wend.reshape(-1)),
            "wave_skew_in_wg": q(wend.max(axis=1) - wend.min(axis=1)),
            "loop_end_by_wave_med": [round(us(float(np.median(wend[:, i]))), 1) for i in range(16)],
            # workgroup i runs on XCD i % 8 (round-robin dispatch): is the end spread per XCD?
            "end_by_xcd": [q((t[:, 3] - t0)[np.nonzero(keep)[0] % 8 == x]) for x in range(8)],
            # the launch if every workgroup ended at the mean end / its waves at their mean
            "end_mean": float(us((t[:, 3] - t0).mean())),
            "wave_end_mean_minus_max": q(wend.mean(axis=1) - wend.max(axis=1))}


def main():
    n = 10_000_000
    wl = generate_c2(n, seed=42)
    dev = torch.device("cuda", 0)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
            for c in wl.batch.columns()]
    s = torch.cuda.Stream(dev)
    out = {}
    for name, fl in [x for x in (("full", 0), ("loads_only", 15), ("no_sketch", 6))
                     if x[0] in os.environ.get("STAMP_SETS", "full,loads_only,no_sketch").split(",")]:
        for v in [int(x) for x in os.environ.get("STAMP_VARS", "0,8").split(",")]:
            os.environ["SPANAGG_VARIANT"] = str(v)
            with Engine(Config(n_services=wl.n_services, n_windows=16, flags=fl, options=_lib.OPT_STAMPS)) as e:
                e.window_advance(wl.first_window)
                for i in range(int(os.environ.get("STAMP_LAUNCHES", "24"))):
                    # a fresh trace-id variant per launch (as bench.py), so HLL raises do not idle
                    c = list(cols)
                    c[3] = cols[3] ^ (0x5DEECE66D * (i + 1))
                    e.ingest_device(*c, n=n, stream=s.cuda_stream)
                torch.cuda.synchronize()
                out[f"{name}/v{v}"] = timeline(e)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
