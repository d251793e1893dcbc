#!/usr/bin/env python3
"""Per-workgroup phases of the exponential-histogram counting kernel
(expo_count_slab_kernel) and of the EXPO-mode ingest kernel before it, from
in-kernel s_memrealtime stamps (SA_OPT_STAMPS; 100 MHz), on the c2expo
workload (10 M C2 spans, max_size 160).  The stamps are the last launch's.
  ingest row slots 0..3: start, prologue done, loop done, end
  counting slots 4..7:   start, prologue (entry selection) done, loop done, end;
                         slot 135: its slab stores issued
Environment: XC_LAUNCHES (default 24), SPANAGG_LIB / SPANAGG_XC_DIAG for the
laboratory build's ablations."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opentelemetry-demo_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spanagg import Config, Engine, _lib  # noqa: E402
from spanagg.synth import generate_c2  # noqa: E402

ROW = 136


def q(a):
    a = np.asarray(a, dtype=np.float64) / 100.0  # 100 MHz ticks -> us
    return {"min": round(float(a.min()), 2), "med": round(float(np.median(a)), 2), "max": round(float(a.max()), 2)}


def phases(e):
    n = C.c_uint64(0)
    e.lib.sa_debug_stamps(e._h, None, 0, C.byref(n))
    buf = np.zeros(n.value, np.uint64)
    e.lib.sa_debug_stamps(e._h, buf.ctypes.data_as(_lib.u64p), n.value, C.byref(n))
    rows = buf.reshape(-1, ROW).astype(np.int64)
    ing = rows[rows[:, 0] > 0][:, :4]
    cnt = rows[rows[:, 4] > 0]
    c, slab = cnt[:, 4:8], cnt[:, ROW - 1]
    zeroed, selected = cnt[:, ROW - 9], cnt[:, ROW - 17]
    wg = np.nonzero(rows[:, 4] > 0)[0]
    loop = c[:, 2] - c[:, 1]
    t0 = ing[:, 0].min()
    return {
        "ingest": {"wgs": int(len(ing)), "prologue": q(ing[:, 1] - ing[:, 0]), "loop": q(ing[:, 2] - ing[:, 1]),
                   "epilogue": q(ing[:, 3] - ing[:, 2]), "end": q(ing[:, 3] - t0)},
        "count": {"wgs": int(len(c)), "start_after_ingest_end": q(c[:, 0] - ing[:, 3].max()),
                  "start_skew": q(c[:, 0] - c[:, 0].min()),
                  "prologue": q(c[:, 1] - c[:, 0]), "pro_to_zeroed": q(zeroed - c[:, 0]),
                  "pro_zeroed_to_selected": q(selected - zeroed), "pro_selected_to_sync": q(c[:, 1] - selected),
                  "loop": q(loop),
                  # workgroup i runs on XCD i % 8: is the loop's spread per XCD?
                  "loop_by_xcd": [q(loop[wg % 8 == x]) for x in range(8)],
                  "loop_slowest_wgs": [int(x) for x in wg[np.argsort(loop)[-8:]]],
                  # the workgroups' tail records (spans of series without an LDS entry; past 4,096: HBM atomics)
                  "tail_records": {"min": int(cnt[:, ROW - 25].min()), "med": float(np.median(cnt[:, ROW - 25])),
                                   "max": int(cnt[:, ROW - 25].max()),
                                   "corr_with_loop": float(np.corrcoef(cnt[:, ROW - 25], loop)[0, 1])},
                  # wave steps that took the rare path (long durations, a risen scale, out of range;
                  # the long ones are deferred to after the loop)
                  "rare_steps": {"min": int(cnt[:, ROW - 33].min()), "med": float(np.median(cnt[:, ROW - 33])),
                                 "max": int(cnt[:, ROW - 33].max()),
                                 "corr_with_loop": float(np.corrcoef(cnt[:, ROW - 33], loop)[0, 1]) if cnt[:, ROW - 33].std() > 0 else 0.0,
                                 "slowest_wgs": [int(x) for x in cnt[np.argsort(loop)[-8:], ROW - 33]],
                                 "deferred_long_med": float(np.median(cnt[:, ROW - 41]))},
                  "slab_issue": q(slab - c[:, 2]), "tail": q(c[:, 3] - slab),
                  "lifetime": q(c[:, 3] - c[:, 0]), "end": q(c[:, 3] - c[:, 0].min())},
    }


def main():
    n = 10_000_000
    wl = generate_c2(n, seed=42)
    dev = torch.device("cuda", 0)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).to(dev)
            for c in wl.batch.columns()]
    s = torch.cuda.Stream(dev)
    cfg = Config(n_services=wl.n_services, n_windows=16, key_capacity=1500, exp_max_size=160,
                 options=_lib.OPT_STAMPS)
    out = {"xc_diag": os.environ.get("SPANAGG_XC_DIAG", "0"), "lib": os.path.basename(os.environ.get("SPANAGG_LIB", ""))}
    with Engine(cfg) as e:
        e.window_advance(wl.first_window)
        for i in range(int(os.environ.get("XC_LAUNCHES", "24"))):
            c = list(cols)
            c[3] = cols[3] ^ (0x5DEECE66D * (i + 1))  # a fresh trace-id variant per launch, as bench.py
            e.ingest_device(*c, n=n, stream=s.cuda_stream)
        torch.cuda.synchronize()
        out.update(phases(e))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
