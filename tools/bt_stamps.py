#!/usr/bin/env python3
"""Per-workgroup timeline of the binned C4 kernels (bt_scatter2_kernel,
bt_aggregate3_kernel, or bt_aggregate2_kernel with SPANAGG_BT_AGG=2) from in-kernel s_memrealtime stamps (SA_OPT_STAMPS
diagnostic engines).  Prints phase durations (us) over workgroups."""
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
from spanagg.synth import generate_highcard  # noqa: E402


def q(a):
    a = np.asarray(a, dtype=float) / 100.0  # 100 MHz ticks -> us
    return {"min": round(float(a.min()), 2), "med": round(float(np.median(a)), 2),
            "p90": round(float(np.percentile(a, 90)), 2), "max": round(float(a.max()), 2)}


def main():
    wk = os.environ.get("WL", "c4")
    n = 10_000_000
    batch, _, first = generate_highcard(n, seed=7, zipf_s=1.1 if wk == "c4zipf" else 0.0)
    cols = [torch.from_numpy(c.view(np.int64) if c.dtype == np.uint64 else c.view(np.int32)).cuda()
            for c in batch.columns()]
    s = torch.cuda.Stream()
    with Engine(Config(n_services=1, n_windows=16, key_capacity=1_200_000, options=_lib.OPT_STAMPS)) as e:
        e.window_advance(first)
        for _ in range(4):
            e.ingest_device(*cols, n=n, stream=s.cuda_stream)
        torch.cuda.synchronize()
        cnt = C.c_uint64(0)
        e.lib.sa_debug_stamps(e._h, None, 0, C.byref(cnt))
        buf = np.zeros(cnt.value, np.uint64)
        e.lib.sa_debug_stamps(e._h, buf.ctypes.data_as(_lib.u64p), cnt.value, C.byref(cnt))
    b = buf.astype(np.int64)
    agg = b[:2048 * 8].reshape(2048, 8)[:, :4]
    sc = b[2048 * 8:2048 * 8 + 256 * 8].reshape(256, 8)[:, :4]
    t0 = sc[:, 0].min()
    out = {
        "scatter": {"start": q(sc[:, 0] - t0), "prologue": q(sc[:, 1] - sc[:, 0]), "loop": q(sc[:, 2] - sc[:, 1]),
                    "epilogue": q(sc[:, 3] - sc[:, 2]), "end": q(sc[:, 3] - t0)},
        "aggregate": {"start": q(agg[:, 0] - t0), "setup": q(agg[:, 1] - agg[:, 0]),
                      "records": q(agg[:, 2] - agg[:, 1]), "rows": q(agg[:, 3] - agg[:, 2]),
                      "life": q(agg[:, 3] - agg[:, 0]), "end": q(agg[:, 3] - t0)},
    }
    # resident aggregate workgroups over time (sweep over start/end stamps):
    # the peak is the occupancy the LDS / register budget really allows
    ev = sorted([(int(a), 1) for a in agg[:, 0]] + [(int(z), -1) for z in agg[:, 3]])
    cur = peak = 0
    for _, d in ev:
        cur += d
        peak = max(peak, cur)
    out["aggregate"]["peak_resident"] = peak
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
