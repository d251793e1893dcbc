#!/usr/bin/env python3
"""profiles/traffic[_<wl>].json from the rocprofv3 FETCH_SIZE / WRITE_SIZE
passes of tools/gpu_job.sh (pmc_<wl>_fetch, pmc_<wl>_write over
tools/prof_driver.py): per ingest launch -- every hot-path kernel's bytes
from the first averaged launch on (the last PMC_LAST launches, else all but
the first), divided by those launches (C2: ingest_v2_kernel; C4: bt_scatter2
+ bt_aggregate3, whose paired dispatches cover two launches; c2expo:
ingest_v2 + the expo_* kernels) -- FETCH_SIZE doubled per
MI355X_MICROARCH.md's gfx950 correction, KB = 1024 B.

  python tools/traffic.py <job dir> <workload> <round> <out.json>"""
import collections
import csv
import json
import os
import sys


def _pick(ids):
    """Dispatches averaged: the last PMC_LAST of them (the settled regime of a
    fresh-variant run), else all but the first."""
    k = int(os.environ.get("PMC_LAST", "0"))
    return ids[-k:] if k else (ids[1:] or ids)


HOT = ("ingest", "bt_scatter", "bt_aggregate", "expo_")


PRIMARY = ("ingest", "bt_scatter")  # one dispatch per ingest launch


def per_launch(path, counter):
    """Bytes per ingest launch: every hot kernel's counter summed over the
    dispatches from the first picked launch on, divided by the number of
    picked launches (a binned aggregate that covers two launches' records --
    the paired aggregates -- is counted once, not once per launch)."""
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if r["Counter_Name"] == counter and any(h in name for h in HOT):
            h = next(h for h in HOT if h in name)
            short = h + name[name.index(h):].split("(")[0][len(h):]
            d[short][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    prim = sorted(i for name, per in d.items() if any(name.startswith(p) for p in PRIMARY) for i in per)
    launches = _pick(prim)
    first = launches[0]
    total, kernels = 0.0, {}
    for name, per in d.items():
        kernels[name] = sum(v for i, v in per.items() if i >= first) / len(launches)
        total += kernels[name]
    return total, kernels


def main():
    root, wl, rnd, out = sys.argv[1:5]
    f, fk = per_launch(f"{root}/pmc_{wl}_fetch/run_counter_collection.csv", "FETCH_SIZE")
    w, wk = per_launch(f"{root}/pmc_{wl}_write/run_counter_collection.csv", "WRITE_SIZE")
    spans = 10_000_000
    t = {"workload": wl, "spans_per_launch": spans, "algorithmic_bytes_per_launch": 44 * spans,
         "fetch_size_kb_per_launch": f, "write_size_kb_per_launch": w,
         "per_kernel_kb": {"fetch": fk, "write": wk},
         "hbm_bytes_per_launch": int((2 * f + w) * 1024),
         "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (tools/gpu_job.sh "
                   "pmc_<wl>_fetch / _write over tools/prof_driver.py: PROF_REPS launches of the 10M-span batch, each "
                   "a fresh trace-id variant; the last PMC_LAST averaged, else all but the first); FETCH_SIZE doubled per MI355X_MICROARCH.md gfx950 correction; KB=1024 B",
         "round": rnd}
    t["traffic_over_algorithmic"] = t["hbm_bytes_per_launch"] / t["algorithmic_bytes_per_launch"]
    json.dump(t, open(out, "w"), indent=1)
    print(json.dumps(t, indent=1))


if __name__ == "__main__":
    main()
