#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 --kernel-trace CSV of a bench.py run
(tools/gpu_job.sh trace_<wl>): mean over every dispatch (what the --stats
summary averages: cold and settling launches included) and mean / median over
the last LAST dispatches of each hot kernel (the settled launches bench.py's
kernel_ms and timed steps cover).

  python tools/trace_summary.py <run_kernel_trace.csv> [LAST=16]"""
import collections
import csv
import json
import statistics
import sys

HOT = ("ingest_v2", "bt_scatter", "bt_aggregate", "expo_")


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        h = next((h for h in HOT if h in name), None)
        if h is None:
            continue
        short = name[name.index(h):].split("(")[0]
        d[short].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    out = {}
    # launch period: the first hot kernel of each launch (the one with the most
    # dispatches that starts earliest) -> start-to-start over the last LAST
    # launches, and their span / count (with overlapping kernels of
    # consecutive launches the period, not the sum of durations, is the rate)
    first = min(d, key=lambda k: (-len(d[k]), min(t for t, _ in d[k])))
    starts = sorted(t for t, _ in d[first])[-(last + 1):]
    if len(starts) > 1:
        out["launch_period_us_last%d" % last] = round((starts[-1] - starts[0]) / 1e3 / (len(starts) - 1), 2)
    for k, v in d.items():
        v.sort()
        us = [x for _, x in v]
        tail = us[-last:]
        out[k] = {"dispatches": len(us), "mean_us_all": round(statistics.mean(us), 2),
                  f"mean_us_last{last}": round(statistics.mean(tail), 2),
                  f"median_us_last{last}": round(statistics.median(tail), 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
