#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs under a directory: mean per ingest launch
(excluding the first launch) for every counter, per label."""
import csv, glob, os, sys, collections


def _pick(ids):
    """Dispatches averaged: the last PMC_LAST of them (the settled regime of a
    fresh-variant run), else all but the first."""
    k = int(os.environ.get("PMC_LAST", "0"))
    return ids[-k:] if k else (ids[1:] or ids)

root = sys.argv[1]
out = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    label = os.path.relpath(f, root).split(os.sep)[0].rsplit(".", 1)[0]
    rows = [r for r in csv.DictReader(open(f)) if "ingest" in r.get("Kernel_Name", "")]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        per[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    for c, d in per.items():
        ids = _pick(sorted(d))
        out[label][c] = sum(d[i] for i in ids) / len(ids)
for label, d in out.items():
    print(label, " ".join(f"{k}={v:.4g}" for k, v in sorted(d.items())))
