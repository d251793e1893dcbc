#!/usr/bin/env python3
"""profiles/traffic.json from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
tools/round_profile.sh: per ingest launch (first launch dropped), FETCH_SIZE
doubled per MI355X_MICROARCH.md's gfx950 correction, KB = 1024 B."""
import csv, json, sys, collections

def per_launch(path, counter):
    d = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if "ingest" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            d[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    ids = sorted(d)[1:] or sorted(d)
    return sum(d[i] for i in ids) / len(ids), len(ids)

root, out, rnd = sys.argv[1], sys.argv[2], sys.argv[3]
f, nf = per_launch(f"{root}/pmc_fetch/run_counter_collection.csv", "FETCH_SIZE")
w, nw = per_launch(f"{root}/pmc_write/run_counter_collection.csv", "WRITE_SIZE")
spans = 10_000_000
t = {"workload": "c2", "kernel": "ingest_v2_kernel<2,2,2,false,11,9,14,-1,true,1> (variant 16)",
     "spans_per_launch": spans, "algorithmic_bytes_per_launch": 44 * spans,
     "fetch_size_kb_per_launch": f, "write_size_kb_per_launch": w,
     "hbm_bytes_per_launch": int((2 * f + w) * 1024),
     "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes "
               "(tools/round_profile.sh, tools/prof_driver.py: 5 launches of the C2 10M-span "
               f"batch, first launch dropped: {nf} / {nw} launches averaged); FETCH_SIZE doubled "
               "per MI355X_MICROARCH.md gfx950 correction; KB=1024 B",
     "round": rnd}
json.dump(t, open(out, "w"), indent=1)
print(json.dumps(t, indent=1))
