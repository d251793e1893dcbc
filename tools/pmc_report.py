#!/usr/bin/env python3
"""profiles/<name>.json from rocprofv3 --pmc passes of tools/gpu_job.sh
(pmc_<wl>_<set> over tools/prof_driver.py with fresh trace-id variants):
per hot-path kernel, each counter averaged over the last PMC_LAST (default 5)
dispatches -- the settled regime bench.py times -- plus per-span figures.

  python tools/pmc_report.py <out.json> <spans_per_launch> <label>=<job dir> ...

Per-span figures: SQ_INSTS_* are wave instructions, so x 64 / spans is the
lane view (instructions each span costs its lane); SQ_ACTIVE_INST_VALU /
SQ_WAVE_CYCLES x waves per SIMD is the VALU issue share of a SIMD; FETCH_SIZE
(KB) is doubled per MI355X_MICROARCH.md's gfx950 correction."""
import collections
import csv
import glob
import json
import os
import sys

HOT = ("ingest", "bt_scatter", "bt_aggregate", "expo_")


def kernel_short(name):
    for h in HOT:
        if h in name:
            rest = name[name.index(h):]
            return rest[: rest.index(">") + 1] if "<" in rest.split("(")[0] else rest.split("(")[0]
    return None


def collect(job):
    last = int(os.environ.get("PMC_LAST", "5"))
    out = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(job, "pmc_*", "*counter_collection.csv"))):
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        meta = {}
        for r in csv.DictReader(open(f)):
            k = kernel_short(r["Kernel_Name"])
            if k is None:
                continue
            per[(k, r["Counter_Name"])][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            meta[k] = {"vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]),
                       "lds": int(r["LDS_Block_Size"]), "wg": int(r["Workgroup_Size"])}
        for (k, c), d in per.items():
            ids = sorted(d)[-last:]
            out[k][c] = sum(d[i] for i in ids) / len(ids)
            out[k].setdefault("_meta", meta[k])
    return out


def main():
    dst, spans = sys.argv[1], int(sys.argv[2])
    rep = {"spans_per_launch": spans, "dispatches_averaged": int(os.environ.get("PMC_LAST", "5")),
           "method": "rocprofv3 --pmc, one counter set per pass (tools/gpu_job.sh pmc_<wl>_<set>), "
                     "tools/prof_driver.py: PROF_REPS launches of the 10M-span batch, each a fresh "
                     "trace-id variant; the last PMC_LAST dispatches of each kernel averaged",
           "runs": {}}
    for arg in sys.argv[3:]:
        label, job = arg.split("=", 1)
        ks = collect(job)
        for k, c in ks.items():
            d = {n: v for n, v in c.items()}
            w = spans / 64.0
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_BRANCH"):
                if n in c:
                    d[n + "_per_span_lane"] = c[n] / w
            if "SQ_ACTIVE_INST_VALU" in c and "SQ_WAVE_CYCLES" in c:
                d["valu_issue_share_per_wave"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
            if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c:
                d["lds_bank_conflict_share"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"] if c["SQ_LDS_IDX_ACTIVE"] else None
            if "FETCH_SIZE" in c:
                d["fetch_bytes_corrected"] = 2 * c["FETCH_SIZE"] * 1024
            if "WRITE_SIZE" in c:
                d["write_bytes"] = c["WRITE_SIZE"] * 1024
            rep["runs"].setdefault(label, {})[k] = d
    json.dump(rep, open(dst, "w"), indent=1)
    print(json.dumps(rep, indent=1)[:4000])


if __name__ == "__main__":
    main()
