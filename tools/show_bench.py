import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "v*.json"))):
    try:
        d = json.load(open(f))
    except Exception as e:
        print(f, "unreadable", e); continue
    r = d["roofline"]
    print(f"{os.path.basename(f):10s} {d['value']/1e9:7.2f} Gspans/s  step {d['ms_per_step']*1e3:7.1f} us  kernel {r['kernel_ms']*1e3:7.1f} us  frac {r['frac']:.3f}  calls_ok {d['calls_check']}")
