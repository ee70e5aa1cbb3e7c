"""Summarise rocprofv3 counter CSVs per kernel (the longest dispatch of each kernel)."""
import csv, collections, glob, sys
for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    agg = collections.OrderedDict()
    for r in rows:
        k = r["Kernel_Name"].split("(")[0]
        d = agg.setdefault((k, r["Dispatch_Id"]), {})
        d[r["Counter_Name"]] = float(r["Counter_Value"])
        d["_dur_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    last = {}
    for (k, _), d in agg.items():
        if k not in last or d["_dur_us"] >= last[k]["_dur_us"]:
            last[k] = d
    for k, d in last.items():
        if k.startswith("__amd"):
            continue
        print(k, " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
