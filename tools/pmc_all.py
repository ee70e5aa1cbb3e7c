"""Print every dispatch of nice:: kernels with its counters (rocprofv3 CSV)."""
import csv, collections, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.OrderedDict()
for r in rows:
    n = re.split(r"[(<]", r["Kernel_Name"])[0]
    if "nice::" not in n:
        continue
    d = agg.setdefault(r["Dispatch_Id"], {"name": n.replace("nice::", "")})
    d[r["Counter_Name"]] = float(r["Counter_Value"])
    d["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, d in agg.items():
    name = d.pop("name")
    print(f"{name:16s}", " ".join(f"{c}={v:.4g}" for c, v in sorted(d.items())))
