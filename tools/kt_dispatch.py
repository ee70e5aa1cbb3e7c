"""Per-dispatch durations (us) of nice:: kernels from a rocprofv3 kernel_trace.csv."""
import csv, re, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
seq = []
for r in rows:
    n = re.split(r"[(<]", r["Kernel_Name"])[0]
    if "nice::" not in n and "fill" not in r["Kernel_Name"].lower() and "memset" not in r["Kernel_Name"].lower():
        continue
    seq.append((int(r["Start_Timestamp"]), n.replace("nice::", ""), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
seq.sort()
for _, n, d in seq[-int(sys.argv[2]) if len(sys.argv) > 2 else 0:]:
    print(f"{n:40s} {d:10.1f}")
