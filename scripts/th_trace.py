"""Per-launch durations of the sequential FGS kernels from a rocprofv3 kernel-trace CSV, grouped by
position within a filter call (launch 0 = coefficient jobs, 1.. = passes).
python scripts/th_trace.py TRACE.csv [launches_per_call]"""
import csv
import statistics as st
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_fgs_th" in r["Kernel_Name"]]
per = int(sys.argv[2]) if len(sys.argv) > 2 else 7
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in rows]
groups = [d[i:i + per] for i in range(0, len(d) - per + 1, per)][3:]
print("launch  median_us  min  max")
for k in range(per):
    v = [g[k] for g in groups]
    print(f"{k:6d} {st.median(v):9.1f} {min(v):6.1f} {max(v):6.1f}")
print(f"total per call (median of sums): {st.median([sum(g) for g in groups]):.1f} us")
