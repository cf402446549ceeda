"""Summarise a rocprofv3 --kernel-trace --stats directory: per-kernel average and the last step's timeline."""
import csv
import sys

d = sys.argv[1]
for r in csv.DictReader(open(f"{d}/run_kernel_stats.csv")):
    print(r["Name"][:48].ljust(48), r["Calls"].rjust(4), f"{float(r['AverageNs']) / 1000:9.1f} us", r["Percentage"])
rows = sorted(csv.DictReader(open(f"{d}/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
last = rows[-14:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"  {r['Kernel_Name'][:40].ljust(40)} start {(s - t0) / 1000:8.1f} us  dur {(e - s) / 1000:7.1f} us")
