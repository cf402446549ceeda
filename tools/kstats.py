"""Summarise a rocprofv3 --kernel-trace --stats directory: per-kernel average and the last step's timeline."""
import csv
import glob
import os
import sys

d = sys.argv[1]
stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
trace = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
for r in csv.DictReader(open(stats[0])):
    print(r["Name"][:48].ljust(48), r["Calls"].rjust(4), f"{float(r['AverageNs']) / 1000:9.1f} us", r["Percentage"])
rows = sorted(csv.DictReader(open(trace[0])), key=lambda r: int(r["Start_Timestamp"]))
last = rows[-14:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"  {r['Kernel_Name'][:40].ljust(40)} start {(s - t0) / 1000:8.1f} us  dur {(e - s) / 1000:7.1f} us")
if len(sys.argv) > 2:   # copy the summary csv to a tracked path
    import shutil
    shutil.copy(stats[0], sys.argv[2])
