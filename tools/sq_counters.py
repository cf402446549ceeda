"""Per-launch averages of rocprofv3 --pmc counters for kernels matching a substring.
Usage: python tools/sq_counters.py PMC_DIR KERNEL_SUBSTRING [KERNEL_SUBSTRING ...]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
for kern in sys.argv[2:]:
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(kern, {k: round(sum(v) / len(v)) for k, v in sorted(acc.items())})
