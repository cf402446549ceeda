"""FETCH_SIZE calibration per load width from a rocprofv3 --pmc FETCH_SIZE run of tools/calib/pmc_calib (1 GiB
read once per launch at 4, 8 and 16 B per lane).  factor = bytes read / (FETCH_SIZE KiB x 1024): the multiplier
tools/pmc_traffic.py applies to a kernel whose streaming loads have that width.
Usage: python tools/pmc_calib.py ROCPROF_DIR OUT_JSON"""
import csv
import glob
import json
import os
import sys

WIDTH = {"k_read<unsigned int>": 4, "k_read<unsigned long>": 8, "k_read<uint4>": 16, "k_read<HIP_vector_type<unsigned int, 4u> >": 16}


def main():
    d, out = sys.argv[1:3]
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "FETCH_SIZE":
                continue
            name = r["Kernel_Name"]
            w = next((v for k, v in WIDTH.items() if k in name), None)
            if w is None:
                if "k_read" in name:
                    w = 16 if "uint4" in name or "vector" in name else (8 if "long" in name else 4)
                else:
                    continue
            vals.setdefault(w, []).append(float(r["Counter_Value"]))
    nbytes = 1 << 30
    res = {"bytes_per_launch": nbytes, "program": "tools/calib/pmc_calib.hip", "counter": "FETCH_SIZE (KiB)",
           "fetch_kib": {str(w): v for w, v in sorted(vals.items())},
           "factor": {str(w): nbytes / (1024.0 * (sum(v) / len(v))) for w, v in sorted(vals.items())}}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
