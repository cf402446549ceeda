"""Per-launch HBM traffic of a kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

MI355X_MICROARCH.md "HBM": FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE undercounts streaming reads (the
guide gives x2 for 16-B/lane reads).  The factor per load width is measured (profiles/pmc_calibration.json, made by
tools/pmc_calib.py from tools/calib/pmc_calib.hip: 1 GiB read once at 4, 8 and 16 B per lane) and applied for the
kernel's streaming load width (LOAD_BYTES; default 16); WRITE_SIZE is taken as exact.  Usage:
  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTRING WORKLOAD_KEY OUT_JSON [LOAD_BYTES]
"""
import csv
import glob
import json
import os
import sys


def per_launch(d, kernel, counter):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None, len(vals)


def main():
    fdir, wdir, kernel, key, out = sys.argv[1:6]
    width = sys.argv[6] if len(sys.argv) > 6 else "16"
    cal_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_calibration.json")
    factor, source = 2.0, "MI355X_MICROARCH.md x2 (16-B reads)"
    if os.path.exists(cal_path):
        cal = json.load(open(cal_path))
        if width in cal.get("factor", {}):
            factor, source = cal["factor"][width], f"profiles/pmc_calibration.json, {width}-B loads"
    fetch, nf = per_launch(fdir, kernel, "FETCH_SIZE")
    write, nw = per_launch(wdir, kernel, "WRITE_SIZE")
    res = {"kernel": kernel, "workload_key": key, "launches": [nf, nw],
           "fetch_size_kib_raw": fetch, "write_size_kib": write}
    if fetch is not None and write is not None:
        res["bytes_per_launch"] = factor * fetch * 1024 + write * 1024
        res["fetch_factor"] = factor
        res["correction"] = f"FETCH_SIZE x {factor:.3f} ({source}), KiB -> bytes"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
