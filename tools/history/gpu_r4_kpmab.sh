#!/bin/bash
# round 4: KPM register variants -- parity of the release build, configs[4] bench lines for release / 3 waves per SIMD /
# the previous commit, and KPM's WRITE_SIZE per launch (rocprofv3 PMC, its own pass) for release and 3 waves
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multisample.py tests/test_gpu_pool.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/kpmab_parity.log 2>&1 || { tail -20 gpurun_out/kpmab_parity.log; exit 1; }
tail -1 gpurun_out/kpmab_parity.log
B="python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 20 --warmup 4"
lib() { case $1 in A) echo $PWD/ngsepcore_amd/lib/libngsep_amd.so;; W3) echo $PWD/ab/kpm3/libngsep_amd.so;; P) echo $PWD/ab/prev/libngsep_amd.so;; esac; }
for v in A W3 P A W3 P; do
  NGSEP_TIME_POSTERIOR=1 NGSEP_LIB_PATH=$(lib $v) timeout -k 10 300 $B > gpurun_out/kpmab_$v.json 2> gpurun_out/kpmab_$v.err || { tail -5 gpurun_out/kpmab_$v.err; exit 1; }
  python - <<PY
import json
d = json.loads(open("gpurun_out/kpmab_$v.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("$v", "step %.3f ms" % d["ms_per_step"], "scan %.3f ms" % r["kernel_avg_ms"], "kpm", r["posterior_kernel_avg_ms"])
PY
done
for v in A W3; do
  NGSEP_LIB_PATH=$(lib $v) timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/kpmab_w_$v -o run --output-format csv -- \
      python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 3 --warmup 1 > gpurun_out/kpmab_w_$v.out 2>&1 || exit 1
  python - <<PY
import csv, glob
vals = []
for f in glob.glob("gpurun_out/kpmab_w_$v/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_posterior_multi" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE":
            vals.append(float(r["Counter_Value"]))
print("$v KPM WRITE_SIZE per launch %.1f MB over %d launches" % (sum(vals) / len(vals) * 1024 / 1e6, len(vals)) if vals else "$v no KPM rows")
PY
done
