#!/bin/bash
# round 6: where KLM's fetched bytes go -- FETCH_SIZE of k_scan_pop<true> under diagnostic ablations (ngsepcore_amd/lib_dg, a DIAG build):
# 0 full, 262144 no exact bound, 524288 loads only (no counters, so no candidates)
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06r}
P="python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 3 --warmup 1"
for AB in 0 262144 524288; do
  NGSEP_LIB_PATH=$PWD/ngsepcore_amd/lib_dg/libngsep_amd.so NGSEP_ABLATE=$AB timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --kernel-include-regex "k_scan_pop" \
      -d gpurun_out/pmc_${TAG}_$AB -o run --output-format csv -- $P > gpurun_out/pmc_${TAG}_$AB.out 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_$AB.out; exit 1; }
  python - <<PY
import csv, glob
f = glob.glob("gpurun_out/pmc_${TAG}_$AB/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))]
t = glob.glob("gpurun_out/pmc_${TAG}_$AB/**/*kernel_trace.csv", recursive=True)[0]
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(t)) if "k_scan_pop" in r["Kernel_Name"]]
print("ablate $AB FETCH GB/launch %.3f" % (sum(v) / len(v) * 2 * 1024 / 1e9), "launches", len(v), "kernel us %.1f" % (sum(d) / len(d) / 1e3))
PY
done
