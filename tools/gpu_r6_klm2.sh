#!/bin/bash
# round 6: KLM with reference-call / other-allele byte counters (no marks, no coverage differences) -- the GPU suite,
# then configs[4] A/B against the previous build (ngsepcore_amd/lib_base, NGSEP_LIB_PATH) and KLM's counters
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06k}
SUITE=${2:-all}
LIBS=${3:-"base new"}
PMCLIB=${4:-new}       # the build whose counters are collected
CFG=${5:-multisample}  # the bench configuration (chr20: the default, KL)
KREGEX=k_scan_pop; [ $CFG = chr20 ] && KREGEX=k_read_scan   # builds to alternate: base = ngsepcore_amd/lib_base, new = ngsepcore_amd/lib, X = ngsepcore_amd/lib_X
if [ "$SUITE" = none ]; then
  true
elif [ "$SUITE" = all ]; then
  timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests \
      > gpurun_out/${TAG}_suite.log 2>&1
else
  timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider -k "$SUITE" tests \
      > gpurun_out/${TAG}_suite.log 2>&1
fi
rc=$?
[ "$SUITE" = none ] || tail -1 gpurun_out/${TAG}_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/${TAG}_suite.log; exit 1; fi
grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_suite.log | head
B="python -u bench.py --config $CFG --no-cpu-baseline --no-cold --no-e2e --steps 40 --warmup 3"
for it in 1 2; do
  for v in $LIBS; do
    if [ $v = new ]; then L=ngsepcore_amd/lib/libngsep_amd.so; else L=ngsepcore_amd/lib_$v/libngsep_amd.so; fi
    NGSEP_LIB_PATH=$PWD/$L timeout -k 10 300 $B > gpurun_out/${TAG}_ab_${v}_$it.json 2> gpurun_out/${TAG}_ab_${v}_$it.err || { tail -5 gpurun_out/${TAG}_ab_${v}_$it.err; exit 1; }
    python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_ab_${v}_$it.json").read().strip().splitlines()[-1])
r = d["roofline"]
print("$v $it", "step %.4f ms" % d["ms_per_step"], "KLM %.4f ms frac %.3f" % (r["kernel_avg_ms"], r["frac"]), "KPM", r.get("posterior_kernel_avg_ms"),
      "cand", d["config"].get("candidates_per_gpu"), "exact", d["config"].get("exact_sites_per_gpu"), "walked", d["config"].get("exact_bound_columns_per_gpu"), "sites", d["config"].get("sites_called_per_gpu"))
PY
  done
done
P="python -u bench.py --config $CFG --no-cpu-baseline --no-cold --no-e2e --steps 3 --warmup 1"
if [ $PMCLIB != new ]; then export NGSEP_LIB_PATH=$PWD/ngsepcore_amd/lib_$PMCLIB/libngsep_amd.so; fi
pass() {   # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "$KREGEX" \
      -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- $P > gpurun_out/pmc_${TAG}_$name.out 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_$name.out; return 1; }
  python - <<PY
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_${TAG}_$name/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"][:28]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print("$name", k, {c: "%.4g" % (sum(v) / len(v)) for c, v in d.items()})
PY
}
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT && \
pass fetch FETCH_SIZE && pass write WRITE_SIZE
