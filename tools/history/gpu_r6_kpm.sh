#!/bin/bash
# round 6: what KPM's second stage waits on -- block 0's phase stamps (DIAG build ngsepcore_amd/lib_dg, NGSEP_TIMING, the
# end-to-end leg's device_run_multi) and the SQ counters of k_posterior_multi / k_stage_a on configs[4]
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06kpm}
NGSEP_LIB_PATH=$PWD/ngsepcore_amd/lib_dg/libngsep_amd.so NGSEP_TIMING=1 NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --config multisample --no-cpu-baseline --no-cold --steps 3 --warmup 1 \
    > gpurun_out/${TAG}_timing.json 2> gpurun_out/${TAG}_timing.err || { tail -20 gpurun_out/${TAG}_timing.err; exit 1; }
grep -a "ngsep timing\|population" gpurun_out/${TAG}_timing.err | head -20
P="python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 3 --warmup 1"
pass() {   # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "k_posterior_multi|k_stage_a" \
      -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- $P > gpurun_out/pmc_${TAG}_$name.out 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_$name.out; return 1; }
  python - <<PY
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_${TAG}_$name/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print("$name", k, {c: "%.4g" % (sum(v) / len(v)) for c, v in d.items()})
PY
}
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS && \
pass sq2 SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH
