#!/bin/bash
# round 5: KL's (k_read_scan, configs[2]) stall and instruction mix -- two SQ counter passes of their own
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05u}
B="python -u bench.py --no-cpu-baseline --no-cold --no-e2e --steps 3 --warmup 1"
pass() {   # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "k_read_scan|k_gather_kl|k_posterior" \
      -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- $B > gpurun_out/pmc_${TAG}_$name.out 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_$name.out; return 1; }
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
pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SMEM
