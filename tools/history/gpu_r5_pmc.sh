#!/bin/bash
# round 5: KLM's (k_scan_pop) stall and instruction mix on configs[4] -- two SQ counter passes of their own, plus the
# HBM bytes (FETCH_SIZE / WRITE_SIZE passes) of KLM and the first-stage / second-stage KPM kernels
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r05p}
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_multisample.py \
    "tests/test_gpu_full_size.py::test_full_size_population_vcf_identical" tests/test_gpu_kpm_stages.py tests/test_gpu_known.py tests/test_gpu_indels.py \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for k in 1 2; do
NGSEP_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --config multisample --no-cold --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/${TAG}_ms$k.json 2> gpurun_out/${TAG}_ms$k.err || { tail -20 gpurun_out/${TAG}_ms$k.err; exit 1; }
python - <<PY
import json
d = json.loads(open("gpurun_out/${TAG}_ms$k.json").read().strip().splitlines()[-1])
print("ms step %.3f ms" % d["ms_per_step"], "population e2e %.3f s" % d["end_to_end"]["wall_s"])
PY
grep -E "population layout|layout [0-9.]+ ms, device upload|population: " gpurun_out/${TAG}_ms$k.err | tail -12
done
B="python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e --steps 3 --warmup 1"
pass() {   # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --kernel-include-regex "k_scan_pop|k_stage_a|k_posterior_multi" \
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
pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VMEM && \
pass fetch FETCH_SIZE && pass write WRITE_SIZE
