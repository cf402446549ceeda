#!/bin/bash
# round 6: KLM without marks (count bound by exception count), block tables from each block's first reaching entry --
# the whole GPU suite, the configs[4] and configs[2] lines, KLM's instruction / traffic counters
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06d}
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests \
    > gpurun_out/${TAG}_suite.log 2>&1
rc=$?
tail -1 gpurun_out/${TAG}_suite.log
# a failing test does not stop the measurements below; a timeout, abort or fault does
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/${TAG}_suite.log; exit 1; fi
grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_suite.log | head
timeout -k 10 400 python -u bench.py --config multisample --no-cpu-baseline > gpurun_out/${TAG}_ms.json 2> gpurun_out/${TAG}_ms.err || { tail -20 gpurun_out/${TAG}_ms.err; exit 1; }
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python - <<PY
import json
for f in ("${TAG}_ms", "${TAG}_bench"):
    d = json.loads(open("gpurun_out/%s.json" % f).read().strip().splitlines()[-1])
    r = d["roofline"]; e = d.get("end_to_end") or {}
    print(f, "value %.4g" % d["value"], "step %.4f ms" % d["ms_per_step"], "kernel %.4f ms frac %.3f" % (r["kernel_avg_ms"], r["frac"]),
          "e2e %s" % e.get("wall_s"), "cand", d["config"]["candidates_per_gpu"], "exact", d["config"]["exact_sites_per_gpu"])
PY
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
pass fetch FETCH_SIZE && pass write WRITE_SIZE
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_ms -o run --output-format csv -- python -u bench.py --config multisample --no-cpu-baseline --no-cold --no-e2e \
    > gpurun_out/prof_${TAG}_ms.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}_ms.out; exit 1; }
python tools/kstats.py gpurun_out/prof_${TAG}_ms gpurun_out/${TAG}_ms_kernel_stats.csv | head -8
