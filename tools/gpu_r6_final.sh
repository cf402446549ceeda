#!/bin/bash
# round 6 evidence on the current tree: the whole GPU suite and smoke(); the default bench line (configs[2]) and the
# configs[4] line, each with its rocprof kernel summary; HBM traffic of KL and KLM (FETCH_SIZE / WRITE_SIZE passes)
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06fin}
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests \
    > gpurun_out/${TAG}_suite.log 2>&1
rc=$?
tail -1 gpurun_out/${TAG}_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -40 gpurun_out/${TAG}_suite.log; exit 1; fi
grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_suite.log | head
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 400 python -u bench.py --config multisample > gpurun_out/${TAG}_ms.json 2> gpurun_out/${TAG}_ms.err || { tail -20 gpurun_out/${TAG}_ms.err; exit 1; }
python - <<PY
import json
for f in ("${TAG}_bench", "${TAG}_ms"):
    d = json.loads(open("gpurun_out/%s.json" % f).read().strip().splitlines()[-1])
    r = d["roofline"]; e = d.get("end_to_end") or {}
    print(f, "value %.4g" % d["value"], "step %.4f ms" % d["ms_per_step"], "kernel %.4f ms frac %.3f" % (r["kernel_avg_ms"], r["frac"]),
          "traffic", r.get("traffic"), "e2e %s" % e.get("wall_s"), "indels %s" % (e.get("indels") or {}).get("wall_s"),
          "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
for cfg in default multisample; do
  a=""; [ $cfg = multisample ] && a="--config multisample"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$cfg -o run --output-format csv -- python -u bench.py $a --no-cpu-baseline --no-cold --no-e2e \
      > gpurun_out/prof_${TAG}_$cfg.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}_$cfg.out; exit 1; }
  python tools/kstats.py gpurun_out/prof_${TAG}_$cfg gpurun_out/${TAG}_${cfg}_kernel_stats.csv > gpurun_out/${TAG}_${cfg}_kstats.txt
  head -5 gpurun_out/${TAG}_${cfg}_kstats.txt
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex "k_read_scan|k_scan_pop" -d gpurun_out/pmc_${TAG}_${cfg}_$ctr -o run --output-format csv \
        -- python -u bench.py $a --no-cpu-baseline --no-cold --no-e2e --steps 3 --warmup 1 > gpurun_out/pmc_${TAG}_${cfg}_$ctr.out 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_${cfg}_$ctr.out; exit 1; }
    python - <<PY
import csv, glob
f = glob.glob("gpurun_out/pmc_${TAG}_${cfg}_$ctr/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))]
print("$cfg $ctr per launch (raw, KB units)", sum(v) / len(v), "launches", len(v))
PY
  done
done
