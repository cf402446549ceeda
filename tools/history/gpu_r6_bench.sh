#!/bin/bash
# round 6: the default bench line (configs[2]), the configs[4] line, the N = 2 rehearsal (gloo, both ranks on the
# one card) and a kernel trace of the deep-population tests (k_scan_pop<false>, KPM's scratch-column variants)
set -o pipefail
export NGSEP_SKIP_BUILD=1
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-r06c}
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
timeout -k 10 400 python -u bench.py --config multisample > gpurun_out/${TAG}_ms.json 2> gpurun_out/${TAG}_ms.err || { tail -20 gpurun_out/${TAG}_ms.err; exit 1; }
NGSEP_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 > gpurun_out/${TAG}_gloo2.json 2> gpurun_out/${TAG}_gloo2.err || { tail -20 gpurun_out/${TAG}_gloo2.err; exit 1; }
python - <<PY
import json
for f in ("${TAG}_bench", "${TAG}_ms", "${TAG}_gloo2"):
    d = json.loads(open("gpurun_out/%s.json" % f).read().strip().splitlines()[-1])
    r = d["roofline"]; e = d.get("end_to_end") or {}; sh = d.get("sharded_end_to_end") or {}
    print(f, "n", d["n_gpus"], "value %.4g" % d["value"], "step %.4f ms" % d["ms_per_step"], "kernel %.4f ms frac %.3f" % (r["kernel_avg_ms"], r["frac"]),
          "e2e %s %s" % (e.get("wall_s"), e.get("value")), "sharded %s" % sh.get("wall_s"), "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_deep -o run --output-format csv -- python -u -m pytest -x -q --timeout 250 -p no:cacheprovider tests/test_gpu_deep_population.py \
    > gpurun_out/prof_${TAG}_deep.out 2>&1 || { tail -5 gpurun_out/prof_${TAG}_deep.out; exit 1; }
python tools/kstats.py gpurun_out/prof_${TAG}_deep gpurun_out/${TAG}_deep_kernel_stats.csv > gpurun_out/${TAG}_deep_kstats.txt && grep -E "scan_pop|posterior_multi|stage_a" gpurun_out/${TAG}_deep_kstats.txt | head -20
